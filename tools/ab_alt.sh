#!/bin/bash
# Alternating A/B bench of library builds on the GPU box (R rounds, each lib once
# per round): bash tools/ab_alt.sh TAG R LIB1 LIB2 [...] -- extra bench args after --
TAG=$1; R=$2; shift 2
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "$1" == "--" ] && shift
mkdir -p gpurun_out/$TAG
for r in $(seq 1 $R); do
  for lib in "${LIBS[@]}"; do
    v=$(basename $lib .so)
    KITE_NMPC_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" \
        > gpurun_out/$TAG/bench_${v}_$r.json 2>gpurun_out/$TAG/bench_${v}_$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_${v}_$r.json'));print('$v',$r,d['value'],d['kernel_ms_per_step'],d['qp_mean_iterations'])"
  done
done
