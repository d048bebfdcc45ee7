#!/bin/bash
# A/B bench of library builds on the GPU box: bash tools/ab_bench.sh TAG LIB1 [LIB2 ...]
# (each LIB a path to a libkite_nmpc.so build; bench.py loads it via KITE_NMPC_LIB)
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  v=$(basename $lib .so)
  KITE_NMPC_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline \
      > gpurun_out/$TAG/bench_$v.json 2>gpurun_out/$TAG/bench_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$v.json'));print('$v',d['value'],d['kernel_ms_per_step'],d['qp_mean_iterations'])"
done
