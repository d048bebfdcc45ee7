#!/bin/bash
# A/B of library builds on the N = 40 workload (BASELINE config 5 horizon, no EKF):
#   bash tools/ab_bench40.sh TAG LIB1 [LIB2 ...]
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  v=$(basename $lib .so)
  KITE_NMPC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --horizon 40 --no-cpu-baseline \
      > gpurun_out/$TAG/bench40_$v.json 2>gpurun_out/$TAG/bench40_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/$TAG/bench40_$v.json'));print('$v',d['value'],d['kernel_ms_per_step'],d['qp_mean_iterations'])"
done
