#!/bin/bash
# Round-6 session R: config 5 evidence at HEAD (the two-wave k_qp_ric with
# Sigma first and the prefetched stage operands): tools/gpu_round.sh at 4096
# and at 512 kites per GPU (bench line, kernel trace, HBM and SQ passes).
# The N = 20 kernels are unchanged since session J (profiles/r06j_*).
set -o pipefail
export TMPDIR=/tmp
SKIP_TESTS=1 bash tools/gpu_round.sh r06rn40 0 "--horizon 40 --ekf" || exit 1
SKIP_TESTS=1 bash tools/gpu_round.sh r06rn40b512 0 "--horizon 40 --ekf --batch 512" || exit 1
for t in r06rn40 r06rn40b512; do python -c "import json;d=json.load(open('gpurun_out/$t/bench.json'));print('$t',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'],d['roofline']['frac'])"; done
