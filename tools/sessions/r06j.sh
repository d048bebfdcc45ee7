#!/bin/bash
# Round-6 session J: final evidence at HEAD -- the GPU suite, the headline
# bench line (+ CPU baseline), its rocprofv3 kernel trace and HBM / SQ passes
# (tools/gpu_round.sh), the same for config 5 at 4096 and at 512 kites per
# GPU (the two-wave k_qp_ric), and the k_qp_tiled phase profile.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r06j || exit 1
SKIP_TESTS=1 bash tools/gpu_round.sh r06jn40 0 "--horizon 40 --ekf" || exit 1
SKIP_TESTS=1 bash tools/gpu_round.sh r06jn40b512 0 "--horizon 40 --ekf --batch 512" || exit 1
timeout -k 10 200 python tools/qp_phase_profile.py 4096 > gpurun_out/r06j/qp_phase_profile.txt 2>&1 || { echo qp prof failed; exit 1; }
tail -14 gpurun_out/r06j/qp_phase_profile.txt
