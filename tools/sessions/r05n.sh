#!/bin/bash
# Round-5 session N: the new GPU tests (collocation golden), config-5 evidence
# at HEAD (trace + HBM / SQ passes), the QP phase profile of the HEAD kernels.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05n; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_colloc.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_colloc.log 2>&1 || { echo "pytest colloc failed"; tail -20 $OUT/pytest_colloc.log; exit 1; }
tail -1 $OUT/pytest_colloc.log
SKIP_TESTS=1 bash tools/gpu_round.sh r05n40 0 "--horizon 40 --ekf" || { echo "config5 round failed"; exit 1; }
timeout -k 10 300 python tools/qp_phase_profile.py 4096 20 > $OUT/qp_phase_profile.txt 2>&1 || { echo "phase profile failed"; exit 1; }
echo done
