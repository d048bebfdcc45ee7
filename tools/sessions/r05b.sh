#!/bin/bash
# Round-5 session B: main-QP-kernel duration vs batch size at N = 20 and 40
# (kernel traces; tools/qp_scaling_probe.py); the N = 40 frozen-QP dump and
# parity tests after k_qp's equilibration.
set -o pipefail
OUT=gpurun_out/r05b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/n40_frozen_dump.py $OUT > $OUT/dump.log 2>&1 || { echo "dump failed"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "n40_qp_kernels or condensed_horizons or qp_kernels_vs_oracle or iteration_sum" > $OUT/pytest_qp.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_qp.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/scal20 -o kt --output-format csv -- python tools/qp_scaling_probe.py 20 10 > $OUT/scal20.log 2>&1 || { echo "scal20 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/scal40 -o kt --output-format csv -- python tools/qp_scaling_probe.py 40 6 1 64 256 512 1024 2048 4096 > $OUT/scal40.log 2>&1 || { echo "scal40 failed"; exit 1; }
echo done
