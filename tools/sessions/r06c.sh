#!/bin/bash
# Round-6 session C: the two-wave k_qp_ric -- bitwise test against the single
# wave, the full GPU suite (every N = 40 test at B <= 512 now runs two waves),
# and the config-5 per-GPU latency probe for both variants in one session
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06c}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -30 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
KITE_RIC_WAVES=1 timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_w1.txt 2>&1 || { echo probe1 failed; exit 1; }
tail -1 $OUT/latency512_w1.txt
timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_w2.txt 2>&1 || { echo probe2 failed; exit 1; }
tail -1 $OUT/latency512_w2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
