#!/bin/bash
# Round-6 session F: two-wave k_qp_ric, closed-loop forward sweeps (+ the
# factorisation overlapping the residual pass): the two-wave test, latency
# probes (single wave, closed-loop only, + overlap), then the full GPU suite
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06f}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -30 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
KITE_RIC_WAVES=1 timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_w1.txt 2>&1 || { echo probe1 failed; exit 1; }
tail -1 $OUT/latency512_w1.txt
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/libkite_acl.so timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_acl.txt 2>&1 || { echo probe-acl failed; exit 1; }
tail -1 $OUT/latency512_acl.txt
timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_w2.txt 2>&1 || { echo probe2 failed; exit 1; }
tail -1 $OUT/latency512_w2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
