#!/bin/bash
# Round-6 session K: the two-wave k_qp_ric with the feedback K and the
# corrector feed-forward moved off the sweep wave (bitwise test, latency
# against the committed pipelined kernel, the GPU suite).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06k; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -30 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
for v in pipe cur pipe cur; do
  if [ $v = cur ]; then L=$PWD/openkite_amd/lib/libkite_nmpc.so; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
