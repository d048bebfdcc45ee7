#!/bin/bash
# Round-6 session M: k_qp_ric two-wave hand-overs without the lgkmcnt(0)
# wait before each counter store (LDS executes one wave's DS instructions in
# order): the bitwise test on that build, latency against the committed kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06m; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
KITE_NMPC_LIB=$AB/libkite_nowait.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave_nowait.log 2>&1 || { echo "two-wave test failed"; tail -30 $OUT/pytest_two_wave_nowait.log; exit 1; }
tail -1 $OUT/pytest_two_wave_nowait.log
for v in kff nowait kff nowait; do
  KITE_NMPC_LIB=$AB/libkite_$v.so timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
