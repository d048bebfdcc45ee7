#!/bin/bash
# Round-6 session S: Sigma handed to the factorisation slot by slot (the
# convergence test's first half computed ahead of it): bitwise two-wave test,
# latency at 512 against the committed build (pfsig), the timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06s2; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
CUR=$PWD/openkite_amd/lib/libkite_nmpc.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -40 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
for v in pfsig cur pfsig cur; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
timeout -k 10 200 python tools/ric_timeline.py 512 40 > $OUT/ric_timeline_512.txt 2>&1 || { echo timeline failed; tail -20 $OUT/ric_timeline_512.txt; exit 1; }
tail -19 $OUT/ric_timeline_512.txt
