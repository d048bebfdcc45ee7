#!/bin/bash
# Round-6 session P (second run: K in LDS for the du fill): closed-loop forward sweeps in the two-wave k_qp_ric --
# clA: du on the sweep wave beside the chain (the corrector's offsets with a
# Z ring on the elementwise wave), cur: du filled in by the elementwise wave --
# against pfsig (open-loop forward).  Two-wave test, latency at 512, timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06p3; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
CUR=$PWD/openkite_amd/lib/libkite_nmpc.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -40 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
for v in pfsig clA cur pfsig clA cur; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
timeout -k 10 200 python tools/ric_timeline.py 512 40 > $OUT/ric_timeline_512.txt 2>&1 || { echo timeline failed; tail -20 $OUT/ric_timeline_512.txt; exit 1; }
tail -19 $OUT/ric_timeline_512.txt
