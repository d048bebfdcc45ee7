#!/bin/bash
# Round-6 session N: the factor stage's LDS operands prefetched one stage
# ahead and the factorisation started on Sigma before the rest of the residual
# pass (bitwise two-wave test, latency at 512 against the previous build,
# config 5 at 4096 for both, the timeline of the new build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06n; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
CUR=$PWD/openkite_amd/lib/libkite_nmpc.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -30 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
for v in nowait cur nowait cur; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
for v in nowait cur; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 300 python bench.py --horizon 40 --ekf --no-cpu-baseline > $OUT/bench5_4096_$v.json 2> $OUT/bench5_4096_$v.err || { echo bench $v failed; tail $OUT/bench5_4096_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench5_4096_$v.json'));print('config5-4096 $v',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
done
timeout -k 10 200 python tools/ric_timeline.py 512 40 > $OUT/ric_timeline_512.txt 2>&1 || { echo timeline failed; tail -20 $OUT/ric_timeline_512.txt; exit 1; }
tail -19 $OUT/ric_timeline_512.txt
