#!/bin/bash
# Round-6 session T: the factor stage's theta-coupling shuffles issued before
# the 4 x 4 Cholesky (tools/experiments/ric_factor_early_shuffles.patch, built
# as lib/ab/libkite_tb.so): bitwise two-wave test on it, latency at 512 and
# config 5 at 4096 against the product build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06t; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
CUR=$PWD/openkite_amd/lib/libkite_nmpc.so
KITE_NMPC_LIB=$AB/libkite_tb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave_tb.log 2>&1 || { echo "two-wave test failed"; tail -40 $OUT/pytest_two_wave_tb.log; exit 1; }
tail -1 $OUT/pytest_two_wave_tb.log
for v in cur tb cur tb; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
for v in cur tb; do
  if [ $v = cur ]; then L=$CUR; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 300 python bench.py --horizon 40 --ekf --no-cpu-baseline > $OUT/bench5_4096_$v.json 2> $OUT/bench5_4096_$v.err || { echo bench $v failed; tail $OUT/bench5_4096_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench5_4096_$v.json'));print('config5-4096 $v',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
done
