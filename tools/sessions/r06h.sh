#!/bin/bash
# Round-6 session H: the pipelined two-wave k_qp_ric + the factorisation
# overlapping the residual pass (bitwise test, latency against the committed
# pipelined kernel), k_qp_tiled's recursive residuals (the GPU suite), and the
# headline bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06h; mkdir -p $OUT
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
timeout -k 10 300 python bench.py --batch 512 --horizon 40 --ekf --no-cpu-baseline > $OUT/bench_config5_512.json 2> $OUT/bench_config5_512.err || { echo bench5 failed; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_config5_512.json'));print('config5-512',d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
timeout -k 10 300 python bench.py --horizon 40 --ekf --no-cpu-baseline > $OUT/bench_config5_4096.json 2> $OUT/bench_config5_4096.err || { echo bench5 4096 failed; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_config5_4096.json'));print('config5-4096',d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('headline 20+5',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'],d['roofline']['frac'],d['gpu_latency_batch1']['median_ms'] if d.get('gpu_latency_batch1') else None)"
