#!/bin/bash
# Round-6 session Q: the two-wave k_qp_ric with the factor stage's LDS
# operands prefetched and the factorisation started on Sigma (the product
# build): bitwise two-wave test, the GPU suite, config 5 at 512 and 4096,
# the timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k two_wave --timeout 120 --timeout-method thread > $OUT/pytest_two_wave.log 2>&1 || { echo "two-wave test failed"; tail -40 $OUT/pytest_two_wave.log; exit 1; }
tail -1 $OUT/pytest_two_wave.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --batch 512 --horizon 40 --ekf --no-cpu-baseline > $OUT/bench5_512.json 2> $OUT/bench5_512.err || { echo bench5 512 failed; tail $OUT/bench5_512.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench5_512.json'));print('config5-512',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
timeout -k 10 300 python bench.py --horizon 40 --ekf --no-cpu-baseline > $OUT/bench5_4096.json 2> $OUT/bench5_4096.err || { echo bench5 failed; tail $OUT/bench5_4096.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench5_4096.json'));print('config5-4096',d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"
timeout -k 10 200 python tools/ric_timeline.py 512 40 > $OUT/ric_timeline_512.txt 2>&1 || { echo timeline failed; tail -20 $OUT/ric_timeline_512.txt; exit 1; }
tail -19 $OUT/ric_timeline_512.txt
