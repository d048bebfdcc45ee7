#!/bin/bash
# Round-5 session O: timing events without the system-scope fence -- the GPU
# suite, three bench lines, a kernel trace (inter-kernel gaps).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05o; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { echo "bench failed"; exit 1; }; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o ktrace --output-format csv -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
