#!/bin/bash
# GPU suite on the product library, then the config-5 bench line, an N = 40
# kernel trace and an N = 40 A/B of candidate builds:
#   bash tools/n40_check.sh TAG [LIB ...]
set -o pipefail
TAG=${1:-n40}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --horizon 40 --ekf --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench failed"; tail $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof40 -o kt --output-format csv -- python bench.py --steps 30 --warmup 3 --horizon 40 --ekf --no-cpu-baseline > $OUT/prof40.log 2>&1 || { echo "rocprof failed"; exit 1; }
[ $# -gt 0 ] && bash tools/ab_bench40.sh $TAG "$@"
echo done
