#!/bin/bash
# A/B of the QP formulations on one GPU: Riccati MS QP (default) vs condensed tiled QP,
# N = 20 and N = 40 + EKF, plus a kernel trace of the default N = 20 bench.
# Usage (GPU box, repo root): bash tools/ric_bench.sh TAG
set -o pipefail
TAG=${1:-rb}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b20_ric.json 2> $OUT/b20_ric.err || { echo "bench 20 ric failed"; tail $OUT/b20_ric.err; exit 1; }
cat $OUT/b20_ric.json
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --qp-kernel 2 > $OUT/b20_tiled.json 2> $OUT/b20_tiled.err || { echo "bench 20 tiled failed"; exit 1; }
cat $OUT/b20_tiled.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --horizon 40 --ekf > $OUT/b40_ric.json 2> $OUT/b40_ric.err || { echo "bench 40 ric failed"; tail $OUT/b40_ric.err; exit 1; }
cat $OUT/b40_ric.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv
