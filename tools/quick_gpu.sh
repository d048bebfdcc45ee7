#!/bin/bash
# Quick GPU check: parity suite + a short bench (no CPU baseline).
# Usage (GPU box, repo root): bash tools/quick_gpu.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-q}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
