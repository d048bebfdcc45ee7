#!/bin/bash
# Round-5 session K: the undamped every-node mode (qp_kernel 3, qp_lm 0, soft
# weight 1e6) at N = 20 -- its GPU parity test and its bench line, nominal and
# with the binding |omega_i| <= 3 box, plus a kernel trace.
set -o pipefail
OUT=gpurun_out/r05k; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
E="--qp-kernel 3 --qp-lm 0 --soft-weight 1e6"
timeout -k 10 600 python -u -m pytest tests/test_state_bounds.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_bounds.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_bounds.log; exit 1; }
tail -2 $OUT/pytest_bounds.log
timeout -k 10 200 $B $E > $OUT/n20_exact.json 2> $OUT/n20_exact.err || { echo "exact failed"; exit 1; }
timeout -k 10 200 $B $E --rate-bound 3 > $OUT/n20_exact_w3.json 2> $OUT/n20_exact_w3.err || { echo "exact w3 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_exact -o ktrace --output-format csv -- $B $E > $OUT/prof_exact.log 2>&1 || { echo "prof exact failed"; exit 1; }
echo done
