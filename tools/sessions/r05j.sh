#!/bin/bash
# Round-5 session J: every-node state bounds (VERDICT r04 Missing #2) -- the
# multiple-shooting QP at N = 20 with the reference box and with a binding
# |omega_i| <= 3 box, beside the condensed QP's lazy rows on the same box; a
# fresh config-3 and config-5 bench with kernel traces at HEAD.
set -o pipefail
OUT=gpurun_out/r05j; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests/test_state_bounds.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_bounds.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_bounds.log; exit 1; }
tail -2 $OUT/pytest_bounds.log
timeout -k 10 200 $B --qp-kernel 3 > $OUT/n20_ric.json 2> $OUT/n20_ric.err || { echo "n20 ric failed"; exit 1; }
timeout -k 10 200 $B --rate-bound 3 > $OUT/n20_lazy_w3.json 2> $OUT/n20_lazy_w3.err || { echo "lazy w3 failed"; exit 1; }
timeout -k 10 200 $B --rate-bound 3 --qp-kernel 3 > $OUT/n20_ric_w3.json 2> $OUT/n20_ric_w3.err || { echo "ric w3 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_ric_w3 -o ktrace --output-format csv -- $B --rate-bound 3 --qp-kernel 3 > $OUT/prof_ric_w3.log 2>&1 || { echo "prof ric w3 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_lazy_w3 -o ktrace --output-format csv -- $B --rate-bound 3 > $OUT/prof_lazy_w3.log 2>&1 || { echo "prof lazy w3 failed"; exit 1; }
timeout -k 10 200 $B --horizon 40 --ekf > $OUT/config5.json 2> $OUT/config5.err || { echo "config5 failed"; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
echo done
