#!/bin/bash
# Round-5 session P: sampled timing ring (ABI 7) -- timing / ABI GPU tests,
# three bench lines, a kernel trace of the same command.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "timing or captured or abi" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { echo "bench failed"; exit 1; }; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o ktrace --output-format csv -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
