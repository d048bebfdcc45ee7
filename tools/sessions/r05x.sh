#!/bin/bash
# Round-5 session X: k_expand20 commit with batched loads (no load behind a
# store to the same array) vs the prologue split -- bitwise outputs, GPU
# suite, alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05x; mkdir -p $OUT
for N in 20 40; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/light.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base$N.npz - 256 60 $N > $OUT/out_base$N.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base$N.log; exit 1; }
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/expand.so timeout -k 10 200 python tools/ab_outputs.py $OUT/light$N.npz $OUT/base$N.npz 256 60 $N > $OUT/out_light$N.log 2>&1 || { echo "light outputs failed"; cat $OUT/out_light$N.log; exit 1; }
  tail -1 $OUT/out_light$N.log
  rm -f $OUT/*.npz
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
bash tools/ab_alt.sh r05x 3 openkite_amd/lib/ab/light.so openkite_amd/lib/ab/expand.so || { echo "ab failed"; exit 1; }

timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/prof
echo done
