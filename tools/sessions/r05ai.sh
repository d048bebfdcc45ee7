#!/bin/bash
# Round-5 session AI: instruction-cache counters (SQC_ICACHE_*) of the hot
# kernels, config 3 and config 5 (separate --pmc passes, kernel trace only).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ai; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || { echo "list failed"; exit 1; }
grep -i "ICACHE\|SQC_" $OUT/list_avail.txt | head -40
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -T -d $OUT/ic3 -o ic --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/ic3.log 2>&1 || { echo "pmc c3 failed"; tail $OUT/ic3.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -T -d $OUT/ic5 -o ic --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --horizon 40 --ekf > $OUT/ic5.log 2>&1 || { echo "pmc c5 failed"; tail $OUT/ic5.log; exit 1; }
find $OUT/ic3 -name "*counter_collection.csv" -exec cp {} $OUT/ic3.csv \;
find $OUT/ic5 -name "*counter_collection.csv" -exec cp {} $OUT/ic5.csv \;
rm -rf $OUT/ic3 $OUT/ic5
echo done
