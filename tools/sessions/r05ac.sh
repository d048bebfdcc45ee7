#!/bin/bash
# Round-5 session AC: single-kite latency -- latency probe
# of HEAD and of the branch-free condensing stores (cstore), and a kernel trace
# of the batch-1 probe (per-kernel device time of one kite).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ac; mkdir -p $OUT
for v in head cstore head cstore; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/$v.so timeout -k 10 200 python tools/latency_probe.py 300 20 1 >> $OUT/lat_$v.jsonl 2> $OUT/lat_$v.err || { echo "probe $v failed"; exit 1; }
  tail -1 $OUT/lat_$v.jsonl
done
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/prof -o ktrace --output-format csv -- python tools/latency_probe.py 100 20 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $OUT/prof -name "*kernel_trace.csv" -exec cp {} $OUT/trace_b1.csv \;
rm -rf $OUT/prof
python tools/trace_means.py $OUT/trace_b1.csv
echo done
