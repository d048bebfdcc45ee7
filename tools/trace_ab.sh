#!/bin/bash
# Kernel-trace A/B of library builds: bash tools/trace_ab.sh TAG LIB1 [LIB2 ...]
# (rocprofv3 --kernel-trace of a 30-step bench per library; per-kernel steady
# means printed by tools/trace_means.py)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for lib in "$@"; do
  v=$(basename $lib .so)
  KITE_NMPC_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/prof_$v -o ktrace --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/prof_$v.log 2>&1 || { echo "rocprof $v failed"; exit 1; }
  find $OUT/prof_$v -name "*kernel_trace.csv" -exec cp {} $OUT/trace_$v.csv \;
  rm -rf $OUT/prof_$v
  echo "== $v"; python tools/trace_means.py $OUT/trace_$v.csv || exit 1
done
