#!/bin/bash
# Round-5 session T: the disturbed loops at HEAD next to the nominal one (same
# session), with kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05t; mkdir -p $OUT
B="python bench.py --no-cpu-baseline"
timeout -k 10 200 $B > $OUT/nominal.json 2> $OUT/nominal.err || { echo "nominal failed"; exit 1; }
timeout -k 10 200 $B --wind-sweep 0.5 > $OUT/wind05.json 2> $OUT/wind05.err || { echo "wind failed"; exit 1; }
timeout -k 10 200 $B --meas-noise 1 > $OUT/noise1.json 2> $OUT/noise1.err || { echo "noise failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profwind -o ktrace --output-format csv -- $B --wind-sweep 0.5 > $OUT/profwind.log 2>&1 || { echo "profwind failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profnoise -o ktrace --output-format csv -- $B --meas-noise 1 > $OUT/profnoise.log 2>&1 || { echo "profnoise failed"; exit 1; }
echo done
