#!/bin/bash
# Round-6 session L: timeline of the two-wave k_qp_ric at 512 kites (both
# waves' hand-over points, tools/ric_timeline.py on the prof2 build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06l; mkdir -p $OUT
timeout -k 10 200 python tools/ric_timeline.py 512 40 > $OUT/ric_timeline_512.txt 2>&1 || { echo timeline failed; tail -20 $OUT/ric_timeline_512.txt; exit 1; }
cat $OUT/ric_timeline_512.txt
