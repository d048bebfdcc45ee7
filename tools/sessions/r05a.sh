#!/bin/bash
# Round-5 session A (GPU box, repo root): the N = 40 frozen-QP dump (VERDICT
# r04 item 1), config 5 at its per-GPU shape (512 kites, item 4), the
# single-kite latency decomposition (item 7) and kernel traces of the
# disturbed loops (item 5: wind sweep 0.5, measurement noise 1).
set -o pipefail
OUT=gpurun_out/r05a; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python -u tools/n40_frozen_dump.py $OUT > $OUT/dump.log 2>&1 || { echo "dump failed"; exit 1; }
timeout -k 10 120 python -u tools/latency_probe.py 300 > $OUT/latency.json 2> $OUT/latency.err || { echo "latency failed"; exit 1; }
timeout -k 10 200 $B --batch 512 --horizon 40 --ekf > $OUT/c5_512.json 2> $OUT/c5_512.err || { echo "c5 512 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/prof512 -o ktrace --output-format csv -- $B --batch 512 --horizon 40 --ekf > $OUT/prof512.log 2>&1 || { echo "prof512 failed"; exit 1; }
timeout -k 10 200 $B > $OUT/nominal.json 2> $OUT/nominal.err || { echo "nominal failed"; exit 1; }
timeout -k 10 200 $B --wind-sweep 0.5 > $OUT/wind05.json 2> $OUT/wind05.err || { echo "wind failed"; exit 1; }
timeout -k 10 200 $B --meas-noise 1 > $OUT/noise1.json 2> $OUT/noise1.err || { echo "noise failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profwind -o ktrace --output-format csv -- $B --wind-sweep 0.5 > $OUT/profwind.log 2>&1 || { echo "profwind failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profnoise -o ktrace --output-format csv -- $B --meas-noise 1 > $OUT/profnoise.log 2>&1 || { echo "profnoise failed"; exit 1; }
echo done
