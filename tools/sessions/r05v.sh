#!/bin/bash
# Round-5 session V: config 4's per-GPU slice (fp32 sensitivities) and config
# 2 (batch 256: the sensitivity kernel's interval integrations/s) at HEAD.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/config3.json 2> $OUT/config3.err || { echo "config3 failed"; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --fp32-sens > $OUT/config4.json 2> $OUT/config4.err || { echo "config4 failed"; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 256 > $OUT/config2.json 2> $OUT/config2.err || { echo "config2 failed"; exit 1; }
echo done
