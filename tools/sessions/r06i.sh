#!/bin/bash
# Round-6 session I: the other bench lines at HEAD in one session -- nominal,
# disturbed (measurement noise 1, wind <= 0.5 m/s), config 4 (fp32
# sensitivities), config 2 (256 kites), every-node state bounds -- plus the
# batch-1 latency probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06i; mkdir -p $OUT
B="python bench.py --no-cpu-baseline"
run() { local tag=$1; shift; timeout -k 10 200 $B "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'])"; }
run nominal
run noise1 --meas-noise 1
run wind05 --wind-sweep 0.5
run nominal_b
run config4 --fp32-sens
run config2 --batch 256
run every_node --qp-kernel 3 --qp-lm 0 --soft-weight 1e6
timeout -k 10 200 python tools/latency_probe.py > $OUT/latency_batch1.txt 2>&1 || { echo latency failed; tail $OUT/latency_batch1.txt; exit 1; }
tail -3 $OUT/latency_batch1.txt
