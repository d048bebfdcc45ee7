#!/bin/bash
# Round-5 session AO: the other bench lines at final HEAD in one session --
# nominal, disturbed (wind <= 0.5 m/s, measurement noise 1), config 4 (fp32
# sensitivities), config 2 (256 kites), config 5 at 512 kites per GPU, and the
# every-node state-bound configuration.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ao; mkdir -p $OUT
B="python bench.py --no-cpu-baseline"
run() { local tag=$1; shift; timeout -k 10 200 $B "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['kernel_ms_per_step'],d['qp_mean_iterations'])"; }
run nominal
run wind05 --wind-sweep 0.5
run noise1 --meas-noise 1
run config4 --fp32-sens
run config2 --batch 256
run config5_512 --horizon 40 --ekf --batch 512
run every_node --qp-kernel 3 --qp-lm 0 --soft-weight 1e6
echo done
