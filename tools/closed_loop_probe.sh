#!/bin/bash
# closed-loop behaviour of the fleet driver under a few settings (summary every 10 steps)
set -o pipefail
mkdir -p gpurun_out/cl
for cfg in "0.1 3" "0.0 3" "0.0 1" "0.1 1"; do
  set -- $cfg
  timeout -k 10 120 ./openkite_amd/bin/nmpf_driver --batch 64 --steps 120 --delay $1 --ctrl-every $2 --sim-dt 0.02 --trace 1 --out gpurun_out/cl/d$1_k$2.jsonl || exit 1
done
