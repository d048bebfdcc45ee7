#!/bin/bash
# Round-5 session AF: the max-ilp machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp)
# on rti_kernels.hip (config 3) and on ric_kernels.hip (config 5) vs HEAD --
# kernel traces and alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05af; mkdir -p $OUT
bash tools/trace_ab.sh r05af openkite_amd/lib/ab/head.so openkite_amd/lib/ab/schedilp.so 2>&1 | grep -E "==|k_qp_tiled |k_condense20|k_rk4|k_expand20|k_prologue_warm" || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05af 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/schedilp.so || { echo "ab failed"; exit 1; }
bash tools/ab_alt.sh r05af/n40 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/schedilp_ric.so -- --horizon 40 --ekf || { echo "ab40 failed"; exit 1; }
echo done
