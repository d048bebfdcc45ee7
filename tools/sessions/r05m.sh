#!/bin/bash
# Round-5 session M: full evidence at HEAD (DPP condensing) + an LDS counter
# pass per kernel at N = 20 and at config 5 (which kernels are LDS-bound).
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r05m || exit 1
OUT=gpurun_out/r05m; B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
L="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $L -T -d $OUT/pmc_lds -o lds --output-format csv -- $B > $OUT/pmc_lds.log 2>&1 || { echo "pmc lds failed"; tail -5 $OUT/pmc_lds.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $L -T -d $OUT/pmc_lds40 -o lds --output-format csv -- $B --horizon 40 --ekf > $OUT/pmc_lds40.log 2>&1 || { echo "pmc lds40 failed"; tail -5 $OUT/pmc_lds40.log; exit 1; }
echo done
