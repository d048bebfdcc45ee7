#!/bin/bash
# One GPU session: parity tests, benches, rocprofv3 kernel stats + HBM PMC passes
# + an SQ pass (wave-cycle breakdown, fp64 MFMA instructions / busy cycles).
# The kernel-trace run uses the bench line's own arguments (--steps 30 --warmup 3),
# so its steady-state means (profiles/<tag>_kernel_steady.json) compare 1:1.
# Usage (on the GPU box, repo root): bash tools/gpu_round.sh TAG [QP_KERNEL [EXTRA_BENCH_ARGS]]
# (SKIP_TESTS=1 skips the parity suite, e.g. for a second configuration)
set -o pipefail
TAG=${1:-r01}; QK=${2:-0}; EXTRA=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-seconds 10 --qp-kernel $QK $EXTRA > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof -o ktrace --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --qp-kernel $QK $EXTRA > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o fetch --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --qp-kernel $QK $EXTRA > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o write --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --qp-kernel $QK $EXTRA > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $OUT/pmc_sq -o sq --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --qp-kernel $QK $EXTRA > $OUT/pmc_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
KITE_PROF_WARMUP=3 timeout -k 10 60 python tools/pmc_summary.py $OUT $TAG > $OUT/pmc_summary.log 2>&1 && cp profiles/${TAG}_* $OUT/ ; echo done
