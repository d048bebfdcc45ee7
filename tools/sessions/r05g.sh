#!/bin/bash
# Round-5 session G: the GPU suite (SURVEY 1e-9 distribution bars, lazy rounds
# restructured), the disturbed loops with their traces, the QP phase profile.
set -o pipefail
OUT=gpurun_out/r05g; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 $B --wind-sweep 0.5 > $OUT/wind05.json 2> $OUT/wind05.err || { echo "wind failed"; exit 1; }
timeout -k 10 200 $B --meas-noise 1 > $OUT/noise1.json 2> $OUT/noise1.err || { echo "noise failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profwind -o ktrace --output-format csv -- $B --wind-sweep 0.5 > $OUT/profwind.log 2>&1 || { echo "profwind failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profnoise -o ktrace --output-format csv -- $B --meas-noise 1 > $OUT/profnoise.log 2>&1 || { echo "profnoise failed"; exit 1; }
timeout -k 10 300 python tools/qp_phase_profile.py 4096 20 > $OUT/qp_phase_profile.txt 2>&1 || { echo "phase profile failed"; exit 1; }
echo done
