#!/bin/bash
# Round-5 session C: the GPU suite and smoke on HEAD, the driver-format bench
# line, the disturbed loops after the lazy round-0 handover (bench lines +
# kernel traces), and a kernel trace of the batch-1 latency loop.
set -o pipefail
OUT=gpurun_out/r05c; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 200 $B --wind-sweep 0.5 > $OUT/wind05.json 2> $OUT/wind05.err || { echo "wind failed"; exit 1; }
timeout -k 10 200 $B --meas-noise 1 > $OUT/noise1.json 2> $OUT/noise1.err || { echo "noise failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profwind -o ktrace --output-format csv -- $B --wind-sweep 0.5 > $OUT/profwind.log 2>&1 || { echo "profwind failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/profnoise -o ktrace --output-format csv -- $B --meas-noise 1 > $OUT/profnoise.log 2>&1 || { echo "profnoise failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/proflat -o kt --output-format csv -- python tools/latency_probe.py 100 > $OUT/proflat.log 2>&1 || { echo "proflat failed"; exit 1; }
echo done
