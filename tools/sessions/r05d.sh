#!/bin/bash
# Round-5 session D: the captured host step (graph vs plain launches, bitwise)
# and the batch-1 latency with and without it; facade test.
set -o pipefail
OUT=gpurun_out/r05d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "captured or step_device or facade" tests/test_cpp_facade.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 120 python -u tools/latency_probe.py 300 > $OUT/latency_graph.json 2> $OUT/latency_graph.err || { echo "latency failed"; exit 1; }
KITE_NMPC_NO_GRAPH=1 timeout -k 10 120 python -u tools/latency_probe.py 300 > $OUT/latency_plain.json 2> $OUT/latency_plain.err || { echo "latency plain failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/proflat -o kt --output-format csv -- python tools/latency_probe.py 100 > $OUT/proflat.log 2>&1 || { echo "proflat failed"; exit 1; }
echo done
