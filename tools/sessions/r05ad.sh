#!/bin/bash
# Round-5 session AD: single-kite latency in episodes (reset + 25 warm steps,
# as the CPU oracle's batch-1 latency is measured) -- latency probe and the
# bench line's gpu_latency_batch1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ad; mkdir -p $OUT
timeout -k 10 300 python tools/latency_probe.py 300 20 1 > $OUT/latency_probe_b1.json 2> $OUT/latency_probe_b1.err || { echo "probe failed"; tail $OUT/latency_probe_b1.err; exit 1; }
cat $OUT/latency_probe_b1.json
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['gpu_latency_batch1'],d['cpu_baseline']['latency_1thread_batch1'])"
echo done
