#!/bin/bash
# Round-6 session G: k_qp_ric two-wave variants at 512 kites / N = 40 (latency
# probe per library: committed pipelined kernel, closed-loop forward sweeps,
# + residual overlap with ring depth 3 / 6 / 8), the phase profile of the
# current kernel, and the headline A/B of k_qp_tiled's recursive residuals
# (current library vs the one before the change), alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06g; mkdir -p $OUT
AB=$PWD/openkite_amd/lib/ab
for v in pipe acl cur cb pd6 pd8; do
  if [ $v = cur ]; then L=$PWD/openkite_amd/lib/libkite_nmpc.so; else L=$AB/libkite_$v.so; fi
  KITE_NMPC_LIB=$L timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512_$v.txt 2>&1 || { echo probe $v failed; tail $OUT/latency512_$v.txt; exit 1; }
  echo "$v $(tail -1 $OUT/latency512_$v.txt)"
done
KITE_NMPC_LIB=$PWD/openkite_amd/lib/libkite_nmpc_prof2.so timeout -k 10 200 python tools/ric_phase_profile.py 512 40 > $OUT/phase512.txt 2>&1 || { echo prof failed; exit 1; }
for r in 1 2; do
  for v in acl cur; do
    if [ $v = cur ]; then L=$PWD/openkite_amd/lib/libkite_nmpc.so; else L=$AB/libkite_$v.so; fi
    KITE_NMPC_LIB=$L timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { echo bench $v failed; tail $OUT/bench_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${v}_$r.json'));print('$v',$r,d['value'],d['ms_per_step'],d['qp_main_kernel_ms_per_step'],d['qp_mean_iterations'],d['roofline']['frac'])"
  done
done
cat $OUT/phase512.txt
