#!/bin/bash
# Round-6 session B: config 5 at 512 kites per GPU -- per-step QP time vs the
# slowest kite's iterations, and the k_qp_ric phase profiles (s_memtime builds:
# with the factor-stage sub-markers, and without them = the stage unserialised)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 200 python tools/ric_latency_probe.py 512 20 5 > $OUT/latency512.txt 2>&1 || { echo probe failed; tail $OUT/latency512.txt; exit 1; }
tail -1 $OUT/latency512.txt
timeout -k 10 200 python tools/ric_phase_profile.py 512 40 > $OUT/phase512_sub.txt 2>&1 || { echo prof failed; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/libkite_nmpc_prof2.so timeout -k 10 200 python tools/ric_phase_profile.py 512 40 > $OUT/phase512_nosub.txt 2>&1 || { echo prof2 failed; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/libkite_nmpc_prof2.so timeout -k 10 200 python tools/ric_phase_profile.py 4096 40 > $OUT/phase4096_nosub.txt 2>&1 || { echo prof2 4096 failed; exit 1; }
cat $OUT/phase512_sub.txt $OUT/phase512_nosub.txt $OUT/phase4096_nosub.txt
