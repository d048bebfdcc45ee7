#!/bin/bash
# Round-5 session AP: gravity and wind rotations written for constant vectors
# (no dual-typed zeros in the RHS) vs HEAD -- GPU suite (parity, batch
# invariance), outputs difference, kernel traces, alternating A/B, wind line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ap; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 512 20 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/grav.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new.npz $OUT/base.npz 512 20 20 > $OUT/out_new.log 2>&1 || { echo "new outputs failed"; exit 1; }
echo "512 kites x 20 steps vs HEAD: $(tail -1 $OUT/out_new.log)"
rm -f $OUT/*.npz
bash tools/trace_ab.sh r05ap openkite_amd/lib/ab/head.so openkite_amd/lib/ab/grav.so 2>&1 | grep -E "==|k_rk4_sens2|k_prologue_cold|k_qp_tiled " || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05ap 3 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/grav.so || { echo "ab failed"; exit 1; }
bash tools/ab_alt.sh r05ap/wind 1 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/grav.so -- --wind-sweep 0.5 || { echo "ab wind failed"; exit 1; }
echo done
