#!/bin/bash
# Round-5 session Z: k_qp_ric's commit with its loads ahead of its stores (four
# elements a lane at a time) -- bitwise outputs at N = 40, alternating A/B at
# config 5 (4096 kites) and at its per-GPU shape (512 kites), kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05z; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/expand.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base40.npz - 256 60 40 > $OUT/out_base40.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base40.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/ric.so timeout -k 10 200 python tools/ab_outputs.py $OUT/ric40.npz $OUT/base40.npz 256 60 40 > $OUT/out_ric40.log 2>&1 || { echo "ric outputs failed"; cat $OUT/out_ric40.log; exit 1; }
tail -1 $OUT/out_ric40.log
rm -f $OUT/*.npz
bash tools/ab_alt.sh r05z 2 openkite_amd/lib/ab/expand.so openkite_amd/lib/ab/ric.so -- --horizon 40 --ekf || { echo "ab4096 failed"; exit 1; }
bash tools/ab_alt.sh r05z/b512 2 openkite_amd/lib/ab/expand.so openkite_amd/lib/ab/ric.so -- --horizon 40 --ekf --batch 512 || { echo "ab512 failed"; exit 1; }
echo done
