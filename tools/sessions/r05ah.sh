#!/bin/bash
# Round-5 session AH: k_qp_ric factorisation sweep run in rounds of RIC_PDF
# stages (the Z_k ring two stages deep, pdf2) vs the same loop with one stage
# (pdf1) and HEAD -- bitwise outputs at N = 40, alternating A/B at config 5
# (4096 kites) and at its per-GPU shape (512 kites).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ah; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base40.npz - 256 60 40 > $OUT/out_base40.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base40.log; exit 1; }
for v in pdf1 pdf2; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/$v.so timeout -k 10 200 python tools/ab_outputs.py $OUT/$v.npz $OUT/base40.npz 256 60 40 > $OUT/out_$v.log 2>&1 || { echo "$v outputs failed"; cat $OUT/out_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/out_$v.log)"
done
rm -f $OUT/*.npz
bash tools/ab_alt.sh r05ah 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/pdf1.so openkite_amd/lib/ab/pdf2.so -- --horizon 40 --ekf || { echo "ab4096 failed"; exit 1; }
bash tools/ab_alt.sh r05ah/b512 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/pdf1.so openkite_amd/lib/ab/pdf2.so -- --horizon 40 --ekf --batch 512 || { echo "ab512 failed"; exit 1; }
echo done
