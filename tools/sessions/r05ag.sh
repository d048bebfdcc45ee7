#!/bin/bash
# Round-5 session AG: k_qp_ric factorisation sweep with a Z_k ring two stages
# deep (RIC_PDF 2) vs HEAD (1) -- bitwise outputs at N = 40, alternating A/B at
# config 5 (4096 kites) and at its per-GPU shape (512 kites).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ag; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base40.npz - 256 60 40 > $OUT/out_base40.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base40.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/pdf2.so timeout -k 10 200 python tools/ab_outputs.py $OUT/pdf40.npz $OUT/base40.npz 256 60 40 > $OUT/out_pdf40.log 2>&1 || { echo "ric outputs failed"; cat $OUT/out_pdf40.log; exit 1; }
tail -1 $OUT/out_pdf40.log
rm -f $OUT/*.npz
bash tools/ab_alt.sh r05ag 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/pdf2.so -- --horizon 40 --ekf || { echo "ab4096 failed"; exit 1; }
bash tools/ab_alt.sh r05ag/b512 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/pdf2.so -- --horizon 40 --ekf --batch 512 || { echo "ab512 failed"; exit 1; }
echo done
