#!/bin/bash
# Round-5 session AN: k_expand20 with 2 and 1 kites per wave (2048 / 4096
# waves, two waves per SIMD) vs HEAD (4 kites per wave, 1024 waves) -- outputs,
# kernel traces, alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05an; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 512 20 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; exit 1; }
for v in kpw2 kpw1; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/$v.so timeout -k 10 200 python tools/ab_outputs.py $OUT/$v.npz $OUT/base.npz 512 20 20 > $OUT/out_$v.log 2>&1 || { echo "$v outputs failed"; exit 1; }
  echo "$v: $(tail -1 $OUT/out_$v.log)"
done
rm -f $OUT/*.npz
bash tools/trace_ab.sh r05an openkite_amd/lib/ab/head.so openkite_amd/lib/ab/kpw2.so openkite_amd/lib/ab/kpw1.so 2>&1 | grep -E "==|k_expand20" || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05an 2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/kpw2.so openkite_amd/lib/ab/kpw1.so || { echo "ab failed"; exit 1; }
echo done
