#!/bin/bash
# Round-5 session AM: k_condense20<2> (node data prefetched two nodes ahead)
# for batches <= 1024 vs HEAD -- batch invariance, outputs at 64 kites,
# batch-1 latency, condensing phase at 64 / 512 / 4096 kites.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05am; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "full_batch_properties" -x -q --timeout 200 --timeout-method thread > $OUT/inv.txt 2>&1 || { echo "invariance failed"; tail -25 $OUT/inv.txt; exit 1; }
tail -1 $OUT/inv.txt
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 64 30 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/cpf2.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new.npz $OUT/base.npz 64 30 20 > $OUT/out_new.log 2>&1 || { echo "new outputs failed"; exit 1; }
echo "64 kites vs HEAD: $(tail -1 $OUT/out_new.log)"
rm -f $OUT/*.npz
for v in head cpf2; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/$v.so timeout -k 10 200 python tools/latency_probe.py 200 20 1 > $OUT/lat_$v.json 2>/dev/null || { echo "probe $v failed"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/lat_$v.json'));print('$v latency',round(d['host_step_median_ms'],4),round(d['device_step_median_ms'],4),{k:round(x,4) for k,x in d['phases_median_ms'].items()})"
done
for bb in 64 512 4096; do
  bash tools/ab_alt.sh r05am/b$bb 1 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/cpf2.so -- --batch $bb || { echo "ab failed"; exit 1; }
done
echo done
