#!/bin/bash
# Round-5 session AK: one-tangent sensitivity kernel for small batches
# (k_rk4_sens1, B <= 128) vs HEAD (k_rk4_sens2 everywhere) -- bitwise outputs at
# 64 kites, batch-1 latency, rk4 phase time at 1 / 64 / 128 kites, GPU suite.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ak; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 64 40 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/sens1.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new.npz $OUT/base.npz 64 40 20 > $OUT/out_new.log 2>&1 || { echo "new outputs failed"; cat $OUT/out_new.log; exit 1; }
tail -1 $OUT/out_new.log
rm -f $OUT/*.npz
for v in head sens1; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/$v.so timeout -k 10 200 python tools/latency_probe.py 200 20 1 > $OUT/lat_$v.json 2>/dev/null || { echo "probe $v failed"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/lat_$v.json'));print('$v latency',round(d['host_step_median_ms'],4),round(d['device_step_median_ms'],4),{k:round(x,4) for k,x in d['phases_median_ms'].items()})"
done
for bb in 64 128; do
  bash tools/ab_alt.sh r05ak/b$bb 1 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/sens1.so -- --batch $bb || { echo "ab failed"; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
echo done
