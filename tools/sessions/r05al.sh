#!/bin/bash
# Round-5 session AL: k_rk4_sens1 with the Dual tangent formulas written as
# Dual2's -- batch invariance (test_full_batch_properties: 4096 kites through
# k_rk4_sens2, 16 through k_rk4_sens1, bitwise), outputs vs HEAD at 4096 kites,
# GPU suite, batch-1 latency.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05al; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "full_batch_properties" -x -q --timeout 200 --timeout-method thread > $OUT/inv.txt 2>&1 || { echo "invariance failed"; tail -25 $OUT/inv.txt; exit 1; }
tail -1 $OUT/inv.txt
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 512 20 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/sens1b.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new.npz $OUT/base.npz 512 20 20 > $OUT/out_new.log 2>&1 || { echo "new outputs failed"; exit 1; }
echo "512 kites (sens2 path) vs HEAD: $(tail -1 $OUT/out_new.log)"
rm -f $OUT/*.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/sens1b.so timeout -k 10 200 python tools/latency_probe.py 200 20 1 > $OUT/lat.json 2>/dev/null || { echo "probe failed"; exit 1; }
python -c "import json;d=json.load(open('$OUT/lat.json'));print('latency',round(d['host_step_median_ms'],4),round(d['device_step_median_ms'],4),{k:round(x,4) for k,x in d['phases_median_ms'].items()})"
echo done
