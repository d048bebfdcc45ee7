#!/bin/bash
# Round-5 session W: the warm-step prologue split (k_prologue_warm at full
# occupancy + k_prologue_cold over the cold-restart list) -- bitwise outputs
# at N = 20 and 40 over 60 closed-loop steps, GPU suite, alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05w; mkdir -p $OUT
for N in 20 40; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base$N.npz - 256 60 $N > $OUT/out_base$N.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base$N.log; exit 1; }
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/light.so timeout -k 10 200 python tools/ab_outputs.py $OUT/light$N.npz $OUT/base$N.npz 256 60 $N > $OUT/out_light$N.log 2>&1 || { echo "light outputs failed"; cat $OUT/out_light$N.log; exit 1; }
  tail -1 $OUT/out_light$N.log
  rm -f $OUT/*.npz
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
bash tools/ab_alt.sh r05w 3 openkite_amd/lib/ab/base.so openkite_amd/lib/ab/light.so || { echo "ab failed"; exit 1; }
echo done
