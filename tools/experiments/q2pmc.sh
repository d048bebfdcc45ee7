#!/bin/bash
# PMC SQ pass on base and q2 libs
mkdir -p gpurun_out/q2p
for v in base q2; do
  KITE_NMPC_LIB=$PWD/abl/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/q2p/$v -o sq --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/q2p/$v.log 2>&1 || exit 1
done
echo done
