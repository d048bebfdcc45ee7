mkdir -p gpurun_out/r02f
for v in O A B; do
  if [ $v = B ]; then lib=openkite_amd/lib/libkite_nmpc.so; else lib=openkite_amd/lib/libkite_nmpc_$v.so; fi
  KITE_NMPC_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r02f/bench_$v.json 2>gpurun_out/r02f/bench_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02f/bench_$v.json'));print('$v',d['value'],d['kernel_ms_per_step'],d['qp_mean_iterations'])"
done
