timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k "chunked or multi_frame or bench_preheat" > gpurun_out/pt_chunk.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pt_chunk.log
for i in 1 2; do for v in old default; do
  if [ $v = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-batch1 --no-latency > gpurun_out/d20_${v}_$i.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.2fM'%(d['value']/1e6), 'step %.4f'%d['ms_per_step'], 'kern %.4f'%d['roofline']['ms_per_frame'], 'fnet %.4f'%d['frame_network_ms_per_frame'], d['pcm_checksum'])" gpurun_out/d20_${v}_$i.log $v
done; done
