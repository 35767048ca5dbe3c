cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2; do for v in base new; do
  if [ $v = base ]; then export LPCNET_LIB_VARIANT=base; else unset LPCNET_LIB_VARIANT; fi
  for B in 128 96; do timeout -k 10 120 python bench.py --streams $B --steps 20 --no-cpu --no-batch1 > gpurun_out/ab128_${v}_${B}_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab128_${v}_${B}_$i.log').read().strip().splitlines()[-1]); print('$v B=$B', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"; done
done; done
