#!/bin/bash
# Warmup-length experiment: the timed multi-frame launch vs the warmup length
# (driver command: --steps 20 --warmup 5).  Prints value and launch ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for w in ${WARMS:-5 40}; do
    timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup $w --no-cpu --no-batch1 --no-latency $EXTRA > gpurun_out/warm_${w}_$i.log 2>&1 || { echo "bench w$w rc=$?"; tail -5 gpurun_out/warm_${w}_$i.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/warm_${w}_$i.log').read().strip().splitlines()[-1])
print('warmup $w', 'value %.2fM'%(d['value']/1e6), 'ms/step %.4f'%d['ms_per_step'], 'kernel ms/frame %.4f'%d['roofline']['ms_per_frame'])"
  done
done
