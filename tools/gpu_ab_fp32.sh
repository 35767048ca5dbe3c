#!/bin/bash
# Alternating A/B of library variants on the batch-1 fp32 configuration
# (BASELINE configs[1]): VARIANTS="prev default" ROUNDS=2 tools/gpu_ab_fp32.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    if [ "$v" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --streams 1 --variant fp32 --steps 20 --no-cpu --no-batch1 --no-latency > gpurun_out/abf_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/abf_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-8s value %.4gK samples/s launch %.4f ms crc %s' % (sys.argv[2], d['value']/1e3, d['roofline']['avg_launch_ms'], d.get('pcm_checksum')))" gpurun_out/abf_${v}_$i.log $v
  done
done
