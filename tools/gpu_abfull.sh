#!/bin/bash
# Alternating full-bench A/B (B=1024 + batch1 + batch1_fp32 + batch256) of
# library variants: VARIANTS="default x" ROUNDS=2 tools/gpu_abfull.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    if [ "$v" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-latency > gpurun_out/abf_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/abf_${v}_$i.log; exit 1; }
    python3 - gpurun_out/abf_${v}_$i.log "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-9s B1024 %7.2fM (%.4f ms, frame %.4f)  b1 %6.1fK  b1fp32 %6.1fK  b256 %6.2fM" % (
    sys.argv[2], d["value"] / 1e6, d["roofline"]["avg_launch_ms"], d["frame_kernel_avg_ms"], d["batch1"]["samples_per_s"] / 1e3,
    d["batch1_fp32"]["samples_per_s"] / 1e3, d["batch256"]["samples_per_s"] / 1e6))
PY
  done
done
