#!/bin/bash
# A/B of two in-tree builds of the native library: liblpcnet_mi355x.so (new)
# vs liblpcnet_mi355x_${AB_BASE:-base}.so, benched alternately so that box
# drift hits both alike.  Usage: tools/gpu_ab.sh [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${1:-3}
for i in $(seq 1 $R); do
  for v in base new; do
    if [ $v = base ]; then export LPCNET_LIB_VARIANT=${AB_BASE:-base}; else unset LPCNET_LIB_VARIANT; fi
    timeout -k 10 200 python bench.py --steps 20 --no-cpu > gpurun_out/ab_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/ab_${v}_$i.log; exit 1; }
    echo "$v $i done"
  done
done
python3 - "$R" <<'PY'
import json, sys
R = int(sys.argv[1])
for v in ("base", "new"):
    rows = []
    for i in range(1, R + 1):
        d = json.loads(open(f"gpurun_out/ab_{v}_{i}.log").read().strip().splitlines()[-1])
        rows.append((d["value"], d["roofline"]["avg_launch_ms"], d["batch1"]["samples_per_s"],
                     d.get("batch1_fp32", {}).get("samples_per_s", 0)))
    for r in rows:
        print(v, "value %.4g  sample_ms %.4f  b1 %.4g  b1fp32 %.4g" % r)
PY
