#!/bin/bash
# Alternating A/B/.. of in-tree library variants at one batch size:
#   VARIANTS="base prio1" B=1024 ROUNDS=3 tools/gpu_abn.sh
# "default" = liblpcnet_mi355x.so.  Prints value, sample-kernel launch ms and
# the stamped critical path per variant and round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-1024}; ROUNDS=${ROUNDS:-3}
for i in $(seq 1 $ROUNDS); do
  for v in $VARIANTS; do
    if [ "$v" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --streams $B --steps 20 --no-cpu --no-batch1 > gpurun_out/abn_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/abn_${v}_$i.log; exit 1; }
    python3 - gpurun_out/abn_${v}_$i.log "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lat = d.get("latency", {})
cp = lat.get("critical_path_cycles", {})
print("%-10s value %7.2fM frame %.4f ms crc %s cyc/sample %6.0f  %s" % (sys.argv[2], d["value"] / 1e6, d["roofline"]["ms_per_frame"], d.get("pcm_checksum"),
      lat.get("cycles_per_sample", 0), " ".join("%s=%.0f" % (k.replace("gru_a_", "A_").replace("sampler_", "S_"), v) for k, v in cp.items())))
PY
  done
done
