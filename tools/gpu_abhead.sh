#!/bin/bash
# Alternating A/B of the working tree against a checkout of an earlier
# commit in ./ab_head (git worktree add ab_head <rev>; make -C ab_head lib):
#   B=1024 ROUNDS=3 tools/gpu_abhead.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-1024}; ROUNDS=${ROUNDS:-3}; STEPS=${STEPS:-20}
for i in $(seq 1 $ROUNDS); do
  for v in head cur; do
    if [ $v = head ]; then d=ab_head; else d=.; fi
    (cd $d && timeout -k 10 150 python bench.py --streams $B --steps $STEPS --no-cpu --no-batch1 --no-latency) > gpurun_out/abh_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/abh_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-5s B=%s value %8.4gM step %.4f ms' % (sys.argv[2], sys.argv[3], d['value']/1e6, d['ms_per_step']))" gpurun_out/abh_${v}_$i.log $v $B
  done
done
