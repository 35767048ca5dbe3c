#!/bin/bash
# round-5 baseline: the bench line at HEAD, then the wide-batch kernel's
# A/B against mf2 and its per-wave work/wait stamps (mfwst build)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py --steps 30 > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench.log; exit 1; }
tail -c 600 gpurun_out/bench.log; echo
timeout -k 10 300 python tools/ab_env.py LPCNET_MFW=0,1 3072,8192,24576 20 2 > gpurun_out/mfw_ab.log 2>&1 || { echo "ab rc=$?"; exit 1; }
cat gpurun_out/mfw_ab.log
timeout -k 10 120 python tools/mfw_probe.py 3072 6 LPCNET_LIB_VARIANT=mfwst > gpurun_out/mfw_st.log 2>&1 || { echo "st rc=$?"; exit 1; }
grep -E "wave|kernel" gpurun_out/mfw_st.log | sort | uniq | head -40
