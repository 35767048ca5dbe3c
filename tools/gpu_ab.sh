#!/bin/bash
# GPU tests, quad vs per-slot LDS A/B bench, phase profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/phase_profile.py > gpurun_out/phase.log 2>&1 || { echo "phase rc=$?"; exit 1; }
cat gpurun_out/phase.log
timeout -k 10 200 python bench.py --steps 20 --no-cpu > gpurun_out/bench_quad.log 2>&1 || exit $?
LPCNET_NO_QUAD=1 timeout -k 10 200 python bench.py --steps 20 --no-cpu > gpurun_out/bench_lds.log 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ("quad","lds"):
    d=json.loads(open(f"gpurun_out/bench_{f}.log").read().strip().splitlines()[-1])
    print(f, "value %.4g"%d["value"], "sample_ms %.3f"%d["roofline"]["avg_launch_ms"], "frame_ms %.3f"%d["frame_kernel_avg_ms"], "b1 %.4g"%d["batch1"]["samples_per_s"], d["kernel_config"])
PY
