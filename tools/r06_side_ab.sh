#!/bin/bash
# Deferred LPC beside the sample kernel (LPCNET_LPC_SIDE=1, on fstream after
# the chunk kernel) vs after it on the tick's stream: the live / deferred
# parity tests with the knob on, the alternating live-tick A/B, and a kernel
# trace of the side form.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
LPCNET_LPC_SIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_constants.py tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "live or deferred or host_views" > gpurun_out/side_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/side_pytest.log; exit 1; }
tail -2 gpurun_out/side_pytest.log
ROUNDS=3 ENVS="base LPCNET_LPC_SIDE=1" bash tools/r06_tick_ab.sh > gpurun_out/side_ab.log 2>&1 || { echo "ab failed"; cat gpurun_out/side_ab.log; exit 1; }
cat gpurun_out/side_ab.log
export TMPDIR=/tmp LPCNET_LPC_SIDE=1
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d "$R/gpurun_out/side_prof" -o run --output-format csv -- python3 "$R/tools/live_probe.py" 1024 100 host > "$R/gpurun_out/side_prof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "trace ok"
