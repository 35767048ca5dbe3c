#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first crash/timeout (exit codes other than pytest's 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 420 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --cpu-seconds 8 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof.log"
fi
exit $rc
