#!/bin/bash
# Round-6 live-tick / drop-in real-time check in one gpurun call: the GPU
# parity tests of the live and drop-in paths, the live tick at 1024 streams
# with the LPC deferred vs eager (alternating), the paced drop-in sweep, and
# a kernel trace of the deferred tick.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_constants.py tests/test_gpu.py tests/test_gpu_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TESTK:-live or deferred or constants or host_views or dropin or placement or thread}" > gpurun_out/r06_live_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r06_live_pytest.log; exit 1; }
tail -2 gpurun_out/r06_live_pytest.log
for k in 1 2 3; do
  for m in ${LIVE_AB:-LPCNET_LPC_EAGER=0 LPCNET_LPC_EAGER=1}; do
    timeout -k 10 120 python tools/live_probe.py ${LIVEB:-1024} 300 host $m >> gpurun_out/r06_live_ab.log 2>&1 || { echo "live probe rc=$?"; exit 1; }
    echo "$m" >> gpurun_out/r06_live_ab.log
  done
done
cat gpurun_out/r06_live_ab.log
for T in ${RT_THREADS-256 960}; do
  for mode in spread burst; do
    timeout -k 10 120 ./tools/dropin_bench $T 300 rt $mode >> gpurun_out/r06_dropin_rt.jsonl 2>gpurun_out/r06_dropin_rt.err || { echo "dropin rt rc=$?"; cat gpurun_out/r06_dropin_rt.err; exit 1; }
  done
done
cat gpurun_out/r06_dropin_rt.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/live_prof" -o run --output-format csv -- python3 "$R/tools/live_probe.py" ${LIVEB:-1024} 100 host > "$R/gpurun_out/live_prof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "trace ok"
