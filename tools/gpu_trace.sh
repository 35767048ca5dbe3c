#!/bin/bash
# rocprofv3 kernel trace of the B=1024 bench command; per-kernel summary.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-20}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
f=$(ls "$R"/gpurun_out/prof/*/run_kernel_trace.csv "$R"/gpurun_out/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 "$R/tools/trace_summary.py" "$f" "$R/gpurun_out/trace_summary.json"
