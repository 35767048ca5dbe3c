#!/bin/bash
# Kernel trace of the batch-1 configurations (fp32 and int8): per-kernel
# durations and the device idle gaps between kernels (host overhead).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for V in fp32 int8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_b1_$V" -o run --output-format csv -- python3 "$R/bench.py" --streams 1 --variant $V --steps 40 --no-cpu --no-batch1 > "$R/gpurun_out/prof_b1_$V.log" 2>&1 || { echo "trace $V rc=$?"; exit 1; }
  tail -1 "$R/gpurun_out/prof_b1_$V.log" | cut -c1-300
  python3 "$R/tools/trace_summary.py" "$R/gpurun_out/prof_b1_$V/run_kernel_trace.csv" "$R/gpurun_out/trace_b1_$V.json" | tail -12
done
