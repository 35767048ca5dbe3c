#!/bin/bash
# kernel + copy timeline of the per-frame host-I/O loop at 1024 and 28672 streams
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 1024 28672; do
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/lt_$B" -o run --output-format csv -- python3 "$R/tools/live_probe.py" $B 24 > "$R/gpurun_out/lt_$B.log" 2>&1 || { echo "trace $B rc=$?"; exit 1; }
  tail -1 "$R/gpurun_out/lt_$B.log"
  f=$(ls "$R"/gpurun_out/lt_$B/*/run_kernel_trace.csv "$R"/gpurun_out/lt_$B/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 "$R/tools/trace_gaps.py" "$f" | head -30
  ls "$R"/gpurun_out/lt_$B/*/ "$R"/gpurun_out/lt_$B/ 2>/dev/null | head
done
