#!/bin/bash
# Launch-gap study: bench value with and without the per-launch HIP events
# (--timers 1 / 0) at 1024 and 1 streams, then one kernel trace of the
# 1024-stream bench for the dispatch timeline (tools/trace_gaps.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gap
export TMPDIR=/tmp
for r in 1 2; do
  for B in 1024 1; do
    for t in 1 0; do
      timeout -k 10 150 python bench.py --streams $B --steps 20 --no-cpu --no-batch1 --timers $t > gpurun_out/gap/b${B}_t${t}_$r.log 2>&1 || { echo "bench B=$B timers=$t rc=$?"; tail -5 gpurun_out/gap/b${B}_t${t}_$r.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('B=%s timers=%s value %.4g step %.4f ms launch %.4f ms' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']))" gpurun_out/gap/b${B}_t${t}_$r.log $B $t
    done
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/trace -o run -- python3 bench.py --streams 1024 --steps 20 --no-cpu --no-batch1 --timers 0 > gpurun_out/gap/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/gap/trace.log; exit 1; }
echo done
