#!/bin/bash
# live path: engine-buffer parity tests, per-frame timeline at 1024 / 28672
# streams, chunk_kernel single-frame stamps (ckst build), the bench's live
# and capacity_live lines
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_constants.py tests/test_gpu_plc.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "live or chunk or constants or golden or frame or plc or delay" > gpurun_out/live_pt.log 2>&1; rc=$?; tail -2 gpurun_out/live_pt.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$CKST" ]; then
  timeout -k 10 120 python tools/live_probe.py 1024 8 LPCNET_LIB_VARIANT=ckst > gpurun_out/ckst.log 2>&1 || { echo "ckst rc=$?"; exit 1; }
  grep "^ck" gpurun_out/ckst.log | tail -2
fi
for B in 1024 28672; do
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/lz_$B" -o run --output-format csv -- python3 "$R/tools/live_probe.py" $B 24 host > "$R/gpurun_out/lz_$B.log" 2>&1 || { echo "trace $B rc=$?"; exit 1; }
  tail -1 "$R/gpurun_out/lz_$B.log"
done
timeout -k 10 400 python bench.py --steps 30 --live-only --no-batch1 --no-cpu --no-latency > gpurun_out/bench_live.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_live.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_live.log').read().strip().splitlines()[-1])
print('value', d['value']); print('live', json.dumps(d.get('live'))[:700]); print('capacity_live', d.get('capacity_live',{}).get('max_realtime_streams'))"
