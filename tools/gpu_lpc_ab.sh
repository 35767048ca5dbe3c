#!/bin/bash
# lpc_kernel A/B: device LPC parity tests with the default library, then the
# kernel's mean duration under rocprofv3 for each library variant (VARIANTS).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_lpc.py tests/test_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "lpc or golden or chunked" > gpurun_out/pt_lpc.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pt_lpc.log
export TMPDIR=/tmp
for v in ${VARIANTS:-old default}; do
  if [ $v = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/lpcab_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu --no-batch1 --no-latency > "$R/gpurun_out/lpcab_$v.log" 2>&1 || { echo "rocprof $v failed"; exit 1; }
  cd "$R"; python3 - "$R/gpurun_out/lpcab_$v/run_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'lpc_kernel' in r['Name'] or 'chunk_kernel' in r['Name']:
        print(sys.argv[2], r['Name'][:40], 'calls', r['Calls'], 'avg_us %.1f' % (float(r['AverageNs']) / 1e3))
PY
done
