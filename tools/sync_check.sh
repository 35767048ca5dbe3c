#!/bin/bash
# drop-in / live parity after the wait change, then the C driver at 64 / 256 threads (default settings)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "dropin or live or plc or decode or boundary" > gpurun_out/sync_pt.log 2>&1; rc=$?; tail -2 gpurun_out/sync_pt.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for T in 64 256 1024; do
    timeout -k 10 120 ./tools/dropin_bench $T 60 > gpurun_out/dropin_c_${T}_$r.json 2> gpurun_out/dropin_c_${T}_$r.err || { echo "dropin $T rc=$?"; tail -3 gpurun_out/dropin_c_${T}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/dropin_c_${T}_$r.json'))
print('T=$T r$r pool %.1f M  batch_host %.1f M (%.4f ms)  device %.1f M' % (d['dropin_c_threads']['samples_per_s']/1e6, d['batch_host_io']['samples_per_s']/1e6, d['batch_host_io']['ms_per_frame'], d['batch_device']['samples_per_s']/1e6))"
  done
done
