#!/bin/bash
# end-of-call wait: blocking (LPCNET_SYNC_BLOCK=1) vs polled with P pause
# instructions between polls, on the drop-in C driver (pool at 64 / 256
# threads, batch host I/O, device-resident)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
for r in 1 2; do
  for mode in block p0 p200 p2000; do
    for T in 64 256; do
      unset LPCNET_SYNC_BLOCK LPCNET_SYNC_PAUSE
      case $mode in block) export LPCNET_SYNC_BLOCK=1;; p*) export LPCNET_SYNC_PAUSE=${mode#p};; esac
      timeout -k 10 120 ./tools/dropin_bench $T 60 > gpurun_out/sync_${mode}_${T}_$r.json 2> gpurun_out/sync_${mode}_${T}_$r.err || { echo "dropin $mode $T rc=$?"; tail -3 gpurun_out/sync_${mode}_${T}_$r.err; exit 1; }
      python3 -c "
import json,sys; d=json.load(open('gpurun_out/sync_${mode}_${T}_$r.json'))
print('%-6s T=$T r$r pool %.1f M  batch_host %.1f M (%.4f ms)  device %.1f M' % ('$mode', d['dropin_c_threads']['samples_per_s']/1e6, d['batch_host_io']['samples_per_s']/1e6, d['batch_host_io']['ms_per_frame'], d['batch_device']['samples_per_s']/1e6))"
    done
  done
done
