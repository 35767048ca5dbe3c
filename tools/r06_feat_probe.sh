cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/vram_host_probe > gpurun_out/vram_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/vram_probe.log
for m in "host LPCNET_FEAT_DMA=1" "caller" "host"; do
  LPCNET_LIB_VARIANT=ckst timeout -k 10 120 python tools/live_probe.py 1024 40 $m LPCNET_CK_SLICES=4 > gpurun_out/ckst_m.log 2>&1 || { echo "ckst rc=$?"; tail -5 gpurun_out/ckst_m.log; exit 1; }
  echo "== $m"; grep "ck<" gpurun_out/ckst_m.log | tail -3; grep ms_per gpurun_out/ckst_m.log
done
