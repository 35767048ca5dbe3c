cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_constants.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "wide_kernel or live_single or chunk or golden or mf" > gpurun_out/sched_pt.log 2>&1; rc=$?; tail -2 gpurun_out/sched_pt.log; [ $rc -eq 0 ] || exit $rc
for v in "" nosched "" nosched; do
  LPCNET_LIB_VARIANT=$v timeout -k 10 200 python tools/ab_env.py LPCNET_MFW=0,1 1024,3072,8192,24576 20 1 > gpurun_out/sched_ab_$v.log 2>&1 || exit 1; echo "variant [$v]"; cat gpurun_out/sched_ab_$v.log | grep frame
done
timeout -k 10 120 python tools/live_probe.py 1024 8 LPCNET_LIB_VARIANT=ckst > gpurun_out/ckst.log 2>&1; grep "^ck" gpurun_out/ckst.log | tail -1
timeout -k 10 120 python tools/live_probe.py 1024 40 > gpurun_out/live_a.log 2>&1 && tail -1 gpurun_out/live_a.log
timeout -k 10 120 python tools/mfw_probe.py 3072 6 LPCNET_LIB_VARIANT=mfwst > gpurun_out/mfw_st.log 2>&1; grep -E "wave (0|5|6|10|12)|kernel" gpurun_out/mfw_st.log | head -20
