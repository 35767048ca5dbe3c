cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "wide_kernel" > gpurun_out/mfw_pt.log 2>&1; rc=$?; tail -3 gpurun_out/mfw_pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_env.py LPCNET_MFW=0,1 3072,8192,12288,24576 20 2 > gpurun_out/mfw_ab.log 2>&1; tail -8 gpurun_out/mfw_ab.log
timeout -k 10 120 python tools/mfw_probe.py 3072 6 LPCNET_LIB_VARIANT=mfwst > gpurun_out/mfw_st.log 2>&1; grep -E "wave (0|5|6|7|10|12)|kernel" gpurun_out/mfw_st.log | head -20
