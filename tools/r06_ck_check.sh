cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_constants.py tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TESTK:-live or deferred or constants or wide}" > gpurun_out/t.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
LPCNET_LIB_VARIANT=ckst timeout -k 10 120 python tools/live_probe.py 1024 40 host > gpurun_out/ckst4.log 2>&1 && grep "ck<" gpurun_out/ckst4.log | tail -3
ENVS="base LPCNET_TICK_FLAG=0" ROUNDS=3 bash tools/r06_tick_ab.sh
