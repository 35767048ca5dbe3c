cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_constants.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "live_single or chunk or golden or constants or range" > gpurun_out/live_pt.log 2>&1; rc=$?; tail -2 gpurun_out/live_pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/live_probe.py 1024 8 LPCNET_LIB_VARIANT=ckst > gpurun_out/ckst.log 2>&1; grep "^ck" gpurun_out/ckst.log | tail -2
timeout -k 10 120 python tools/live_probe.py 1024 40 > gpurun_out/live_a.log 2>&1 && tail -1 gpurun_out/live_a.log &&
timeout -k 10 120 python tools/live_probe.py 28672 12 > gpurun_out/live_c.log 2>&1 && tail -1 gpurun_out/live_c.log &&
timeout -k 10 200 python bench.py --steps 20 --no-batch1 --no-capacity --no-cpu --no-latency > gpurun_out/bench_live.log 2>&1; grep -o '"value": [0-9.]*\|"frame_network_ms_per_frame": [0-9.]*' gpurun_out/bench_live.log
