cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "live_single or chunk or golden" > gpurun_out/live_pt.log 2>&1; rc=$?; tail -2 gpurun_out/live_pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/live_probe.py 1024 40 > gpurun_out/live_a.log 2>&1 && tail -1 gpurun_out/live_a.log &&
timeout -k 10 120 python tools/live_probe.py 28672 12 > gpurun_out/live_c.log 2>&1 && tail -1 gpurun_out/live_c.log &&
export TMPDIR=/tmp && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/live_prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/live_probe.py 1024 40 > $GRAFT_REPO_ROOT/gpurun_out/live_prof.log 2>&1 && echo prof ok && cd $GRAFT_REPO_ROOT && timeout -k 10 200 python bench.py --steps 20 --no-batch1 --no-capacity --no-cpu --no-latency > gpurun_out/bench_live.log 2>&1; tail -c 600 gpurun_out/bench_live.log
