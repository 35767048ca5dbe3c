#!/bin/bash
# PMC passes of tools/pmc_ab.py on the default and skewed models at 1024 streams
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out/pmcab"
for m in default skewed; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES -d "$R/gpurun_out/pmcab/lds_$m" -o run --output-format csv -- python3 "$R/tools/pmc_ab.py" $m 1024 8 > "$R/gpurun_out/pmcab/lds_$m.log" 2>&1 || { echo "lds $m rc=$?"; exit 1; }
done
for m in default skewed; do
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d "$R/gpurun_out/pmcab/ic_$m" -o run --output-format csv -- python3 "$R/tools/pmc_ab.py" $m 1024 8 > "$R/gpurun_out/pmcab/ic_$m.log" 2>&1 || { echo "ic $m rc=$?"; exit 1; }
done
LPCNET_FINE_STAMPS=1 timeout -k 10 200 python3 "$R/tools/split_latency.py" 1024 > "$R/gpurun_out/pmcab/waves.log" 2>&1 || { echo "waves rc=$?"; exit 1; }
echo ok
