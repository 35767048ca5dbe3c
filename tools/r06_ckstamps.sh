#!/bin/bash
# Stamped one-frame chunk kernel (CK_STAMPS variant library) at 1024 streams,
# slices 1 / 4, and the wide kernel's wave-state / LDS PMC passes at 8192
# streams (scratch under gpurun_out/).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
for s in 1 4; do
  LPCNET_LIB_VARIANT=ckst timeout -k 10 120 python tools/live_probe.py 1024 40 host LPCNET_CK_SLICES=$s > gpurun_out/ckst_$s.log 2>&1 || { echo "ckst $s rc=$?"; tail -5 gpurun_out/ckst_$s.log; exit 1; }
  grep "ck<" gpurun_out/ckst_$s.log | tail -4
done
export TMPDIR=/tmp; cd /tmp
for pass in "lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "waves:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "valu:SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  pn=${pass%%:*}; ctr=${pass#*:}
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d "$R/gpurun_out/mfwp_$pn" -o run --output-format csv -- python3 "$R/tools/pmc_ab.py" default 8192 6 > "$R/gpurun_out/mfwp_$pn.log" 2>&1 || { echo "pmc $pn rc=$?"; exit 1; }
done
echo pmc ok
