cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
# instruction mix and busy cycles of one 3072-stream, 6-frame launch: mfw_kernel (LPCNET_MFW=1) and mf2_kernel (0)
for v in 1 0; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/mfwpmc_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mfw_probe.py 3072 6 LPCNET_MFW=$v > $GRAFT_REPO_ROOT/gpurun_out/mfwpmc_$v.log 2>&1 || { echo "pmc $v failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/mfwpmc_$v.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/mfwpmc2_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mfw_probe.py 3072 6 LPCNET_MFW=$v > $GRAFT_REPO_ROOT/gpurun_out/mfwpmc2_$v.log 2>&1 || { echo "pmc2 $v failed rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/mfwpmc2_$v.log; exit 1; }
done
echo pmc done
