cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in default notab; do
  if [ $v = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $GRAFT_REPO_ROOT/gpurun_out/ab_lds_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_ab.py default 8192 6 > gpurun_out/ab_lds_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
done
python3 - <<'PY'
import csv,glob,collections
for v in ('default','notab'):
    tot=collections.defaultdict(float)
    for f in glob.glob(f'gpurun_out/ab_lds_{v}/**/*counter_collection.csv',recursive=True):
        for r in csv.DictReader(open(f)):
            if 'mfw' in r['Kernel_Name']: tot[r['Counter_Name']]+=float(r['Counter_Value'])
    print(v, dict(tot), tot['SQ_LDS_BANK_CONFLICT']/max(tot['SQ_ACTIVE_INST_LDS'],1))
PY
