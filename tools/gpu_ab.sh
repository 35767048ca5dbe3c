#!/bin/bash
# Same-box A/B measurements in one gpurun call (every GPU step under its own
# time limit; the script stops at the first failing step).  MODE selects:
#
#   MODE=lib    alternating in-tree library variants (tools/ab_build.sh) on the
#               device-resident frame step (tools/ab_env.py):
#               VARIANTS="default base" BS=1024,1 ROUNDS=3 [MODEL=int8|int8_skewed|fp32] [AB_VAR=ENV=a,b]
#   MODE=env    alternating engine environment settings through bench.py:
#               ENVS="base LPCNET_NO_MULTIFRAME=1" B=1024 ROUNDS=3
#   MODE=head   the working tree against a checkout of an earlier commit in
#               ./ab_head (git worktree add ab_head <rev>; make -C ab_head lib)
#   MODE=stamps per library variant: stamped per-wave critical path
#               (LPCNET_FINE_STAMPS) of the default and skewed models at $B,
#               their throughput at $TB (tools/split_latency.py, skew_tput.py)
#   MODE=pmc    one rocprofv3 PMC pass per model (default, skewed) of $CTR over
#               tools/pmc_ab.py at $B streams
#
# "default" = liblpcnet_mi355x.so; <name> = liblpcnet_mi355x_<name>.so.
# With K set, the GPU tests matching K run first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}; B=${B:-1024}; STEPS=${STEPS:-20}
use() { if [ "$1" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$1; fi; }
line() {  # bench.py JSON line -> one summary line
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-28s value %8.4gM step %.4f ms kernel/frame %.4f ms" % (sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["ms_per_frame"]))
PY
}
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pt_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_ab.log; [ $rc -eq 0 ] || exit $rc
fi
case "${MODE:-lib}" in
lib)
  for r in $(seq 1 $ROUNDS); do
    for v in $VARIANTS; do
      use $v
      timeout -k 10 200 python tools/ab_env.py ${AB_VAR:-LPCNET_AB_ROUND=$r} ${BS:-1024} $STEPS 1 ${MODEL:-int8} > gpurun_out/ablib_${v}_$r.log 2>&1 || { echo "ab $v $r rc=$?"; tail -5 gpurun_out/ablib_${v}_$r.log; exit 1; }
      sed "s/^/$v r$r /" gpurun_out/ablib_${v}_$r.log | grep frame
    done
  done ;;
env)
  for i in $(seq 1 $ROUNDS); do
    for e in $ENVS; do
      tag=$(echo "$e" | tr -c 'A-Za-z0-9_\n' '_')
      if [ "$e" = base ]; then envs=(); else envs=("$e"); fi
      env "${envs[@]}" timeout -k 10 150 python bench.py --streams $B --steps $STEPS --no-cpu --no-batch1 --no-latency --no-capacity > gpurun_out/abe_${tag}_$i.log 2>&1 || { echo "bench $e $i rc=$?"; tail -5 gpurun_out/abe_${tag}_$i.log; exit 1; }
      line gpurun_out/abe_${tag}_$i.log "$e"
    done
  done ;;
head)
  for i in $(seq 1 $ROUNDS); do
    for v in head cur; do
      if [ $v = head ]; then d=ab_head; else d=.; fi
      (cd $d && timeout -k 10 150 python bench.py --streams $B --steps $STEPS --no-cpu --no-batch1 --no-latency --no-capacity) > gpurun_out/abh_${v}_$i.log 2>&1 || { echo "bench $v $i rc=$?"; tail -5 gpurun_out/abh_${v}_$i.log; exit 1; }
      line gpurun_out/abh_${v}_$i.log "$v"
    done
  done ;;
stamps)
  for v in ${VARIANTS:-default}; do
    use $v
    echo "== $v"
    LPCNET_FINE_STAMPS=1 timeout -k 10 120 python tools/split_latency.py $B default,skewed || exit 1
    timeout -k 10 200 python tools/skew_tput.py ${TB:-1024,2048} || exit 1
  done ;;
pmc)
  export TMPDIR=/tmp
  CTR=${CTR:-"SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES"}
  mkdir -p "$R/gpurun_out/pmcab"
  for m in default skewed; do
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $CTR -d "$R/gpurun_out/pmcab/$m" -o run --output-format csv -- python3 "$R/tools/pmc_ab.py" $m $B 8) > "$R/gpurun_out/pmcab/$m.log" 2>&1 || { echo "pmc $m rc=$?"; exit 1; }
  done
  python3 - <<'PY'
import csv, glob, collections
for m in ("default", "skewed"):
    f = glob.glob(f"gpurun_out/pmcab/{m}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        if "kernel" in k:
            print(m, k, {c: round(v) for c, v in d.items()})
PY
  ;;
*) echo "unknown MODE $MODE"; exit 2 ;;
esac
echo "gpu_ab done"
