#!/bin/bash
# Per-stage cost of the kernel on several configs: diagnostic builds cut
# after staging / parse / descent (DIAG_*ONLY) and the full kernel; for each
# build and config, one rocprofv3 --pmc pass (instruction counts per tile) and
# the kernel time from bench.py (one stream).  Usage: tools/diag_stages.sh TAG "CFGS"
set -o pipefail
TAG=$1
CFGS=${2:-"3 4 5"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/diag_$TAG
mkdir -p $OUT
i=0
for v in DIAG_STAGEONLY DIAG_PARSEONLY DIAG_DESCENTONLY VB_FULL; do
  d=/tmp/dg_$i
  timeout -k 10 300 python -m odp_amd._build $d $v > /dev/null || { echo "build $v failed"; exit 1; }
  for c in $CFGS; do
    ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 \
      --timed-only > $OUT/t${i}_c$c.json 2>/dev/null || { echo "bench $v $c failed"; exit 1; }
    ( cd /tmp && export TMPDIR=/tmp && ODP_AMD_LIB_DIR=$d timeout -s KILL 120 rocprofv3 \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAVES \
      --output-format csv -d $OUT/b${i}_c$c -o p -- python3 $ROOT/bench.py --config $c --steps 5 \
      --warmup 2 --timed-only > $OUT/b${i}_c$c.log 2>&1 ) || { echo "pmc $v $c failed"; exit 1; }
    python3 - $OUT/b${i}_c$c "$v" $c $OUT/t${i}_c$c.json <<'PY'
import csv, glob, sys, collections, json
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mi_cls" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
t = 15625.0
kms = json.load(open(sys.argv[4]))["roofline"]["kernel_ms"]
print(f"[{sys.argv[2]:>16s}] config{sys.argv[3]:>3s} kernel_us={kms*1e3:6.1f} " + " ".join(
    f"{k.replace('SQ_INSTS_', '').replace('SQ_', '')}={sum(v)/len(v)/t:.1f}" for k, v in sorted(agg.items())
    if k != "SQ_WAVES"))
PY
  done
  i=$((i+1))
done
for c in ${NOWIDE_CFGS:-}; do
  MI_CLS_NO_WIDE=1 timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --timed-only > $OUT/nowide_c$c.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$OUT/nowide_c$c.json')); print('nowide config $c', d['roofline']['kernel_ms'])"
done
