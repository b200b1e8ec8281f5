#!/bin/bash
# Instruction counts per 64-packet tile of the in-tree build (one --pmc pass
# per config).  Usage: tools/pmc_quick.sh TAG "CFGS"
set -o pipefail
TAG=$1
CFGS=${2:-"3 4"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmcq_$TAG
mkdir -p $OUT
for c in $CFGS; do
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
    n=$(echo $set | md5sum | cut -c1-6)
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv \
      -d $OUT/c${c}_$n -o p -- python3 $ROOT/bench.py --config $c --steps 5 --warmup 2 --timed-only > $OUT/c${c}_$n.log 2>&1 ) || { echo "pmc $c failed"; exit 1; }
  done
  python3 - $OUT $c <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/c{sys.argv[2]}_*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mi_cls" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
t = 15625.0
print(f"config{sys.argv[2]}: " + " ".join(f"{k.replace('SQ_INSTS_', '').replace('SQ_', '')}={sum(v)/len(v)/t:.1f}" for k, v in sorted(agg.items()) if k != "SQ_WAVES"))
PY
done
