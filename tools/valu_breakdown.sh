#!/bin/bash
# Instructions per tile by kernel stage: SQ_INSTS_* of diagnostic builds
# (stage only / parse only / full) on config 20 and config 2.  One --pmc pass
# per build, kernel trace off.  Usage: tools/valu_breakdown.sh [extra defines]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/valu
mkdir -p $OUT
i=0
for v in "DIAG_STAGEONLY $*" "DIAG_PARSEONLY $*" "DIAG_DESCENTONLY $*" "VB_FULL $*"; do
  d=/tmp/vb_$i
  timeout -k 10 300 python -m odp_amd._build $d $v > /dev/null || exit 1
  for c in ${VB_CFGS:-20 2}; do
    ( cd /tmp && export TMPDIR=/tmp && ODP_AMD_LIB_DIR=$d timeout -k 10 200 rocprofv3 \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES \
      --output-format csv -d $OUT/b${i}_c$c -o p -- python3 $ROOT/bench.py --config $c --steps 5 \
      --warmup 2 --no-cpu --no-extra --streams 1 > $OUT/b${i}_c$c.log 2>&1 ) || exit 1
    python3 - $OUT/b${i}_c$c "$v" $c <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mi_cls" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
t = 15625.0
print(f"[{sys.argv[2]:>24s}] config{sys.argv[3]:>3s}  " + "  ".join(
    f"{k.replace('SQ_INSTS_', '')}={sum(v)/len(v)/t:.1f}" for k, v in sorted(agg.items())
    if k != "SQ_WAVES"))
PY
  done
  i=$((i+1))
done
