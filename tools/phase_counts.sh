#!/bin/bash
# Instruction counts per 64-packet tile for the stage-only, parse-only and
# full kernels on one config (attributes instructions to pipeline phases).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CFG:-20}
cd /tmp; export TMPDIR=/tmp
for v in "DIAG_STAGEONLY=1" "DIAG_PARSEONLY=1" "FULL=1"; do
  d=/tmp/pc_${v%%=*}
  (cd $ROOT && timeout -k 10 300 python -m odp_amd._build $d $v > /dev/null) || exit 1
  ODP_AMD_LIB_DIR=$d timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH \
    --output-format csv -d $d/pmc -o p -- python3 $ROOT/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu --no-extra > $d/log 2>&1 || exit 1
  python3 - $d/pmc/p_counter_collection.csv "$v" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "mi_cls" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], " ".join(f"{k.replace('SQ_INSTS_','')}={sum(v)/len(v)/15625:.0f}" for k, v in sorted(agg.items())))
PY
done
