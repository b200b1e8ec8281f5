#!/bin/bash
# Instruction-cache / issue-stall counters for one bench config (separate
# --pmc passes).  Also saves the list of available counters once.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/icache_$1; shift
ARGS=${*:-"--config 20 --steps 10 --warmup 3 --no-cpu --no-extra"}
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
[ -f $ROOT/gpurun_out/counters_avail.txt ] || timeout -k 10 120 rocprofv3 --list-avail > $ROOT/gpurun_out/counters_avail.txt 2>&1
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p \
    -- python3 $ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1 || echo "pass $i failed: $set"
  i=$((i+1))
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mi_cls" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v)/len(v):16.1f}  per-tile {sum(v)/len(v)/15625:10.1f}")
PY
