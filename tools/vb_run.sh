#!/bin/bash
# Instructions per tile by kernel stage from prebuilt diagnostic builds
# (build/vb_stage: -DDIAG_STAGEONLY, build/vb_parse: -DDIAG_PARSEONLY,
# build/vb_desc: -DDIAG_DESCENTONLY, and the in-tree full kernel), one --pmc
# pass each.  Usage (via gpurun): tools/vb_run.sh "4 5 3"
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/vb
mkdir -p $OUT
for c in ${1:-4 5 3}; do
  for d in build/vb_stage build/vb_parse build/vb_desc odp_amd; do
    tag=$(basename $d)_c$c
    ( cd /tmp && export TMPDIR=/tmp && ODP_AMD_LIB_DIR=$ROOT/$d timeout -k 10 120 rocprofv3 \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES \
      --output-format csv -d $OUT/$tag -o p -- python3 $ROOT/bench.py --config $c --steps 5 \
      --warmup 2 --timed-only --no-parity > $OUT/$tag.log 2>&1 ) || { echo "$tag failed"; exit 1; }
    python3 - $OUT/$tag $tag <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mi_cls" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
t = 15625.0
print(f"{sys.argv[2]:>22s}  " + "  ".join(
    f"{k.replace('SQ_INSTS_', '')}={sum(v)/len(v)/t:.1f}" for k, v in sorted(agg.items())
    if k != "SQ_WAVES"))
PY
  done
done
