#!/bin/bash
# Profile the bench's dominant kernel on the GPU box (run through gpurun from
# the repo root).  Separate rocprofv3 runs, as MI355X_MICROARCH.md
# prescribes: kernel trace + stats, then one PMC pass per counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; no trace domains are
# combined with --pmc).
# Usage: tools/profile.sh <tag> <config> [n]
set -o pipefail
TAG=${1:-r02}
CFG=${2:-3}
N=${3:-1000000}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_c${CFG}${PROF_SUFFIX}
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
# PROF_EXTRA: more bench arguments (e.g. "--pktin-opt 0x3C" for the checksum path)
ARGS="--config $CFG --n $N --steps 20 --warmup 5 --timed-only $PROF_EXTRA"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
  -- python3 "$ROOT/bench.py" $ARGS > "$OUT/kt.log" 2>&1 || { echo "kt failed"; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p \
    -- python3 "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed: $set"; exit 1; }
  i=$((i+1))
done
echo done
