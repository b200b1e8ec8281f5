#!/bin/bash
# One GPU-box session: GPU tests, the default bench line, then rocprofv3
# kernel-trace + PMC summaries for the listed configs.
# Usage (repo root, through gpurun): tools/gpu_round.sh TAG "CONFIGS" [skip-tests]
set -o pipefail
TAG=$1
CFGS=${2:-"3 33 2 4 5"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
  tail -3 $OUT/pytest.txt
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for c in $CFGS; do
  timeout -k 10 900 tools/profile.sh $TAG $c > $OUT/prof_c$c.log 2>&1 || { echo "profile $c failed"; cat $OUT/prof_c$c.log; exit 1; }
  echo "profiled $c"
done
