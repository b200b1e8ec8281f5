#!/bin/bash
# PC sampling of the dominant kernel (stochastic, gfx950), one config.
# Usage (via gpurun): tools/pcsamp.sh <config>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pcs_c$1
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d $OUT -o pcs \
  -- python3 $ROOT/bench.py --config $1 --steps 20 --warmup 3 --timed-only --no-parity \
  > $OUT/run.log 2>&1; rc=$?
ls -la $OUT $OUT/* | head -20
tail -5 $OUT/run.log
exit $rc
