#!/bin/bash
# Profile the bench's dominant kernel on the GPU box (run through gpurun from
# the repo root).  Three separate rocprofv3 runs, as MI355X_MICROARCH.md
# prescribes: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS=("$@")
if [ ${#ARGS[@]} -eq 0 ]; then
  ARGS=(--steps 20 --warmup 5 --no-cpu --no-extra --streams 1)
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/write.log" 2>&1
find "$OUT" -name "*.csv" | sort > "$OUT/files.txt"
echo done
