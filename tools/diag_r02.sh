#!/bin/bash
# Per-phase cycles (DIAG_STAMPS build in build/diag, made on the CPU side by
# `python -m odp_amd._build build/diag DIAG_STAMPS`) and SQ/TA/TCC counters
# for configs 2-5.  Usage (repo root, via gpurun): tools/diag_r02.sh
set -o pipefail
for c in ${DIAG_CFGS:-2 3 4 5}; do
  echo "== config $c"
  ODP_AMD_LIB_DIR=build/diag timeout -k 10 120 python bench.py --config $c --steps 3 --warmup 1 \
    --timed-only 2>&1 >/dev/null | grep DIAG | tail -1 || exit 1
done
for c in ${CTR_CFGS:-4 5}; do
  tools/counters.sh c$c "--config $c --steps 5 --warmup 2 --timed-only" || exit 1
done
