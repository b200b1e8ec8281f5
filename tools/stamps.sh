#!/bin/bash
# Per-phase cycle sums per wave (-DDIAG_STAMPS build): p0 = wait for the
# tile's window + LDS staging, p1 = next tile's loads issued, p2 = parse,
# p3 = CoS descent, p4 = outcome / record.  Run from the repo root via gpurun.
set -o pipefail
timeout -k 10 300 python -m odp_amd._build /tmp/vdiag DIAG_STAMPS $STAMP_DEFS > /dev/null || exit 1
for args in "--config 20" "--config 2" "--config 33" "--config 2 --n 4000000"; do
  echo "== $args"
  ODP_AMD_LIB_DIR=/tmp/vdiag timeout -k 10 200 python bench.py $args --steps 3 --warmup 1 --no-cpu \
    --no-extra --streams 1 2>&1 >/dev/null | grep DIAG | tail -1 || exit 1
done
