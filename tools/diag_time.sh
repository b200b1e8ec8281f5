#!/bin/bash
# Where a launch's time goes: per-phase cycles per wave (-DDIAG_STAMPS: p5
# block setup, p0 wait for the tile's window + LDS staging, p1 next loads
# issued, p2 parse, p3 descent, p4 outcome, p6 final store), stage-only and
# full kernel time at 1 M and 4 M packets.  Usage: tools/diag_time.sh "CFGS"
set -o pipefail
CFGS=${1:-"3"}
timeout -k 10 300 python -m odp_amd._build /tmp/vst DIAG_STAMPS > /dev/null || exit 1
timeout -k 10 300 python -m odp_amd._build /tmp/vso DIAG_STAGEONLY > /dev/null || exit 1
for c in $CFGS; do
  for n in 1000000 4000000; do
    for d in /tmp/vso $(pwd)/odp_amd; do
      ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config $c --n $n --steps 20 --warmup 3 --timed-only > /tmp/t.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('/tmp/t.json')); print('config $c n=$n lib=$d kernel_us', round(d['roofline']['kernel_ms']*1e3,2))"
    done
  done
  ODP_AMD_LIB_DIR=/tmp/vst timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --timed-only 2>&1 >/dev/null | grep DIAG | tail -1 || exit 1
done
