#!/bin/bash
# A/B on config 5: window forced on, port merge off
set -o pipefail
timeout -k 10 300 python -m odp_amd._build /tmp/vhi DIAG_FORCE_HI > /dev/null || exit 1
for v in "NONE=1|$(pwd)/odp_amd" "MI_CLS_NO_PORTMERGE=1|$(pwd)/odp_amd" "NONE=1|/tmp/vhi" "MI_CLS_DIV=1|$(pwd)/odp_amd"; do
  e=${v%%|*}; d=${v#*|}
  for c in ${CFGS:-5}; do
  env $e ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --timed-only > /tmp/t.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/t.json')); print('$e $d config $c kernel_us', round(d['roofline']['kernel_ms']*1e3,2))"
  done
done
