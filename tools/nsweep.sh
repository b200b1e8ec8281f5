#!/bin/bash
# Kernel time vs batch size (fixed per-launch cost = intercept).  Usage: tools/nsweep.sh "CFGS"
set -o pipefail
for c in ${1:-3}; do
  for n in 250000 500000 1000000 2000000 4000000; do
    timeout -k 10 200 python bench.py --config $c --n $n --steps 20 --warmup 3 --timed-only > /tmp/t.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('/tmp/t.json')); print('config $c n=$n kernel_us', round(d['roofline']['kernel_ms']*1e3,2))"
  done
done
