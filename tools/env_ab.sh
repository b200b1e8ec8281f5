#!/bin/bash
# Kernel time per launch (single stream) with and without one environment
# setting.  Usage (via gpurun): tools/env_ab.sh "VAR=value" "3 2"
set -o pipefail
for c in ${2:-3}; do
  for e in "" "$1"; do
    r=$(env $e timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --timed-only \
        --no-parity 2>/dev/null) || { echo "config $c $e failed"; exit 1; }
    echo "config $c ${e:-default}: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["value"])')"
  done
done
