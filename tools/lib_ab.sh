#!/bin/bash
# Kernel time per launch (single stream, HIP events) for an alternative
# build (ODP_AMD_LIB_DIR) against the in-tree one, per config.
# Usage (via gpurun): tools/lib_ab.sh build/variant "3 4 5"
set -o pipefail
V=$1
for c in ${2:-3 4 5}; do
  for lib in "" "$V"; do
    r=$(ODP_AMD_LIB_DIR=${lib:-odp_amd} timeout -k 10 120 python bench.py --config $c --steps 20 \
        --warmup 5 --timed-only --no-parity 2>/dev/null) || { echo "config $c $lib failed"; exit 1; }
    echo "config $c ${lib:-in-tree}: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
