#!/bin/bash
# Per-launch kernel time vs batch size (single stream, HIP events): the
# fixed per-launch cost is the intercept.  Usage (via gpurun): tools/nscale.sh "3 2"
set -o pipefail
for c in ${1:-3}; do
  for n in 250000 1000000 2000000 4000000; do
    r=$(timeout -k 10 120 python bench.py --config $c --n $n --steps 10 --warmup 3 --timed-only \
        --no-parity 2>/dev/null) || { echo "config $c n $n failed"; exit 1; }
    echo "config $c n $n: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
# same-buffer launches (warm translations; 4 M packets keep the header bytes
# well past the 256 MiB Infinity Cache)
for c in ${1:-3}; do
  r=$(timeout -k 10 120 python bench.py --config $c --n 4000000 --rotate 1 --steps 10 --warmup 3 \
      --timed-only --no-parity 2>/dev/null) || { echo "config $c rotate 1 failed"; exit 1; }
  echo "config $c n 4000000 rotate 1: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
