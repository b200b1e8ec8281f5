#!/bin/bash
# Block-shape A/B for one or more configs: kernel time per launch (HIP events,
# single stream) with MI_CLS_WPB forcing 4 / 8 / 12 / 16-wave blocks, beside
# the automatic choice.  Usage (repo root, via gpurun): tools/shape_ab.sh "4 5"
set -o pipefail
for c in ${1:-4 5}; do
  for w in auto 4 8 12 16; do
    if [ $w = auto ]; then unset MI_CLS_WPB; else export MI_CLS_WPB=$w; fi
    r=$(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --timed-only \
        --no-parity 2>/dev/null) || { echo "config $c wpb $w failed"; exit 1; }
    echo "config $c wpb $w: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
unset MI_CLS_WPB
