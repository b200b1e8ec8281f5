#!/bin/bash
# A/B kernel variants on the GPU box: build each -D set into its own dir and
# time the bench's kernel for several workloads.  "DEFS|ENV" runs the build
# with -D DEFS under environment ENV; "env ENV" uses the in-tree build.
#   tools/variants.sh "WIN=128" "WIN=96 WAVES_PER_BLOCK=16|MI_CLS_LDS_HOT_MAX=52000"
set -o pipefail
CFGS=${CFGS:-"20 2 3 5"}
mkdir -p gpurun_out
i=0
for v in "$@"; do
  d=$(pwd)/odp_amd
  envs=""
  defs=""
  if [[ "$v" == env\ * ]]; then
    envs=${v#env }
  else
    defs=${v%%|*}
    [[ "$v" == *"|"* ]] && envs=${v#*|}
    d=/tmp/variant_$i
    timeout -k 10 300 python -m odp_amd._build $d $defs > /dev/null || exit 1
  fi
  for c in $CFGS; do
    env $envs ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 \
      --no-cpu --no-extra $BENCH_EXTRA > /tmp/v.json || exit 1
    python -c "import json; d=json.load(open('/tmp/v.json')); print('$v', d['config']['workload'], d['config']['rules'], d['roofline']['kernel_ms'], d['value'])"
  done
  i=$((i+1))
done
