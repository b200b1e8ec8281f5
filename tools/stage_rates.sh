#!/bin/bash
# Kernel time of the diagnostic builds (stage only / parse only / descent
# only / full) at two batch sizes, so the marginal cost per packet of each
# stage can be read off (config 2, one stream, rotation as in the bench).
set -o pipefail
mkdir -p gpurun_out
i=0
for v in DIAG_STAGEONLY DIAG_PARSEONLY DIAG_DESCENTONLY VB_FULL; do
  d=/tmp/sr_$i
  timeout -k 10 300 python -m odp_amd._build $d $v > /dev/null || exit 1
  for n in 1000000 4000000; do
    for st in 1 2; do
      ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config ${CFG:-2} --n $n --steps 30 --warmup 5 \
        --no-cpu --no-extra --streams $st > /tmp/v.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('/tmp/v.json')); print('$v n=$n streams=$st', d['roofline']['kernel_ms'], d['ms_per_step'])"
    done
  done
  i=$((i+1))
done
