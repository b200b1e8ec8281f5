set -o pipefail
for v in "" "MI_CLS_BLOCKS_PER_CU=1" "MI_CLS_BLOCKS_PER_CU=2" "MI_CLS_BLOCKS_PER_CU=3"; do
 for c in "--config 2" "--config 2 --n 4000000" "--config 33" "--config 20"; do
  env $v timeout -k 10 200 python bench.py $c --steps 30 --warmup 5 --no-cpu --no-extra > /tmp/v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/v.json')); print('$v', '$c', d['roofline']['kernel_ms'], round(d['roofline']['kernel_ms']*1e6/d['config']['packets_per_gpu'],3), 'ns/pkt')"
 done
done
