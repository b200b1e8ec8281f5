set -o pipefail
for r in 1 4; do
 for c in "--config 2" "--config 20" "--config 33" "--config 3"; do
  timeout -k 10 200 python bench.py $c --rotate $r --steps 30 --warmup 5 --no-cpu --no-extra > /tmp/v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/v.json')); print('rotate $r', '$c', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'])"
 done
done
timeout -k 10 300 python -m odp_amd._build /tmp/vstage DIAG_STAGEONLY > /dev/null || exit 1
for r in 1 4; do
  ODP_AMD_LIB_DIR=/tmp/vstage timeout -k 10 200 python bench.py --config 2 --rotate $r --steps 30 --warmup 5 --no-cpu --no-extra > /tmp/v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/v.json')); print('stageonly rotate $r', d['roofline']['kernel_ms'])"
  ODP_AMD_LIB_DIR=/tmp/vstage timeout -k 10 200 python bench.py --config 2 --n 4096 --rotate $r --steps 30 --warmup 5 --no-cpu --no-extra > /tmp/v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/v.json')); print('stageonly n=4096 rotate $r', d['roofline']['kernel_ms'])"
done
