set -o pipefail
for st in 1 2 4; do
 for c in "--config 2" "--config 33" "--config 2 --n 250000"; do
  timeout -k 10 200 python bench.py $c --streams $st --steps 60 --warmup 5 --no-cpu --no-extra > /tmp/v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/v.json')); print('streams $st', '$c', d['roofline']['kernel_ms'], d['ms_per_step'], d['value'])"
 done
done
