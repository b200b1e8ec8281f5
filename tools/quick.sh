#!/bin/bash
# Quick GPU check: GPU tests, then kernel time (one stream) per config.
# Usage: tools/quick.sh TAG "CFGS" [skip-tests] [pytest -k expr]
set -o pipefail
TAG=$1
CFGS=${2:-"3 33 2 4 5"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$3" != "skip-tests" ]; then
  K=${4:+-k "$4"}
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K \
    > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
for c in $CFGS; do
  timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --timed-only > $OUT/c$c.json 2> $OUT/c$c.err \
    || { echo "bench $c failed"; tail $OUT/c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c$c.json')); print('config $c', d['config']['workload'], 'kernel_us', round(d['roofline']['kernel_ms']*1e3,2), 'frac', d['roofline']['frac'], 'Mpkt/s', d['value'])"
done
