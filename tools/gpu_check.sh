#!/bin/bash
# One GPU-box round trip: GPU tests, then a short bench.  Each GPU step has
# its own time limit; steps are chained so a failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_runtime.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest_rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --cpu-seconds 3} > gpurun_out/bench.log 2>&1
