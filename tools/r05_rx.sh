#!/bin/bash
# round 5: receive-path GPU tests, then the receive rates (tools/rx_rate.sh)
set -o pipefail
TAG=${1:-r05rx}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -60 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 tools/rx_rate.sh gpurun_out/${TAG} 200000 10 > gpurun_out/${TAG}_rate.txt 2>&1 || { cat gpurun_out/${TAG}_rate.txt; exit 1; }
cat gpurun_out/${TAG}_rate.txt
