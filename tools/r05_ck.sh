#!/bin/bash
# round 5: checksum-path parity tests and kernel times (config 3 UDP/TCP and
# config 3 with a third SCTP, pktin option 0x3C)
set -o pipefail
TAG=${1:-r05ck}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_chksum.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python -u tools/ab.py --libs odp_amd --configs 3,35 --bench-args "--pktin-opt 0x3C" > gpurun_out/${TAG}_ab.txt 2>&1 || { cat gpurun_out/${TAG}_ab.txt; exit 1; }
cat gpurun_out/${TAG}_ab.txt
