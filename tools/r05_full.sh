#!/bin/bash
# round 5: full GPU suite, then A/B kernel times of the BASELINE configs
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -60 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 400 python -u tools/ab.py --libs odp_amd --configs 3,33,2,4,5 > gpurun_out/${TAG}_ab.txt 2>&1 || { cat gpurun_out/${TAG}_ab.txt; exit 1; }
cat gpurun_out/${TAG}_ab.txt
