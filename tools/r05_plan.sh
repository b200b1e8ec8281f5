#!/bin/bash
# round 5: tree-plan kernel parity + timing (config 5)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifecycle.py -x -q --timeout 300 --timeout-method thread -k "config5 or joint or fuzz or configs_small or lifecycle or bench_order or many_classes" > gpurun_out/r05d_pytest.txt 2>&1 || { tail -40 gpurun_out/r05d_pytest.txt; exit 1; }
tail -3 gpurun_out/r05d_pytest.txt
timeout -k 10 300 python -u tools/ab.py --libs odp_amd --configs 5 > gpurun_out/r05d_ab.txt 2>&1 || { cat gpurun_out/r05d_ab.txt; exit 1; }
timeout -k 10 300 python -u tools/ab.py --libs odp_amd --configs 5 --env MI_CLS_NO_PLAN=1 >> gpurun_out/r05d_ab.txt 2>&1
cat gpurun_out/r05d_ab.txt
