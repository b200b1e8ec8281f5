set -o pipefail
bash tools/variants.sh "WIN=128" "WIN=64" || exit 1
for g in 2 8 16; do MI_CLS_BLOCKS_PER_CU=$g CFGS="20 2" bash tools/variants.sh "WIN=64" | sed "s/^/bpc=$g /" || exit 1; done
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
