set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/variants.sh "WIN=128" "WIN=64" || exit 1
