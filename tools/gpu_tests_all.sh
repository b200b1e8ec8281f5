set -o pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=30 > gpurun_out/r02h/pytest.txt 2>&1
grep -E "FAILED|passed|failed" gpurun_out/r02h/pytest.txt | tail -40
exit 0
