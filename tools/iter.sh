#!/bin/bash
# One kernel iteration on the GPU box: parity tests, then kernel times of the
# in-tree build for the bench configs (one stream), then the phase stamps.
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_parity.py} NO_BENCH=1 bash tools/gpu_check.sh || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
CFGS=${CFGS:-"2 33 3 4 5"} BENCH_EXTRA="--streams 1" bash tools/variants.sh "env X=1" 2>&1 | grep -v amdgpu.ids || exit 1
[ -n "$NO_STAMPS" ] || bash tools/stamps.sh
