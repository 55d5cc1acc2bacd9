#!/bin/bash
# Direct solve check on the GPU: direct / C4 / group tests, C3 + C4 timing and C4 accuracy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_c4.py tests/test_gpu_group.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_direct_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_direct_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/direct_timing.py 15 15 50 2>&1 | grep -v amdgpu.ids | tee gpurun_out/direct_timing_c3.log || exit $?
timeout -k 10 400 python -u scripts/direct_accuracy.py 18 19 2>&1 | grep -v amdgpu.ids | tee gpurun_out/direct_accuracy_c4.log || exit $?
timeout -k 10 400 python -u scripts/direct_timing.py 18 19 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/direct_timing_c4.log
