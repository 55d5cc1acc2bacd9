#!/bin/bash
# Round 3: the (k, 0) direct solve through the condensed system -- FE tests, the direct
# tests (shared sweeps, mass pivots), FE timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03y}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fe.py tests/test_gpu_direct.py tests/test_gpu_dstep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/fe_timing.py 9 8 > gpurun_out/${T}_fe_timing.log 2>&1; rc=$?
echo fe_timing rc=$rc; cat gpurun_out/${T}_fe_timing.log
exit $rc
