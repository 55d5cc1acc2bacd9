#!/bin/bash
# Round 3: the (k, 0) direct solve at the C3 tree (depth 14, N = 15): timing against plain
# MINRES, P1/DG0 beside it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03ae}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_fe_tests.log 2>&1; rc=$?
echo fe tests rc=$rc; tail -2 gpurun_out/${T}_fe_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/fe_timing.py 15 15 "1,0;2,0;3,0" > gpurun_out/${T}_fe_timing_c3.log 2>&1; rc=$?
echo rc=$rc; cat gpurun_out/${T}_fe_timing_c3.log
exit $rc
