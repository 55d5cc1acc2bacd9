#!/bin/bash
# Round 3: unit-stride x / rhs stores in k_dir_step -- direct tests, phases, bench, profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03aa}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dstep.py tests/test_gpu_direct.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1; rc=$?
echo bench rc=$rc; tail -c 300 gpurun_out/${T}_bench.log
[ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh $T > gpurun_out/${T}_profile.log 2>&1; echo profile rc=$?
