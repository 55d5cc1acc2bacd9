#!/bin/bash
# Round 3: tests of the direct paths, the fused step's phases, bench, then rocprofv3 stats +
# PMC passes of the bench workload (scripts/profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dstep.py tests/test_gpu_direct.py tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1; echo bench rc=$?
bash scripts/profile.sh $T > gpurun_out/${T}_profile.log 2>&1; echo profile rc=$?
