#!/bin/bash
# Round 3: group (team kernel) tests first, then the fused step's tests, phases, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03v}
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_dstep.py tests/test_gpu_direct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1; echo bench rc=$?
TAG=$T bash scripts/rehearsal_profile.sh > /dev/null 2>&1; echo reh rc=$?
python scripts/rank_times.py gpurun_out/prof_reh_$T/trace_kernel_trace.csv 8 > gpurun_out/${T}_rank_times.txt 2>&1; cat gpurun_out/${T}_rank_times.txt
