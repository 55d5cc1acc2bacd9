#!/bin/bash
# Round 3 validation: the whole GPU suite, smoke, the fused step's phases, the default bench
# (with the CPU baseline leg), then the rocprofv3 trace + PMC passes (scripts/profile.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03z}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/${T}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${T}_smoke.log 2>&1; rc=$?
echo smoke rc=$rc; tail -2 gpurun_out/${T}_smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?
echo bench rc=$rc; tail -c 400 gpurun_out/${T}_bench.log
[ $rc -ne 0 ] && exit $rc
[ -n "$SKIP_PROF" ] || { bash scripts/profile.sh $T > gpurun_out/${T}_profile.log 2>&1; echo profile rc=$?; }
