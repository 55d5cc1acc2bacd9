#!/bin/bash
# Round 3: the whole GPU suite, the fused step's phase stamps, the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -5 gpurun_out/${T}_gpu_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1; echo bench rc=$?
tail -c 600 gpurun_out/${T}_bench.log
