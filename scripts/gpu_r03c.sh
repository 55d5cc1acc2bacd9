#!/bin/bash
# Round 3: the fused direct step (deferred stores) and the cycle correction, phases, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03f}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dstep.py tests/test_gpu_direct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -5 gpurun_out/${T}_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
timeout -k 10 200 python bench.py --no-cpu-baseline --api-steps 0 --steps 200 > gpurun_out/${T}_bench_fused.log 2>&1 && \
NXHIP_DIR_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline --api-steps 0 --steps 200 > gpurun_out/${T}_bench_launches.log 2>&1
echo rc=$?
