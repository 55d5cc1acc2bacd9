#!/bin/bash
# Round 3: multi-rank fused up kernel (k_dir_team_up): group/RCCL/direct tests, the 8-rank
# C4 rehearsal's per-rank kernel times, then the bench workload's rocprofv3 stats + PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_dstep.py tests/test_gpu_direct.py tests/test_gpu_c4.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -4 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
TAG=$T bash scripts/rehearsal_profile.sh; rc=$?
[ $rc -ne 0 ] && exit $rc
python scripts/rank_times.py gpurun_out/prof_reh_$T/trace_kernel_trace.csv 8 > gpurun_out/${T}_rank_times.txt 2>&1; cat gpurun_out/${T}_rank_times.txt
[ -n "$SKIP_PROF" ] && exit 0
bash scripts/profile.sh $T
