set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/direct_timing.py 18 19 20 > gpurun_out/direct_timing_c4.log 2>&1; cat gpurun_out/direct_timing_c4.log
