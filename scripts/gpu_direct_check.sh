set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/direct_tests.log 2>&1; rc=$?; tail -5 gpurun_out/direct_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/direct_timing.py 15 15 50 > gpurun_out/direct_timing.log 2>&1 && cat gpurun_out/direct_timing.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_direct -o dt --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/direct_timing.py 15 15 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_direct.log 2>&1; echo prof rc=$?
