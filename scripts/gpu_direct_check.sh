set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/direct_timing.py 15 15 50 > gpurun_out/direct_timing.log 2>&1 && cat gpurun_out/direct_timing.log
timeout -k 10 300 python -u scripts/phase_timing.py 15 15 direct > gpurun_out/phase_direct.log 2>&1; tail -6 gpurun_out/phase_direct.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_direct -o dt --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/direct_timing.py 15 15 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_direct.log 2>&1; echo prof rc=$?
