set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/phase_timing.py 15 15 direct > gpurun_out/phase_direct.log 2>&1; cat gpurun_out/phase_direct.log
