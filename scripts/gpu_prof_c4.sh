set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o c4 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/direct_timing.py 18 19 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1; echo prof rc=$?
