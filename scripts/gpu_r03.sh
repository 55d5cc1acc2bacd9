#!/bin/bash
# Round 3 checks: the fused direct step and the RCCL direct tests, then a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step ${TAG:-r03}_dstep 300 python -u -m pytest tests/test_gpu_dstep.py -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS}
step ${TAG:-r03}_rccl 300 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread -k rccl
step ${TAG:-r03}_bench 300 python bench.py --no-cpu-baseline --api-steps 0 ${BENCH_ARGS}
