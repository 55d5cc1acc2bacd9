#!/bin/bash
# Round 3: top-part indices issued before the arrival (k_dir_step) -- tests, phases, then an
# A/B of the bench on one box: the new library, the previous one (libnxhip_ab.so), the new.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03ad}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dstep.py tests/test_gpu_direct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo tests rc=$rc; tail -2 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dstep_phases.py > gpurun_out/${T}_phases.log 2>&1; echo phases rc=$?
grep -E "top part by|top values|published" gpurun_out/${T}_phases.log
for v in new ab new ab; do
  if [ $v = ab ]; then L=networks_fenicsx_amd/libnxhip_ab.so; else L=networks_fenicsx_amd/libnxhip.so; fi
  NXHIP_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench_$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
