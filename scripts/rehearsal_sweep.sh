#!/bin/bash
# group rehearsal over (ranks, levels); stops at the first crash/timeout (rc other than 0/1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# CFGS="ranks:levels ..." (default below)
for cfg in ${CFGS:-2:12 2:15 4:12 4:15 8:8 8:10 8:12 8:14}; do
  set -- ${cfg/:/ }
  timeout -k 10 300 python -u scripts/group_rehearsal.py --ranks $1 --levels $2 --reps 1 > gpurun_out/reh_$1_$2.log 2>&1
  rc=$?
  echo "ranks $1 levels $2 rc=$rc: $(grep -h 'REHEARSAL\|diverged\|Error' gpurun_out/reh_$1_$2.log | tail -1 | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
