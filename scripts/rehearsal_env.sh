#!/bin/bash
# failing rehearsal config under each alternative kernel path (env toggles)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${R:-4}; L=${L:-15}
for ev in NONE=1 NXHIP_PC_LIN=0 NXHIP_PC_GLOBAL=1 NXHIP_BETA_P2P=0 NXHIP_PC_DENSE=0 NXHIP_PC_FACTOR=0 NXHIP_PC_FUSE=0 NXHIP_LEAN=0; do
  env $ev timeout -k 10 300 python -u scripts/group_rehearsal.py --ranks $R --levels $L --reps 1 > gpurun_out/rehenv_$ev.log 2>&1
  rc=$?
  echo "$ev rc=$rc: $(grep -h 'REHEARSAL\|diverged\|Error\|first solve' gpurun_out/rehenv_$ev.log | tail -2 | tr '\n' ' ' | cut -c1-250)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for cfg in "4 13" "4 14" "16 12"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/group_rehearsal.py --ranks $1 --levels $2 --reps 1 > gpurun_out/reh_$1_$2.log 2>&1
  rc=$?
  echo "ranks $1 levels $2 rc=$rc: $(grep -h 'REHEARSAL\|diverged\|Error' gpurun_out/reh_$1_$2.log | tail -1 | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
