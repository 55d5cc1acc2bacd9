#!/bin/bash
# Round 3: k_dir_team_up phase stamps with the helpers (debug build), 8-rank C4 rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r03ac}
timeout -k 10 200 python scripts/team_phases.py 8 15 19 > gpurun_out/${T}_team_phases.log 2>&1; rc=$?
echo phases rc=$rc; cat gpurun_out/${T}_team_phases.log
exit $rc
