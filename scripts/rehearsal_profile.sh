#!/bin/bash
# kernel trace of the 8-rank group rehearsal (depth-17 bench workload): per-rank launch
# times of the preconditioner sweeps show the ranks' load balance
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_reh_${TAG:-a}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace --output-format csv -- \
  python3 "$R/scripts/group_rehearsal.py" --ranks 8 --levels 15 --reps 3 ${REH_ARGS} > "$OUT/run.log" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$OUT/run.log"; exit $rc
