#!/bin/bash
# Round 3: rocprofv3 kernel stats of the (2, 0) direct solve at the C3 tree.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/prof_r03af"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace --output-format csv -- python3 "$R/scripts/fe_timing.py" 15 15 "2,0" > "$OUT/run.log" 2>&1
rc=$?; echo rc=$rc; tail -3 "$OUT/run.log"
find "$OUT" -name '*kernel_stats.csv' | head -2
exit $rc
