#!/bin/bash
# Kernel trace of the bench's direct step + its per-step timeline (gaps between dispatches).
# Usage: scripts/gpu_timeline.sh <tag> [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r02}; shift
OUT="$R/gpurun_out/tl_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- \
  python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --api-steps 0 "$@" > "$OUT/bench.log" 2>&1 || exit $?
F=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/scripts/timeline.py" "$F" k_assemble_seg 5 > "$OUT/timeline.txt" || exit $?
cat "$OUT/timeline.txt"
