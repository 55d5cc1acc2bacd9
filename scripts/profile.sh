#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
# Usage: scripts/profile.sh <tag> [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "=== $name"; date
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@"
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@"
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@"
find "$OUT" -name '*.csv' | head -20
