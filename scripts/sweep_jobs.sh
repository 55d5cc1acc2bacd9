#!/bin/bash
# Bench at several preconditioner job counts (NXHIP_PC_JOBS); one line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for j in ${JOBS:-128 256 384 512}; do
  echo "=== jobs $j"
  NXHIP_PC_JOBS=$j timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/sweep_jobs_$j.log 2>&1 || { echo "rc=$?"; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_jobs_$j.log | head -1
done
