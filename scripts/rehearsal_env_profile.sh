#!/bin/bash
# per-rank kernel times of the 8-rank rehearsal under alternative multi-rank paths
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for ev in NONE=1 NXHIP_PC_FUSE=0 NXHIP_PC_LIN=0 NXHIP_PC_DENSE=0; do
  echo "=== $ev"
  env $ev TAG="env_${ev%%=*}" bash "$R/scripts/rehearsal_profile.sh" > /dev/null 2>&1 || { echo "rc=$?"; exit 1; }
  python3 "$R/scripts/rank_times.py" "$R/gpurun_out/prof_reh_env_${ev%%=*}/trace_kernel_trace.csv" | grep "k_pc\|k_mr\|coarse\|cpart\|group"
done
