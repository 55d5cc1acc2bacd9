#!/bin/bash
# A/B step time of the direct solve under env settings: scripts/gpu_ab.sh "ENV=.. ENV=.." "..." ...
# (C3, 200 steps each, then C4 50 steps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "=== $cfg"
  env $cfg timeout -k 10 200 python -u scripts/direct_timing.py 15 15 200 2>&1 | grep -v amdgpu.ids || exit $?
done
