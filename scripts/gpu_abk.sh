#!/bin/bash
# A/B per-kernel times of the direct step under env settings (scripts/direct_kernels.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "$@"; do
  echo "=== $cfg"
  env $cfg timeout -k 10 200 python -u scripts/direct_kernels.py 15 15 200 2>&1 | grep -v amdgpu.ids || exit $?
done
