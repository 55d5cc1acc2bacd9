#!/bin/bash
# A/B step time of the direct solve at C4 on one GPU under env settings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "$@"; do
  echo "=== $cfg"
  env $cfg timeout -k 10 300 python -u scripts/direct_timing.py 18 19 20 2>&1 | grep -v amdgpu.ids || exit $?
done
