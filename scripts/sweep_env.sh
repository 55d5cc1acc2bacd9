#!/bin/bash
# Bench under several values of one environment variable: VAR=NAME VALUES="a b c".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VALUES}; do
  echo "=== ${VAR}=$v"
  env "${VAR}=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    > "gpurun_out/sweep_${VAR}_$v.log" 2>&1 || { echo "rc=$?"; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"assembly_kernel_ms": [0-9.]*' "gpurun_out/sweep_${VAR}_$v.log" | head -2 | tr '\n' ' '; echo
done
