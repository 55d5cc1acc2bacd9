#!/bin/bash
# PC chain-variant sweep: phase timing + bench per (W, CPL) variant (NXHIP_PC_VARIANT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 5 6 7}; do
  echo "=== variant $v"
  NXHIP_PC_VARIANT=$v timeout -k 10 300 python scripts/phase_timing.py > gpurun_out/phase_v$v.log 2>&1 || exit $?
  grep -E "k_pc|^up|^down" gpurun_out/phase_v$v.log
  NXHIP_PC_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]); print('ms/step', round(d['ms_per_step'],4), 'it', d['config']['minres_iterations'])"
done
