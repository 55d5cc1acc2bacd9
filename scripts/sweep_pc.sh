#!/bin/bash
# decomposition sweep of the tree preconditioner on the bench workload
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for j in ${JOBS:-64 128 256 512 1024}; do
  echo -n "NXHIP_PC_JOBS=$j: "
  NXHIP_PC_JOBS=$j timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sw.json 2>/dev/null || { echo fail; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(round(d['ms_per_step'],3),'ms', d['config']['minres_iterations'],'its')"
done
