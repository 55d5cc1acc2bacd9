#!/bin/bash
# geometry sweep of the MINRES kernels on the bench workload (one process per setting)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for a in 1 2 4; do for b in 256 512 1024; do
  echo -n "A_CHUNKS=$a B_BLOCKS=$b: "
  NXHIP_A_CHUNKS=$a NXHIP_B_BLOCKS=$b timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sw.json 2>/dev/null || { echo fail; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(round(d['ms_per_step'],3),'ms', d['config']['minres_iterations'],'its', round(d['roofline']['avg_launch_ms']*1e3,2),'us k_mr_a')"
done; done
