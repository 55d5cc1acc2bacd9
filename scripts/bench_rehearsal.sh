#!/bin/bash
# The multi-rank bench path (bench.py --gpus 2) on ONE GPU: two processes, the library's host
# transport in place of RCCL (NXHIP_TRANSPORT=host; RCCL refuses two ranks on one device), a
# small tree so that both ranks' one-launch exchange steps are co-resident. Checks bench.py's
# N > 1 code end to end (rendezvous, partition, exchange step, timing, the JSON line).
# C4=1 adds the configs[4] leg (its two ranks' launches cannot be co-resident on one GPU, so
# their exchange gives up and the ranks take the graph path together).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
LEVELS=${LEVELS:-8}
C4ARG=--no-c4
[ "${C4:-0}" = 1 ] && C4ARG=
NXHIP_TRANSPORT=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
  --steps 20 --warmup 5 --levels "$LEVELS" --N 15 $C4ARG --api-steps 2
