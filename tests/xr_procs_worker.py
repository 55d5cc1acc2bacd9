"""One rank of tests/test_gpu_xr_procs.py: a partitioned network problem with one process per
rank, several processes on ONE GPU.

RCCL refuses two ranks on one device, so the ranks use the library's host transport
(``NXHIP_TRANSPORT=host`` -> ``nx_comm_init_host``): the RCCL ranks' host logic unchanged --
the exchange step's mailboxes IPC-mapped between the processes, the per-rank give-up and
agreement, the graph path -- with its collectives through shared memory. Host control
(graph broadcast, IPC handle all-gather) goes over gloo, as in bench.py.

Each step: assemble + solve (the direct solve), then a gloo barrier (a host collective
between steps, as a user's code would have). Writes ``rank<r>.json`` (per step: residual,
path, exchange status) and ``rank<r>.npz`` (global rows, x per step) into ``--out``.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="depth6_N40")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--give-up-rank", type=int, default=-1)
    ap.add_argument("--give-up-which", type=int, default=1, help="0: exchange 1, 1: exchange 2")
    ap.add_argument("--give-up-step", type=int, default=2)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()

    import numpy as np
    import torch  # noqa: F401  (first: libnxhip binds to torch's HIP runtime)
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)

    import distributed_model as DM
    from cases import CASES
    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
    from networks_fenicsx_amd.comm import TorchComm

    make, N, strategy, pbc = CASES[args.case]
    G = make() if rank == 0 else None
    mesh = NetworkMesh(G, N=N, color_strategy=strategy, comm=TorchComm())
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=pbc)
    asm.set_direct(True)
    h = asm.handle
    rows = DM.global_rows(asm.local_problem, mesh.num_edges, mesh.bifurcation_index)
    steps, xs = [], []
    for k in range(args.steps):
        if rank == args.give_up_rank and k in (args.give_up_step, args.give_up_step + 1):
            h.xr_polls(args.give_up_which, 0 if k == args.give_up_step else 1 << 20)
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 50000, 4)
        steps.append({"step": k, "iterations": it, "relres": rr, "converged": conv,
                      "solver": "direct" if h.solver()[1] == 1 else "minres",
                      "path": h.direct_path(), "xr": h.xr_status()})
        xs.append(h.solution())
        dist.barrier()
    out = Path(args.out)
    np.savez(out / f"rank{rank}.npz", rows=rows, x=np.stack(xs))
    (out / f"rank{rank}.json").write_text(json.dumps({"rank": rank, "steps": steps}))
    dist.barrier()
    asm.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
