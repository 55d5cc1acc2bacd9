"""One rank of tests/test_gpu_fe_ranks.py: a (k, m) problem partitioned over processes, several
on ONE GPU, through the library's host transport (``NXHIP_TRANSPORT=host``: the RCCL ranks'
host logic with the collectives through shared memory; host control over gloo).

Each step: assemble + solve ((k, 0): the condensed direct solve -- condense per edge, the
ranks' direct tree solve of the auxiliary P1/DG0 system, expand, the residual over the
ranks; continuous pressure: plain MINRES over the halo), a gloo barrier; then one
plain-MINRES solve (``--minres``). Writes ``rank<r>.json`` and
``rank<r>.npz`` (one-rank layout rows of the owned rows, x per solve) into ``--out``.
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
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--m", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--minres", type=int, default=0)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()

    import numpy as np
    import torch  # noqa: F401  (first: libnxhip binds to torch's HIP runtime)
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)

    from cases import CASES
    from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh
    from networks_fenicsx_amd.comm import TorchComm
    from networks_fenicsx_amd.layout_fe import fe_global_rows

    make, N, strategy, pbc = CASES[args.case]
    G = make() if rank == 0 else None
    mesh = NetworkMesh(G, N=N, color_strategy=strategy, comm=TorchComm())
    asm = HydraulicNetworkAssembler(mesh, flux_degree=args.k, pressure_degree=args.m)
    E = mesh.num_edges
    asm.compute_forms(p_bc_ex=pbc, f=0.3, R=1.0 + 0.5 * (np.arange(E) % 3))
    asm.set_direct(True)
    h = asm.handle
    rows = fe_global_rows(asm.fe_layout, mesh.degrees)
    steps, xs = [], []
    for k in range(args.steps):
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 50000, 4)
        steps.append({"step": k, "iterations": it, "relres": rr, "converged": conv,
                      "solver": "direct" if h.solver()[1] == 1 else "minres",
                      "path": h.direct_path(), "direct_available": asm.fe_direct_available})
        xs.append(h.solution())
        dist.barrier()
    if args.minres:
        asm.set_direct(False)
        it, rr, conv = h.solve(1e-12, 50000, 4)
        steps.append({"step": "minres", "iterations": it, "relres": rr, "converged": conv,
                      "solver": "direct" if h.solver()[1] == 1 else "minres"})
        xs.append(h.solution())
    out = Path(args.out)
    np.savez(out / f"rank{rank}.npz", rows=rows, x=np.stack(xs))
    (out / f"rank{rank}.json").write_text(json.dumps({"rank": rank, "steps": steps}))
    dist.barrier()
    asm.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
