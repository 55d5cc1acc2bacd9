"""Accuracy of one direct pass vs one refinement step on a tree (GPU): true residual and
error against the analytic resistor-network answer. python scripts/direct_accuracy.py [levels N]"""

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from oracle import nx_oracle as O  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 else 18
N = int(sys.argv[2]) if len(sys.argv) > 2 else 19
mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
asm = HydraulicNetworkAssembler(mesh)
asm.compute_forms(p_bc_ex=lambda x: x[1])
src, dst = mesh.edges
P = O.build_problem(mesh.node_coordinates, src, dst, N)
xa = O.resistor_network_solution(P, lambda x: x[1])[O.build_permutation(P)[0]]
h = asm.handle
for direct, rtol in ((True, 1e-12), (True, 1e-9), (False, 1e-12)):
    asm.set_direct(direct)
    asm.assemble()
    it, rr, conv = h.solve(rtol, 1000, 4)
    x = h.solution()
    print(f"{'direct' if direct else 'minres'} rtol {rtol:g}: it {it} reported {rr:.2e} "
          f"true {h.true_residual():.2e} err vs analytic {np.linalg.norm(x - xa) / np.linalg.norm(xa):.2e}",
          flush=True)
asm.close()
