"""Step time of the direct tree solve vs preconditioned MINRES (assemble + solve, inputs
resident), C3 by default: python scripts/direct_timing.py [levels N steps]."""

import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (HIP runtime first)

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 else 15
N = int(sys.argv[2]) if len(sys.argv) > 2 else 15
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
asm = HydraulicNetworkAssembler(mesh)
asm.compute_forms(p_bc_ex=lambda x: x[1])
h = asm.handle
for direct in (True, False, True):
    asm.set_direct(direct)
    for _ in range(5):
        h.assemble(True, True)
        h.solve(1e-12, 100, 4)
    h.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        h.assemble(True, True)
        it, rr, conv = h.solve(1e-12, 100, 4)
    h.sync()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    print(f"{'direct' if direct else 'minres'}: {ms:.4f} ms/step, it {it}, relres {rr:.2e}, "
          f"solver {h.solver()}, true {h.true_residual():.2e}", flush=True)
asm.close()
