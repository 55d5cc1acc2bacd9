"""Per-kernel times of the direct step (HIP events bound to each dispatch, eager profiled
steps), C3 by default: python scripts/direct_kernels.py [levels N steps]."""

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (HIP runtime first)

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 else 15
N = int(sys.argv[2]) if len(sys.argv) > 2 else 15
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
asm = HydraulicNetworkAssembler(mesh)
asm.compute_forms(p_bc_ex=lambda x: x[1])
h = asm.handle
asm.set_direct(True)
for _ in range(5):
    h.assemble(True, True)
    h.solve(1e-12, 100, 4)
h.set_profiling(True)
h.reset_profile()
for _ in range(steps):
    h.assemble(True, True)
    h.solve(1e-12, 100, 4)
pd, pr = h.profile_direct(), h.profile()
h.set_profiling(False)
n = max(pd["count"], 1)
t = {"asm": 1e3 * pr["asm_ms"] / max(pr["asm_count"], 1), "up": 1e3 * pd["up_ms"] / n,
     "top": 1e3 * pd["top_ms"] / n, "down": 1e3 * pd["down_ms"] / n,
     "publish": 1e3 * pd["residual_ms"] / n}
print("us per launch: " + "  ".join(f"{k} {v:6.2f}" for k, v in t.items())
      + f"  sum {sum(t.values()):6.2f}  (true residual {h.true_residual():.2e})", flush=True)
asm.close()
