#!/usr/bin/env python3
"""Where the public surface's host time goes (GPU box): ``Solver.assemble()`` +
``Solver.solve()`` on the bench workload, timed plain and under cProfile.

    python scripts/api_profile.py [steps]
"""

from __future__ import annotations

import cProfile
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (HIP runtime first)

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, Solver  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402


def main() -> int:
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    mesh = NetworkMesh(ng.make_tree(15, 15, 15), N=15, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    solver = Solver(asm)
    h = asm.handle

    def loop(n):
        for _ in range(n):
            solver.assemble()
            solver.solve()
        h.sync()

    loop(50)
    for _ in range(3):
        t0 = time.perf_counter()
        loop(steps)
        print(f"api: {1e3 * (time.perf_counter() - t0) / steps:.4f} ms/step", flush=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        h.assemble(True, True)
        h.solve(1e-12, 50000, 4)
    h.sync()
    print(f"handle: {1e3 * (time.perf_counter() - t0) / steps:.4f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    loop(steps)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    asm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
