#!/usr/bin/env python3
"""A/B of k_dir_step variants switched per launch by environment variables (GPU box): the
bench workload (C3 by default), every arm timed in several interleaved rounds so box drift
falls on all arms alike. Per arm: ms per step (assemble + solve, inputs resident) and the
kernel's own time (HIP events bound to its dispatch).

    python scripts/dstep_ab.py [levels N steps rounds] -- NAME=VAR=VAL[,VAR=VAL] ...
    e.g. python scripts/dstep_ab.py 15 15 200 5 -- plain=NXHIP_DIR_SUP=0 sup=NXHIP_DIR_SUP=1
"""

from __future__ import annotations

import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (HIP runtime first)

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402


def main() -> int:
    argv = sys.argv[1:]
    arms_at = argv.index("--") if "--" in argv else len(argv)
    pos = [int(a) for a in argv[:arms_at]]
    levels, N, steps, rounds = (pos + [15, 15, 200, 5][len(pos):])[:4]
    arms = []
    for spec in argv[arms_at + 1:]:
        name, _, kv = spec.partition("=")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        arms.append((name, env))
    if not arms:
        arms = [("default", {})]
    mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    h = asm.handle
    res = {name: {"ms": [], "kern": []} for name, _ in arms}
    for r in range(rounds):
        for name, env in arms:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                for _ in range(10):
                    h.assemble(True, True)
                    h.solve(1e-12, 100, 4)
                h.sync()
                t0 = time.perf_counter()
                for _ in range(steps):
                    h.assemble(True, True)
                    it, rr, conv = h.solve(1e-12, 100, 4)
                h.sync()
                res[name]["ms"].append(1e3 * (time.perf_counter() - t0) / steps)
                h.set_profiling(True)
                h.assemble(True, True)
                h.solve(1e-12, 100, 4)
                h.reset_profile()
                for _ in range(20):
                    h.assemble(True, True)
                    h.solve(1e-12, 100, 4)
                pd = h.profile_direct()
                h.set_profiling(False)
                res[name]["kern"].append(pd["up_ms"] / max(pd["count"], 1))
                assert conv and h.direct_path() == "fused", (name, h.direct_path())
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            print(f"round {r} {name}: {res[name]['ms'][-1]:.4f} ms/step, kernel "
                  f"{1e3 * res[name]['kern'][-1]:.2f} us, relres {rr:.2e}", flush=True)
    for name, _ in arms:
        ms, kern = sorted(res[name]["ms"]), sorted(res[name]["kern"])
        print(f"{name:12s} ms/step median {ms[len(ms) // 2]:.4f} min {ms[0]:.4f} | kernel us "
              f"median {1e3 * kern[len(kern) // 2]:.2f} min {1e3 * kern[0]:.2f}", flush=True)
    asm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
