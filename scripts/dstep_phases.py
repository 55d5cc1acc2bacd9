#!/usr/bin/env python3
"""Per-workgroup phase stamps of the fused direct step k_dir_step (debug build, GPU box).

Loads ``libnxhip_phase.so`` (``python -c 'from networks_fenicsx_amd import build;
build.build(phase_timing=True)'``), runs the bench workload's direct step a few times and
prints, for the last launch, the distribution over workgroups (wall_clock64, 100 MHz, in us
from the earliest workgroup start) of: start, phase-1 arrival, top values received, phase-2
arrival; and when the last workgroup finished the top part and published.

    python scripts/dstep_phases.py [levels] [N]
"""

from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("NXHIP_LIB", str(REPO / "networks_fenicsx_amd" / "libnxhip_phase.so"))
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402

from networks_fenicsx_amd import HydraulicNetworkAssembler, NetworkMesh, _lib  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402


def main() -> int:
    levels = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    mesh = NetworkMesh(ng.make_tree(levels, levels, levels), N=N, color_strategy="smallest_last")
    asm = HydraulicNetworkAssembler(mesh)
    asm.compute_forms(p_bc_ex=lambda x: x[1])
    asm.set_direct(True)
    h = asm.handle
    for _ in range(5):
        asm.assemble()
        it, rr, conv = h.solve(1e-12, 100, 4)
    assert h.direct_path() == "fused", h.direct_path()
    nj = asm.tree_preconditioner.n_jobs
    report(nj, rr)
    return 0


def report(nj: int, rr: float) -> None:
    """Print the last launch's per-workgroup stamps (nx_debug_dstep) of nj workgroups."""
    buf = (C.c_ulonglong * (48 * 512))()
    fn = _lib.lib().nx_debug_dstep
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    _lib.check(fn(buf))
    g = np.array(buf, dtype=np.float64).reshape(48, 512)[:, :nj]
    t0 = g[0].min()
    us = (g - t0) / 100.0  # 100 MHz ticks -> us
    names = ["start", "phase-1 arrival", "top values in", "phase-2 arrival", "published",
             "top part solved"]
    print(f"{nj} workgroups, residual {rr:.2e}; us from the first workgroup start")
    for k in (0, 1, 2, 3):
        v = us[k]
        print(f"  {names[k]:16s} min {v.min():7.2f}  med {np.median(v):7.2f}  max {v.max():7.2f}")
    last1 = int(np.argmax(g[5]))  # the workgroup that solved the top part (latest stamp 5)
    print(f"  top part by wg {last1}: arrival {us[1][last1]:7.2f}, inputs loaded "
          f"{us[6][last1]:7.2f}, solved {us[7][last1]:7.2f}, values out {us[5][last1]:7.2f}")
    print(f"  top part phases: set-up {us[9][last1]:7.2f}, up levels {us[10][last1]:7.2f}, "
          f"down levels {us[11][last1]:7.2f}")
    lv = [f"{us[12 + q][last1]:.2f}" for q in range(8)]
    print(f"  up levels (deepest first) end at: {' '.join(reversed(lv))}")
    v = us[8]
    print(f"  {'stores issued':16s} min {v.min():7.2f}  med {np.median(v):7.2f}  max {v.max():7.2f}")
    late = np.argsort(us[2])[-4:][::-1]  # the latest to receive the top values
    print("  latest top values in: " + ", ".join(
        f"wg {w} at {us[2][w]:.2f} (arrived {us[1][w]:.2f}, stores issued {us[8][w]:.2f}"
        f"{', top solver' if w == last1 else ''})" for w in late))
    pub = np.argmax(g[4])
    print(f"  published by wg {pub} at {us[4][pub]:7.2f}")
    print(f"  publisher: phase-2 arrival {us[3][pub]:.2f}, loads summed {us[23][pub]:.2f}, "
          f"state formed {us[24][pub]:.2f}, published {us[4][pub]:.2f}; last phase-2 arrival "
          f"{us[3].max():.2f}")
    d1 = us[1] - us[0]
    d2 = us[3] - us[2]
    print(f"  phase 1 per wg: min {d1.min():.2f} med {np.median(d1):.2f} max {d1.max():.2f}")
    print(f"  phase 2 per wg: min {d2.min():.2f} med {np.median(d2):.2f} max {d2.max():.2f}")
    # inside the phases (thread 0 of every workgroup; medians over workgroups)
    inner = [(32, 0, "phase 1: chains assembled + condensed"), (33, 32, "phase 1: junction set-up"),
             (34, 33, "phase 1: junction levels"), (35, 34, "phase 1: posts"),
             (36, 2, "phase 2: set-up"), (37, 36, "phase 2: junction levels"),
             (38, 37, "phase 2: chains (x, residual)"), (3, 38, "phase 2: rows + partials"),
             (40, 3, "end of the workgroup after phase 2")]
    if os.environ.get("NXHIP_DIR_SUP", "1") != "0":  # phase 2 by superposition (round 6)
        inner = inner[:4] + [
            (20, 1, "sup: u-independent part (waiting wgs)"), (8, 1, "stores issued"),
            (21, 2, "sup: slot values"), (22, 21, "sup: chains (x, residual)"),
            (25, 22, "sup: rows + partials"), (3, 25, "hand-off 2 drain + barrier"),
            (40, 3, "end of the workgroup after phase 2")]
    for k, k0, name in inner:
        d = us[k] - us[k0]
        print(f"  {name:38s} med {np.median(d):6.2f}  max {d.max():6.2f}")
    if g[41].max() > 0:  # several ranks (k_dir_xr): the top solver's exchange, the publisher's
        t, pb = last1, pub
        print(f"  xr: top part up {us[41][t]:.2f}, partials read {us[42][t]:.2f}, exchange 1 done "
              f"{us[43][t]:.2f}, values out {us[5][t]:.2f}; publish: exchange 2 from "
              f"{us[44][pb]:.2f} to {us[45][pb]:.2f}, published {us[4][pb]:.2f}")
        print(f"  xr: coarse forest solved {us[46][t]:.2f}, top part's values {us[47][t]:.2f}")
    e = us[40]
    print(f"  {'workgroup end':16s} min {e.min():7.2f}  med {np.median(e):7.2f}  max {e.max():7.2f}")


if __name__ == "__main__":
    sys.exit(main())
