#!/usr/bin/env python3
"""Per-workgroup phase stamps of the several-rank fused up kernel k_dir_team_up (debug build,
GPU box): the 8-rank group rehearsal's last rank (the stamps of the last launch win).

    python scripts/team_phases.py [ranks] [levels-at-one-rank] [N]
"""
from __future__ import annotations

import ctypes as C
import math
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("NXHIP_LIB", str(REPO / "networks_fenicsx_amd" / "libnxhip_phase.so"))
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402

from networks_fenicsx_amd import _lib  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402


def main() -> int:
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    lv = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 19
    levels = lv + int(round(math.log2(P)))
    grp = RankGroup(ng.make_tree(levels, levels, levels), N, P, color_strategy="smallest_last")
    try:
        grp.compute_forms(p_bc_ex=lambda x: x[1])
        grp.set_direct(True)
        for _ in range(4):
            grp.assemble()
            it, rr, conv = grp.solve(1e-12, 50000, 4)
        nj = grp.assemblers[-1].tree_preconditioner.n_jobs
        buf = (C.c_ulonglong * (32 * 512))()
        fn = _lib.lib().nx_debug_dstep
        fn.argtypes = [C.POINTER(C.c_ulonglong)]
        _lib.check(fn(buf))
        g = np.array(buf, dtype=np.float64).reshape(32, 512)[:, :nj]
        t0 = g[0].min()
        us = (g - t0) / 100.0
        last = int(np.argmax(g[7]))
        print(f"rank {P - 1}: {nj} workgroups, solver {grp.solver_used}, residual {rr:.2e}")
        for k, name in ((0, "start"), (1, "arrival")):
            v = us[k]
            print(f"  {name:10s} min {v.min():7.2f}  med {np.median(v):7.2f}  max {v.max():7.2f}")
        ok = us[8][us[8] > 0]
        print(f"  stores done (non-last) med {np.median(us[8]):7.2f} max {us[8].max():7.2f}")
        print(f"  last wg {last}: arrival {us[1][last]:.2f}, inputs loaded {us[6][last]:.2f}, "
              f"top part + coarse partials {us[7][last]:.2f}")
        print(f"  up levels of the top part (deepest first) end at: "
              f"{' '.join(f'{us[12 + q][last]:.2f}' for q in reversed(range(8)))}")
    finally:
        grp.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
