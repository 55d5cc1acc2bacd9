#!/usr/bin/env python3
"""Per-workgroup phase stamps of one rank's exchange step (k_dir_xr, debug build) in the
multi-GPU rehearsal: the group's graph-path direct solve, then rank ``--rank`` alone
(nx_debug_xr_rehearse, its exchanges emulated), then its stamps as scripts/dstep_phases.py
prints them.

    python scripts/xr_phases.py [--ranks 8] [--levels 15] [--N 19] [--rank 7]
"""

from __future__ import annotations

import argparse
import math
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("NXHIP_LIB", str(REPO / "networks_fenicsx_amd" / "libnxhip_phase.so"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "scripts"))

import torch  # noqa: E402,F401  (HIP runtime before libnxhip.so)

from dstep_phases import report  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--levels", type=int, default=15)
    ap.add_argument("--N", type=int, default=19)
    ap.add_argument("--rank", type=int, default=7)
    args = ap.parse_args()
    levels = args.levels + int(round(math.log2(args.ranks)))
    grp = RankGroup(ng.make_tree(levels, levels, levels), args.N, args.ranks,
                    color_strategy="smallest_last")
    try:
        grp.compute_forms(p_bc_ex=lambda x: x[1])
        grp.set_direct(True)
        os.environ["NXHIP_DIR_XR"] = "0"  # the graph path leaves the sums the rehearsal reads
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        a = grp.assemblers[args.rank]
        ms = a.handle.xr_rehearse(1e-12, 3)
        print(f"rank {args.rank}: {1e3 * ms:.1f} us per launch (exchanges emulated)")
        report(a.tree_preconditioner.n_jobs, rr)
        return 0
    finally:
        grp.close()


if __name__ == "__main__":
    sys.exit(main())
