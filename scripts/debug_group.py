"""Diagnose a multi-rank (in-process group) solve: iterations / relres / error per env."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import numpy as np  # noqa: E402

from cases import CASES  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402

case, P = sys.argv[1], int(sys.argv[2])
make, N, strategy, pbc = CASES[case]
grp = RankGroup(make(), N, P, color_strategy=strategy)
grp.compute_forms(p_bc_ex=pbc)
grp.assemble()
try:
    it, rr, conv = grp.solve(1e-12, 2000, 32)
    print(f"{os.environ.get('TAG', '')}: it {it} relres {rr:.3e} conv {conv}")
except Exception as e:  # noqa: BLE001
    print(f"{os.environ.get('TAG', '')}: ERROR {e}")
grp.close()
