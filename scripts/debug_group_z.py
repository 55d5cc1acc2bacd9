"""Dump z (preconditioned residual) of every rank after `maxit` iterations of a group solve."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import numpy as np  # noqa: E402

from cases import CASES  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402

case, P, maxit, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
make, N, strategy, pbc = CASES[case]
grp = RankGroup(make(), N, P, color_strategy=strategy)
grp.compute_forms(p_bc_ex=pbc)
grp.assemble()
try:
    print(grp.solve(1e-12, maxit, 2))
except Exception as e:  # noqa: BLE001
    print("ERR", e)
np.savez(out, **{f"z{r}": a.handle.vector(2) for r, a in enumerate(grp.assemblers)},
         **{f"x{r}": a.handle.vector(0) for r, a in enumerate(grp.assemblers)})
grp.close()
