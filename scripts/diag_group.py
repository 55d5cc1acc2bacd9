"""Diagnostic (GPU box): the residual reported by the several-rank direct solve across the
variants of tests/test_gpu_group.py::test_group_direct_cut_rows_in_one_allreduce, with and
without the fused first half (NXHIP_DIR_FUSED)."""
import hashlib
import os
import sys

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

from cases import CASES  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402


def main(fused: str) -> None:
    os.environ["NXHIP_DIR_FUSED"] = fused
    make, N, strategy, pbc = CASES["arterial5_N40"]
    grp = RankGroup(make(), N, 3, color_strategy=strategy)
    grp.compute_forms(p_bc_ex=pbc)
    grp.set_direct(True)

    def run(tag):
        grp.assemble()
        it, rr, conv = grp.solve(1e-12, 50000, 4)
        h = hashlib.md5(np.concatenate(grp.solutions()).tobytes()).hexdigest()[:8]
        print(f"fused={fused} {tag:14s} it={it} rr={rr!r} {grp.solver_used} x={h}", flush=True)

    run("default")
    os.environ["NXHIP_DIR_CUT"] = "0"
    run("cut0")
    del os.environ["NXHIP_DIR_CUT"]
    os.environ["NXHIP_DIR_COARSE_DOWN"] = "0"
    run("coarse_down0")
    run("coarse_down0")
    del os.environ["NXHIP_DIR_COARSE_DOWN"]
    run("default")
    grp.close()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "1")
