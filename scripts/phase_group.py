"""Phase stamps (debug build, workgroup 0 of the LAST rank's launch) of the multi-rank direct
solve's sweeps through the in-process group (8 ranks, C4 by default):
python scripts/phase_group.py [ranks levels N]"""

import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("NXHIP_LIB", str(REPO / "networks_fenicsx_amd" / "libnxhip_phase.so"))
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

from networks_fenicsx_amd import _lib  # noqa: E402
from networks_fenicsx_amd import network_generation as ng  # noqa: E402
from networks_fenicsx_amd.group import RankGroup  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
levels = int(sys.argv[2]) if len(sys.argv) > 2 else 18
N = int(sys.argv[3]) if len(sys.argv) > 3 else 19
grp = RankGroup(ng.make_tree(levels, levels, levels), N, P, color_strategy="smallest_last")
grp.compute_forms(p_bc_ex=lambda x: x[1])
grp.set_direct(True)
for _ in range(3):
    grp.assemble()
    grp.solve(1e-12, 50000, 4)
fn = _lib.lib().nx_debug_phases
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32]
buf = (C.c_ulonglong * 128)()
_lib.check(fn(buf, 128))
g = list(buf)
for base, names in ((16, ["start", "chains", "phase A", "levels+store", "levels"]),
                    (32, ["start", "A1/A2", "A3", "up levels", "back-sub"]),
                    (48, ["start", "phase A", "levels+slots", "chains"])):
    t0 = g[base]
    print(base, "  ".join(f"{n}={(g[base + i] - t0) / 100.0:7.2f}" for i, n in enumerate(names)),
          f"| end {(g[base + 15] - t0) / 100.0:7.2f}", flush=True)
grp.close()
