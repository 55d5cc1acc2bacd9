"""General degrees on several ranks, one process per rank (several processes on one
GPU through the host transport, as in test_gpu_xr_procs.py; the RCCL ranks' host logic).

Checked: every rank takes the condensed direct solve (the ranks' direct tree solve of the
auxiliary P1/DG0 system) and converges in one pass; the gathered solution equals the
oracle's one-rank direct solve of the (k, 0) system (``oracle/nx_oracle_fe.py``) to 1e-10;
every rank publishes the same residual bits; plain MINRES across the ranks reaches the same
solution, for (k, 0) and for continuous pressure (whose shared node rows are partitioned by
ownership), to the forward-error bound of its residual: ||x - x*|| / ||x*|| <=
kappa_2(A) ||b - A x|| / ||b||, kappa_2 of the symmetric system from its extreme eigenvalues
(ARPACK, shift-invert at 0) -- MINRES stops on rtol 1e-12 of the residual, so its forward
error is not 1e-10 by construction; north_star's 1e-10 is the direct solve's bar."""

from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import scipy.sparse.linalg as spla

from cases import CASES
from networks_fenicsx_amd import NetworkMesh
from networks_fenicsx_amd.layout_fe import build_fe_layout
from oracle import nx_oracle as O
from oracle import nx_oracle_fe as OF

pytestmark = pytest.mark.gpu

HERE = Path(__file__).resolve().parent
SOL_TOL = 1e-10


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _run(tmp_path, case, P, k, steps=3, minres=0, timeout=240, m=0):
    port = _free_port()
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(P), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NXHIP_TRANSPORT="host")
        cmd = [sys.executable, "-u", str(HERE / "fe_procs_worker.py"), "--case", case,
               "--k", str(k), "--m", str(m), "--steps", str(steps), "--minres", str(minres),
               "--out", str(tmp_path)]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, start_new_session=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{out[-4000:]}"
    ranks = [json.loads((tmp_path / f"rank{r}.json").read_text())["steps"] for r in range(P)]
    data = [np.load(tmp_path / f"rank{r}.npz") for r in range(P)]
    return ranks, data


def _reference(case, k, m=0, system=False):
    """The oracle's one-rank solve, in the one-rank (k, m) layout's row order (and with
    ``system`` the oracle's A, b and the layout-to-oracle row order)."""
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = mesh.edges
    E = mesh.num_edges
    F = OF.build_problem_fe(mesh.node_coordinates, src, dst, N, k, m, mesh.edge_colors)
    A, b = OF.assemble_reference_fe(F, pbc, f=0.3, R=1.0 + 0.5 * (np.arange(E) % 3))
    x_ref = O.solve_reference(A, b)
    lay = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, N, k, m)
    colors = mesh.edge_colors
    blocks = [lay.flux_rows[np.flatnonzero(colors == c)].ravel()
              for c in range(mesh.num_edge_colors)] + [lay.p_rows, lay.lm_rows]
    order = np.concatenate(blocks)
    x = np.empty(lay.n_rows)
    x[order] = x_ref
    return (x, A, b, order) if system else x


def _minres_bound(x, A, b, order):
    """kappa_2(A) * ||b - A x|| / ||b|| for the gathered x (layout order): the forward-error
    bound of a solution with that residual; x_ref's own error (the LU's, ~kappa u) is added
    as 4 kappa u."""
    A = A.tocsc()
    lmax = abs(spla.eigsh(A, k=1, which="LM", return_eigenvectors=False, tol=1e-6)[0])
    lmin = abs(spla.eigsh(A, k=1, sigma=0.0, which="LM", return_eigenvectors=False,
                          tol=1e-6)[0])
    kappa = 1.05 * lmax / lmin  # (ARPACK's tol 1e-6 on both ends)
    r = b - A @ x[order]
    return kappa * (np.linalg.norm(r) / np.linalg.norm(b) + 4 * np.finfo(float).eps)


def _gather(data, j, n):
    x = np.full(n, np.nan)
    for d in data:
        x[d["rows"]] = d["x"][j]
    assert not np.isnan(x).any(), "every row owned by some rank"
    return x


@pytest.mark.parametrize("case,P,k", [("depth6_N40", 2, 2), ("depth6_N40", 3, 3),
                                      ("arterial5_N40", 2, 2), ("double_Y_N5", 2, 3),
                                      # cycles (round 6): the auxiliary handle's team Woodbury
                                      ("edge_info_N10", 2, 2), ("edge_info_N10", 3, 3)])
def test_fe_ranks_direct(tmp_path, case, P, k):
    ranks, data = _run(tmp_path, case, P, k)
    x_ref = _reference(case, k)
    for s in range(len(ranks[0])):
        for r in range(P):
            st = ranks[r][s]
            assert st["direct_available"] and st["solver"] == "direct", (r, st)
            assert st["path"] == "condensed" and st["converged"] and st["iterations"] == 1, (r, st)
            assert st["relres"] == ranks[0][s]["relres"]  # one all-reduce: the same bits
        x = _gather(data, s, x_ref.size)
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL, s


def test_fe_ranks_minres(tmp_path):
    ranks, data = _run(tmp_path, "double_Y_N5", 2, 2, steps=1, minres=1)
    x_ref, A, b, order = _reference("double_Y_N5", 2, system=True)
    for r in range(2):
        assert ranks[r][-1]["solver"] == "minres" and ranks[r][-1]["converged"]
    x = _gather(data, 1, x_ref.size)
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert err <= _minres_bound(x, A, b, order), err


@pytest.mark.parametrize("case,P,km", [("double_Y_N5", 2, (2, 1)), ("depth6_N40", 3, (3, 2)),
                                       ("arterial5_N40", 2, (2, 1)), ("Y_N4", 2, (3, 1))])
def test_fe_ranks_continuous_pressure(tmp_path, case, P, km):
    """Continuous pressure over the ranks (``build_fe_partition``: shared node rows owned
    once, ghost edges for their remote terms) on a forest: the node-condensed direct solve
    (every rank's border blocks and node rhs summed, the node forest on every rank) to the
    one-rank LU's answer, then plain MINRES to the same."""
    ranks, data = _run(tmp_path, case, P, km[0], steps=2, minres=1, m=km[1])
    x_ref, A, b, order = _reference(case, *km, system=True)
    for s in range(2):
        for r in range(P):
            st = ranks[r][s]
            assert st["direct_available"] and st["solver"] == "direct", (r, st)
            assert st["path"] == "node-condensed" and st["converged"], (r, st)
            assert st["relres"] == ranks[0][s]["relres"]
        x = _gather(data, s, x_ref.size)
        assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) <= SOL_TOL, s
    for r in range(P):
        assert ranks[r][2]["solver"] == "minres" and ranks[r][2]["converged"], ranks[r][2]
    x = _gather(data, 2, x_ref.size)
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert err <= _minres_bound(x, A, b, order), err


def test_fe_ranks_continuous_pressure_cycles(tmp_path):
    """A graph with cycles (the reference's edge_info graph): plain MINRES over the ranks."""
    ranks, data = _run(tmp_path, "edge_info_N10", 3, 3, steps=1, m=2)
    x_ref, A, b, order = _reference("edge_info_N10", 3, 2, system=True)
    for r in range(3):
        assert ranks[r][0]["solver"] == "minres" and ranks[r][0]["converged"], ranks[r][0]
    x = _gather(data, 0, x_ref.size)
    err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert err <= _minres_bound(x, A, b, order), err
