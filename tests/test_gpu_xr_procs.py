"""The exchange step (k_dir_xr) across PROCESSES: one process per rank, several on one GPU.

The multi-GPU path runs one process per GPU; its ranks' kernels exchange the coarse
partials and the residual through mailboxes IPC-mapped between the processes. RCCL refuses
two ranks on one device, so these ranks run the library's host transport
(``nx_comm_init_host``: the same host logic with the collectives through shared memory) and
``tests/xr_procs_worker.py`` drives each rank. What runs for real here and nowhere else on a
one-GPU box: the IPC export / import of the fine-grained mailboxes between processes, the
one-handle launches with the communicator's exchange width, the per-rank give-up, the host
finishing an exchange 2 that its kernel gave up, the agreement, and the graph path's
collectives after it.

Checked per step: the gathered solution against the oracle's direct solve (1e-10), every
rank's published residual the same bits, every rank on the same path; and that the
steps are bit-identical while the exchange step runs.
"""

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

from cases import CASES
from networks_fenicsx_amd import NetworkMesh
from oracle import nx_oracle as O

pytestmark = pytest.mark.gpu

HERE = Path(__file__).resolve().parent
SOL_TOL = 1e-10


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _run(tmp_path, case, P, steps=6, give_up_rank=-1, which=1, give_up_step=2, timeout=240):
    port = _free_port()
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(P), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NXHIP_TRANSPORT="host")
        cmd = [sys.executable, "-u", str(HERE / "xr_procs_worker.py"), "--case", case,
               "--steps", str(steps), "--give-up-rank", str(give_up_rank),
               "--give-up-which", str(which), "--give-up-step", str(give_up_step),
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


def _reference(case):
    make, N, strategy, pbc = CASES[case]
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = mesh.edges
    P = O.build_problem(mesh.node_coordinates, src, dst, N, mesh.edge_colors)
    A, b = O.assemble_reference(P, pbc)
    Ab, bb, perm, _ = O.to_build_layout(P, A, b)
    return Ab, O.solve_reference(A, b)[perm]


def _gather(data, k, n):
    x = np.zeros(n)
    for d in data:
        x[d["rows"]] = d["x"][k]
    return x


def _check_steps(ranks, data, Ab, x_ref):
    xs = []
    for k in range(len(ranks[0])):
        st = [r[k] for r in ranks]
        assert all(s["converged"] and s["solver"] == "direct" for s in st), st
        assert len({s["relres"] for s in st}) == 1, [s["relres"] for s in st]
        assert len({s["path"] for s in st}) == 1, [s["path"] for s in st]
        x = _gather(data, k, Ab.shape[0])
        err = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
        assert err <= SOL_TOL, (k, err)
        xs.append(x)
    return xs


@pytest.mark.parametrize("case,P", [("depth6_N40", 2), ("arterial5_N40", 3), ("tree5_N15", 4)])
def test_processes_exchange_step(tmp_path, case, P):
    """Every step by the exchange step (one launch per rank, no collective), the oracle's
    answer, the same bits on every step and rank."""
    Ab, x_ref = _reference(case)
    ranks, data = _run(tmp_path, case, P)
    xs = _check_steps(ranks, data, Ab, x_ref)
    assert {s["path"] for r in ranks for s in r} == {"exchange"}
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])
    assert all(s["xr"]["why"] == 0 and not s["xr"]["off"] for r in ranks for s in r)


@pytest.mark.parametrize("P", [2, 3])
def test_processes_one_rank_gives_up_exchange2(tmp_path, P):
    """Rank 1's exchange 2 gives up at once at step 2 (after its own slots and flags went
    out), while the other ranks finish it: rank 1's host finishes exchange 2 from its
    mailbox (the same residual bits), so every rank ends step 2 on the exchange path with
    the oracle's answer; the steps after it run the exchange step again."""
    case = "depth6_N40"
    Ab, x_ref = _reference(case)
    ranks, data = _run(tmp_path, case, P, give_up_rank=1, which=1, give_up_step=2)
    xs = _check_steps(ranks, data, Ab, x_ref)
    assert {s["path"] for r in ranks for s in r} == {"exchange"}
    assert ranks[1][2]["xr"]["why"] & 2, ranks[1][2]
    assert not any(s["xr"]["off"] for r in ranks for s in r)
    for x in xs[1:]:
        np.testing.assert_array_equal(x, xs[0])


@pytest.mark.parametrize("P", [2, 3])
def test_processes_one_rank_gives_up_exchange1(tmp_path, P):
    """Rank 1's exchange 1 gives up at once at step 2: no rank can finish that step (rank 1
    never sends its residual share), every rank's launch gives up -- the others at once, on
    rank 1's abort word -- the ranks agree (one max-all-reduce) and every rank solves step 2
    and every later step on the graph path: the same path on every rank at every step."""
    case = "depth6_N40"
    Ab, x_ref = _reference(case)
    ranks, data = _run(tmp_path, case, P, give_up_rank=1, which=0, give_up_step=2)
    _check_steps(ranks, data, Ab, x_ref)
    for k, st in enumerate(zip(*ranks)):
        want = "exchange" if k < 2 else "launches"
        assert {s["path"] for s in st} == {want}, (k, st)
        assert all(s["xr"]["off"] == (k >= 2) for s in st), (k, st)
    assert all(r[-1]["xr"]["agreed"] == 1 for r in ranks)
    assert ranks[1][2]["xr"]["why"] & 1
    assert all(r[2]["xr"]["why"] & 4 for q, r in enumerate(ranks) if q != 1)
