"""All ranks of a partitioned network problem in ONE process, on one GPU.

The multi-GPU path runs one process per GPU over RCCL (``assembly.py`` +
``nx_comm_init``). RCCL refuses two ranks on one device, so this module drives the same
per-rank handles -- same partition, halo plans, preconditioner decomposition with the
coarse step, kernels and MINRES schedule -- through the library's in-process group
transport (``nx_group_*`` in ``include/nxhip.h``), where the halo exchange is a device
copy and every all-reduce a fixed-order device sum. It exists to check the multi-rank
algorithm on a single GPU against the single-rank solve; it is not a performance path.
"""

from __future__ import annotations

import networkx as nx
import numpy as np

from . import _lib
from .assembly import HydraulicNetworkAssembler
from .comm import LocalGroup
from .mesh import NetworkMesh

__all__ = ["RankGroup"]


class RankGroup:
    """``nranks`` ranks of the network problem on graph ``graph``.

    Args:
        graph: the network (built once; the other ranks receive it by the group's bcast)
        N: cells per edge
        nranks: number of simulated ranks (<= 16)
        color_strategy: edge colouring strategy, as for :class:`NetworkMesh`
    """

    def __init__(self, graph: nx.DiGraph, N: int, nranks: int, color_strategy=None):
        group = LocalGroup(nranks)
        self.meshes = [NetworkMesh(graph if r == 0 else None, N=N, color_strategy=color_strategy,
                                   comm=group.comm(r)) for r in range(nranks)]
        self.assemblers = [HydraulicNetworkAssembler(m) for m in self.meshes]
        self._agree_kernels()
        self._team_cycles()
        self._group: _lib.Group | None = None
        self.iterations = 0
        self.relres = float("nan")
        self.converged = False

    @property
    def nranks(self) -> int:
        return len(self.assemblers)

    def compute_forms(self, **kwargs) -> None:
        for a in self.assemblers:
            a.compute_forms(**kwargs)

    def assemble(self) -> None:
        for a in self.assemblers:
            a.assemble()

    def set_preconditioner(self, enable: bool) -> None:
        self._close_group()
        for a in self.assemblers:
            a.set_preconditioner(enable)
        if enable:
            self._agree_kernels()
            self._team_cycles()

    def _agree_kernels(self) -> None:
        """The ranks' sweep kernels (LDS or global memory, chosen per rank from its
        decomposition) must agree -- their exchange schedules differ: if any rank cannot run
        the LDS kernels, every rank takes the global-memory ones (what
        HydraulicNetworkAssembler.set_preconditioner does over a real communicator)."""
        pcs = [a for a in self.assemblers if a.preconditioned]
        if len(pcs) < 2:
            return
        lds = [a.handle.pc_lds() for a in pcs]
        if all(lds) or not any(lds):
            return
        for a, on in zip(pcs, lds):
            if on:
                a.handle.set_pc_kernels(True)
                a.handle.set_preconditioner(a.tree_preconditioner)

    def _team_cycles(self) -> None:
        """A graph with cycles: every rank's share of the direct solve's Woodbury correction
        of all ranks' cycle chains (what HydraulicNetworkAssembler.set_preconditioner does
        over a real communicator, here from every rank's pairs at once)."""
        if self.nranks < 2:
            return
        pairs = [p for a in self.assemblers for p in a.cycle_pairs()]
        for a in self.assemblers:
            if a.preconditioned:
                a.set_team_cycles(pairs)

    def set_direct(self, enable: bool) -> None:
        """The direct tree solve over all ranks (``nx_set_solver`` on every handle; it runs
        where every rank can run it exactly, else MINRES)."""
        for a in self.assemblers:
            a.set_direct(enable)

    @property
    def solver_used(self) -> str:
        """What the last solve ran: ``"direct"`` or ``"minres"``."""
        return "direct" if self.assemblers[0].handle.solver()[1] == 1 else "minres"

    def solve(self, rtol: float = 1e-12, maxit: int = 50000, check_every: int = 4):
        """MINRES (or the direct solve, see :meth:`set_direct`) over all ranks; returns
        ``(iterations, relres, converged)``."""
        if self._group is None:
            self._group = _lib.Group([a.handle for a in self.assemblers])
        it, rr, conv = self._group.solve(rtol, maxit, check_every)
        self.iterations, self.relres, self.converged = it, rr, conv
        return it, rr, conv

    def solutions(self) -> list[np.ndarray]:
        """Device-layout solution of every rank (owned DoFs)."""
        return [a.handle.solution() for a in self.assemblers]

    def _close_group(self) -> None:
        if self._group is not None:
            self._group.close()
            self._group = None

    def close(self) -> None:
        self._close_group()
        for a in self.assemblers:
            a.close()

    def __del__(self):
        try:
            self._close_group()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
