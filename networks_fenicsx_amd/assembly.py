"""Device assembly of the hydraulic network system.

Mirrors ``HydraulicNetworkAssembler`` of the reference
(``src/networks_fenicsx/assembly.py:95-398``): same constructor, ``compute_forms``,
``assemble`` and accessors. The forms are fixed by the model, so instead of
generating code from UFL at run time (``assembly.py:288-299``) the closed-form P1/DG0
element tensors are evaluated by the HIP kernel ``k_assemble`` (``csrc/nxhip.hip``),
one wavefront per graph edge, straight into a CSR matrix resident in HBM:

====================  =============================  ==========================
reference form        element tensor (cell length h)  device rows
====================  =============================  ==========================
``R q v dx``          ``R h/3, R h/6``                flux rows (mass)
``phi dq/ds dx``      ``[-1, +1]`` up/downstream      pressure rows (negated)
``-p dv/ds dx``       ``[+1, -1]^T``                  flux rows
``+-mu q ds``         ``+1`` in-edge end, ``-1`` out   multiplier rows
``+-lmbda v ds``      same, transposed                flux end rows
``p_bc v ds(in/out)`` ``+p_bc`` leaves, ``-p_bc`` roots rhs of flux end rows
``f phi dx``          ``f h``                         rhs of pressure rows (negated)
====================  =============================  ==========================

The pressure rows (and their rhs) are negated so the matrix is symmetric; this does
not change the solution and lets MINRES replace the direct solve.
"""

from __future__ import annotations

import logging
import os
import secrets
import typing

import numpy as np

from . import _lib
from .comm import MIN, GroupRankComm
from .fem import Constant, Function, FunctionSpace
from .element import condensed_flux_mass, stable_pair
from .layout import (LocalProblem, build_local_problem, cycle_pairs_global, partition_edges,
                     team_cycle_tables)
from .layout_fe import (FeLayout, build_cp_rank_tables, build_cp_tables, build_fe_aux_maps,
                        build_fe_layout, build_fe_partition, build_fe_rank_layout, fe_aux_slots)
from .mesh import NetworkMesh
from .precond import TreePreconditioner, build_tree_preconditioner
from .timing import timed

__all__ = ["HydraulicNetworkAssembler", "DeviceMatrix", "DeviceVector", "evaluate_nodal",
           "edge_boundary_rhs"]


def _device_for_rank() -> int:
    env = os.environ.get("NXHIP_DEVICE")
    if env is not None:
        return int(env)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = _lib.device_count()
    if n < 1:
        raise _lib.NxError("no HIP device visible: the network assembler runs on the GPU only")
    return local % n


def evaluate_nodal(p_bc_ex, pos: np.ndarray) -> np.ndarray:
    """Nodal values of the pressure boundary data at the graph nodes.

    The reference interpolates ``p_bc_ex`` into P1 on the network mesh
    (``assembly.py:225-234``); only vertex values at boundary nodes reach the rhs, so
    evaluating at the graph nodes is exact. Accepted forms: a callable ``x -> values``
    with DOLFINx's ``x`` of shape ``(3, n)``; an object with ``eval(x)``
    (``PressureFunction`` protocol, ``assembly.py:24-25``); an array of nodal values;
    or a scalar.
    """
    n = pos.shape[0]
    x = np.zeros((3, n), dtype=np.float64)
    x[: pos.shape[1], :] = pos.T
    if hasattr(p_bc_ex, "eval") and not callable(p_bc_ex):
        vals = p_bc_ex.eval(x)
    elif callable(p_bc_ex):
        vals = p_bc_ex(x)
    else:
        vals = p_bc_ex
    vals = np.asarray(vals, dtype=np.float64)
    if vals.ndim == 0:
        vals = np.full(n, float(vals))
    vals = vals.reshape(-1)
    if vals.size != n:
        raise ValueError(f"p_bc gave {vals.size} values for {n} nodes")
    return vals


def edge_boundary_rhs(mesh: NetworkMesh, edge_ids: np.ndarray, pbc: np.ndarray) -> np.ndarray:
    """rhs of the flux end rows of every listed edge, ``(E, 2)``: ``-p_bc(source)`` at an
    inlet root's ``q_0`` and ``+p_bc(target)`` at an outlet leaf's ``q_N``, 0 elsewhere --
    the weak boundary terms ``+p_bc v ds(in) - p_bc v ds(out)`` (``assembly.py:258-260``)
    with the markers of ``mesh.py:402-420``."""
    src, dst = mesh.edges
    s, d = src[edge_ids], dst[edge_ids]
    leaf = np.zeros(mesh.num_nodes, dtype=bool)
    leaf[mesh.boundary_in_nodes] = True
    root = np.zeros(mesh.num_nodes, dtype=bool)
    root[mesh.boundary_out_nodes] = True
    edge_bc = np.zeros((edge_ids.size, 2), dtype=np.float64)
    edge_bc[:, 0] = np.where(root[s], -pbc[s], 0.0)  # - p_bc ds(out_marker)
    edge_bc[:, 1] = np.where(leaf[d], pbc[d], 0.0)  # + p_bc ds(in_marker)
    return edge_bc


def _scalar(c, name: str, default: float) -> float:
    if c is None:
        return default
    if isinstance(c, Constant):
        return float(c.value)
    if hasattr(c, "value"):
        return float(np.asarray(c.value))
    return float(c)


class DeviceVector:
    """The rhs ``b`` resident on the device (returned where PETSc returned a ``Vec``)."""

    def __init__(self, handle: _lib.Handle):
        self._handle = handle

    def getArray(self) -> np.ndarray:  # noqa: N802 (petsc4py spelling)
        return self._handle.rhs()

    @property
    def array(self) -> np.ndarray:
        return self._handle.rhs()

    def getSize(self) -> int:  # noqa: N802
        return self._handle.n_rows


class DeviceMatrix:
    """The assembled CSR matrix resident on the device (stands in for a PETSc ``Mat``)."""

    def __init__(self, handle: _lib.Handle, kind=None):
        self._handle = handle
        self.kind = kind

    def getType(self) -> str:  # noqa: N802
        return "nest" if self.kind == "nest" else "aij"

    def getSize(self):  # noqa: N802
        return (self._handle.n_rows, self._handle.n_cols)

    def csr(self):
        return self._handle.csr()

    def to_scipy(self):
        import scipy.sparse as sp

        rp, col, val = self._handle.csr()
        return sp.csr_matrix((val, col, rp), shape=(self._handle.n_rows, self._handle.n_cols))

    def mult(self, x: np.ndarray) -> np.ndarray:
        return self._handle.spmv(x)


class FormBlock:
    """Block ``a[i][j]`` (bilinear, ``j`` given) or ``L[i]`` (linear) of the reference's
    nested forms (``assembly.py:194-299``: row block = test space ``i``, column block =
    trial space ``j``, spaces ordered ``[flux_color_0 .., pressure, multiplier]``).

    ``kind`` names the term of ``compute_forms`` it holds: ``"mass"`` (``R q v dx``, a[c][c],
    ``:253``), ``"divergence"`` (``phi dq/ds``, a[M][c], ``:254``), ``"gradient"``
    (``-p dv/ds``, a[c][M], ``:255``), ``"junction"`` (``+-mu q`` / ``+-lambda v``,
    a[M+1][c] and a[c][M+1], ``:271-277``), ``"boundary"`` (``+-p_bc v ds``, L[c], ``:258``),
    ``"source"`` (``f phi dx``, L[M], ``:262``) or ``"zero"`` (L[M+1]). Blocks the reference
    sets to ``None`` (``:284-287``) are ``None`` here too.

    :meth:`assemble` extracts the block from the device-assembled system in the reference's
    signs (the device stores the pressure rows negated, which makes the system symmetric):
    a ``scipy.sparse.csr_matrix`` over this rank's owned rows/columns, or the rhs slice."""

    def __init__(self, assembler: "HydraulicNetworkAssembler", kind: str, i: int,
                 j: int | None = None):
        self._asm = assembler
        self.kind = kind
        self.i, self.j = i, j
        self.rank = 2 if j is not None else 1

    @property
    def function_spaces(self):
        V = self._asm.function_spaces
        return [V[self.i]] if self.j is None else [V[self.i], V[self.j]]

    def assemble(self):
        asm = self._asm
        rows = asm._block_rows(self.i)
        sign = -1.0 if self.i == len(asm.function_spaces) - 2 else 1.0  # pressure rows
        if self.j is None:
            return sign * asm.handle.rhs()[rows]
        import scipy.sparse as sp

        h = asm.handle
        rp, col, val = h.csr()
        A = sp.csr_matrix((val, col, rp), shape=(h.n_rows, h.n_cols))
        return (sign * A[rows][:, asm._block_rows(self.j)]).tocsr()

    def __repr__(self) -> str:
        idx = f"[{self.i}]" if self.j is None else f"[{self.i}][{self.j}]"
        return f"FormBlock{idx}({self.kind})"


def _block_kind(i: int, j: int, M: int) -> str | None:
    """Which term of compute_forms block a[i][j] holds (None: the reference's None)."""
    if i < M and j == i:
        return "mass"
    if i == M and j < M:
        return "divergence"
    if i < M and j == M:
        return "gradient"
    if (i == M + 1 and j < M) or (i < M and j == M + 1):
        return "junction"
    return None


class _BilinearBlocks:
    """The nested ``a[i][j]`` of the reference (``assembly.py:194-196, 284-293``) without
    storing its (M + 2)^2 entries: with ``color_strategy=None`` M is the edge count, and a
    list of lists would need O(E^2) memory (the reference's own structure)."""

    def __init__(self, asm: "HydraulicNetworkAssembler", M: int):
        self._asm, self._M = asm, M

    def __len__(self) -> int:
        return self._M + 2

    def __getitem__(self, i: int) -> "_BilinearRow":
        if not -len(self) <= i < len(self):
            raise IndexError(i)
        return _BilinearRow(self._asm, i % len(self), self._M)

    def __iter__(self):
        return (self[i] for i in range(len(self)))


class _BilinearRow:
    def __init__(self, asm, i: int, M: int):
        self._asm, self._i, self._M = asm, i, M

    def __len__(self) -> int:
        return self._M + 2

    def __getitem__(self, j: int):
        if not -len(self) <= j < len(self):
            raise IndexError(j)
        j %= len(self)
        kind = _block_kind(self._i, j, self._M)
        return None if kind is None else FormBlock(self._asm, kind, self._i, j)

    def __iter__(self):
        return (self[j] for j in range(len(self)))


class HydraulicNetworkAssembler:
    """Assembler for the mixed hydraulic network problem

    ``R q + dp/ds = 0``, ``dq/ds = f`` on every edge, with flux conservation at the
    bifurcations enforced by Lagrange multipliers (reference ``assembly.py:95-118``).

    Args:
        mesh: the :class:`NetworkMesh`
        flux_degree: degree k of the equispaced Lagrange flux on every edge (default 1)
        pressure_degree: 0 for DG0 pressure (default), m >= 1 for continuous P_m (needs
            k > m); other pairs than (1, 0) run without the tree preconditioner, on one or
            several ranks, with their direct solves on forests
    """

    @timed("nxfx:HydraulicNetworkAssembler:__init__")
    def __init__(self, mesh: NetworkMesh, flux_degree: int = 1, pressure_degree: int = 0):
        self._network_mesh = mesh
        comm = mesh.comm
        self._rank, self._nranks = comm.rank, comm.size
        self._degrees = (int(flux_degree), int(pressure_degree))
        self._a = None
        self._L = None
        self._pc: TreePreconditioner | None = None
        if self._degrees != (1, 0):
            self._init_general_degrees()
            return
        src, dst = mesh.edges
        self._local: LocalProblem = build_local_problem(
            mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, self._rank, self._nranks
        )
        lp = self._local
        self._handle = _lib.Handle(_device_for_rank(), mesh.N, lp.edge_x, lp.edge_lm,
                                   lp.lm_rowptr, lp.lm_col, lp.lm_val, lp.n_ghost)
        if self._nranks > 1:
            self._init_comm()
        self._edge_ids = lp.edges
        # MINRES preconditioner (tree Schur complement); topology-only, built once
        if mesh.N <= 1024 and np.any(np.asarray(mesh.degrees) > 1):
            # (no junction anywhere -- one edge, or separate edges: plain MINRES)
            # 256 jobs = one workgroup per CU (swept on MI355X: 64..1024)
            self._pc = build_tree_preconditioner(lp, src, dst, mesh.degrees, target_jobs=256)
        self.set_preconditioner(True)
        self._make_spaces()

    def _init_general_degrees(self) -> None:
        """Flux P_k / pressure DG0 or continuous P_m (``layout_fe.py``): gather assembly
        (``nx_create_fe``), the condensed direct solves, plain MINRES otherwise -- the tree
        preconditioner is P1/DG0's. Several ranks, one process per rank: (k, 0) on the edges
        of the P1/DG0 rank layout (``layout_fe.build_fe_rank_layout``) with the condensed
        direct solve across the ranks; continuous pressure by row ownership
        (``layout_fe.build_fe_partition``: a node's shared pressure row with one rank, the
        remote edges at the node as ghost edges) with the node-condensed direct solve across
        the ranks (``layout_fe.build_cp_rank_tables``); MINRES over the halo otherwise."""
        mesh = self._network_mesh
        k, m = self._degrees
        if not stable_pair(k, m):
            raise ValueError(
                f"flux_degree={k}, pressure_degree={m}: with continuous pressure the flux degree "
                "must exceed the pressure degree (otherwise the system is singular)")
        ranks = self._nranks > 1
        if ranks and isinstance(mesh.comm, GroupRankComm):
            raise NotImplementedError("general degrees on several ranks run one process per "
                                      "rank (RCCL), not an in-process group")
        src, dst = mesh.edges
        if ranks:  # (every rank decides the same from the same partition: no rank is left
            # waiting in a collective for one that raised)
            owner = partition_edges(src, dst, mesh.node_coordinates.shape[0], self._nranks)
            if (np.bincount(owner, minlength=self._nranks) == 0).any():
                raise ValueError(f"general element degrees on {self._nranks} ranks need at least "
                                 f"one edge per rank ({mesh.num_edges} edges)")
        self._local = None
        self._fe_lp = None
        n_rows_edges = None  # edges whose rows this rank owns (the rest: ghost edges)
        full = None
        if ranks and m == 0:
            self._fe_lp = build_local_problem(mesh.node_coordinates, src, dst, mesh.degrees,
                                              mesh.N, self._rank, self._nranks)
            self._fe = build_fe_rank_layout(mesh.node_coordinates, src, dst, mesh.N, k,
                                            self._fe_lp)
            self._edge_ids = np.asarray(self._fe_lp.edges)
        elif ranks:
            full = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, k, m)
            owner = partition_edges(src, dst, mesh.node_coordinates.shape[0], self._nranks)
            self._fe = build_fe_partition(full, src, dst, owner, self._rank, self._nranks)
            self._edge_ids = np.asarray(self._fe.edges)  # coefficients: own + ghost edges
            n_rows_edges = self._fe.n_own_edges
        else:
            self._fe = build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, mesh.N, k, m)
            self._edge_ids = np.arange(mesh.num_edges)
        self._handle = _lib.Handle.create_fe(_device_for_rank(), self._fe)
        fe = self._fe
        if ranks:
            self._join_comm(self._handle, fe.peers, fe.send_off, fe.send_idx, fe.recv_off)
        self._pc_on = False
        own_ids = self._edge_ids[:n_rows_edges]
        colors = mesh.edge_colors[own_ids]
        self._flux_spaces, self._flux_idx = [], []
        for c in range(mesh.num_edge_colors):
            slots = np.flatnonzero(colors == c)  # graph.edges() order inside a colour
            edges = own_ids[slots]
            self._flux_spaces.append(
                FunctionSpace(mesh, "flux", "P", k, False, edges.size * (k * mesh.N + 1), edges, c))
            self._flux_idx.append(fe.flux_rows[slots].ravel())
        if m == 0:
            self._pressure_space = FunctionSpace(mesh, "pressure", "DG", 0, True,
                                                 fe.p_rows.size, own_ids)
        else:
            self._pressure_space = FunctionSpace(mesh, "pressure", "P", m, False,
                                                 fe.p_rows.size, own_ids)
            self._pressure_space.nodes = np.asarray(fe.p_nodes)  # the shared node values first
        self._lm_space = FunctionSpace(mesh, "multiplier", "DG", 0, True, fe.lm_nodes.size)
        self._lm_space.nodes = np.asarray(fe.lm_nodes)
        self._p_idx = fe.p_rows
        self._lm_idx = fe.lm_rows
        self._set_output_map()
        self._fe_aux = None
        self._fe_cp = None
        if m == 0 and mesh.N <= 1024 and np.any(np.asarray(mesh.degrees) > 1):
            self._init_fe_direct(src, dst)
        elif m >= 1:
            # continuous pressure on a forest: the direct solve by condensation onto the graph
            # nodes (nx_fe_set_cp; several ranks: every rank's border blocks summed, the node
            # forest solved on every rank, nx_fe_cp_ranks); a graph with cycles runs MINRES
            tab = build_cp_tables(full if ranks else fe, src, dst)
            if tab is not None and ranks:
                # the ranks attach it together or not at all: a rank whose tables or
                # allocation fail would otherwise leave the others in fe_cp_solve's
                # all-reduce alone (RCCL has no timeout) -- the (k, 0) path's rule
                ok = 1
                try:
                    tab, gid, nrowx = build_cp_rank_tables(tab, fe)
                    self._handle.fe_cp_ranks(fe.n_own_edges, mesh.num_edges, gid, nrowx)
                    self._handle.fe_set_cp(tab)
                except (_lib.NxError, ValueError, AssertionError, IndexError) as err:
                    logging.error("rank %d: the continuous-pressure direct solve could not be "
                                  "attached (%s); every rank runs MINRES", self._rank, err)
                    ok = 0
                if int(mesh.comm.allreduce(ok, MIN)) != 1:
                    self._handle.fe_set_cp(None)
                    tab = None
                self._fe_cp = tab
            elif tab is not None:
                self._handle.fe_set_cp(tab)
                self._fe_cp = tab

    def _init_fe_direct(self, src, dst) -> None:
        """(k, 0): the direct solve through the condensed P1/DG0 system (``nx_fe_set_direct``).
        An auxiliary P1/DG0 handle of the same edges carries the tree decomposition; its flux
        mass becomes the condensed ``R h [[a, b], [b, a]]`` (``element.condensed_flux_mass``),
        whose ratios are integers: ``a / b = (-1)^(k+1) (k+1)``. A graph with cycles (one
        rank, up to ``MAX_CYCLES`` cycle chains): the auxiliary tree solve is corrected by the
        Woodbury step of its dropped couplings (``fe_cyc_build``). Several ranks:
        the auxiliary handle is the rank's P1/DG0 handle (its halo, cut rows, coarse step),
        and the ranks attach it only if every rank can run its direct tree solve."""
        mesh, fe = self._network_mesh, self._fe
        k = self._degrees[0]
        ranks = self._nranks > 1
        lp = self._fe_lp if ranks else build_local_problem(mesh.node_coordinates, src, dst,
                                                           mesh.degrees, mesh.N, 0, 1)
        pc = build_tree_preconditioner(lp, src, dst, mesh.degrees, target_jobs=256)
        aux = None
        # a graph with cycles: the auxiliary handle's Woodbury correction of its cycle chains
        # (one rank: nx_set_cycles, set with its decomposition; several: every rank's share of
        # all ranks' chains, nx_set_cycles_team, the pairs gathered on the host), as P1/DG0's
        # direct solve
        ncyc = int(np.asarray(pc.cyc_rows).reshape(-1, 2).shape[0])
        gpairs = []
        if ranks:  # (collective: every rank, in the same order)
            gpairs = [p for ps in mesh.comm.allgather(
                cycle_pairs_global(lp, pc.cyc_rows, mesh.num_edges, mesh.bifurcation_index))
                for p in ps]
            ok = (bool(pc.tree_exact) and not gpairs) or 0 < len(gpairs) <= _lib.MAX_CYCLES
        else:
            ok = bool(pc.tree_exact) or 0 < ncyc <= _lib.MAX_CYCLES
        if ranks:  # (every rank makes the same collective calls below: decide together)
            ok = int(self._network_mesh.comm.allreduce(int(ok), MIN)) == 1
        if ok:
            aux = _lib.Handle(_device_for_rank(), mesh.N, lp.edge_x, lp.edge_lm, lp.lm_rowptr,
                              lp.lm_col, lp.lm_val, lp.n_ghost)
            if ranks:
                self._join_comm(aux, lp.peers, lp.send_off, lp.send_idx, lp.recv_off)
                aux.set_cut(lp.n_cut, lp.lm_cut, lp.gk_off, lp.gk_row, lp.gk_coef)
            aux.set_preconditioner(pc)
            ok = aux.pc_lds()
            if ok and gpairs:
                own, qloc, lcol = team_cycle_tables(lp, pc.cyc_rows, gpairs, mesh.num_edges,
                                                    mesh.bifurcation_index)
                aux.set_cycles_team(own, qloc, lcol)
        if ok:
            alpha, beta, C, K, Mii = condensed_flux_mass(k)
            ratio = round(alpha / beta)
            assert abs(alpha / beta - ratio) < 1e-12, (alpha, beta)
            aux.set_cell_mass(float(ratio), float(ratio + 1))
            aux.set_solver(True, True)  # (its sweeps invert an exact forest decomposition)
            maps = build_fe_aux_maps(fe, lp)
            cst = np.concatenate([C.ravel(), K.ravel(), Mii.ravel()])
            try:
                self._handle.fe_set_direct(aux, k, fe_aux_slots(fe, lp), maps, cst, alpha + beta)
            except _lib.NxError:
                if not ranks:
                    raise
                ok = False
        if ranks and int(self._network_mesh.comm.allreduce(int(ok), MIN)) == 0:
            if ok:  # another rank cannot: every rank runs MINRES
                self._handle.fe_set_direct(None, k, None, None, None, 0.0)
            ok = False
        if not ok:
            if aux is not None:
                aux.close()
            return
        self._fe_aux = aux
        self._fe_aux_pc = pc

    @property
    def fe_direct_available(self) -> bool:
        """A general-degree assembler with a direct solve: (k, 0) through the condensed P1/DG0
        system, continuous pressure (k > m >= 1) by condensation onto the graph nodes (forest
        graphs)."""
        return (getattr(self, "_fe_aux", None) is not None
                or getattr(self, "_fe_cp", None) is not None)

    def _join_comm(self, handle: _lib.Handle, peers, send_off, send_idx, recv_off) -> None:
        """``handle`` joins the ranks' communicator with this halo plan (rank 0 makes the id,
        the mesh's communicator broadcasts it; every rank calls this in the same order)."""
        comm = self._network_mesh.comm
        if os.environ.get("NXHIP_TRANSPORT", "rccl") == "host":
            # tests: several ranks' processes on ONE GPU (RCCL refuses that) -- the same
            # host logic with its collectives through shared memory (nx_comm_init_host)
            uid = f"/nxhip_{os.getpid()}_{secrets.token_hex(6)}" if self._rank == 0 else None
        else:
            uid = _lib.comm_unique_id() if self._rank == 0 else None
        uid = comm.bcast(uid, root=0)
        handle.comm_init(self._nranks, self._rank, uid, peers, send_off, send_idx, recv_off)

    def _init_comm(self) -> None:
        comm = self._network_mesh.comm
        lp = self._local
        if isinstance(comm, GroupRankComm):  # in-process group: plan only (RankGroup)
            self._handle.set_halo(self._nranks, self._rank, lp.peers, lp.send_off, lp.send_idx,
                                  lp.recv_off)
        else:
            self._join_comm(self._handle, lp.peers, lp.send_off, lp.send_idx, lp.recv_off)
            # the exchange step's mailboxes (nx_xch_*): every rank maps every rank's; a rank
            # that cannot export one leaves every rank on the graph path (RCCL all-reduces)
            try:
                mine = self._handle.xch_export()
            except _lib.NxError:
                mine = None
            handles = comm.allgather(mine)
            if all(hd is not None for hd in handles):
                try:  # (a rank left unlinked turns the step off everywhere: check_schedules)
                    self._handle.xch_import(handles)
                except _lib.NxError:
                    pass
        # the direct solve completes the cut multiplier rows in its residual all-reduce
        self._handle.set_cut(lp.n_cut, lp.lm_cut, lp.gk_off, lp.gk_row, lp.gk_coef)

    def _make_spaces(self) -> None:
        mesh, lp, N = self._network_mesh, self._local, self._network_mesh.N
        colors = mesh.edge_colors[lp.edges]
        order = np.argsort(colors, kind="stable")  # graph.edges() order inside a colour
        bounds = np.searchsorted(colors[order], np.arange(mesh.num_edge_colors + 1))
        self._flux_spaces = []
        for c in range(mesh.num_edge_colors):
            edges = lp.edges[order[bounds[c]:bounds[c + 1]]]
            self._flux_spaces.append(
                FunctionSpace(mesh, "flux", "P", 1, False, edges.size * (N + 1), edges, c))
        self._pressure_space = FunctionSpace(mesh, "pressure", "DG", 0, True,
                                             lp.edges.size * N, lp.edges)
        self._lm_space = FunctionSpace(mesh, "multiplier", "DG", 0, True, lp.lm_nodes.size)
        self._lm_space.nodes = np.asarray(lp.lm_nodes)
        # gather maps: device vector -> function arrays
        per = 2 * N + 1
        slot = np.full(mesh.num_edges, -1, dtype=np.int64)
        slot[lp.edges] = np.arange(lp.edges.size)
        all_q = (np.arange(lp.edges.size)[:, None] * per + 2 * np.arange(N + 1)[None, :])
        q_sorted = all_q[slot[lp.edges[order]]].ravel()  # flux DoFs grouped by colour
        cuts = bounds * (N + 1)
        self._flux_idx = [q_sorted[cuts[c]:cuts[c + 1]] for c in range(mesh.num_edge_colors)]
        self._p_idx = (np.arange(lp.edges.size)[:, None] * per
                       + 2 * np.arange(N)[None, :] + 1).ravel()
        self._lm_idx = lp.n_edge_dofs + np.arange(lp.lm_nodes.size)
        self._set_output_map()

    def _set_output_map(self) -> None:
        """Upload the function-block order of the owned rows (``nx_set_output_map``): the
        solution then reaches the host already split into ``[flux_color_0 .., pressure,
        global_flux]`` (``solver.py:120-134``), each function a slice of one buffer."""
        blocks = [*self._flux_idx, self._p_idx, self._lm_idx]
        self._out_off = np.concatenate([[0], np.cumsum([b.size for b in blocks])]).astype(np.int64)
        self._handle.set_output_map(np.concatenate(blocks))
        self._out_pool = _lib.PinnedPool(self._handle.n_rows)
        self._snap_pool = _lib.SnapshotPool(self._handle, self._out_pool)

    def set_preconditioner(self, enable: bool) -> bool:
        """Switch the device MINRES between preconditioned and plain; returns the state
        (always plain for general degrees: the tree preconditioner is P1/DG0's)."""
        on = bool(enable) and self._pc is not None
        self._handle.set_preconditioner(self._pc if on else None)
        comm = self._network_mesh.comm
        if on and self._nranks > 1 and not isinstance(comm, GroupRankComm):
            # the sweep kernels are chosen per rank from its decomposition (LDS caps); the
            # ranks' exchange schedules must agree: global-memory kernels everywhere if any
            # rank cannot run the LDS ones (RankGroup does the same for its ranks)
            lds = int(self._handle.pc_lds())
            if int(comm.allreduce(lds, MIN)) == 0 and lds:
                self._handle.set_pc_kernels(True)
                self._handle.set_preconditioner(self._pc)
            # a graph with cycles: every rank's share of the Woodbury correction of all
            # ranks' cycle chains (nx_set_cycles_team; the pairs gathered on the host)
            pairs = [p for ps in comm.allgather(self.cycle_pairs()) for p in ps]
            self.set_team_cycles(pairs)
        self._pc_on = on
        return on

    def cycle_pairs(self) -> list:
        """This rank's cycle chains' dropped couplings (flux end, multiplier) as rows of the
        single-rank layout (several ranks; ``TreePreconditioner.cyc_rows``)."""
        if self._pc is None or self._local is None:
            return []
        mesh = self._network_mesh
        return cycle_pairs_global(self._local, self._pc.cyc_rows, mesh.num_edges,
                                  mesh.bifurcation_index)

    def set_team_cycles(self, all_pairs) -> None:
        """Several ranks: this rank's share of the direct solve's Woodbury correction of every
        rank's cycle chains (``nx_set_cycles_team``); beyond ``MAX_CYCLES`` chains (or none)
        it is cleared and a cyclic graph runs MINRES."""
        if self._nranks < 2 or not self._pc_on_pending():
            return
        pairs = list(all_pairs)
        if not pairs or len(pairs) > _lib.MAX_CYCLES:
            self._handle.set_cycles_team([], [], [])
            return
        mesh = self._network_mesh
        own, qloc, lcol = team_cycle_tables(self._local, self._pc.cyc_rows, pairs,
                                            mesh.num_edges, mesh.bifurcation_index)
        self._handle.set_cycles_team(own, qloc, lcol)

    def _pc_on_pending(self) -> bool:
        return self._pc is not None and self._handle is not None

    @property
    def preconditioned(self) -> bool:
        return self._pc_on

    def set_direct(self, enable: bool) -> None:
        """Ask ``nx_solve`` for the direct tree solve (``nx_set_solver``); the device runs it
        only where it is exact -- exact preconditioner; a forest (the decomposition's
        ``tree_exact``) or up to ``MAX_CYCLES`` cycle-closing chains corrected by a Woodbury
        step (``nx_set_cycles``, one rank; ``nx_set_cycles_team``, several); with several
        ranks the LDS sweeps with the coarse step on every rank (the ranks decide together)
        -- and MINRES otherwise."""
        exact = (self._pc is not None and self._pc.tree_exact) or self.fe_direct_available
        want = (bool(enable), bool(exact))
        if getattr(self, "_direct_state", None) != want:
            self._handle.set_solver(*want)
            self._direct_state = want

    # ------------------------------------------------------------------ forms
    @timed("nxfx:HydraulicNetworkAssembler:compute_forms")
    def compute_forms(
        self,
        p_bc_ex: typing.Any,
        f: typing.Any = None,
        R: typing.Any = None,
        jit_options: dict | None = None,
        form_compiler_options: dict | None = None,
    ) -> None:
        """Evaluate the coefficients of the forms and upload them to the device.

        Args:
            p_bc_ex: pressure boundary data (callable ``x -> values``, object with
                ``eval``, nodal array or scalar), imposed weakly at inlet/outlet nodes.
            f: source of the mass-conservation equation -- a constant (default 0,
                ``assembly.py:201-202``) or one value per graph edge (``graph.edges()`` order).
            R: resistance -- a constant (default 1, ``assembly.py:204-205``) or one
                value per graph edge (``graph.edges()`` order).
            jit_options, form_compiler_options: accepted for API compatibility; the
                element tensors are compiled into the HIP library ahead of time.
        """
        del jit_options, form_compiler_options
        mesh, edge_ids = self._network_mesh, self._edge_ids
        f_val, f_edge = 0.0, None
        fv = f.value if isinstance(f, Constant) else f
        if fv is not None and np.ndim(fv) > 0:  # one value per graph edge
            fv = np.asarray(fv, dtype=np.float64).reshape(-1)
            if fv.size != mesh.num_edges:
                raise ValueError("f must be a constant or one value per graph edge")
            f_edge = np.ascontiguousarray(fv[edge_ids])
        else:
            f_val = _scalar(f, "f", 0.0)
        R_const, R_edge = 1.0, None
        if R is not None:
            Rv = R.value if isinstance(R, Constant) else R
            Rv = np.asarray(Rv, dtype=np.float64)
            if Rv.ndim == 0:
                R_const = float(Rv)
            elif Rv.size == mesh.num_edges:
                R_edge = np.ascontiguousarray(Rv[edge_ids])
            else:
                raise ValueError("R must be a constant or one value per graph edge")
        pbc = evaluate_nodal(p_bc_ex, mesh.node_coordinates)
        edge_bc = edge_boundary_rhs(mesh, edge_ids, pbc)
        self._handle.set_coefficients(R_edge, R_const, f_val, edge_bc)
        self._handle.set_source(f_edge)
        self._coefficients = {"R": R_const if R_edge is None else "per-edge",
                              "f": f_val if f_edge is None else "per-edge", "p_bc": pbc}
        M = len(self._flux_spaces)
        self._a = _BilinearBlocks(self, M)  # (M + 2)^2 blocks, materialised on access
        self._L = [FormBlock(self, "boundary", c) for c in range(M)]
        self._L += [FormBlock(self, "source", M), FormBlock(self, "zero", M + 1)]

    # ---------------------------------------------------------------- assemble
    @timed("nxfx:HydraulicNetworkAssembler:assemble")
    def assemble(self, A=None, b=None, assemble_lhs: bool = True, assemble_rhs: bool = True,
                 kind=None):
        """Assemble the system matrix and/or rhs on the device.

        Returns ``(A, b)`` views of the device-resident CSR matrix and rhs (the
        reference returns PETSc objects, ``assembly.py:329-368``). ``kind`` is
        recorded; the device storage is always one CSR matrix.
        """
        if self._a is None:
            raise RuntimeError("compute_forms() must be called before assemble()")
        # enqueued on the handle's stream: the solve (same stream) and every host read of
        # the matrix / rhs order after it, so the host does not wait here
        self._handle.assemble(assemble_lhs, assemble_rhs)
        if A is None and assemble_lhs:
            A = DeviceMatrix(self._handle, kind)
        if b is None and assemble_rhs:
            b = DeviceVector(self._handle)
        return (A, b)

    # --------------------------------------------------------------- accessors
    @property
    def handle(self) -> _lib.Handle:
        return self._handle

    @property
    def local_problem(self) -> LocalProblem | None:
        """The P1/DG0 rank layout (``layout.py``); None for general degrees."""
        return self._local

    @property
    def tree_preconditioner(self) -> TreePreconditioner | None:
        """The host decomposition of the tree preconditioner (``precond.py``), or None."""
        return self._pc

    @property
    def fe_layout(self) -> FeLayout | None:
        """The general-degree layout (``layout_fe.py``); None for P1/DG0."""
        return getattr(self, "_fe", None)

    @property
    def degrees(self) -> tuple[int, int]:
        """``(flux_degree, pressure_degree)``."""
        return self._degrees

    @property
    def lm_space(self) -> FunctionSpace:
        return self._lm_space

    @property
    def pressure_space(self) -> FunctionSpace:
        return self._pressure_space

    @property
    def flux_spaces(self) -> list[FunctionSpace]:
        return self._flux_spaces

    @property
    def function_spaces(self) -> list[FunctionSpace]:
        return [*self._flux_spaces, self._pressure_space, self._lm_space]

    @property
    def network(self) -> NetworkMesh:
        return self._network_mesh

    @property
    def bilinear_forms(self):
        if self._a is None:
            logging.error("Bilinear forms haven't been computed. Need to call compute_forms()")
            return None
        return self._a

    def bilinear_form(self, i: int, j: int):
        """Block ``a[i][j]`` (reference ``assembly.py:378-383``): a :class:`FormBlock`, or
        None where the reference's block is None; out of range logs an error and raises."""
        a = self.bilinear_forms
        if a is None:
            return None
        if i >= len(a) or j >= len(a[i]):
            logging.error("Bilinear form a[%d][%d] out of range", i, j)
        return a[i][j]

    @property
    def linear_forms(self):
        if self._L is None:
            logging.error("Linear forms haven't been computed. Need to call compute_forms()")
            return None
        return self._L

    def linear_form(self, i: int):
        """Block ``L[i]`` (reference ``assembly.py:393-398``)."""
        L = self.linear_forms
        if L is None:
            return None
        if i >= len(L):
            logging.error("Linear form L[%d] out of range", i)
        return L[i]

    def _block_rows(self, i: int) -> np.ndarray:
        """Owned device rows of function block ``i`` in the block's DoF order."""
        blocks = [*self._flux_idx, self._p_idx, self._lm_idx]
        return np.asarray(blocks[i], dtype=np.int64)

    def scatter_solution(self, x: np.ndarray, functions: list) -> list:
        """Split a host device-layout vector into ``[flux..., pressure, multiplier]``."""
        for fn, idx in zip(functions[:-2], self._flux_idx):
            fn.x.array[:] = x[idx]
        functions[-2].x.array[:] = x[self._p_idx]
        functions[-1].x.array[:] = x[self._lm_idx]
        return functions

    def solution_functions(self, functions: list | None = None, deferred: bool = True) -> list:
        """The device solution as ``[flux_color_0 .., pressure, global_flux]`` (the
        reference's ``assign``, ``solver.py:120-134``), in the block order by one gather
        kernel. New functions (``deferred``, the default) hold a device snapshot of it and
        read it into a pinned buffer -- one DMA for all of them -- when the first one's
        ``x.array`` is used; ``deferred=False`` copies at once. Given ``functions`` are
        filled at once."""
        off = self._out_off
        spaces = self.function_spaces
        if functions is None:
            names = [f"flux_color_{i}" for i in range(len(self._flux_spaces))]
            names += ["pressure", "global_flux"]
            if deferred:
                src = self._snap_pool.take()
                return [Function(V, name=nm, deferred=(src, int(off[i]), int(off[i + 1])))
                        for i, (V, nm) in enumerate(zip(spaces, names))]
            buf = self._out_pool.take()
            self._handle.solution_blocks(buf)
            return [Function(V, name=nm, array=buf[off[i]:off[i + 1]])
                    for i, (V, nm) in enumerate(zip(spaces, names))]
        if len(functions) != len(spaces):
            raise ValueError(f"expected {len(spaces)} functions, got {len(functions)}")
        buf = self._out_pool.take()
        self._handle.solution_blocks(buf)
        for i, fn in enumerate(functions):
            np.copyto(fn.x.array, buf[off[i]:off[i + 1]])
        return functions

    def close(self) -> None:
        snaps = getattr(self, "_snap_pool", None)
        if snaps is not None and getattr(self._handle, "_h", None):
            snaps.materialize_all()  # returned functions stay valid after close
        pool = getattr(self, "_out_pool", None)
        if pool is not None:
            pool.close()
        self._handle.close()
        aux = getattr(self, "_fe_aux", None)
        if aux is not None:  # (after the handle that used it)
            aux.close()
            self._fe_aux = None
