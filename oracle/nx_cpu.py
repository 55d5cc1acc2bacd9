"""CPU PORT wrapper -- test infrastructure only.

ctypes binding of ``oracle/libnxcpu.so`` (``oracle/nx_cpu.c``, built by ``oracle/Makefile``):
an OpenMP restatement of one full step of the hot path on the host cores -- assembly of
the reference's forms in the device layout (``assembly.py:243-277``, pressure rows negated)
plus MINRES with the same exact tree Schur-complement preconditioner as the GPU, or the
same direct tree solve as the GPU's default (``nxc_direct``). Only
``bench.py``'s ``cpu_baseline`` leg and ``tests/`` use it; the product path never does.
"""

from __future__ import annotations

import ctypes as C
import os
import time
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "libnxcpu.so"
_lib = None

_pd = C.POINTER(C.c_double)
_pi = C.POINTER(C.c_int32)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise FileNotFoundError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(str(LIB))
        L.nxc_threads.restype = C.c_int
        L.nxc_set_threads.restype = None
        L.nxc_set_threads.argtypes = [C.c_int]
        L.nxc_nnz.restype = C.c_int64
        L.nxc_nnz.argtypes = [C.c_int, C.c_int64, _pi, C.c_int64, _pi]
        L.nxc_assemble.restype = None
        L.nxc_assemble.argtypes = [C.c_int, C.c_int64, _pd, _pi, _pd, C.c_double, _pd, C.c_double,
                                   C.c_int64, _pi, _pi, _pd, C.c_int, _pi, _pi, _pd, _pd, _pd]
        L.nxc_direct.restype = C.c_int
        L.nxc_direct.argtypes = ([C.c_int64, _pi, _pi, _pd, _pd, C.c_double, C.c_int, _pd,
                                  C.c_int64] + [_pi] * 4 + [C.c_int64] + [_pi] * 5
                                 + [C.c_int] + [_pi] * 3 + [C.c_int, _pi, _pd, _pd])
        L.nxc_minres.restype = C.c_int
        L.nxc_minres.argtypes = ([C.c_int64, _pi, _pi, _pd, _pd, C.c_double, C.c_int, C.c_int, _pd,
                                  C.c_int, C.c_int64] + [_pi] * 4 + [C.c_int64] + [_pi] * 5
                                 + [C.c_int] + [_pi] * 3 + [C.c_int, _pi, _pd, _pd])
        _lib = L
    return _lib


def threads() -> int:
    return int(lib().nxc_threads())


def set_threads(n: int) -> None:
    """The OpenMP thread count of the following calls (``omp_set_num_threads``)."""
    lib().nxc_set_threads(int(n))


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class CpuStep:
    """One rank-local problem (``layout.LocalProblem`` + ``precond.TreePreconditioner``)
    held in host memory; ``assemble()`` + ``solve()`` is one step of the hot path."""

    def __init__(self, lp, pc, edge_bc: np.ndarray, R: float = 1.0, f: float = 0.0,
                 exact: bool = True):
        L = lib()
        self.lp, self.pc, self.exact = lp, pc, exact
        self.N, self.E, self.B = lp.N, lp.edges.size, lp.lm_nodes.size
        self.n = lp.n_own
        self.edge_x = np.ascontiguousarray(lp.edge_x, dtype=np.float64)
        self.edge_lm = np.ascontiguousarray(lp.edge_lm, dtype=np.int32)
        self.lm_rowptr = np.ascontiguousarray(lp.lm_rowptr, dtype=np.int32)
        self.lm_col = np.ascontiguousarray(lp.lm_col, dtype=np.int32)
        self.lm_val = np.ascontiguousarray(lp.lm_val, dtype=np.float64)
        self.edge_bc = np.ascontiguousarray(edge_bc, dtype=np.float64).reshape(-1)
        self.R, self.f = float(R), float(f)
        nnz = int(L.nxc_nnz(self.N, self.E, _p(self.edge_lm, C.c_int32), self.B,
                            _p(self.lm_rowptr, C.c_int32)))
        self.rowptr = np.zeros(self.n + 1, np.int32)
        self.col = np.zeros(nnz, np.int32)
        self.val = np.zeros(nnz)
        self.rhs = np.zeros(self.n)
        self.dq = np.zeros(self.E * (self.N + 1))
        self.x = np.zeros(self.n)
        self._pc = {k: np.ascontiguousarray(getattr(pc, k), dtype=np.int32) for k in (
            "chain_edge", "chain_flip", "chain_up", "chain_lo", "slot_lam", "slot_pchain",
            "slot_parent", "slot_dc_off", "slot_dc", "job_chain_off", "job_lvl_off",
            "lvl_slot_off", "top_lvl_off")}
        self._assemble(pattern=True)

    def _assemble(self, pattern: bool) -> None:
        lib().nxc_assemble(self.N, self.E, _p(self.edge_x, C.c_double),
                           _p(self.edge_lm, C.c_int32), None, self.R,
                           _p(self.edge_bc, C.c_double), self.f, self.B,
                           _p(self.lm_rowptr, C.c_int32), _p(self.lm_col, C.c_int32),
                           _p(self.lm_val, C.c_double), int(pattern),
                           _p(self.rowptr, C.c_int32), _p(self.col, C.c_int32),
                           _p(self.val, C.c_double), _p(self.rhs, C.c_double),
                           _p(self.dq, C.c_double))

    def assemble(self) -> None:
        self._assemble(pattern=False)

    def solve(self, rtol: float = 1e-12, maxit: int = 50000):
        q = self._pc
        pc = self.pc
        rr = C.c_double(0.0)
        it = lib().nxc_minres(
            self.n, _p(self.rowptr, C.c_int32), _p(self.col, C.c_int32), _p(self.val, C.c_double),
            _p(self.rhs, C.c_double), float(rtol), int(maxit), self.N, _p(self.dq, C.c_double),
            int(self.exact), int(pc.n_chains), _p(q["chain_edge"], C.c_int32),
            _p(q["chain_flip"], C.c_int32), _p(q["chain_up"], C.c_int32),
            _p(q["chain_lo"], C.c_int32), int(pc.n_slots), _p(q["slot_lam"], C.c_int32),
            _p(q["slot_pchain"], C.c_int32), _p(q["slot_parent"], C.c_int32),
            _p(q["slot_dc_off"], C.c_int32), _p(q["slot_dc"], C.c_int32), int(pc.n_jobs),
            _p(q["job_chain_off"], C.c_int32), _p(q["job_lvl_off"], C.c_int32),
            _p(q["lvl_slot_off"], C.c_int32), int(q["top_lvl_off"].size - 1),
            _p(q["top_lvl_off"], C.c_int32), _p(self.x, C.c_double), C.byref(rr))
        return int(it), float(rr.value)

    def solve_direct(self, rtol: float = 1e-12):
        """The direct tree solve (``nxc_direct``): (passes, true relative residual)."""
        q = self._pc
        pc = self.pc
        rr = C.c_double(0.0)
        it = lib().nxc_direct(
            self.n, _p(self.rowptr, C.c_int32), _p(self.col, C.c_int32), _p(self.val, C.c_double),
            _p(self.rhs, C.c_double), float(rtol), self.N, _p(self.dq, C.c_double),
            int(pc.n_chains), _p(q["chain_edge"], C.c_int32),
            _p(q["chain_flip"], C.c_int32), _p(q["chain_up"], C.c_int32),
            _p(q["chain_lo"], C.c_int32), int(pc.n_slots), _p(q["slot_lam"], C.c_int32),
            _p(q["slot_pchain"], C.c_int32), _p(q["slot_parent"], C.c_int32),
            _p(q["slot_dc_off"], C.c_int32), _p(q["slot_dc"], C.c_int32), int(pc.n_jobs),
            _p(q["job_chain_off"], C.c_int32), _p(q["job_lvl_off"], C.c_int32),
            _p(q["lvl_slot_off"], C.c_int32), int(q["top_lvl_off"].size - 1),
            _p(q["top_lvl_off"], C.c_int32), _p(self.x, C.c_double), C.byref(rr))
        return int(it), float(rr.value)

    def time_steps(self, budget_s: float, rtol: float = 1e-12, max_runs: int = 200,
                   direct: bool = False):
        """Repeat assemble + solve for about ``budget_s`` seconds; (ms per step, runs, its)."""
        runs, total, its = 0, 0.0, 0
        while runs < 1 or (total < budget_s and runs < max_runs):
            t0 = time.perf_counter()
            self.assemble()
            its, _ = self.solve_direct(rtol) if direct else self.solve(rtol)
            total += time.perf_counter() - t0
            runs += 1
        return 1e3 * total / runs, runs, its


def omp_threads_env() -> int:
    v = os.environ.get("OMP_NUM_THREADS")
    return int(v) if v and v.isdigit() else (os.cpu_count() or 1)
