"""ctypes binding of ``libnxhip.so`` (C ABI declared in ``include/nxhip.h``).

There is no CPU fallback: if the library cannot be loaded, or no HIP device is
visible, the device entry points raise. The library is loaded from the package
directory (built in-tree by :mod:`networks_fenicsx_amd.build`).
"""

from __future__ import annotations

import ctypes as C
import os
import threading
import weakref
from pathlib import Path

import numpy as np

__all__ = ["lib", "NxError", "NxNotConverged", "check", "Handle", "Group", "PinnedPool",
           "EXPORTED_SYMBOLS"]

_LIB_PATH = Path(os.environ.get("NXHIP_LIB") or Path(__file__).resolve().parent / "libnxhip.so")
_lock = threading.Lock()
_lib = None

NX_OK, NX_ERR_ARG, NX_ERR_HIP, NX_ERR_RCCL, NX_ERR_STATE, NX_ERR_NOCONV = 0, -1, -2, -3, -4, -5
UNIQUE_ID_BYTES = 128
XCH_HANDLE_BYTES = 64  # NX_XCH_HANDLE_BYTES

_i32, _i64, _f64 = C.c_int32, C.c_int64, C.c_double
_pd = C.POINTER(C.c_double)
_pi32 = C.POINTER(C.c_int32)
_pi64 = C.POINTER(C.c_int64)
_pu8 = C.POINTER(C.c_ubyte)
_h = C.c_void_p

# name -> (restype, argtypes); mirrors include/nxhip.h
_SIGS = {
    "nx_version": (C.c_int, []),
    "nx_last_error": (C.c_char_p, []),
    "nx_device_count": (C.c_int, [_pi32]),
    "nx_create": (C.c_int, [_i32, _i32, _i64, _pd, _pi32, _i64, _pi32, _pi32, _pd, _i64,
                            C.POINTER(_h)]),
    "nx_create_fe": (C.c_int, [_i32, _i32, _i64, _pd, _i64, _pi32, _pi32, _i64, _i32, _pi32, _pd,
                               _pi32, _pi32, _pi32, _pi32, _pi32, _pi32, C.POINTER(_h)]),
    "nx_fe_struct_degree": (C.c_int, [_i32, _i64, _i64, _pi32, _pi32, _i32, _pi32, _pi32,
                                      _pi32, _pi32, _pi32, _pi32, _pi32]),
    "nx_fe_templates": (C.c_int, [_h, _pi32, _pi32]),
    "nx_destroy": (C.c_int, [_h]),
    "nx_dims": (C.c_int, [_h, _pi64, _pi64, _pi64]),
    "nx_set_coefficients": (C.c_int, [_h, _pd, _f64, _f64, _pd]),
    "nx_set_source": (C.c_int, [_h, _pd]),
    "nx_assemble": (C.c_int, [_h, _i32, _i32]),
    "nx_solve": (C.c_int, [_h, _f64, _i32, _i32, _pi32, _pd, _pi32]),
    "nx_get_solution": (C.c_int, [_h, _pd]),
    "nx_get_rhs": (C.c_int, [_h, _pd]),
    "nx_set_output_map": (C.c_int, [_h, _i64, _pi32]),
    "nx_get_solution_blocks": (C.c_int, [_h, C.c_void_p]),
    "nx_snapshot_solution": (C.c_int, [_h, _i32]),
    "nx_fetch_snapshot": (C.c_int, [_h, _i32, C.c_void_p]),
    "nx_host_alloc": (C.c_int, [_i64, C.POINTER(C.c_void_p)]),
    "nx_host_free": (C.c_int, [C.c_void_p]),
    "nx_get_vector": (C.c_int, [_h, _i32, _pd]),
    "nx_get_csr": (C.c_int, [_h, _pi32, _pi32, _pd]),
    "nx_spmv_host": (C.c_int, [_h, _pd, _pd]),
    "nx_true_residual": (C.c_int, [_h, _pd]),
    "nx_sync": (C.c_int, [_h]),
    "nx_set_profiling": (C.c_int, [_h, _i32]),
    "nx_get_profile": (C.c_int, [_h, _pd, _pi64, _pd, _pi64]),
    "nx_get_profile_direct": (C.c_int, [_h, _pd, _pi64]),
    "nx_get_direct_info": (C.c_int, [_h, _pi32, _pi32]),
    "nx_get_direct_path": (C.c_int, [_h, _pi32]),
    "nx_get_direct_sup": (C.c_int, [_h, _pi32]),
    "nx_debug_set_wait_polls": (C.c_int, [_h, C.c_uint32]),
    "nx_debug_xr_rehearse": (C.c_int, [_h, _f64, _i32, _pd]),
    "nx_reset_profile": (C.c_int, [_h]),
    "nx_bench_spmv": (C.c_int, [_h, _i32, _pd]),
    "nx_bench_spmv_cold": (C.c_int, [_h, _i32, _pi32, _pd]),
    "nx_get_graph_mode": (C.c_int, [_h, _pi32]),
    "nx_set_preconditioner": (C.c_int, [_h, _i32, _i64, _pi32, _pi32, _pi32, _pi32, _i64, _pi32,
                                        _pi32, _pi32, _pi32, _pi32, _pi32, _pi32, _i32, _pi32,
                                        _pi32, _i32, _pi32, _i32, _pi32]),
    "nx_comm_unique_id": (C.c_int, [_pu8]),
    "nx_comm_init": (C.c_int, [_h, _i32, _i32, _pu8, _i32, _pi32, _pi32, _pi32, _pi32]),
    "nx_comm_init_host": (C.c_int, [_h, _i32, _i32, C.c_char_p, _i32, _pi32, _pi32, _pi32,
                                    _pi32]),
    "nx_set_coarse": (C.c_int, [_h, _i32, _pi32, _i32, _pi32, _pi32, _pi32, _pi32, _pi32, _pi32,
                                _i32, _pi32]),
    "nx_comm_count": (C.c_int, [_h, _pi32]),
    "nx_xch_export": (C.c_int, [_h, _pu8]),
    "nx_xch_import": (C.c_int, [_h, _pu8]),
    "nx_set_halo": (C.c_int, [_h, _i32, _i32, _i32, _pi32, _pi32, _pi32, _pi32]),
    "nx_set_cut": (C.c_int, [_h, _i32, _pi32, _pi32, _pi32, _pd]),
    "nx_set_pc_kernels": (C.c_int, [_h, _i32]),
    "nx_get_pc_kernels": (C.c_int, [_h, _pi32]),
    "nx_set_pc_dense": (C.c_int, [_h, _i32, _i32, _pi32, _pi32, _pi32, _pi32, _pi32, _pi32,
                                  _pi32, _pi32, _pi32, _pi32]),
    "nx_set_pc_exact": (C.c_int, [_h, _i32]),
    "nx_get_pc_exact": (C.c_int, [_h, _pi32]),
    "nx_set_solver": (C.c_int, [_h, _i32, _i32]),
    "nx_set_cycles": (C.c_int, [_h, _i32, _pi32]),
    "nx_set_cycles_team": (C.c_int, [_h, _i32, _pi32, _pi32, _pi32]),
    "nx_set_cell_mass": (C.c_int, [_h, _f64, _f64]),
    "nx_fe_set_direct": (C.c_int, [_h, _h, _i32, _i64, _pi32, _pi32, _pi32, _pi32, _pi32, _pi32,
                                   _pi32, _pi32, _pd, _f64]),
    "nx_fe_cp_ranks": (C.c_int, [_h, _i64, _i64, _pi32, _i64, _pi32]),
    "nx_fe_set_cp": (C.c_int, [_h, _i32, _i32, _i32, _pd, _pi32, _i64, _pi32, _pi32, _i32,
                               _pi32, _pi32, _pi32, _pi32, _pi32, _pi32, _pi32, _pi32]),
    "nx_get_solver": (C.c_int, [_h, _pi32, _pi32]),
    "nx_set_lean": (C.c_int, [_i32]),
    "nx_group_create": (C.c_int, [_i32, C.POINTER(_h), C.POINTER(_h)]),
    "nx_group_solve": (C.c_int, [_h, _f64, _i32, _i32, _pi32, _pd, _pi32]),
    "nx_debug_xr_separate": (C.c_int, [_h, _f64, _pd]),
    "nx_debug_xr_polls": (C.c_int, [_h, _i32, C.c_uint32]),
    "nx_get_xr_status": (C.c_int, [_h, _pi32]),
    "nx_group_destroy": (C.c_int, [_h]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)
MAX_CYCLES = 2048  # kMaxCyc of csrc/nxhip.hip: cycle-closing chains the direct solve corrects


class NxError(RuntimeError):
    """A failure reported by libnxhip (the message is ``nx_last_error()``)."""


class NxNotConverged(NxError):
    """MINRES did not reach the tolerance (mirrors ``ksp_error_if_not_converged``)."""


def _import_torch_first() -> bool:
    """Load torch's HIP runtime and RCCL before ``libnxhip.so``.

    torch bundles its own ``libamdhip64`` / ``librccl`` (same SONAMEs as ``/opt/rocm``), and
    a process that maps ``libnxhip.so`` before torch's HIP libraries aborts at exit ("double
    free or corruption"), even when both bind to the same runtime copy (measured: preloading
    torch's runtime libraries by path does not avoid it; importing torch first does). So when
    torch is importable it is imported here, before the library is mapped, whatever order
    the caller imports things in (``tests/test_lib.py`` runs the "wrong" order in a
    subprocess). ``NXHIP_NO_TORCH=1`` skips this for processes that never import torch."""
    import importlib.util
    import sys

    if "torch" in sys.modules or os.environ.get("NXHIP_NO_TORCH", "0") not in ("", "0"):
        return False
    try:
        if importlib.util.find_spec("torch") is None:
            return False
    except (ImportError, ValueError):
        return False
    import torch  # noqa: F401

    return True


def lib():
    """Load ``libnxhip.so`` once; raise loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not _LIB_PATH.exists():
                raise NxError(
                    f"{_LIB_PATH} is missing: build it with "
                    "`python -m networks_fenicsx_amd.build` (there is no CPU fallback)"
                )
            _import_torch_first()
            handle = C.CDLL(str(_LIB_PATH), mode=C.RTLD_GLOBAL)
            for name, (res, args) in _SIGS.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


_FAST = None  # the _nxfast extension bound to lib()'s entry points, or False (ctypes)


def _fast():
    """The ``_nxfast`` extension (csrc/nxfast.c) bound to this library's ``nx_assemble`` /
    ``nx_solve``; None when it is not built (then ctypes makes the calls) or
    ``NXHIP_CTYPES=1``."""
    global _FAST
    if _FAST is None:
        _FAST = False
        if os.environ.get("NXHIP_CTYPES", "0") == "0":
            try:
                from . import _nxfast  # type: ignore[attr-defined]

                L = lib()
                _nxfast.bind(C.cast(L.nx_assemble, C.c_void_p).value,
                             C.cast(L.nx_solve, C.c_void_p).value)
                _FAST = _nxfast
            except ImportError:
                pass
    return _FAST or None


def check(rc: int) -> None:
    if rc != NX_OK:
        msg = lib().nx_last_error().decode(errors="replace")
        raise NxError(f"libnxhip error {rc}: {msg}")


def _ptr(a: np.ndarray | None, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


def fe_struct_degree(lay) -> int:
    """k when ``lay`` (a :class:`layout_fe.FeLayout`) is a (k, 0) layout whose terms the
    structured kernel forms in closed form, else 0 (``nx_fe_struct_degree``; no device)."""
    a = [np.ascontiguousarray(x, dtype=np.int32) for x in
         (lay.rowptr, lay.col, lay.a_ptr, lay.a_idx, lay.a_ent, lay.b_ptr, lay.b_idx, lay.b_ent)]
    k = C.c_int32()
    check(lib().nx_fe_struct_degree(int(lay.N), int(lay.E), int(lay.n_rows),
                                    *[_ptr(x, C.c_int32) for x in a[:2]],
                                    int(lay.table_kind.size),
                                    *[_ptr(x, C.c_int32) for x in a[2:]], C.byref(k)))
    return int(k.value)


def device_count() -> int:
    n = C.c_int32(0)
    check(lib().nx_device_count(C.byref(n)))
    return int(n.value)


class Handle:
    """Owning wrapper of an ``nx_network_t*`` (one local problem on one device)."""

    def __init__(self, device: int, N: int, edge_x: np.ndarray, edge_lm: np.ndarray,
                 lm_rowptr: np.ndarray, lm_col: np.ndarray, lm_val: np.ndarray, n_ghost: int = 0):
        L = lib()
        self._keep = []
        edge_x = np.ascontiguousarray(edge_x, dtype=np.float64).reshape(-1)
        edge_lm = np.ascontiguousarray(edge_lm, dtype=np.int32).reshape(-1)
        lm_rowptr = np.ascontiguousarray(lm_rowptr, dtype=np.int32)
        lm_col = np.ascontiguousarray(lm_col, dtype=np.int32)
        lm_val = np.ascontiguousarray(lm_val, dtype=np.float64)
        n_edges = edge_x.size // 6
        if edge_x.size != 6 * n_edges or edge_lm.size != 2 * n_edges:
            raise ValueError("edge_x must be (E, 6) and edge_lm (E, 2)")
        n_lm = lm_rowptr.size - 1
        h = C.c_void_p()
        check(L.nx_create(int(device), int(N), int(n_edges), _ptr(edge_x, C.c_double),
                          _ptr(edge_lm, C.c_int32), int(n_lm), _ptr(lm_rowptr, C.c_int32),
                          _ptr(lm_col, C.c_int32), _ptr(lm_val, C.c_double), int(n_ghost),
                          C.byref(h)))
        self._h = h
        self.device = int(device)
        self.N = int(N)
        self.n_edges = int(n_edges)
        self.n_lm = int(n_lm)
        r, c, z = C.c_int64(), C.c_int64(), C.c_int64()
        check(L.nx_dims(h, C.byref(r), C.byref(c), C.byref(z)))
        self.n_rows, self.n_cols, self.nnz = int(r.value), int(c.value), int(z.value)

    @classmethod
    def create_fe(cls, device: int, lay) -> "Handle":
        """Handle for general element degrees from a :class:`layout_fe.FeLayout`
        (``nx_create_fe``: CSR pattern and term tables from the host; a rank layout's ghost
        columns follow its owned rows)."""
        L = lib()
        self = cls.__new__(cls)
        self._keep = []
        edge_x = np.ascontiguousarray(lay.edge_x, dtype=np.float64).reshape(-1)
        h = C.c_void_p()
        arrays = [np.ascontiguousarray(a, dtype=np.int32) for a in
                  (lay.rowptr, lay.col, lay.table_kind, lay.a_ptr, lay.a_idx, lay.a_ent,
                   lay.b_ptr, lay.b_idx, lay.b_ent)]
        rp, col, kind, ap, ai, ae, bp, bi, be = arrays
        tval = np.ascontiguousarray(lay.table_val, dtype=np.float64)
        check(L.nx_create_fe(int(device), int(lay.N), int(lay.E), _ptr(edge_x, C.c_double),
                             int(lay.n_rows), _ptr(rp, C.c_int32), _ptr(col, C.c_int32),
                             int(getattr(lay, "n_ghost", 0)), int(kind.size), _ptr(kind, C.c_int32), _ptr(tval, C.c_double),
                             _ptr(ap, C.c_int32), _ptr(ai, C.c_int32), _ptr(ae, C.c_int32),
                             _ptr(bp, C.c_int32), _ptr(bi, C.c_int32), _ptr(be, C.c_int32),
                             C.byref(h)))
        self._h = h
        self.device = int(device)
        self.N = int(lay.N)
        self.n_edges = int(lay.E)
        self.n_lm = int(lay.lm_nodes.size)
        r, c, z = C.c_int64(), C.c_int64(), C.c_int64()
        check(L.nx_dims(h, C.byref(r), C.byref(c), C.byref(z)))
        self.n_rows, self.n_cols, self.nnz = int(r.value), int(c.value), int(z.value)
        return self

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        self.__dict__.pop("_addr_v", None)
        if getattr(self, "_h", None):
            lib().nx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ptr(self):
        if not self._h:
            raise NxError("handle is closed")
        return self._h

    # ------------------------------------------------------------------ calls
    def set_coefficients(self, edge_R: np.ndarray | None, R_const: float, f: float,
                         edge_bc: np.ndarray) -> None:
        eR = None if edge_R is None else np.ascontiguousarray(edge_R, dtype=np.float64)
        bc = np.ascontiguousarray(edge_bc, dtype=np.float64).reshape(-1)
        if bc.size != 2 * self.n_edges or (eR is not None and eR.size != self.n_edges):
            raise ValueError("edge_bc must be (E, 2) and edge_R (E,)")
        check(lib().nx_set_coefficients(self.ptr, _ptr(eR, C.c_double), float(R_const), float(f),
                                        _ptr(bc, C.c_double)))

    def set_source(self, edge_f: np.ndarray | None) -> None:
        """Per-edge source values (``nx_set_source``); None: the constant of set_coefficients."""
        ef = None if edge_f is None else np.ascontiguousarray(edge_f, dtype=np.float64)
        if ef is not None and ef.size != self.n_edges:
            raise ValueError("edge_f must have one value per local edge")
        check(lib().nx_set_source(self.ptr, _ptr(ef, C.c_double)))

    def assemble(self, lhs: bool = True, rhs: bool = True) -> None:
        fast = _fast()
        if fast is not None:  # (the per-step calls without ctypes: csrc/nxfast.c)
            rc = fast.assemble(self._addr, 1 if lhs else 0, 1 if rhs else 0)
        else:
            rc = lib().nx_assemble(self.ptr, 1 if lhs else 0, 1 if rhs else 0)
        if rc != NX_OK:
            check(rc)

    def solve(self, rtol: float, maxit: int, check_every: int = 4):
        fast = _fast()
        if fast is not None:
            rc, it, rr, conv = fast.solve(self._addr, float(rtol), int(maxit), int(check_every))
            if rc != NX_OK:
                check(rc)
            return it, rr, conv
        # out-parameters allocated once per handle: this call sits in every step's host path
        out = self.__dict__.get("_solve_out")
        if out is None:
            vals = (C.c_int32(), C.c_double(), C.c_int32())
            out = self._solve_out = (vals, tuple(C.byref(v) for v in vals))
        rc = lib().nx_solve(self.ptr, float(rtol), int(maxit), int(check_every), *out[1])
        if rc != NX_OK:
            check(rc)
        it, rr, conv = out[0]
        return int(it.value), float(rr.value), bool(conv.value)

    @property
    def _addr(self) -> int:
        # (the handle's address for _nxfast, cached until close(); a closed handle fails
        # loudly, as the ctypes path does)
        a = self.__dict__.get("_addr_v")
        if a is None:
            h = self._h
            if not h:
                raise NxError("handle is closed")
            a = self._addr_v = int(C.cast(h, C.c_void_p).value or 0)
        return a

    def solution(self) -> np.ndarray:
        x = np.empty(self.n_rows, dtype=np.float64)
        check(lib().nx_get_solution(self.ptr, _ptr(x, C.c_double)))
        return x

    def set_output_map(self, rows: np.ndarray) -> None:
        """Owned rows in output order (``nx_set_output_map``): the solver's function blocks."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        check(lib().nx_set_output_map(self.ptr, int(rows.size),
                                      _ptr(rows if rows.size else np.zeros(1, np.int32), C.c_int32)))

    def solution_blocks(self, out: np.ndarray) -> np.ndarray:
        """The solution permuted by the output map into ``out`` (n_rows doubles; pinned
        memory from :class:`PinnedPool` makes the device-to-host copy one DMA)."""
        if out.dtype != np.float64 or out.size != self.n_rows or not out.flags.c_contiguous:
            raise ValueError(f"out must be a contiguous float64 array of {self.n_rows} entries")
        check(lib().nx_get_solution_blocks(self.ptr, C.c_void_p(out.ctypes.data)))
        return out

    def snapshot_solution(self, slot: int) -> None:
        """Gather the solution in the output order into device snapshot ``slot`` (async)."""
        check(lib().nx_snapshot_solution(self.ptr, int(slot)))

    def fetch_snapshot(self, slot: int, out: np.ndarray) -> np.ndarray:
        """Copy device snapshot ``slot`` into ``out`` (n_rows doubles, ideally pinned)."""
        if out.dtype != np.float64 or out.size != self.n_rows or not out.flags.c_contiguous:
            raise ValueError(f"out must be a contiguous float64 array of {self.n_rows} entries")
        check(lib().nx_fetch_snapshot(self.ptr, int(slot), C.c_void_p(out.ctypes.data)))
        return out

    def rhs(self) -> np.ndarray:
        b = np.empty(self.n_rows, dtype=np.float64)
        check(lib().nx_get_rhs(self.ptr, _ptr(b, C.c_double)))
        return b

    def csr(self):
        rp = np.empty(self.n_rows + 1, dtype=np.int32)
        col = np.empty(self.nnz, dtype=np.int32)
        val = np.empty(self.nnz, dtype=np.float64)
        check(lib().nx_get_csr(self.ptr, _ptr(rp, C.c_int32), _ptr(col, C.c_int32),
                               _ptr(val, C.c_double)))
        return rp, col, val

    def spmv(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.size != self.n_cols:
            raise ValueError(f"x must have {self.n_cols} entries")
        y = np.empty(self.n_rows, dtype=np.float64)
        check(lib().nx_spmv_host(self.ptr, _ptr(x, C.c_double), _ptr(y, C.c_double)))
        return y

    def true_residual(self) -> float:
        r = C.c_double()
        check(lib().nx_true_residual(self.ptr, C.byref(r)))
        return float(r.value)

    def sync(self) -> None:
        check(lib().nx_sync(self.ptr))

    def set_profiling(self, enable: bool) -> None:
        check(lib().nx_set_profiling(self.ptr, int(bool(enable))))

    def profile(self):
        a, b, c, d = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        check(lib().nx_get_profile(self.ptr, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"spmv_ms": a.value, "spmv_count": b.value, "asm_ms": c.value, "asm_count": d.value}

    def profile_direct(self):
        """Direct solves under profiling: summed ms of up / top / down sweeps and residual."""
        ms = (C.c_double * 4)()
        n = C.c_int64(0)
        check(lib().nx_get_profile_direct(self.ptr, ms, C.byref(n)))
        return {"up_ms": ms[0], "top_ms": ms[1], "down_ms": ms[2], "residual_ms": ms[3],
                "count": int(n.value)}

    def direct_info(self) -> dict:
        """How the direct solve checks its residual (nx_get_direct_info)."""
        f, n = C.c_int32(0), C.c_int32(0)
        check(lib().nx_get_direct_info(self.ptr, C.byref(f), C.byref(n)))
        return {"fused_residual": bool(f.value), "n_left": int(n.value)}

    def fe_templates(self) -> tuple[int, int]:
        """(shapes, rows per edge) of a general-degree handle's edge templates
        (nx_fe_templates); (0, 0) when it kept the gather tables."""
        n, per = C.c_int32(0), C.c_int32(0)
        check(lib().nx_fe_templates(self.ptr, C.byref(n), C.byref(per)))
        return int(n.value), int(per.value)

    def direct_sup(self) -> bool:
        """Whether the last one-launch step ran phase 2 by superposition
        (nx_get_direct_sup)."""
        v = C.c_int32(0)
        check(lib().nx_get_direct_sup(self.ptr, C.byref(v)))
        return bool(v.value)

    def direct_path(self) -> str:
        """What the last direct solve ran (nx_get_direct_path): ``"fused"`` (k_dir_step, one
        launch), ``"launches"`` (assembly, up, down, publish) or ``"condensed"`` (the (k, 0)
        route through the auxiliary P1/DG0 handle)."""
        v = C.c_int32(0)
        check(lib().nx_get_direct_path(self.ptr, C.byref(v)))
        return {1: "fused", 2: "condensed", 3: "exchange", 4: "node-condensed"}.get(v.value,
                                                                                  "launches")

    def xr_rehearse(self, rtol: float = 1e-12, reps: int = 20) -> float:
        """Rehearsal hook (``nx_debug_xr_rehearse``): ms per launch of this group member's
        exchange step alone, its exchanges emulated from the group's last graph-path solve."""
        ms = C.c_double(0.0)
        check(lib().nx_debug_xr_rehearse(self.ptr, float(rtol), int(reps), C.byref(ms)))
        return float(ms.value)

    def set_wait_polls(self, polls: int) -> None:
        """Test hook (``nx_debug_set_wait_polls``): the fused step's wait bound; 0 forces
        the give-up fallback to the separate launches."""
        check(lib().nx_debug_set_wait_polls(self.ptr, int(polls)))

    def reset_profile(self) -> None:
        check(lib().nx_reset_profile(self.ptr))

    def bench_spmv(self, reps: int) -> float:
        ms = C.c_double()
        check(lib().nx_bench_spmv(self.ptr, int(reps), C.byref(ms)))
        return float(ms.value)

    def vector(self, which: int) -> np.ndarray:
        """0 = solution, 1 = rhs, 2 = latest preconditioned residual (owned rows)."""
        out = np.empty(self.n_rows, dtype=np.float64)
        check(lib().nx_get_vector(self.ptr, int(which), _ptr(out, C.c_double)))
        return out

    def graph_mode(self) -> bool:
        """True if the last solve replayed HIP graphs."""
        g = C.c_int32(0)
        check(lib().nx_get_graph_mode(self.ptr, C.byref(g)))
        return bool(g.value)

    def bench_spmv_cold(self, reps: int = 200):
        """(ms per SpMV, number of rotated copies) with operands streamed from HBM."""
        ms = C.c_double(0.0)
        k = C.c_int32(0)
        check(lib().nx_bench_spmv_cold(self.ptr, int(reps), C.byref(k), C.byref(ms)))
        return float(ms.value), int(k.value)

    def set_preconditioner(self, pc) -> None:
        """Upload a :class:`precond.TreePreconditioner` (``None`` disables it)."""
        self._pcx = None  # (nx_set_preconditioner resets the flux mass choice)
        if pc is None:
            z = np.zeros(1, np.int32)
            check(lib().nx_set_preconditioner(self.ptr, 0, 0, *([_ptr(z, C.c_int32)] * 4), 0,
                                              *([_ptr(z, C.c_int32)] * 7), 0, _ptr(z, C.c_int32),
                                              _ptr(z, C.c_int32), 0, _ptr(z, C.c_int32), 0,
                                              _ptr(z, C.c_int32)))
            return
        arr = {k: np.ascontiguousarray(getattr(pc, k), dtype=np.int32) for k in (
            "chain_edge", "chain_flip", "chain_up", "chain_lo", "slot_lam", "slot_pchain",
            "slot_parent", "slot_dc_off", "slot_dc", "dc_lo", "slot_plam", "job_chain_off",
            "job_lvl_off", "lvl_slot_off", "top_lvl_off")}
        arr = {k: (v if v.size else np.zeros(1, np.int32)) for k, v in arr.items()}
        self._pc_keep = arr
        p = {k: _ptr(v, C.c_int32) for k, v in arr.items()}
        check(lib().nx_set_preconditioner(
            self.ptr, 1, int(pc.n_chains), p["chain_edge"], p["chain_flip"], p["chain_up"],
            p["chain_lo"], int(pc.n_slots), p["slot_lam"], p["slot_pchain"], p["slot_parent"],
            p["slot_dc_off"], p["slot_dc"], p["dc_lo"], p["slot_plam"], int(pc.n_jobs),
            p["job_chain_off"], p["job_lvl_off"],
            int(pc.lvl_slot_off.size - 1), p["lvl_slot_off"], int(pc.top_lvl_off.size - 1),
            p["top_lvl_off"]))
        if getattr(pc, "job_tslot", None) is not None and pc.job_tslot.size:
            keys = ("job_tslot_off", "job_tslot", "job_need_off", "job_need", "top_uoff",
                    "slot_uy", "chain_uit", "chain_uib", "job_root_u", "job_root_dc")
            da = {k: np.ascontiguousarray(getattr(pc, k), dtype=np.int32) for k in keys}
            da = {k: (v if v.size else np.zeros(1, np.int32)) for k, v in da.items()}
            self._pc_keep_d = da
            check(lib().nx_set_pc_dense(self.ptr, 1, int(pc.n_jobs),
                                        *[_ptr(da[k], C.c_int32) for k in keys]))
        nC = int(getattr(pc, "n_coarse", 0))
        if nC:
            ca = {k: np.ascontiguousarray(getattr(pc, k), dtype=np.int32) for k in (
                "slot_cidx", "cc_chain", "cc_top", "cc_bot", "c_parent", "c_child_off",
                "c_child", "c_lvl_off")}
            ca = {k: (v if v.size else np.zeros(1, np.int32)) for k, v in ca.items()}
            self._pc_keep_c = ca
            q = {k: _ptr(v, C.c_int32) for k, v in ca.items()}
            check(lib().nx_set_coarse(
                self.ptr, nC, q["slot_cidx"], int(pc.cc_chain.size), q["cc_chain"], q["cc_top"],
                q["cc_bot"], q["c_parent"], q["c_child_off"], q["c_child"],
                int(pc.c_lvl_off.size - 1), q["c_lvl_off"]))
        cyc = np.ascontiguousarray(getattr(pc, "cyc_rows", np.zeros((0, 2))), dtype=np.int32)
        multi = getattr(self, "_multi", False) or self.n_cols > self.n_rows
        if cyc.size and nC == 0 and not multi and cyc.shape[0] <= MAX_CYCLES:
            # one rank, a graph with cycles: the direct solve corrects for the couplings its
            # tree solve drops (nx_set_cycles; past MAX_CYCLES the solve runs MINRES)
            self._pc_keep_y = cyc
            check(lib().nx_set_cycles(self.ptr, int(cyc.shape[0]), _ptr(cyc, C.c_int32)))

    def set_cycles_team(self, own, qloc, lcol) -> None:
        """Several ranks, a graph with cycles (``nx_set_cycles_team``): this rank's share of
        the Woodbury correction of all ranks' K cycle chains (``own``: 2K, ``qloc`` /
        ``lcol``: K; see include/nxhip.h). Empty arrays clear it."""
        arrs = [np.ascontiguousarray(a, dtype=np.int32) for a in (own, qloc, lcol)]
        K = int(arrs[1].size)
        if arrs[0].size != 2 * K or arrs[2].size != K:
            raise ValueError("own must hold 2K entries, qloc and lcol K")
        arrs = [a if a.size else np.zeros(1, np.int32) for a in arrs]
        self._cyc_team_keep = arrs
        check(lib().nx_set_cycles_team(self.ptr, K, *[_ptr(a, C.c_int32) for a in arrs]))

    def fe_set_cp(self, tab) -> None:
        """``nx_fe_set_cp``: the continuous-pressure direct solve's tables
        (``layout_fe.build_cp_tables``); ``None`` detaches it."""
        if tab is None:
            z = np.zeros(1, np.int32)
            check(lib().nx_fe_set_cp(self.ptr, 0, 0, 0, None, None, 0, *([_ptr(z, C.c_int32)] * 2),
                                     0, *([_ptr(z, C.c_int32)] * 8)))
            return
        i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
        arrs = [i32(x) if x.size else np.zeros(1, np.int32) for x in (
            tab.tI, tab.nrow, tab.eb, tab.lev_off, tab.order, tab.inc_off, tab.inc, tab.parent,
            tab.child_off, tab.child, tab.nown)]
        cst = np.ascontiguousarray(tab.cst, dtype=np.float64)
        self._cp_keep = (arrs, cst)
        p = [_ptr(a, C.c_int32) for a in arrs]
        check(lib().nx_fe_set_cp(self.ptr, int(tab.k), int(tab.m), int(tab.nI),
                                 _ptr(cst, C.c_double), p[0], int(tab.n_nodes), p[1], p[2],
                                 int(tab.lev_off.size - 1), p[3], p[4], p[5], p[6], p[7], p[8],
                                 p[9], p[10]))

    def fe_cp_ranks(self, n_own_edges: int, n_edges_global: int, gid, nrowx) -> None:
        """``nx_fe_cp_ranks`` (several ranks, before :meth:`fe_set_cp`): this rank's edges'
        global ids and the local rows of the node rows it owns (2 per node, -1 elsewhere)."""
        gid = np.ascontiguousarray(gid, dtype=np.int32)
        nrowx = np.ascontiguousarray(nrowx, dtype=np.int32).ravel()
        self._cp_rank_keep = (gid, nrowx)
        check(lib().nx_fe_cp_ranks(self.ptr, int(n_own_edges), int(n_edges_global),
                                   _ptr(gid if gid.size else np.zeros(1, np.int32), C.c_int32),
                                   int(nrowx.size // 2), _ptr(nrowx, C.c_int32)))

    def set_pc_exact(self, enable: bool) -> None:
        """Consistent (exact Schur complement, default) or lumped flux mass in P."""
        check(lib().nx_set_pc_exact(self.ptr, int(bool(enable))))
        self._pcx = bool(enable)

    def pc_exact(self) -> bool:
        """The flux mass P uses (nx_get_pc_exact; remembered after the first query or the
        last set_pc_exact through this handle -- the per-solve check costs no C call)."""
        v = getattr(self, "_pcx", None)
        if v is None:
            e = C.c_int32(0)
            check(lib().nx_get_pc_exact(self.ptr, C.byref(e)))
            v = self._pcx = bool(e.value)
        return v

    def set_cell_mass(self, ratio: float, mo_div: float) -> None:
        """``nx_set_cell_mass``: this (auxiliary) handle's sweeps invert the condensed flux
        mass ``R h [[a, b], [b, a]]`` (ratio = a / b, mo_div = (a + b) / b)."""
        check(lib().nx_set_cell_mass(self.ptr, float(ratio), float(mo_div)))

    def fe_set_direct(self, aux: "Handle | None", k: int, slot, maps, cst, ab: float) -> None:
        """``nx_fe_set_direct``: attach the auxiliary P1/DG0 handle that solves this (k, 0)
        handle's condensed system (``maps``: :class:`layout_fe.FeAuxMaps`)."""
        if aux is None:
            z = _ptr(np.zeros(1, np.int32), C.c_int32)
            check(lib().nx_fe_set_direct(self.ptr, None, 0, 0, *([z] * 8), None, 0.0))
            self._fe_aux = None
            return
        i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
        arrs = [i32(slot), i32(maps.v_fe), i32(maps.v_aux), i32(maps.i_fe), i32(maps.p_fe),
                i32(maps.p_aux), i32(maps.l_fe) if maps.l_fe.size else np.zeros(1, np.int32),
                i32(maps.l_aux) if maps.l_aux.size else np.zeros(1, np.int32)]
        cst = np.ascontiguousarray(cst, dtype=np.float64)
        check(lib().nx_fe_set_direct(self.ptr, aux.ptr, int(k), int(maps.l_fe.size),
                                     *[_ptr(a, C.c_int32) for a in arrs],
                                     _ptr(cst, C.c_double), float(ab)))
        self._fe_aux = aux  # the auxiliary handle lives as long as this one uses it

    def set_solver(self, direct: bool, tree_exact: bool) -> None:
        """``nx_set_solver``: the direct tree solve (where exact) or MINRES."""
        check(lib().nx_set_solver(self.ptr, int(bool(direct)), int(bool(tree_exact))))

    def solver(self):
        """(requested, last run): 0 = MINRES, 1 = direct tree solve."""
        a, b = C.c_int32(0), C.c_int32(0)
        check(lib().nx_get_solver(self.ptr, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def set_halo(self, nranks: int, rank: int, peers, send_off, send_idx, recv_off):
        """Halo plan without a transport (in-process group members)."""
        self._multi = int(nranks) > 1
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        send_off = np.ascontiguousarray(send_off, dtype=np.int32)
        send_idx = np.ascontiguousarray(send_idx, dtype=np.int32)
        recv_off = np.ascontiguousarray(recv_off, dtype=np.int32)
        check(lib().nx_set_halo(self.ptr, int(nranks), int(rank), int(peers.size),
                                _ptr(peers if peers.size else np.zeros(1, np.int32), C.c_int32),
                                _ptr(send_off, C.c_int32),
                                _ptr(send_idx if send_idx.size else np.zeros(1, np.int32),
                                     C.c_int32),
                                _ptr(recv_off, C.c_int32)))

    def set_pc_kernels(self, global_kernels: bool) -> None:
        """The next preconditioner upload takes the global-memory sweeps (ranks agreeing)."""
        check(lib().nx_set_pc_kernels(self.ptr, int(bool(global_kernels))))

    def pc_lds(self) -> bool:
        """The uploaded preconditioner runs the LDS sweep kernels."""
        v = C.c_int32(0)
        check(lib().nx_get_pc_kernels(self.ptr, C.byref(v)))
        return bool(v.value)

    def set_cut(self, n_cut: int, lm_cut, gk_off, gk_row, gk_coef) -> None:
        """Cut bifurcations of a multi-rank problem (``nx_set_cut``): their multiplier rows
        are completed inside the direct solve's residual all-reduce."""
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in (
            (lm_cut, np.int32), (gk_off, np.int32), (gk_row, np.int32), (gk_coef, np.float64))]
        arrs = [a if a.size else np.zeros(1, a.dtype) for a in arrs]
        self._cut_keep = arrs
        check(lib().nx_set_cut(self.ptr, int(n_cut), _ptr(arrs[0], C.c_int32),
                               _ptr(arrs[1], C.c_int32), _ptr(arrs[2], C.c_int32),
                               _ptr(arrs[3], C.c_double)))

    def xch_export(self) -> bytes:
        """This rank's exchange mailbox handle (``nx_xch_export``, after comm_init)."""
        buf = (C.c_ubyte * XCH_HANDLE_BYTES)()
        check(lib().nx_xch_export(self.ptr, buf))
        return bytes(buf)

    def xch_import(self, handles) -> None:
        """Every rank's mailbox handle in rank order (``nx_xch_import``)."""
        raw = b"".join(handles)
        buf = (C.c_ubyte * len(raw)).from_buffer_copy(raw)
        check(lib().nx_xch_import(self.ptr, buf))

    def comm_count(self) -> int:
        """Ranks of the RCCL communicator (``ncclCommCount``), else the plan's rank count."""
        n = C.c_int32(0)
        check(lib().nx_comm_count(self.ptr, C.byref(n)))
        return int(n.value)

    def comm_init(self, nranks: int, rank: int, uid, peers, send_off, send_idx, recv_off):
        """Join the ranks' communicator: RCCL (``uid``: the unique id bytes, ``nx_comm_init``)
        or, with ``uid`` a ``str`` shared-memory name, the host transport of the tests
        (``nx_comm_init_host``: several ranks' processes on one GPU)."""
        self._multi = True  # (a communicator, even of one rank: no cycle correction)
        peers = np.ascontiguousarray(peers, dtype=np.int32)
        send_off = np.ascontiguousarray(send_off, dtype=np.int32)
        send_idx = np.ascontiguousarray(send_idx, dtype=np.int32)
        recv_off = np.ascontiguousarray(recv_off, dtype=np.int32)
        plan = (int(peers.size), _ptr(peers, C.c_int32), _ptr(send_off, C.c_int32),
                _ptr(send_idx if send_idx.size else np.zeros(1, np.int32), C.c_int32),
                _ptr(recv_off, C.c_int32))
        if isinstance(uid, str):
            check(lib().nx_comm_init_host(self.ptr, int(nranks), int(rank), uid.encode(), *plan))
            return
        uid_arr = (C.c_ubyte * UNIQUE_ID_BYTES).from_buffer_copy(uid)
        check(lib().nx_comm_init(self.ptr, int(nranks), int(rank), uid_arr, *plan))

    def xr_polls(self, which: int, polls: int) -> None:
        """Test hook (``nx_debug_xr_polls``): the poll bound of this rank's exchange
        ``which`` (0 coarse partials, 1 residual); 0 gives it up at once."""
        check(lib().nx_debug_xr_polls(self.ptr, int(which), int(polls)))

    def xr_status(self) -> dict:
        """``nx_get_xr_status``: whether the exchange step is off for good, the last launch's
        give-up reasons (bits 1 exchange 1, 2 exchange 2, 4 abort seen, 8 tag, 16 local),
        the agreements taken part in, the last launch's tag."""
        out = (C.c_int32 * 4)()
        check(lib().nx_get_xr_status(self.ptr, out))
        return {"off": bool(out[0]), "why": int(out[1]), "agreed": int(out[2]),
                "tag": int(out[3]) & 0xFFFFFFFF}


class Group:
    """In-process rank group (``nx_group_*``): handles of all ranks on one device."""

    def __init__(self, handles):
        self._handles = list(handles)  # keeps the handles alive while the group exists
        arr = (_h * len(self._handles))(*[h.ptr for h in self._handles])
        out = _h()
        check(lib().nx_group_create(len(self._handles), arr, C.byref(out)))
        self._g = out

    def solve(self, rtol: float = 1e-12, maxit: int = 50000, check_every: int = 4):
        it = C.c_int32(0)
        rr = C.c_double(0.0)
        conv = C.c_int32(0)
        check(lib().nx_group_solve(self._g, float(rtol), int(maxit), int(check_every),
                                   C.byref(it), C.byref(rr), C.byref(conv)))
        return int(it.value), float(rr.value), bool(conv.value)

    def xr_separate(self, rtol: float = 1e-12) -> float:
        """Debug / tests: every rank's exchange step as its own launch on its own stream
        (the RCCL ranks' shape; ``nx_debug_xr_separate``); the published residual."""
        rr = C.c_double(0.0)
        check(lib().nx_debug_xr_separate(self._g, float(rtol), C.byref(rr)))
        return float(rr.value)

    def close(self) -> None:
        if getattr(self, "_g", None):
            lib().nx_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class _PinnedView:
    """numpy base object of one pinned buffer: while any array (or view of one) made from it
    is alive, the pool does not hand the buffer out again."""

    def __init__(self, ptr: int, n: int):
        self.__array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False),
                                    "version": 3}


def _host_free(ptr: int) -> None:
    try:
        lib().nx_host_free(C.c_void_p(ptr))
    except Exception:  # noqa: BLE001 - interpreter shutdown
        pass


class PinnedPool:
    """Page-locked host buffers of ``n`` doubles (``nx_host_alloc``), reused once every array
    handed out from a buffer has been dropped. The solver's output functions are views into
    one such buffer, so a solve costs one gather kernel and one DMA instead of a pageable copy
    plus a host-side split per colour."""

    def __init__(self, n: int):
        self._n = int(n)
        self._slots: list[list] = []  # [ptr, weakref to the live _PinnedView or None]

    def take(self) -> np.ndarray:
        for s in self._slots:
            if s[1] is None or s[1]() is None:
                return self._wrap(s)
        p = C.c_void_p()
        check(lib().nx_host_alloc(8 * max(self._n, 1), C.byref(p)))
        s = [int(p.value), None]
        self._slots.append(s)
        return self._wrap(s)

    def _wrap(self, s) -> np.ndarray:
        v = _PinnedView(s[0], self._n)
        s[1] = weakref.ref(v)
        return np.asarray(v)

    def close(self) -> None:
        for ptr, ref in self._slots:
            v = ref() if ref is not None else None
            if v is None:
                _host_free(ptr)
            else:  # still viewed by a caller's arrays: free when the last one goes
                weakref.finalize(v, _host_free, ptr)
        self._slots = []

    def __del__(self):
        self.close()


_MAX_SNAPSHOTS = 64  # csrc/nxhip.hip kMaxSnap


class DeferredSolution:
    """One solve's output, held in a device snapshot slot until it is first read.

    ``array()`` copies the slot into a pinned buffer (one DMA, on the handle's copy stream)
    and frees the slot; until then later solves on the handle do not disturb it."""

    def __init__(self, pool: "SnapshotPool", slot: int):
        self._pool = pool
        self._slot = slot
        self._buf = None

    @property
    def ready(self) -> bool:
        return self._buf is not None

    def array(self) -> np.ndarray:
        if self._buf is None:
            buf = self._pool.pinned.take()
            self._pool.handle.fetch_snapshot(self._slot, buf)
            self._buf = buf
            self._pool.release(self._slot, self)
        return self._buf

    def __del__(self):
        try:
            if self._buf is None:
                self._pool.release(self._slot, self)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class SnapshotPool:
    """Device snapshot slots of one handle (``nx_snapshot_solution``): ``take()`` gathers the
    current solution into a free slot and returns its :class:`DeferredSolution`. With every
    slot in use the oldest unread snapshot is read first (frees its slot).

    Device memory: a slot's buffer (one solution, ``8 n_rows`` bytes) is allocated on its
    first use and kept until the handle is destroyed, so a handle holds at most
    ``_MAX_SNAPSHOTS`` (64) solutions' worth of HBM for snapshots -- 0.5 GB at the 1 M-row
    C3 problem, the high-water mark of unread results, not a leak."""

    def __init__(self, handle: "Handle", pinned: PinnedPool):
        self.handle = handle
        self.pinned = pinned
        self._free = list(range(_MAX_SNAPSHOTS - 1, -1, -1))
        self._live: dict[int, weakref.ref] = {}  # slot -> unread DeferredSolution (oldest first)

    def take(self) -> DeferredSolution:
        if not self._free:
            oldest = next(iter(self._live.values()))()
            if oldest is not None:
                oldest.array()
            else:  # collected without __del__ running yet
                self._free.append(next(iter(self._live)))
                del self._live[next(iter(self._live))]
        slot = self._free.pop()
        self.handle.snapshot_solution(slot)
        d = DeferredSolution(self, slot)
        self._live[slot] = weakref.ref(d)
        return d

    def release(self, slot: int, owner: DeferredSolution) -> None:
        ref = self._live.get(slot)
        if ref is not None and ref() in (owner, None):
            del self._live[slot]
            self._free.append(slot)

    def materialize_all(self) -> None:
        """Read every unread snapshot (before the handle goes away)."""
        for ref in list(self._live.values()):
            d = ref()
            if d is not None:
                d.array()
        self._live.clear()


def set_lean(enable: bool) -> None:
    """Process-wide: one graph per solve (default) or the general chunked path."""
    check(lib().nx_set_lean(int(bool(enable))))


def comm_unique_id() -> bytes:
    buf = (C.c_ubyte * UNIQUE_ID_BYTES)()
    check(lib().nx_comm_unique_id(buf))
    return bytes(buf)
