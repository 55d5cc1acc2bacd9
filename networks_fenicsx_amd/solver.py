"""Device MINRES solver for the hydraulic network system.

Mirrors ``Solver`` of the reference (``src/networks_fenicsx/solver.py:16-143``):
same constructor signature, ``assemble``, ``solve``, ``A``, ``b``, ``ksp`` and
``assembler`` accessors. The reference factorises the system with MUMPS
(``preonly`` + ``lu``, ``solver.py:58-65``). Here both KSP types run on the GPU
(``nx_solve`` in ``csrc/nxhip.hip``):

* ``ksp_type="preonly"`` (the reference default): a direct solve -- the block LU of the
  saddle-point system whose Schur complement the tree preconditioner inverts exactly
  (``nx_set_solver``), checked by the true residual. Used where it is exact: a tree, on one
  rank or on several (every rank's decomposition must run the LDS sweeps with the coarse
  step; the ranks decide together); otherwise, or with a residual above ``ksp_rtol`` after
  one refinement step, MINRES runs;
* ``ksp_type="minres"`` (or any other iterative type): preconditioned MINRES -- CSR SpMV,
  fused vector updates and deterministic reductions in HIP graphs.

PETSc options understood (with or without the options prefix):

``ksp_rtol``                      relative residual tolerance (default 1e-12, chosen so the
                                  solution matches a direct solve to <= 1e-10 rel. norm)
``ksp_max_it``                    iteration cap (default 50000)
``ksp_error_if_not_converged``    raise :class:`NxNotConverged` (default True)
``ksp_monitor``                   print iterations / residual after each solve
``ksp_check_every``               iterations per host convergence check (default 4 with the
                                  preconditioner -- the exact one converges in 3, + 1 launch for
                                  the last update -- and 32 for plain MINRES)

``pc_type``                       ``"none"`` runs plain MINRES; anything else (the reference's
                                  default ``"lu"`` included) uses the tree Schur-complement
                                  preconditioner (``precond.py``)
``pc_mass``                       ``"consistent"`` (default: exact Schur complement, 3 MINRES
                                  iterations) or ``"lumped"``

``ksp_type``                      ``"preonly"`` (default): the direct tree solve where exact,
                                  else MINRES; anything else: MINRES.
``pc_factor_mat_solver_type`` is accepted and recorded. ``ksp.solver_used`` tells which
solve ran last (``"direct"`` or ``"minres"``).
"""

from __future__ import annotations

import sys
import typing

import numpy as np

from . import _lib
from .assembly import DeviceMatrix, DeviceVector, HydraulicNetworkAssembler
from .timing import timed

__all__ = ["Solver", "KSPInfo"]

_DEFAULTS = {
    "ksp_type": "preonly",
    "pc_type": "lu",
    "pc_factor_mat_solver_type": "mumps",
    "ksp_monitor": None,
    "ksp_error_if_not_converged": True,
}


class KSPInfo:
    """What ``solver.ksp`` exposes: options and the last solve's statistics."""

    def __init__(self, prefix: str, options: dict):
        self.prefix = prefix
        self.options = options
        self.iterations = 0
        self.residual_estimate = float("nan")
        self.converged = False
        self.solver_used = ""

    def getOptionsPrefix(self) -> str:  # noqa: N802
        return self.prefix

    def getIterationNumber(self) -> int:  # noqa: N802
        return self.iterations

    def getResidualNorm(self) -> float:  # noqa: N802
        return self.residual_estimate

    def getConvergedReason(self) -> int:  # noqa: N802
        return 2 if self.converged else -3  # KSP_CONVERGED_RTOL / KSP_DIVERGED_ITS

    def destroy(self) -> None:
        return None


def _truthy(v) -> bool:
    if v is None:
        return True  # PETSc flag options given as None mean "set"
    if isinstance(v, str):
        return v.strip().lower() not in ("0", "false", "no", "off")
    return bool(v)


class Solver:
    """GPU solver interface for the network problem.

    Args:
        assembler: the hydraulic network assembler
        petsc_options_prefix: options prefix (kept for API compatibility)
        petsc_options: dictionary of PETSc-style options (see module docstring)
        kind: matrix kind (None, "mpi" or "nest"); recorded, storage is device CSR
    """

    def __init__(
        self,
        assembler: HydraulicNetworkAssembler,
        petsc_options_prefix: str = "NetworkSolver_",
        petsc_options: dict | None = None,
        kind: str | typing.Sequence[typing.Sequence[str]] | None = None,
    ):
        self._assembler = assembler
        opts = dict(_DEFAULTS if petsc_options is None else petsc_options)
        clean = {}
        for k, v in opts.items():
            key = k[len(petsc_options_prefix):] if k.startswith(petsc_options_prefix) else k
            clean[key.lstrip("-")] = v
        self._rtol = float(clean.get("ksp_rtol", 1e-12))
        self._maxit = int(clean.get("ksp_max_it", 50000))
        ce = clean.get("ksp_check_every")
        self._check_every = None if ce is None else int(ce)
        self._raise = _truthy(clean.get("ksp_error_if_not_converged", True))
        self._monitor = "ksp_monitor" in clean and _truthy(clean["ksp_monitor"])
        self._ksp = KSPInfo(petsc_options_prefix, clean)
        self._pc = str(clean.get("pc_type", "lu")).lower() != "none"
        self._pc_exact = str(clean.get("pc_mass", "consistent")).lower() != "lumped"
        self._direct = str(clean.get("ksp_type", "preonly")).lower() == "preonly"
        self._kind = kind
        self._A = DeviceMatrix(assembler.handle, kind)
        self._b = DeviceVector(assembler.handle)
        self._closed = False

    @property
    def assembler(self) -> HydraulicNetworkAssembler:
        return self._assembler

    @property
    def A(self) -> DeviceMatrix:  # noqa: N802
        return self._A

    @property
    def b(self) -> DeviceVector:
        return self._b

    @property
    def ksp(self) -> KSPInfo:
        return self._ksp

    @property
    def rtol(self) -> float:
        return self._rtol

    def assemble(self, lhs: bool = True, rhs: bool = True) -> None:
        """Assemble the system matrix and/or rhs (values are overwritten, not added)."""
        self.assembler.assemble(self._A, self._b, assemble_lhs=lhs, assemble_rhs=rhs)

    @timed("nxfx:Solver:solve")
    def solve(self, functions: list | None = None) -> list:
        """Solve on the device and return ``[flux_color_0.., pressure, global_flux]``
        (``solver.py:107-135``). One gather kernel snapshots the solution on the device in
        the functions' order; new functions read it -- one DMA into a pinned buffer for all
        of them -- when the first ``x.array`` is used, so later solves never change them
        (``HydraulicNetworkAssembler.solution_functions``). Given ``functions`` are filled
        at once."""
        if self._closed:
            raise RuntimeError("the solver has been destroyed")
        h = self.assembler.handle
        if self.assembler.preconditioned != self._pc:
            self.assembler.set_preconditioner(self._pc)
        if self.assembler.preconditioned and h.pc_exact() != self._pc_exact:
            h.set_pc_exact(self._pc_exact)
        self.assembler.set_direct(self._direct and (self.assembler.preconditioned
                                                    or self.assembler.fe_direct_available))
        ce = self._check_every or (4 if self.assembler.preconditioned else 32)
        it, relres, conv = h.solve(self._rtol, self._maxit, ce)
        self._ksp.iterations, self._ksp.residual_estimate, self._ksp.converged = it, relres, conv
        used = "direct" if h.solver()[1] == 1 else "minres"
        self._ksp.solver_used = used
        if self._monitor:
            what = ("direct tree solve, true residual" if used == "direct"
                    else f"MINRES: {it} iterations, residual estimate")
            print(f"  {what} {relres:.3e} ({'converged' if conv else 'NOT converged'})",
                  file=sys.stdout)
        if not conv and self._raise:
            raise _lib.NxNotConverged(
                f"MINRES did not converge: {it} iterations, relative residual {relres:.3e} "
                f"> rtol {self._rtol:.1e}")
        return self.assembler.solution_functions(functions)

    def solution_vector(self) -> np.ndarray:
        """Device-layout solution (owned DoFs of this rank)."""
        return self.assembler.handle.solution()

    def true_residual(self) -> float:
        return self.assembler.handle.true_residual()

    def destroy(self) -> None:
        """Release what the solver owns (the reference destroys its KSP, b and x,
        ``solver.py:137-143``). The device matrix, rhs and Krylov vectors belong to the
        assembler's handle (shared by every solver of that assembler) and go with
        ``assembler.close()``; functions returned by :meth:`solve` stay valid."""
        self._closed = True
        self._ksp.destroy()
        self._A = None
        self._b = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
