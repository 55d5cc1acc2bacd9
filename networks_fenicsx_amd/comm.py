"""Minimal communicator used by the host-side classes.

The reference passes an ``mpi4py`` communicator around (``mesh.py:89, 113-115``) and uses
``bcast``/``barrier``/``allreduce`` on it (``mesh.py:227-250``,
``demos/demo_tree.py:64-71``). There is no MPI here: one process per GPU is
launched by ``torch.distributed.run`` and host-side control messages go over
``torch.distributed`` (gloo for objects). The device data path (Krylov dot
products and the cut-vertex halo) does NOT go through this object -- it uses
RCCL directly inside the HIP library (see ``csrc/nxhip.hip``).
"""

from __future__ import annotations

import operator
from typing import Any

__all__ = ["Comm", "SerialComm", "TorchComm", "LocalGroup", "GroupRankComm", "COMM_WORLD",
           "SUM", "MAX", "MIN"]

SUM = "sum"
MAX = "max"
MIN = "min"

_PY_OPS = {SUM: operator.add, MAX: max, MIN: min}


def _op_name(op: Any) -> str:
    if op is None:
        return SUM
    if isinstance(op, str):
        return op.lower()
    # mpi4py-like op objects (e.g. the demo shim's MPI.MAX) carry a name
    name = getattr(op, "name", None) or getattr(op, "__name__", None) or str(op)
    name = str(name).lower()
    for k in (SUM, MAX, MIN):
        if k in name:
            return k
    raise ValueError(f"unsupported reduction op {op!r}")


class Comm:
    rank: int = 0
    size: int = 1

    def bcast(self, obj: Any, root: int = 0) -> Any:  # pragma: no cover - interface
        raise NotImplementedError

    def allreduce(self, value: Any, op: Any = None) -> Any:  # pragma: no cover
        raise NotImplementedError

    def barrier(self) -> None:  # pragma: no cover
        raise NotImplementedError

    def allgather(self, obj: Any) -> list:  # pragma: no cover
        raise NotImplementedError


class SerialComm(Comm):
    """Single-process communicator (the ``mpiexec -n 1`` case)."""

    rank = 0
    size = 1

    def bcast(self, obj: Any, root: int = 0) -> Any:
        return obj

    def allreduce(self, value: Any, op: Any = None) -> Any:
        _op_name(op)  # validate
        return value

    def barrier(self) -> None:
        return None

    def allgather(self, obj: Any) -> list:
        return [obj]

    # mpi4py spellings used by demo code
    Get_rank = lambda self: self.rank  # noqa: E731
    Get_size = lambda self: self.size  # noqa: E731


class TorchComm(Comm):
    """Host-side messages over an initialised ``torch.distributed`` process group."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self._dist = dist
        self._group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)

    def bcast(self, obj: Any, root: int = 0) -> Any:
        box = [obj if self.rank == root else None]
        self._dist.broadcast_object_list(box, src=root, group=self._group)
        return box[0]

    def allgather(self, obj: Any) -> list:
        out: list = [None] * self.size
        self._dist.all_gather_object(out, obj, group=self._group)
        return out

    def allreduce(self, value: Any, op: Any = None) -> Any:
        fn = _PY_OPS[_op_name(op)]
        vals = self.allgather(value)
        acc = vals[0]
        for v in vals[1:]:
            acc = fn(acc, v)
        return acc

    def barrier(self) -> None:
        self._dist.barrier(group=self._group)

    Get_rank = lambda self: self.rank  # noqa: E731
    Get_size = lambda self: self.size  # noqa: E731


class LocalGroup:
    """Ranks of a partitioned problem simulated inside ONE process on one device (the
    in-process group transport of the HIP library, ``nx_group_create``). The host objects
    of every rank are built one after the other, rank 0 first, from one thread."""

    def __init__(self, size: int):
        if size < 1:
            raise ValueError("group size must be >= 1")
        self.size = int(size)
        self._store: dict[int, Any] = {}

    def comm(self, rank: int) -> "GroupRankComm":
        return GroupRankComm(self, rank)


class GroupRankComm(Comm):
    """Communicator of one rank of a :class:`LocalGroup`. ``bcast`` works when the root
    rank's call comes first (rank-order construction); collectives that need every rank's
    value at once cannot run from one thread and raise."""

    def __init__(self, group: LocalGroup, rank: int):
        if not 0 <= rank < group.size:
            raise ValueError(f"rank {rank} outside group of {group.size}")
        self.group = group
        self.rank = int(rank)
        self.size = group.size
        self._calls = 0

    def bcast(self, obj: Any, root: int = 0) -> Any:
        k = self._calls
        self._calls += 1
        if self.rank == root:
            self.group._store[k] = obj
            return obj
        if k not in self.group._store:
            raise RuntimeError("in-process group: build the root rank's objects first")
        return self.group._store[k]

    def allreduce(self, value: Any, op: Any = None) -> Any:
        raise NotImplementedError("in-process group ranks run one after the other; "
                                  "reduce over the ranks' results on the host instead")

    def allgather(self, obj: Any) -> list:
        raise NotImplementedError("in-process group: gather the ranks' results on the host")

    def barrier(self) -> None:
        return None

    Get_rank = lambda self: self.rank  # noqa: E731
    Get_size = lambda self: self.size  # noqa: E731


def as_comm(comm: Any) -> Comm:
    """Normalise ``None`` / a :class:`Comm` / a torch process group to a :class:`Comm`."""
    if comm is None:
        # Only consult torch.distributed if the caller already imported torch: the
        # package itself never imports torch (one HIP runtime per process -- the one
        # libnxhip.so is linked against -- unless the caller loads torch first).
        import sys

        dist = sys.modules.get("torch.distributed")
        if dist is not None and dist.is_available() and dist.is_initialized() \
                and dist.get_world_size() > 1:
            return TorchComm()
        return SerialComm()
    if isinstance(comm, Comm):
        return comm
    if hasattr(comm, "bcast") and hasattr(comm, "allreduce"):
        return comm  # duck-typed (e.g. a demo shim comm)
    return TorchComm(comm)


COMM_WORLD = SerialComm()
