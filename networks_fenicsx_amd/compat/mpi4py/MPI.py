"""``mpi4py.MPI`` subset: ``COMM_WORLD`` and the reduction ops.

``COMM_WORLD`` is the host control plane of :mod:`networks_fenicsx_amd.comm`: this
process alone, or the initialised ``torch.distributed`` world when the script runs under
``torch.distributed.run`` (one process per GPU). Its ``allreduce(value, op=MAX)`` etc.
accept the ops below.
"""

from __future__ import annotations

from networks_fenicsx_amd.comm import SerialComm, as_comm


class Op:
    def __init__(self, name: str):
        self.name = name

    def __repr__(self) -> str:
        return f"<mpi4py.MPI.Op {self.name}>"


SUM = Op("MPI_SUM")
MAX = Op("MPI_MAX")
MIN = Op("MPI_MIN")

COMM_WORLD = as_comm(None)
COMM_SELF = SerialComm()
