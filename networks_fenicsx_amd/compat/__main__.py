"""``python -m networks_fenicsx_amd.compat script.py [args]``: run a networks_fenicsx
script with the stand-in ``dolfinx`` / ``ufl`` / ``mpi4py`` / ``networks_fenicsx``."""

from __future__ import annotations

import os
import runpy
import sys

from networks_fenicsx_amd.compat import install


def _init_distributed() -> None:
    """Under ``torch.distributed.run`` (WORLD_SIZE > 1) the demos' ``MPI.COMM_WORLD`` is
    the torch.distributed world: gloo for host messages, one GPU per local rank (RCCL
    inside the library). torch is imported before libnxhip.so is loaded."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group("gloo")
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))


def main() -> int:
    if len(sys.argv) < 2:
        print(__doc__, file=sys.stderr)
        return 2
    _init_distributed()
    install()
    script = sys.argv[1]
    sys.argv = sys.argv[1:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
