"""``python -m networks_fenicsx_amd.compat script.py [args]``: run a networks_fenicsx
script with the stand-in ``dolfinx`` / ``ufl`` / ``mpi4py`` / ``networks_fenicsx``."""

from __future__ import annotations

import runpy
import sys

from networks_fenicsx_amd.compat import install


def main() -> int:
    if len(sys.argv) < 2:
        print(__doc__, file=sys.stderr)
        return 2
    install()
    script = sys.argv[1]
    sys.argv = sys.argv[1:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
