"""Every ``<reference file>.py:N[-M]`` citation in the code, the C header, the oracle and the
design documents must point inside the cited reference file, and the boundary citations
must point at the code they name ("citation drift").

Reads ``/root/reference`` when present (the build container); skipped elsewhere."""

from __future__ import annotations

import re
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")

pytestmark = pytest.mark.skipif(not (REF / "src" / "networks_fenicsx").is_dir(),
                                reason="reference checkout not present")

REF_FILES = {
    "assembly.py": "src/networks_fenicsx/assembly.py",
    "mesh.py": "src/networks_fenicsx/mesh.py",
    "solver.py": "src/networks_fenicsx/solver.py",
    "network_generation.py": "src/networks_fenicsx/network_generation.py",
    "post_processing.py": "src/networks_fenicsx/post_processing.py",
    "__init__.py": "src/networks_fenicsx/__init__.py",
    "demo_Y_bifurcation.py": "demos/demo_Y_bifurcation.py",
    "demo_double_Y_bifurcation.py": "demos/demo_double_Y_bifurcation.py",
    "demo_arterial_tree.py": "demos/demo_arterial_tree.py",
    "demo_tree.py": "demos/demo_tree.py",
    "demo_perf.py": "demos/demo_perf.py",
    "test_edge_info.py": "tests/test_edge_info.py",
    "test_make_tree.py": "tests/test_make_tree.py",
    "test_orientation.py": "tests/test_orientation.py",
}

SCANNED = ["include", "networks_fenicsx_amd", "oracle", "tests", "bench.py", "__graft_entry__.py",
           "DESIGN.md", "INTEGRATION.md", "README.md"]
SUFFIXES = {".py", ".h", ".hip", ".c", ".md"}

CITE = re.compile(
    r"(?P<path>[A-Za-z0-9_/]*?)(?P<file>" + "|".join(re.escape(f) for f in REF_FILES) +
    r"):(?P<nums>\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")

# citation -> text that must appear in the cited lines (the boundary and the forms)
ANCHORS = [
    ("mesh.py", 29, 42, "def color_graph"),
    ("mesh.py", 45, 538, "class NetworkMesh"),
    ("mesh.py", 175, 225, "bifurcation_values"),
    ("mesh.py", 269, 322, "internal_line_coords"),
    ("mesh.py", 365, 400, "orientation"),
    ("mesh.py", 402, 420, "_in_marker"),
    ("solver.py", 32, 73, "def __init__"),
    ("solver.py", 58, 65, "mumps"),
    ("solver.py", 90, 101, "def assemble"),
    ("solver.py", 107, 135, "def solve"),
    ("solver.py", 127, 127, "ksp.solve"),
    ("solver.py", 137, 143, "def __del__"),
    ("assembly.py", 28, 92, "def compute_integration_data"),
    ("assembly.py", 121, 146, "pressure_degree"),
    ("assembly.py", 253, 253, "R * qs[i] * vs[i]"),
    ("assembly.py", 254, 254, "ufl.grad(qs[i])"),
    ("assembly.py", 255, 255, "-p * ufl.dot(ufl.grad(vs[i])"),
    ("assembly.py", 258, 260, "p_bc * vs[i]"),
    ("assembly.py", 268, 277, "mu * qs[color]"),
    ("assembly.py", 328, 368, "def assemble"),
    ("assembly.py", 378, 383, "def bilinear_form"),
    ("assembly.py", 393, 398, "def linear_form"),
    ("post_processing.py", 19, 52, "def extract_global_flux"),
    ("network_generation.py", 41, 42, "def make_tree"),
    ("network_generation.py", 157, 158, "def make_arterial_tree"),
]


def _lines(name: str) -> list[str]:
    return (REF / REF_FILES[name]).read_text().splitlines()


def _sources():
    for entry in SCANNED:
        p = REPO / entry
        files = [p] if p.is_file() else sorted(q for q in p.rglob("*") if q.suffix in SUFFIXES)
        for f in files:
            if "__pycache__" in f.parts or f.name == "test_citations.py":
                continue
            yield f


def _citations():
    for f in _sources():
        for ln, line in enumerate(f.read_text(errors="replace").splitlines(), 1):
            for m in CITE.finditer(line):
                if "networks_fenicsx_amd" in m.group("path") or "csrc" in m.group("path"):
                    continue  # a citation of this repository's own file
                if m.group("path") and not m.group("path").rstrip("/").endswith(
                        ("networks_fenicsx", "demos", "tests", "src")):
                    continue
                for part in re.split(r",\s?", m.group("nums")):
                    a, _, b = part.partition("-")
                    yield f.relative_to(REPO), ln, m.group("file"), int(a), int(b or a)


def test_citations_found():
    assert sum(1 for _ in _citations()) > 100


def test_every_citation_inside_the_cited_file():
    bad = []
    for where, ln, name, a, b in _citations():
        n = len(_lines(name))
        if not (1 <= a <= b <= n):
            bad.append(f"{where}:{ln}: {name}:{a}-{b} (file has {n} lines)")
    assert not bad, "dangling reference citations:\n" + "\n".join(bad)


@pytest.mark.parametrize("name,a,b,text", ANCHORS)
def test_anchor_lines_hold_the_named_code(name, a, b, text):
    assert text in "\n".join(_lines(name)[a - 1:b]), (name, a, b, text)


def test_cited_ranges_match_the_anchors():
    """A citation whose range overlaps an anchor's code must not be shifted off it: every
    cited range naming one of the anchored mesh/solver items starts within the anchor."""
    anchored = {(n, a, b) for n, a, b, _ in ANCHORS}
    stale = {("mesh.py", 54, 67), ("mesh.py", 200, 250), ("mesh.py", 295, 347),
             ("mesh.py", 390, 425), ("mesh.py", 427, 445), ("solver.py", 456, 463),
             ("solver.py", 488, 499), ("solver.py", 505, 533), ("solver.py", 441, 447)}
    found = [(str(w), ln, n, a, b) for w, ln, n, a, b in _citations() if (n, a, b) in stale]
    assert not found, found
    assert anchored  # the anchors themselves are checked above
