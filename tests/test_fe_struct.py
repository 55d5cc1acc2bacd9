"""The (k, 0) structured assembly's closed form (CPU; nx_fe_struct_degree, no device).

fe_s_terms gives every CSR entry and rhs row of a (k, 0) layout from (row, col) alone.
nx_create_fe builds its edge templates (k_fe_tasm, k_fe_tres) only after
nx_fe_struct_degree has found every entry's term list -- (index, table entry), in summation
order -- equal to the gather tables layout_fe builds, so the template kernels add the same
terms in the same order as k_assemble_fe (the CSR stays bit-exact against
layout_fe.evaluate_terms, tests/test_gpu_fe.py). Here: the check
accepts every (k, 0) layout of the test graphs, rejects continuous pressure and any table
that differs in one term."""

from __future__ import annotations

import numpy as np
import pytest

from cases import CASES
from networks_fenicsx_amd import NetworkMesh, _lib
from networks_fenicsx_amd.layout_fe import build_fe_layout


def _layout(case, k, m):
    make, N, strategy, _ = CASES[case]
    N = min(N, 12)
    mesh = NetworkMesh(make(), N=N, color_strategy=strategy)
    src, dst = mesh.edges
    return build_fe_layout(mesh.node_coordinates, src, dst, mesh.degrees, N, k, m)


@pytest.mark.parametrize("case", ["Y_N4", "double_Y_N5", "tree5_N15", "arterial5_N40",
                                  "edge_info_N10"])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_struct_degree_accepts_k0_layouts(case, k):
    assert _lib.fe_struct_degree(_layout(case, k, 0)) == k


@pytest.mark.parametrize("k,m", [(2, 1), (3, 1), (3, 2)])
def test_struct_degree_rejects_continuous_pressure(k, m):
    assert _lib.fe_struct_degree(_layout("tree5_N15", k, m)) == 0


def test_struct_degree_rejects_a_changed_term():
    lay = _layout("tree5_N15", 2, 0)
    assert _lib.fe_struct_degree(lay) == 2
    lay.a_ent = lay.a_ent.copy()
    lay.a_ent[len(lay.a_ent) // 2] ^= 1  # one term's table entry
    assert _lib.fe_struct_degree(lay) == 0
    lay = _layout("tree5_N15", 2, 0)
    lay.b_idx = lay.b_idx.copy()
    lay.b_idx[-1] += 1  # one rhs term's index
    assert _lib.fe_struct_degree(lay) == 0
