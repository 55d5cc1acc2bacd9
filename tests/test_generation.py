"""Graph generators vs. the reference's own outputs (tests/golden/graphs.npz)."""

import numpy as np
import pytest

from networks_fenicsx_amd import network_generation as ng

TREES = {
    "Y": (2, 1, 3, 3),
    "demo_tree": (2, 1, 1, 3),
    "double_Y": (2, 3.1, 7.3, 3),
    "depth6": (7, 7, 7, 3),
    "tree5_2d": (5, 2, 1, 2),
    "depth11": (12, 12, 12, 3),
}


def _arrays(G):
    pos = np.asarray([G.nodes[v]["pos"] for v in G.nodes()], dtype=np.float64)
    edges = np.asarray(list(G.edges()), dtype=np.int64).reshape(-1, 2)
    return pos, edges


@pytest.mark.parametrize("name", sorted(TREES))
def test_make_tree_bit_exact(graphs, name):
    n, H, W, dim = TREES[name]
    pos, edges = _arrays(ng.make_tree(n, H, W, dim=dim))
    np.testing.assert_array_equal(pos, graphs[f"{name}/pos"])
    np.testing.assert_array_equal(edges, graphs[f"{name}/edges"])


@pytest.mark.parametrize("name,kw", [("arterial5", dict(N=5, direction=np.array([0.1, 1, 0]))),
                                     ("arterial7", dict(N=7))])
def test_arterial_tree_bit_exact(graphs, name, kw):
    G = ng.make_arterial_tree(**kw)
    pos, edges = _arrays(G)
    np.testing.assert_array_equal(pos, graphs[f"{name}/pos"])
    np.testing.assert_array_equal(edges, graphs[f"{name}/edges"])
    radius = np.asarray([G.edges[e]["radius"] for e in G.edges()])
    np.testing.assert_array_equal(radius, graphs[f"{name}/radius"])


def test_arterial_random_seeded(graphs):
    np.random.seed(1234)
    G = ng.make_arterial_tree(6, random=True)
    pos, edges = _arrays(G)
    np.testing.assert_array_equal(pos, graphs["arterial6_random_seed1234/pos"])
    np.testing.assert_array_equal(edges, graphs["arterial6_random_seed1234/edges"])


def test_arterial_gamma_error():
    with pytest.raises(ValueError):
        ng.make_arterial_tree(3, gamma=1.5)


@pytest.mark.parametrize("n", [1, 2, 5, 9])
def test_tree_arrays_structure(n):
    if n == 1:  # the reference divides by zero for a single generation
        with pytest.raises(ZeroDivisionError):
            ng.tree_arrays(1, 1, 1)
        return
    pos, src, dst = ng.tree_arrays(n, 1.0, 1.0)
    assert src.size == 2**n - 1 and pos.shape == (2**n, 3)
    assert src[0] == 0 and dst[0] == 1
    np.testing.assert_array_equal(src[1:], dst[1:] // 2)
    # generations sorted by x within each level
    for g in range(1, n):
        lvl = pos[2**g : 2 ** (g + 1), 0]
        assert np.all(np.diff(lvl) > 0)
