"""The networkx-free graph core (graph_core.py + csrc/matching.cpp) against networkx itself.

The reference's decomposition (graph_manager.py:57-83) is pinned by the reference's own outputs
in test_graph_host.py (decomposition.json).  Here the pieces are compared with networkx 3.4.2 --
the library the reference calls -- where it is importable: the matching set returned (its
iteration order included: list(M) feeds subGraphs), is_perfect_matching, the edge view order
after removals / shuffled re-insertions, and gnp_random_graph's edges.  CPU only."""
import itertools
import random

import pytest

nx = pytest.importorskip("networkx")


@pytest.fixture(scope="module")
def gc(pkg):
    import importlib
    return importlib.import_module(pkg.__name__ + ".graph_core")


def _pair(edges, weights=None):
    G = nx.Graph()
    for k, (u, v) in enumerate(edges):
        if weights is None:
            G.add_edge(u, v)
        else:
            G.add_edge(u, v, weight=weights[k])
    return G


def _ours(gc, edges, weights=None):
    H = gc.OrderedGraph()
    H.add_edges_from(edges)
    if weights is not None:
        for (u, v), w in zip(edges, weights):
            H._adj[u][v]["weight"] = w
    return H


def _random_graphs():
    rng = random.Random(7)
    out = []
    for n in (2, 3, 5, 8, 9, 16, 17, 31, 64):
        for p in (0.1, 0.3, 0.6, 0.9):
            nodes = list(range(n))
            rng.shuffle(nodes)                    # node insertion order != id order
            pairs = [(a, b) for a, b in itertools.combinations(nodes, 2) if rng.random() < p]
            rng.shuffle(pairs)
            pairs = [(b, a) if rng.random() < 0.5 else (a, b) for a, b in pairs]
            out.append(pairs)
    out.append([(i, (i + 1) % 9) for i in range(9)])                      # odd cycle
    out.append(list(nx.petersen_graph().edges()))
    out.append(list(nx.complete_graph(7).edges()))
    out.append([(0, 1), (1, 2), (2, 0), (2, 3), (3, 4), (4, 5), (5, 3), (5, 6), (6, 7), (7, 8), (8, 6)])
    return [e for e in out if e]


@pytest.mark.parametrize("maxcard", [False, True])
@pytest.mark.parametrize("weighted", [False, True])
def test_max_weight_matching_equals_networkx(gc, maxcard, weighted):
    rng = random.Random(11)
    for edges in _random_graphs():
        w = [rng.randint(1, 9) for _ in edges] if weighted else None
        want = nx.max_weight_matching(_pair(edges, w), maxcardinality=maxcard)
        got = gc.max_weight_matching(_ours(gc, edges, w), maxcardinality=maxcard)
        assert list(got) == list(want), (edges, w)          # same set, same iteration order


def test_edges_view_and_perfect_matching_equal_networkx(gc):
    rng = random.Random(3)
    for edges in _random_graphs():
        G, H = _pair(edges), _ours(gc, edges)
        assert list(G.edges) == H.edges and list(G) == H.nodes()
        for _ in range(4):                                  # the getSubGraphs moves
            M = nx.max_weight_matching(G)
            assert gc.is_perfect_matching(H, M) == nx.is_perfect_matching(G, M)
            if rng.random() < 0.5:
                G.remove_edges_from(list(M))
                H.remove_edges_from(list(M))
            else:
                order = list(G.edges)
                rng.shuffle(order)
                G.remove_edges_from(order)
                G.add_edges_from(order)
                H.remove_edges_from(order)
                H.add_edges_from(order)
            assert list(G.edges) == H.edges and list(G) == H.nodes()
            assert [list(G.neighbors(v)) for v in G] == [list(H.neighbors(v)) for v in H]


@pytest.mark.parametrize("n,p,seed", [(64, 0.1, 1234), (32, 0.2, 7), (10, 0.5, 0), (5, 1.0, 1), (5, 0.0, 1)])
def test_gnp_random_graph_equals_networkx(gc, n, p, seed):
    assert gc.gnp_random_graph(n, p, seed) == list(nx.gnp_random_graph(n, p, seed=seed).edges())


def test_matching_abi_rejects_bad_input(pkg):
    import ctypes
    import numpy as np
    off = np.array([0, 1, 2], np.int64)
    adj = np.array([1, 5], np.int32)                        # neighbour 5 of a 2-node graph
    mate = np.empty(2, np.int32)
    order = np.empty(2, np.int32)
    cnt = ctypes.c_int(0)
    assert pkg.lib.mx_max_weight_matching(2, off.ctypes.data, adj.ctypes.data, None, 0, mate.ctypes.data,
                                          order.ctypes.data, ctypes.byref(cnt)) != 0
