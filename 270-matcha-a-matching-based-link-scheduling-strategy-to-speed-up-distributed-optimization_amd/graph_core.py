"""The graph machinery the reference's decomposition uses, without networkx.

graph_manager.py:51-83 builds an nx.Graph from the subgraph edge lists, peels perfect matchings
with nx.max_weight_matching / nx.is_perfect_matching, re-inserts the edge list in a shuffled order
when a matching is not perfect, and hands list(G.edges) to the greedy decomposition.  Which
matchings come out depends on networkx's visiting orders (node insertion order, each node's
adjacency insertion order, the order G.edges walks them, the order the returned matching set
iterates in), so this module keeps exactly those:

  OrderedGraph           the adjacency-dict semantics of nx.Graph (add_edges_from,
                         remove_edges_from, nodes, neighbors, edges, has_edge)
  max_weight_matching    the blossom algorithm networkx 3.4.2 runs, native (csrc/matching.cpp,
                         mx_max_weight_matching), returned as the same set, same iteration order
  is_perfect_matching    networkx's check
  gnp_random_graph       nx.gnp_random_graph's edge draw (random.Random(seed), one draw per pair
                         in itertools.combinations order) for the ER topologies of BASELINE config 5

Pinned by tests/golden/decomposition.json (the reference's own decomposition for graphs 0-5 and
a 64-node ER graph over three Python `random` seeds) and, where networkx happens to be installed,
against networkx itself on random graphs (tests/test_graph_core.py).
"""
import ctypes
import itertools
import random

import numpy as np

from ._lib import check, lib


class OrderedGraph:
    """nx.Graph's storage: node -> {neighbour -> edge data}, both in insertion order."""

    def __init__(self, edges=None):
        self._adj = {}
        if edges is not None:
            self.add_edges_from(edges)

    def add_edges_from(self, ebunch):
        adj = self._adj
        for e in ebunch:
            u, v = e[0], e[1]
            if u not in adj:
                adj[u] = {}
            if v not in adj:
                adj[v] = {}
            data = adj[u].get(v, {})
            adj[u][v] = data
            adj[v][u] = data

    def remove_edges_from(self, ebunch):
        adj = self._adj
        for e in ebunch:
            u, v = e[0], e[1]
            if u in adj and v in adj[u]:
                del adj[u][v]
                if u != v:
                    del adj[v][u]

    def __iter__(self):
        return iter(self._adj)

    def __len__(self):
        return len(self._adj)

    def __contains__(self, n):
        return n in self._adj

    def nodes(self):
        return list(self._adj)

    def neighbors(self, n):
        return iter(self._adj[n])

    def has_edge(self, u, v):
        return u in self._adj and v in self._adj[u]

    @property
    def edges(self):
        """nx's EdgeView order: per node in insertion order, its neighbours not yet visited."""
        seen = set()
        out = []
        for n, nbrs in self._adj.items():
            for nbr in nbrs:
                if nbr not in seen:
                    out.append((n, nbr))
            seen.add(n)
        return out

    def weight(self, u, v, key="weight"):
        return self._adj[u][v].get(key, 1)


def max_weight_matching(G, maxcardinality=False, weight="weight"):
    """nx.max_weight_matching(G) (integer weights, default 1), as the set networkx returns."""
    nodes = G.nodes()
    if not nodes:
        return set()
    index = {v: i for i, v in enumerate(nodes)}
    off = np.zeros(len(nodes) + 1, np.int64)
    adj, wts = [], []
    for i, v in enumerate(nodes):
        for w in G.neighbors(v):
            adj.append(index[w])
            wt = G.weight(v, w, weight)
            if int(wt) != wt:
                raise TypeError("max_weight_matching: integer edge weights only")
            wts.append(int(wt))
        off[i + 1] = len(adj)
    adj = np.asarray(adj if adj else [0], np.int32)
    wts = np.asarray(wts if wts else [1], np.int64)
    mate = np.empty(len(nodes), np.int32)
    order = np.empty(len(nodes), np.int32)
    cnt = ctypes.c_int(0)
    check(lib.mx_max_weight_matching(len(nodes), off.ctypes.data, adj.ctypes.data, wts.ctypes.data,
                                     int(bool(maxcardinality)), mate.ctypes.data, order.ctypes.data,
                                     ctypes.byref(cnt)), "mx_max_weight_matching")
    # networkx's mate dict in its insertion order, then matching_dict_to_set over it
    mate_dict = {nodes[int(k)]: nodes[int(mate[k])] for k in order[:cnt.value]}
    edges = set()
    for u, v in mate_dict.items():
        if (v, u) in edges or (u, v) in edges:
            continue
        edges.add((u, v))
    return edges


def is_perfect_matching(G, matching):
    """nx.is_perfect_matching for a set of 2-tuples."""
    seen = set()
    for u, v in matching:
        if u not in G or v not in G:
            raise ValueError(f"matching contains edge {(u, v)} with node not in G")
        if u == v or not G.has_edge(u, v):
            return False
        if u in seen or v in seen:
            return False
        seen.update((u, v))
    return len(seen) == len(G)


def gnp_random_graph(n, p, seed):
    """nx.gnp_random_graph(n, p, seed) edges: random.Random(seed), one random() per pair of
    itertools.combinations(range(n), 2), edge kept if < p (p >= 1: complete; p <= 0: none)."""
    if p >= 1:
        return list(itertools.combinations(range(n), 2))
    if p <= 0:
        return []
    rng = random.Random(seed)
    return [e for e in itertools.combinations(range(n), 2) if rng.random() < p]
