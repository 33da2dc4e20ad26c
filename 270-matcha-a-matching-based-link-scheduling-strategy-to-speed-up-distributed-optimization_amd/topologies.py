"""Base topologies of the reference (util.py:275-342, `select_graph`) -- data, not code paths.

Each graph is a list of matchings (edge lists); pass it to FixedProcessor / MatchaProcessor
with issubgraph=True to use the matchings as given, or issubgraph=False to re-decompose.
"""
from .graph_core import gnp_random_graph

_GRAPHS = [
    # graph 0: 8-node Erdos-Renyi graph, Fig. 1(a) of the MATCHA paper
    [[(1, 5), (6, 7), (0, 4), (2, 3)], [(1, 7), (3, 6)], [(1, 0), (3, 7), (5, 6)], [(1, 2), (7, 0)],
     [(3, 1)]],
    # graph 1: 16-node geometric graph, Fig. A.3(a)
    [[(4, 8), (6, 11), (7, 13), (0, 12), (5, 14), (10, 15), (2, 3), (1, 9)],
     [(11, 13), (14, 2), (5, 6), (15, 3), (10, 9)], [(11, 8), (2, 5), (13, 4), (14, 3), (0, 10)],
     [(11, 5), (15, 14), (13, 8)], [(2, 11)]],
    # graph 2: 16-node geometric graph, Fig. A.3(b)
    [[(2, 7), (12, 15), (3, 13), (5, 6), (8, 0), (9, 4), (11, 14), (1, 10)],
     [(8, 6), (0, 11), (3, 2), (5, 4), (15, 14), (1, 9)], [(8, 3), (0, 6), (11, 2), (4, 1), (12, 14)],
     [(8, 11), (6, 3), (0, 5)], [(8, 2), (0, 3), (6, 7), (11, 12)], [(8, 5), (6, 4), (0, 2), (11, 7)],
     [(8, 15), (3, 7), (0, 4), (6, 2)], [(8, 14), (5, 3), (11, 6), (0, 9)],
     [(8, 7), (15, 11), (2, 5), (4, 3), (1, 0), (13, 6)], [(12, 8)]],
    # graph 3: 16-node geometric graph, Fig. A.3(c)
    [[(3, 12), (4, 8), (1, 13), (5, 7), (9, 10), (11, 14), (6, 15), (0, 2)],
     [(7, 14), (2, 6), (5, 13), (8, 10), (1, 15), (0, 11), (3, 9), (4, 12)],
     [(2, 7), (3, 15), (9, 13), (6, 11), (4, 14), (10, 12), (1, 8), (0, 5)],
     [(5, 14), (1, 12), (13, 8), (9, 4), (2, 11), (7, 0)], [(5, 1), (14, 8), (13, 12), (10, 4), (6, 7)],
     [(5, 9), (14, 1), (13, 3), (8, 2), (11, 7)], [(5, 12), (14, 13), (1, 9), (8, 0)],
     [(5, 2), (14, 10), (1, 3), (9, 8), (13, 15)], [(5, 8), (14, 12), (1, 4), (13, 10)],
     [(5, 3), (14, 2), (9, 12), (1, 10), (13, 4)], [(5, 6), (14, 0), (8, 12), (1, 2)], [(5, 15), (9, 14)],
     [(11, 5)]],
    # graph 4: 16-node Erdos-Renyi graph, Fig. 3(b)
    [[(2, 7), (3, 15), (13, 14), (8, 9), (1, 5), (0, 10), (6, 12), (4, 11)],
     [(12, 11), (5, 6), (14, 1), (9, 10), (15, 2), (8, 13)], [(12, 5), (11, 6), (1, 8), (9, 3), (2, 10)],
     [(12, 14), (11, 9), (5, 15), (0, 6), (1, 7)], [(12, 8), (5, 2), (11, 14), (1, 6)],
     [(12, 15), (13, 11), (10, 5), (3, 14)], [(12, 9)], [(0, 12)]],
    # graph 5: 8-node ring
    [[(0, 1), (2, 3), (4, 5), (6, 7)], [(0, 7), (2, 1), (4, 3), (6, 5)]],
]

GRAPH_SIZES = [8, 16, 16, 16, 16, 8]


def select_graph(graphid):
    """util.py:275-342."""
    return [list(m) for m in _GRAPHS[graphid]]


def erdos_renyi(n, p, seed):
    """A base graph given as one edge list (decompose with issubgraph=False): the edges of
    nx.gnp_random_graph(n, p, seed) (graph_core.gnp_random_graph, no networkx), sorted."""
    return [sorted(tuple(sorted(e)) for e in gnp_random_graph(n, p, seed))]
