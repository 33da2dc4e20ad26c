"""Drop-in schedule processors: GraphProcessor / FixedProcessor / MatchaProcessor.

Same class names, constructor signature and attributes as the reference's graph_manager.py
(graph_manager.py:15-309) so train_mpi.py:72-75 and README.md:31-37 work unchanged:

    GP = MatchaProcessor(subGraphs, budget, rank, size, iterations, issubgraph)
    GP.subGraphs, GP.L_matrices, GP.neighbors_info, GP.probabilities, GP.neighbor_weight,
    GP.active_flags  (list of iterations+1 rows, one 0/1 entry per matching)

Host side (as in the reference): matching decomposition (max_weight_matching plus the greedy
colouring), Laplacians, partner table, FixedProcessor's closed-form alpha and the MATCHA
probability / alpha solves (solver.py; cvxpy/CVXOPT are absent).  No networkx: the graph and the
blossom matching are restated in graph_core.py / csrc/matching.cpp with networkx 3.4.2's visiting
orders, so the decomposition is the reference's (pinned by tests/golden/decomposition.json).

GPU side: the per-iteration Bernoulli flags.  They are drawn on the MI355X from numpy's
global MT19937 state (mx_flags_binomial), bit-exact with np.random.binomial, and numpy's
global state is advanced exactly as the reference's draws would advance it.  The flag table
stays resident in HBM (``flags_dev``, uint8 [iterations+1][M]) for the gossip engine; the host
list ``active_flags`` is a copy for the reference API.
"""
import collections
import ctypes
import random
import sys

import numpy as np

from . import solver
from .graph_core import OrderedGraph, is_perfect_matching, max_weight_matching
from ._lib import check, lib, require_device, stream_ptr


class GraphProcessor(object):
    """graph_manager.py:15-180 -- decomposition, Laplacians and the partner table."""

    def __init__(self, base_graph, commBudget, rank, size, iterations, issubgraph):
        self.rank = rank
        self.size = size
        self.comm = None            # the reference holds MPI.COMM_WORLD here; unused by it
        self.commBudget = commBudget
        if issubgraph:
            self.base_graph = self.getGraphFromSub(base_graph)
            self.subGraphs = base_graph
        else:
            self.base_graph = self.getGraphFromSub(base_graph)
            self.subGraphs = self.getSubGraphs()
        self.L_matrices = self.graphToLaplacian()
        self.neighbors_info = self.drawer()

    # the reference's base class `raise NotImplemented` (a TypeError); subclasses override
    def getProbability(self):
        raise NotImplementedError

    def getAlpha(self):
        raise NotImplementedError

    def set_flags(self, iterations):
        raise NotImplementedError

    def getGraphFromSub(self, subGraphs):
        """graph_manager.py:51-55: union of the edge lists (nx.Graph's insertion-ordered
        adjacency, graph_core.OrderedGraph)."""
        G = OrderedGraph()
        for edges in subGraphs:
            G.add_edges_from(edges)
        return G

    def getSubGraphs(self):
        """graph_manager.py:57-83.  Peel perfect matchings with max_weight_matching for up to
        size-1 rounds (re-ordering the edge list with Python's global `random` when the matching
        is not perfect, which changes the blossom search's tie-breaking), then colour the rest
        greedily.  Mutates self.base_graph exactly as the reference does."""
        G = self.base_graph
        found = []
        for _ in range(self.size - 1):
            matching = max_weight_matching(G)
            if is_perfect_matching(G, matching):
                G.remove_edges_from(list(matching))
                found.append(list(matching))
            else:
                order = list(G.edges)
                random.shuffle(order)
                G.remove_edges_from(order)
                G.add_edges_from(order)
        return found + self.decomposition(list(G.edges))

    def graphToLaplacian(self):
        """graph_manager.py:86-93: one dense n x n Laplacian per matching over nodes range(size).
        (nx.laplacian_matrix over nodelist range(size); built directly -- networkx>=3 would reject
        nodes missing from a matching, networkx 2.x returned zero rows for them, as here.)"""
        out = []
        for edges in self.subGraphs:
            L = np.zeros((self.size, self.size), dtype=np.int64)
            seen = set()
            for a, b in edges:
                a, b = int(a), int(b)
                key = (min(a, b), max(a, b))
                if a == b or key in seen:     # a Graph collapses duplicates; self loops cancel
                    continue
                seen.add(key)
                L[a, a] += 1
                L[b, b] += 1
                L[a, b] -= 1
                L[b, a] -= 1
            out.append(L)
        return out

    def decomposition(self, graph):
        """graph_manager.py:95-154: greedy edge colouring of the remainder into matchings.

        Nodes are visited in descending current degree (a stable ascending sort, then reversed,
        re-done after every colour); each visited node still free in this colour takes the first
        later-visited free neighbour.  Colours repeat until no edge is left."""
        n = self.size
        order = [[v, 0] for v in range(n)]                  # [node, remaining degree]
        adj = [[] for _ in range(n)]
        remaining = collections.defaultdict(int)
        pending = set()
        for a, b in graph:
            order[a][1] += 1
            order[b][1] += 1
            if a in adj[b] or b in adj[a]:
                print("Invalid input graph! Double edge! (" + str(a) + ", " + str(b) + ")")
                sys.exit()
            if a == b:
                print("Invalid input graph! Circle! (" + str(a) + ", " + str(b) + ")")
                sys.exit()
            adj[a].append(b)
            adj[b].append(a)
            remaining[a] += 1
            remaining[b] += 1
            pending.update((a, b))

        def by_degree_desc(rows):
            rows = sorted(rows, key=lambda r: r[1])
            rows.reverse()
            return rows

        order = by_degree_desc(order)
        colours = []
        while pending:
            colour = []
            for i in range(n):
                u = order[i][0]
                if u not in pending:
                    continue
                for j in range(i + 1, n):
                    w = order[j][0]
                    if w in pending and w in adj[u]:
                        colour.append((u, w))
                        order[i][1] -= 1
                        order[j][1] -= 1
                        remaining[u] -= 1
                        remaining[w] -= 1
                        adj[u].remove(w)
                        adj[w].remove(u)
                        pending.discard(u)
                        pending.discard(w)
                        break
            colours.append(colour)
            pending.update(v for v, d in remaining.items() if d > 0)
            order = by_degree_desc(order)
        return colours

    def drawer(self):
        """graph_manager.py:157-180: neighbors_info[g][i] = partner of i in matching g, or -1.
        A subgraph that is not a matching prints the reference's message and exits, as it does."""
        table = []
        for number, edges in enumerate(self.subGraphs, start=1):
            row = [-1] * self.size
            for a, b in edges:
                if row[a] != -1 or row[b] != -1:
                    print("invalide graph! graph: " + str(number))
                    sys.exit()
                row[a] = b
                row[b] = a
            table.append(row)
        return table

    # -------------------------------------------------------------- GPU flag generation
    def _draw_flags_on_gpu(self, probs, iterations):
        """np.random.binomial(1, probs[m], iterations) for every m, matching-major, drawn on the
        GPU from numpy's global MT19937 state; returns the device table uint8 [iterations][M]
        and advances numpy's global state exactly as the reference's draws would."""
        import torch
        require_device()
        probs = np.ascontiguousarray(probs, dtype=np.float64)
        M = probs.shape[0]
        name, key, pos, has_gauss, gauss = np.random.get_state()
        assert name == "MT19937"
        key = np.ascontiguousarray(key, dtype=np.uint32)
        key_out = np.empty(624, dtype=np.uint32)
        pos_out = ctypes.c_int(0)
        flags = torch.empty((iterations, M), dtype=torch.uint8, device="cuda")
        check(lib.mx_flags_binomial(key.ctypes.data, int(pos), probs.ctypes.data, M, iterations,
                                    flags.data_ptr(), key_out.ctypes.data, ctypes.byref(pos_out),
                                    stream_ptr()), "mx_flags_binomial")
        np.random.set_state((name, key_out, pos_out.value, has_gauss, gauss))
        return flags


def _host_rows(flags_dev):
    """Reference container type: list of rows, each a list of numpy int64 scalars."""
    arr = flags_dev.cpu().numpy().astype(np.int64)
    return [list(r) for r in arr]


class FixedProcessor(GraphProcessor):
    """graph_manager.py:183-225 (D-PSGD schedule)."""

    def __init__(self, base_graph, commBudget, rank, size, iterations, issubgraph):
        super(FixedProcessor, self).__init__(base_graph, commBudget, rank, size, iterations, issubgraph)
        self.probabilities = self.getProbability()
        self.neighbor_weight = self.getAlpha()
        self.active_flags = self.set_flags(iterations + 1)

    def getProbability(self):
        return self.commBudget

    def getAlpha(self):
        """graph_manager.py:196-206: alpha = 2 / (lambda_2 + lambda_max) of the summed Laplacian."""
        L_base = np.zeros((self.size, self.size))
        for L in self.L_matrices:
            L_base += L
        w, _ = np.linalg.eig(L_base)
        lam = list(sorted(w))
        if len(w) > 1:
            alpha = 2 / (lam[1] + lam[-1])
        return alpha

    def set_flags(self, iterations):
        """graph_manager.py:208-225: `iterations` binomial draws are made and discarded (they only
        advance numpy's global RNG -- done on the GPU here), then the schedule alternates
        [0, 1] / [1, 0]: only matchings 0 and 1 are ever used."""
        import torch
        self._draw_flags_on_gpu(np.array([self.probabilities], dtype=np.float64), iterations)
        t = torch.arange(iterations, device="cuda")
        odd = (t % 2).to(torch.uint8)
        self.flags_dev = torch.stack([odd, 1 - odd], dim=1).contiguous()
        return [[0, 1] if i % 2 == 0 else [1, 0] for i in range(iterations)]


class MatchaProcessor(GraphProcessor):
    """graph_manager.py:228-309 (MATCHA: a random subset of matchings per iteration)."""

    def __init__(self, base_graph, commBudget, rank, size, iterations, issubgraph):
        super(MatchaProcessor, self).__init__(base_graph, commBudget, rank, size, iterations, issubgraph)
        self.probabilities = self.getProbability()
        self.neighbor_weight = self.getAlpha()
        self.active_flags = self.set_flags(iterations + 1)
        self.rank = rank

    def getProbability(self):
        """graph_manager.py:240-266 (cvxpy/CVXOPT SDP in the reference; solver.py here)."""
        return solver.matcha_probabilities(self.L_matrices, self.commBudget)

    def getAlpha(self):
        """graph_manager.py:268-296 (cvxpy/CVXOPT SDP in the reference; solver.py here)."""
        return solver.matcha_alpha(self.L_matrices, self.probabilities)

    def set_flags(self, iterations):
        """graph_manager.py:298-309 on the GPU (NaN / negative probabilities -> 0 first)."""
        for i in range(len(self.L_matrices)):
            if np.isnan(self.probabilities[i]) or self.probabilities[i] < 0:
                self.probabilities[i] = 0
        self.flags_dev = self._draw_flags_on_gpu(np.asarray(self.probabilities, dtype=np.float64),
                                                 iterations)
        return _host_rows(self.flags_dev)
