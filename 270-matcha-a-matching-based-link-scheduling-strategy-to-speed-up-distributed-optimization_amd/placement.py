"""Worker placement over GPUs for the multi-worker-per-GPU mode (VirtualWorkerGroup /
ChocoWorkerGroup with nranks > 1).

The reference runs one MPI rank per worker (train_mpi.py:40-45), so "which GPU holds which
worker" never comes up there.  When several workers share a GPU the choice decides how many rows
cross each xGMI link per round: a row crosses a link once per (worker, destination GPU)
(mx_exchange_plan), so the link load of a placement is

    rows(a -> b) = |{ w on GPU a : some matching pairs w with a worker on GPU b }|

and a round's exchange time is set by the busiest directed pair.  `best_placement` searches the
balanced assignments (block sizes as engine.partition) for the smallest busiest pair, then the
smallest total, over every matching active (the worst round of any MATCHA schedule).

A placement is applied by renumbering: position i of the relabeled topology is worker perm[i],
so the engine keeps its contiguous blocks [row_base, row_base + n_local) and every kernel and
plan is unchanged.  Each worker's mixing chain is the same sequence of partner terms in the same
(matching) order, so a relabeled round is bit-identical to the original, row for row.
"""
import numpy as np

from .engine import partition


def _counts(partner, owner, nranks):
    """Directed pair loads [nranks, nranks] (rows) of one assignment, every matching active."""
    M, n = partner.shape
    valid = partner >= 0
    w = np.broadcast_to(np.arange(n), partner.shape)[valid]
    dst = owner[partner[valid]]
    src = owner[w]
    cross = src != dst
    reach = np.zeros((n, nranks), bool)
    reach[w[cross], dst[cross]] = True
    load = np.zeros((nranks, nranks), np.int64)
    np.add.at(load, (np.repeat(owner, nranks).reshape(n, nranks)[reach],
                     np.broadcast_to(np.arange(nranks), (n, nranks))[reach]), 1)
    return load


def placement_cost(partner, owner, nranks):
    """(busiest directed pair, total rows moved) of an assignment worker -> GPU."""
    load = _counts(np.asarray(partner, np.int64), np.asarray(owner, np.int64), nranks)
    return int(load.max()) if load.size else 0, int(load.sum())


def _owner_of(perm, nranks):
    n = len(perm)
    own = np.empty(n, np.int64)
    for r, (b, c) in enumerate(partition(n, nranks)):
        own[np.asarray(perm[b:b + c], np.int64)] = r
    return own


def best_placement(partner, nranks, restarts=None, seed=0):
    """Worker order (position -> worker id) whose contiguous blocks minimise the busiest xGMI
    pair.  Deterministic (seeded swap-descent from the identity and `restarts` random starts,
    default 16 up to 32 workers, 4 beyond: about a second at 64 workers), so every rank computes
    the same answer independently; the identity wins ties."""
    partner = np.asarray(partner, np.int64)
    n = partner.shape[1]
    if restarts is None:
        restarts = 16 if n <= 32 else 4
    if nranks <= 1 or n <= 1:
        return list(range(n))

    def cost(own):
        load = _counts(partner, own, nranks)
        return (int(load.max()), int(load.sum()))

    def descend(own):
        best = cost(own)
        improved = True
        while improved:
            improved = False
            for a in range(n):
                for b in range(a + 1, n):
                    if own[a] == own[b]:
                        continue
                    own[a], own[b] = own[b], own[a]
                    c = cost(own)
                    if c < best:
                        best, improved = c, True
                    else:
                        own[a], own[b] = own[b], own[a]
        return best, own

    rng = np.random.RandomState(seed)
    best_c, best_own = descend(_owner_of(list(range(n)), nranks))
    for _ in range(restarts):
        c, own = descend(_owner_of(list(rng.permutation(n)), nranks))
        if c < best_c:
            best_c, best_own = c, own
    # blocks in GPU order, workers ascending inside each block
    return [int(w) for r in range(nranks) for w in np.flatnonzero(best_own == r)]


def check_permutation(perm, n):
    perm = [int(w) for w in perm]
    if sorted(perm) != list(range(n)):
        raise ValueError(f"placement must be a permutation of the {n} workers")
    return perm


class RelabeledTopology:
    """A FixedProcessor / MatchaProcessor seen with position i standing for worker perm[i]:
    neighbors_info is renumbered, the schedule (active_flags, flags_dev, neighbor_weight,
    probabilities) is the processor's own.  Other attributes are the processor's, unrenumbered."""

    def __init__(self, topology, perm):
        self.base = topology
        self.size = int(topology.size)
        self.perm = check_permutation(perm, self.size)
        pos = np.empty(self.size, np.int64)
        pos[np.asarray(self.perm)] = np.arange(self.size)
        part = np.asarray(topology.neighbors_info, np.int64).reshape(-1, self.size)
        new = np.full_like(part, -1)
        for g in range(part.shape[0]):
            for w in range(self.size):
                q = part[g, w]
                if q >= 0:
                    new[g, pos[w]] = pos[q]
        self.neighbors_info = new.tolist()
        self.neighbor_weight = topology.neighbor_weight
        self.active_flags = topology.active_flags
        self.flags_dev = getattr(topology, "flags_dev", None)

    def __getattr__(self, name):
        return getattr(self.__dict__["base"], name)


def resolve(topology, nranks, placement):
    """placement None / "contiguous" -> None (workers stay in id order); "auto" -> best_placement;
    a sequence -> that worker order.  Returns the order (or None) for VirtualWorkerGroup."""
    n = int(topology.size)
    if placement is None or placement == "contiguous":
        return None
    if isinstance(placement, str):
        if placement != "auto":
            raise ValueError(f"unknown placement {placement!r}")
        part = np.asarray(topology.neighbors_info, np.int64).reshape(-1, n)
        M = np.asarray(topology.active_flags).shape[1]
        perm = best_placement(part[:M], nranks)
    else:
        perm = check_permutation(placement, n)
    return None if perm == list(range(n)) else perm


def place(topology, nranks, placement):
    """(topology the engine should see, worker order or None) for a group's `placement` argument."""
    perm = resolve(topology, nranks, placement)
    return (topology if perm is None else RelabeledTopology(topology, perm)), perm


def block_workers(perm, row_base, n_local):
    """Worker ids held by rows [row_base, row_base + n_local) of a group."""
    if perm is None:
        return list(range(row_base, row_base + n_local))
    return list(perm[row_base:row_base + n_local])
