"""Worker placement over GPUs (placement.py): the search against brute force, the native exchange
plan's link volumes under a placement, and that a relabeled round is the original round with its
rows permuted, bit for bit (oracle; CPU only)."""
import ctypes
import itertools
import random

import numpy as np
import pytest


def _partner(pkg, gid):
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    return np.asarray(gp.neighbors_info, np.int32), n


def _brute_force(pkg, partner, n, nranks):
    """smallest cost over every balanced assignment worker -> GPU (block sizes of
    engine.partition; GPU labels are interchangeable, so blocks are enumerated canonically)"""
    sizes = [c for _, c in pkg.partition(n, nranks)]
    best = None

    def rec(left, blocks):
        nonlocal best
        if len(blocks) == nranks:
            own = np.empty(n, np.int64)
            for r, b in enumerate(blocks):
                own[list(b)] = r
            c = pkg.placement_cost(partner, own, nranks)
            best = c if best is None or c < best else best
            return
        size = sizes[len(blocks)]
        first = min(left)           # canonical: the smallest free worker opens the next block
        for rest in itertools.combinations(sorted(left - {first}), size - 1):
            blk = (first,) + rest
            rec(left - set(blk), blocks + [blk])

    rec(set(range(n)), [])
    return best


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_best_placement_is_optimal_on_graph0(pkg, nranks):
    partner, n = _partner(pkg, 0)
    perm = pkg.best_placement(partner, nranks)
    assert sorted(perm) == list(range(n))
    own = pkg.placement._owner_of(perm, nranks)
    assert pkg.placement_cost(partner, own, nranks) == _brute_force(pkg, partner, n, nranks)
    contiguous = pkg.placement_cost(partner, pkg.engine.owner_table(n, nranks), nranks)
    assert pkg.placement_cost(partner, own, nranks) <= contiguous
    # graph 0 over 2 GPUs: busiest direction 4 -> 3 rows, total 7 -> 6
    if nranks == 2:
        assert contiguous == (4, 7) and pkg.placement_cost(partner, own, nranks) == (3, 6)


def test_best_placement_deterministic_and_never_worse(pkg):
    random.seed(0)
    for n, p, nranks in [(16, 0.3, 4), (32, 0.2, 8), (24, 0.25, 3)]:
        gp = pkg.GraphProcessor(pkg.erdos_renyi(n, p, 7), 1.0, 0, n, 4, False)
        partner = np.asarray(gp.neighbors_info, np.int32)
        a = pkg.best_placement(partner, nranks)
        b = pkg.best_placement(partner, nranks)
        assert a == b
        own = pkg.placement._owner_of(a, nranks)
        assert np.bincount(own, minlength=nranks).tolist() == [c for _, c in pkg.partition(n, nranks)]
        assert pkg.placement_cost(partner, own, nranks) <= \
            pkg.placement_cost(partner, pkg.engine.owner_table(n, nranks), nranks)
    assert pkg.best_placement(partner, 1) == list(range(n))


def _plan_ops(pkg, flags, partner, n, owner, rank, base, nl):
    M = partner.shape[0]
    cnt = ctypes.c_int(0)
    assert pkg.lib.mx_exchange_plan(flags.ctypes.data, M, partner.ctypes.data, n, owner.ctypes.data, rank,
                                    base, nl, None, 0, ctypes.byref(cnt)) == 0
    ops = np.zeros((max(1, cnt.value), 4), np.int32)
    assert pkg.lib.mx_exchange_plan(flags.ctypes.data, M, partner.ctypes.data, n, owner.ctypes.data, rank,
                                    base, nl, ops.ctypes.data, cnt.value, ctypes.byref(cnt)) == 0
    return ops[:cnt.value]


@pytest.mark.parametrize("gid,nranks", [(0, 2), (0, 4), (2, 4), (1, 8), (4, 3)])
def test_native_plan_volumes_follow_the_placement(pkg, gid, nranks):
    """With the relabeled table the engine would see, the native exchange plan sends exactly the
    rows placement_cost counts, per directed pair, every matching active."""
    partner, n = _partner(pkg, gid)
    perm = pkg.best_placement(partner, nranks)
    rel = pkg.placement.RelabeledTopology(type("T", (), {"size": n, "neighbors_info": partner.tolist(),
                                                          "neighbor_weight": 0.2,
                                                          "active_flags": [[1] * len(partner)]})(), perm)
    rp = np.ascontiguousarray(np.asarray(rel.neighbors_info, np.int32))
    owner = pkg.engine.owner_table(n, nranks)
    flags = np.ones(rp.shape[0], np.uint8)
    load = np.zeros((nranks, nranks), int)
    for rank, (base, nl) in enumerate(pkg.partition(n, nranks)):
        for op in _plan_ops(pkg, flags, rp, n, owner, rank, base, nl):
            if op[0] == 0:
                load[rank, op[1]] += 1
    own = pkg.placement._owner_of(perm, nranks)
    assert (load.max(), load.sum()) == pkg.placement_cost(partner, own, nranks)


@pytest.mark.parametrize("gid", [0, 1, 2, 3, 4])
def test_relabeled_round_is_permuted_round(pkg, O, gid):
    """Decen and Choco rounds on the relabeled table are the original rounds with rows permuted,
    bit-exact: every worker's chain keeps its partner terms in matching order."""
    partner, n = _partner(pkg, gid)
    rng = np.random.RandomState(gid)
    perm = list(rng.permutation(n))
    rel = pkg.placement.RelabeledTopology(type("T", (), {"size": n, "neighbors_info": partner.tolist(),
                                                          "neighbor_weight": 0.2,
                                                          "active_flags": [[1] * len(partner)]})(), perm)
    rp = np.asarray(rel.neighbors_info, np.int32)
    P = 257
    X = np.stack([O.synth(50 + i, P) for i in range(n)])
    for t in range(3):
        f = (rng.uniform(size=len(partner)) < 0.7).astype(np.uint8)
        want = O.decen_round(X, partner, f, 0.2)
        got = O.decen_round(np.ascontiguousarray(X[perm]), rp, f, 0.2)
        assert np.array_equal(got.view(np.uint32), want[perm].view(np.uint32))
        X = want
    XA, XHA, SA = X.copy(), np.zeros_like(X), np.zeros_like(X)
    XB, XHB, SB = np.ascontiguousarray(X[perm]), np.zeros_like(X), np.zeros_like(X)
    k = O.topk_k(P, 0.9)
    for t in range(3):
        f = (rng.uniform(size=len(partner)) < 0.7).astype(np.uint8)
        O.choco_round(XA, XHA, SA, partner, f, 0.2, k, 0.3)
        O.choco_round(XB, XHB, SB, rp, f, 0.2, k, 0.3)
        assert np.array_equal(XB.view(np.uint32), XA[perm].view(np.uint32))
        assert np.array_equal(XHB.view(np.uint32), XHA[perm].view(np.uint32))


def test_placement_argument_validation(pkg):
    partner, n = _partner(pkg, 0)
    topo = type("T", (), {"size": n, "neighbors_info": partner.tolist(), "neighbor_weight": 0.2,
                          "active_flags": [[1] * len(partner)]})()
    assert pkg.placement.resolve(topo, 2, None) is None
    assert pkg.placement.resolve(topo, 2, "contiguous") is None
    assert pkg.placement.resolve(topo, 2, list(range(n))) is None
    assert pkg.placement.resolve(topo, 2, "auto") == pkg.best_placement(partner, 2)
    with pytest.raises(ValueError):
        pkg.placement.resolve(topo, 2, [0, 0, 1, 2, 3, 4, 5, 6])
    with pytest.raises(ValueError):
        pkg.placement.resolve(topo, 2, "random")
    assert pkg.placement.block_workers([3, 1, 0, 2], 1, 2) == [1, 0]
    assert pkg.placement.block_workers(None, 4, 2) == [4, 5]


def test_flags_row_reference_walk(pkg):
    """engine.flags_row: the row averaging(active_flags) walks (communicator.py:99-110) as one entry
    per matching -- a shorter row (FixedProcessor's [0, 1] / [1, 0], graph_manager.py:208-225) names
    the first matchings, non-zero entries count as active, a longer row is refused like the
    reference's neighbors_info[graph_id] lookup would fail."""
    fr = pkg.engine.flags_row
    assert fr([0, 1], 5).tolist() == [0, 1, 0, 0, 0]
    assert fr(np.array([2, 0, -1], np.int64), 3).tolist() == [1, 0, 1]
    assert fr([], 4).tolist() == [0, 0, 0, 0]
    with pytest.raises(IndexError):
        fr([1] * 6, 5)
    with pytest.raises(IndexError):
        fr([[1, 0]], 5)
