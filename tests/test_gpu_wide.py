"""Wide layouts: more than 64 slots per GPU or more than 32 matchings (the 64-slot /
32-matching hard caps).  mix_kernel_wide takes 65-156 slots and any matching count; bit-exact vs
the oracle on ER topologies decomposed by the host path, 1 process and 2-3 loopback ranks, plus
ChocoSGD on 96 workers."""
import random

import numpy as np
import pytest

from conftest import LoopbackHub, Topo

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _er(pkg, n, p, seed):
    random.seed(0)
    gp = pkg.GraphProcessor(pkg.erdos_renyi(n, p, seed), 1.0, 0, n, 4, False)
    return np.asarray(gp.neighbors_info, np.int32)


@pytest.mark.parametrize("n,p,seed,P", [(96, 0.06, 1, 9_001), (128, 0.05, 2, 5_000), (150, 0.04, 3, 3_001),
                                        (48, 0.9, 4, 7_777), (24, 0.3, 5, 1_000)])
@pytest.mark.parametrize("idle_rows", ["skip", "canonical"])
def test_wide_slots_and_matchings(pkg, O, n, p, seed, P, idle_rows):
    partner = _er(pkg, n, p, seed)
    M = partner.shape[0]
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(4, M)) < 0.5).astype(np.uint8)
    flags[0] = 1
    topo = Topo(partner, 0.5 / M, flags)
    grp = pkg.VirtualWorkerGroup(topo, numel=P, idle_rows=idle_rows)
    wide = n > 64 or M > 32
    if wide:
        assert grp.engine.n_slots > 64 or M > 32
    X = np.stack([O.synth(17 * seed + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X))
    for f in flags:
        grp.communicate()
        X = O.decen_round(X, partner, f, topo.neighbor_weight)
    got = grp.rows.cpu().numpy()          # (synth has no -0.0: "skip" idle rows equal the oracle too)
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


@pytest.mark.parametrize("nranks", [2, 3])
def test_wide_multirank_loopback(pkg, O, nranks):
    """150 workers over 2-3 ranks: local rows + many remote slab slots per rank."""
    n, P = 150, 4_097
    partner = _er(pkg, n, 0.04, 9)
    M = partner.shape[0]
    rng = np.random.RandomState(3)
    flags = (rng.uniform(size=(3, M)) < 0.6).astype(np.uint8)
    flags[0] = 1
    topo = Topo(partner, 0.3 / M, flags)
    hub = LoopbackHub(nranks)
    groups = [pkg.VirtualWorkerGroup(topo, numel=P, rank=r, nranks=nranks, comm=hub.comm(r)) for r in range(nranks)]
    assert max(g.engine.n_slots for g in groups) > 64
    X = np.stack([O.synth(300 + i, P) for i in range(n)])
    for g in groups:
        g.rows.copy_(torch.from_numpy(X[g.row_base:g.row_base + g.n_local]))
        hub.register(g.row_base, g._row_ptrs)
    for it, f in enumerate(flags):
        for g in groups:
            g.step(it)
        torch.cuda.synchronize()
        X = O.decen_round(X, partner, f, topo.neighbor_weight)
    got = np.concatenate([g.rows.cpu().numpy() for g in groups])
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


def test_wide_choco(pkg, O):
    n, P, ratio = 96, 20_011, 0.9
    partner = _er(pkg, n, 0.06, 1)
    M = partner.shape[0]
    flags = np.ones((2, M), np.uint8)
    flags[1, ::2] = 0
    topo = Topo(partner, 0.5 / M, flags)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.2)
    X = np.stack([O.synth(40 + i, P) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X))
    k = O.topk_k(P, ratio)
    for f in flags:
        grp.communicate()
        O.choco_round(X, XH, S, partner, f, topo.neighbor_weight, k, 0.2)
    assert np.array_equal(grp.rows.cpu().numpy().view(np.uint32), X.view(np.uint32))


def test_slot_limit_message(pkg):
    partner = _er(pkg, 160, 0.05, 5)
    topo = Topo(partner, 0.01, np.ones((2, partner.shape[0]), np.uint8))
    with pytest.raises(pkg.MXError, match="156"):
        pkg.VirtualWorkerGroup(topo, numel=100)


@pytest.mark.parametrize("ns48,pf2,tpb", [(0, 0, 256), (1, 0, 256), (0, 1, 256), (1, 1, 256), (0, 2, 256),
                                          (0, 2, 1024), (1, 2, 1024), (0, 1, 1024), (0, 0, 512), (1, 1, 512)])
@pytest.mark.parametrize("nranks,P", [(8, 70_001), (4, 512 * 9 + 3), (2, 33_333), (1, 20_011)])
def test_er64_shares_slot_classes(pkg, O, nranks, P, ns48, pf2, tpb):
    """Config 5's topology, ER(64, 0.1, 1234), split over 8 / 4 / 2 loopback ranks (placement
    "auto", as the bench): the per-rank shares of 35-53 slots run the 64-slot row class or the
    48-slot one (ns48), with one or two tiles' loads in flight (rows_pf2 0 / 1, 2 = by the staged
    share of the class), in 256 / 512 / 1024-thread workgroups (rows_tpb); and all 64 workers on
    one rank.  3 MATCHA-like rounds, ragged P, bit-exact vs the oracle."""
    n = 64
    random.seed(0)
    base = pkg.erdos_renyi(n, 0.1, 1234)
    gp0 = pkg.GraphProcessor(base, 1.0, 0, n, 4, False)
    partner0 = np.asarray(gp0.neighbors_info, np.int32)
    M = partner0.shape[0]
    rng = np.random.RandomState(5)
    flags = (rng.uniform(size=(3, M)) < 0.6).astype(np.uint8)
    flags[0] = 1
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(ns48=ns48, rows_pf2=pf2, rows_tpb=tpb)
    try:
        topo = Topo(partner0, 0.4 / M, flags)
        if nranks == 1:
            groups = [pkg.VirtualWorkerGroup(topo, numel=P)]
            hub = None
        else:
            hub = LoopbackHub(nranks)
            groups = [pkg.VirtualWorkerGroup(topo, numel=P, rank=r, nranks=nranks, comm=hub.comm(r), placement="auto")
                      for r in range(nranks)]
        if nranks == 8:
            assert any(33 <= g.engine.n_slots <= 48 for g in groups)
        X = np.stack([O.synth(700 + i, P) for i in range(n)])
        for g in groups:
            w = np.asarray(g.workers)
            g.rows.copy_(torch.from_numpy(X[w]))
            if hub is not None:
                hub.register(g.row_base, g._row_ptrs)
        for it, f in enumerate(flags):
            for g in groups:
                g.step(it)
            torch.cuda.synchronize()
            X = O.decen_round(X, partner0, f, topo.neighbor_weight)
        for g in groups:
            w = np.asarray(g.workers)
            assert np.array_equal(g.rows.cpu().numpy().view(np.uint32), X[w].view(np.uint32))
    finally:
        pkg.engine.set_mix_tuning(**saved)


@pytest.mark.parametrize("lds_kb,plan_lds,tpb,nt,pf2", [(40, 0, 256, 2, 0), (80, 1, 256, 2, 0), (158, 1, 256, 2, 0),
                                                        (158, 0, 256, 2, 0), (40, 1, 1024, 2, 0), (158, 1, 1024, 2, 0),
                                                        (80, 0, 512, 2, 0), (40, 1, 512, 2, 0), (158, 1, 1024, 0, 0),
                                                        (40, 1, 256, 0, 0), (158, 1, 1024, 2, 1), (80, 0, 1024, 0, 1),
                                                        (40, 1, 1024, 2, 1)])
@pytest.mark.parametrize("n,p,seed,P", [(96, 0.06, 1, 9_001), (150, 0.04, 3, 3_001), (72, 0.08, 6, 70_003)])
def test_wide_lds_budget(pkg, O, n, p, seed, P, lds_kb, plan_lds, tpb, nt, pf2):
    """mix_kernel_wide with a bigger LDS budget per piece (mx_mix_set "wide_lds_kb"): 128- / 256-column
    pieces of every slot (VEC 2 / 4 past 40 / 80 slots, fewer workgroups per CU), and with the plan
    record read from global memory instead of LDS ("wide_plan_lds" 0), and with 512 / 1024-thread
    workgroups ("wide_tpb"), with ordinary instead of streaming accesses, and with two pieces' loads
    in flight ("wide_pf2"); 4 MATCHA-like rounds,
    ragged P, bit-exact vs the oracle."""
    partner = _er(pkg, n, p, seed)
    M = partner.shape[0]
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(4, M)) < 0.5).astype(np.uint8)
    flags[0] = 1
    topo = Topo(partner, 0.5 / M, flags)
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(wide_lds_kb=lds_kb, wide_plan_lds=plan_lds, wide_tpb=tpb, nontemporal=nt, wide_pf2=pf2)
    try:
        grp = pkg.VirtualWorkerGroup(topo, numel=P)
        X = np.stack([O.synth(23 * seed + i, P) for i in range(n)])
        grp.rows.copy_(torch.from_numpy(X))
        for f in flags:
            grp.communicate()
            X = O.decen_round(X, partner, f, topo.neighbor_weight)
        got = grp.rows.cpu().numpy()
    finally:
        pkg.engine.set_mix_tuning(**saved)
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


@pytest.mark.parametrize("tpb,pf2", [(512, 0), (1024, 0), (1024, 1)])
@pytest.mark.parametrize("n,p,seed", [(32, 0.15, 2), (48, 0.1, 4), (64, 0.1, 1234)])
def test_rows_tpb_full_tiles(pkg, O, n, p, seed, tpb, pf2):
    """The 32 / 48 / 64-slot row classes on unsplit tiles (more layout tiles than the persistent
    grid) in 512 / 1024-thread workgroups (rows_tpb: the items of a tile dealt to 8 / 16 waves),
    one or two tiles in flight; 4 MATCHA-like rounds with skipped matchings, ragged P, bit-exact."""
    partner = _er(pkg, n, p, seed)
    M = partner.shape[0]
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(4, M)) < 0.5).astype(np.uint8)
    flags[0] = 1
    topo = Topo(partner, 0.5 / M, flags)
    P = 700 * 512 + 77
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(rows_tpb=tpb, rows_pf2=pf2, ns48=1 if n == 48 else 0)
    try:
        grp = pkg.VirtualWorkerGroup(topo, numel=P)
        assert pkg.engine.mix_kernel_name(grp.engine.n_slots) == "mix_kernel_rows"
        X = np.stack([O.synth(31 * seed + i, P) for i in range(n)])
        grp.rows.copy_(torch.from_numpy(X))
        for f in flags:
            grp.communicate()
            X = O.decen_round(X, partner, f, topo.neighbor_weight)
        got = grp.rows.cpu().numpy()
    finally:
        pkg.engine.set_mix_tuning(**saved)
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))
