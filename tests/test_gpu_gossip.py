"""GPU parity: the HIP path against the golden fixtures and the CPU oracle (bit-exact)."""
import ctypes

import numpy as np
import pytest

from conftest import Topo, golden_json, golden_npz
from planref import py_plan

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _set_state(key, pos):
    np.random.set_state(("MT19937", np.asarray(key, np.uint32), int(pos), 0, 0.0))


# ------------------------------------------------------------------------------------ flags
@pytest.mark.parametrize("ci", range(8))
def test_gpu_flags_vs_reference(pkg, ci):
    g, meta = golden_npz("flags"), golden_json("flags")["matcha"][ci]
    gp = object.__new__(pkg.GraphProcessor)
    p = np.array(meta["p"], np.float64)
    p[np.isnan(p) | (p < 0)] = 0
    _set_state(g[f"matcha{ci}_key0"], meta["pos0"])
    flags = gp._draw_flags_on_gpu(p, meta["T"] + 1)
    assert np.array_equal(flags.cpu().numpy(), g[f"matcha{ci}_flags"])
    st = np.random.get_state()
    assert np.array_equal(st[1], g[f"matcha{ci}_key1"]) and st[2] == meta["pos1"]


@pytest.mark.parametrize("ci", [0, 4, 7])
def test_gpu_flags_sequential_path(pkg, ci):
    """The resample-aware sequential walk gives the same flags and state as the parallel path."""
    g, meta = golden_npz("flags"), golden_json("flags")["matcha"][ci]
    p = np.ascontiguousarray(np.nan_to_num(np.array(meta["p"], np.float64), nan=0.0).clip(0, None))
    T = meta["T"] + 1
    key = np.ascontiguousarray(g[f"matcha{ci}_key0"])
    out = torch.empty((T, len(p)), dtype=torch.uint8, device="cuda")
    k1 = np.empty(624, np.uint32)
    pos = ctypes.c_int(0)
    rc = pkg.lib.mx_flags_binomial_sequential(key.ctypes.data, meta["pos0"], p.ctypes.data, len(p), T,
                                              out.data_ptr(), k1.ctypes.data, ctypes.byref(pos), None)
    assert rc == 0
    assert np.array_equal(out.cpu().numpy(), g[f"matcha{ci}_flags"])
    assert np.array_equal(k1, g[f"matcha{ci}_key1"]) and pos.value == meta["pos1"]


def test_matcha_processor_gpu_flags_and_state(pkg, O):
    np.random.seed(1234)
    st0 = np.random.get_state()
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, 8, 500, True)
    flags, key, pos = O.matcha_flags(st0[1], st0[2], np.asarray(GP.probabilities), 501)
    assert np.array_equal(np.asarray(GP.active_flags, np.uint8), flags)
    assert np.array_equal(GP.flags_dev.cpu().numpy(), flags)
    st1 = np.random.get_state()
    assert np.array_equal(st1[1], key) and st1[2] == pos
    assert isinstance(GP.active_flags[0][0], np.int64)


def test_fixed_processor_gpu(pkg, O):
    np.random.seed(77)
    st0 = np.random.get_state()
    GP = pkg.FixedProcessor(pkg.select_graph(0), 0.37, 0, 8, 99, True)
    flags, key, pos = O.fixed_flags(st0[1], st0[2], 0.37, 100)
    assert GP.active_flags == flags.tolist()
    st1 = np.random.get_state()
    assert np.array_equal(st1[1], key) and st1[2] == pos
    assert GP.neighbor_weight == 0.2857142857142856


# ------------------------------------------------------------------------------------ plans
@pytest.mark.parametrize("gid,nranks", [(0, 1), (0, 2), (0, 8), (2, 4), (3, 3)])
def test_plan_vs_python(pkg, gid, nranks):
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    partner = np.asarray(gp.neighbors_info, np.int32)
    M = partner.shape[0]
    rng = np.random.RandomState(gid * 10 + nranks)
    flags = (rng.uniform(size=(64, M)) < 0.5).astype(np.uint8)
    flags[0] = 1
    flags[1] = 0
    alpha = 0.123456789
    fd = torch.from_numpy(flags).cuda()
    pd = torch.from_numpy(partner).cuda()
    for row_base, n_local in pkg.partition(n, nranks):
        W = pkg.lib.mx_plan_words(n_local, M)
        plan = torch.empty(64 * W, dtype=torch.int32, device="cuda")
        assert pkg.lib.mx_plan_build(fd.data_ptr(), 64, M, pd.data_ptr(), n, None, 0, row_base, n_local,
                                     alpha, plan.data_ptr(), None) == 0
        P = plan.cpu().numpy().reshape(64, W)
        for t in range(64):
            any_, remote, src, sw, _ = py_plan(flags[t], partner, row_base, n_local, alpha)
            rec = P[t]
            assert rec[0] == any_ and rec[1] == remote
            deg = rec[4:4 + n_local]
            assert deg.tolist() == [len(s) for s in src]
            assert np.array_equal(rec[4 + n_local:4 + 2 * n_local].view(np.float32), np.array(sw, np.float32))
            S = rec[4 + 2 * n_local:].reshape(n_local, M)
            for r in range(n_local):
                assert S[r, :len(src[r])].tolist() == src[r]


# ------------------------------------------------------------------------------------ mixing
@pytest.mark.parametrize("case", ["g0", "g5", "g2"])
def test_mix_vs_reference_golden(pkg, case):
    d = golden_npz("decen")
    meta = {m["name"]: m for m in golden_json("decen")}[case]
    topo = Topo(d[case + "_partner"], meta["alpha"], d[case + "_flags"])
    grp = pkg.VirtualWorkerGroup(topo, numel=meta["P"])
    grp.rows.copy_(torch.from_numpy(d[case + "_X0"]))
    for r in range(meta["rounds"]):
        grp.communicate()
        got = grp.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), d[case + "_Y"][r].view(np.uint32)), f"round {r}"


def test_mix_models_adopted_in_place(pkg, O):
    """Workers as nn.Modules: parameters re-homed into the arena (identity kept), mixed in place."""
    n = 8
    torch.manual_seed(0)
    models = [torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.ReLU(), torch.nn.Linear(17, 5)).cuda()
              for _ in range(n)]
    ids = [[id(p) for p in m.parameters()] for m in models]
    X = np.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy() for m in models])
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 0, 1, 0], [0, 0, 0, 0, 0], [0, 1, 1, 0, 1]], np.uint8)
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    grp = pkg.VirtualWorkerGroup(topo, models)
    for f in flags:
        grp.communicate()
        X = O.decen_round(X, topo.neighbors_info, f, 2 / 7)
    got = np.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy() for m in models])
    assert np.array_equal(got, X)
    assert ids == [[id(p) for p in m.parameters()] for m in models]
    out = models[3](torch.ones(2, 33, device="cuda"))          # still a working module
    assert out.shape == (2, 5)


def test_mix_segmented_unaligned_layout(pkg, O):
    """Per-tensor pointer table (no arena): odd lengths, unaligned bases, multi-segment tiles."""
    n = 8
    lens = [1, 3, 1024, 1027, 5, 4096 + 3, 0, 77]
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [0, 1, 0, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 0.3, flags)
    eng = pkg.GossipEngine(topo)
    P = sum(lens)
    X = np.stack([O.synth(900 + i, P) for i in range(n)])
    big = torch.from_numpy(np.concatenate([X, X[:, :3]], axis=1)).cuda()   # odd offsets
    base = 1                                                            # misalign by 4 bytes
    ptrs, cuts = [], np.cumsum([0] + lens)
    for i in range(n):
        ptrs.append([big[i].data_ptr() + 4 * (base + int(cuts[s])) for s in range(len(lens))])
    big[:, base:base + P] = torch.from_numpy(X).cuda()
    lay = pkg.Layout(lens, ptrs, eng.n_slots)
    for it, f in enumerate(flags):
        eng.mix(it, lay)
        X = O.decen_round(X, topo.neighbors_info, f, 0.3)
    torch.cuda.synchronize()
    got = big[:, base:base + P].cpu().numpy()
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


@pytest.mark.parametrize("gid", [0, 3])
def test_mix_full_size_headline(pkg, O, gid):
    """25.6M params x n workers (the headline shape) bit-exact vs the oracle."""
    n = pkg.GRAPH_SIZES[gid]
    P = 25_600_000 if gid == 0 else 3_000_001
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    flags = np.ones((2, M), np.uint8)
    flags[1, ::2] = 0
    topo = Topo(gp.neighbors_info, 0.2857142857142856, flags)
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        assert pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None) == 0
    X = np.stack([O.synth(1234 + i, P) for i in range(n)])
    assert np.array_equal(grp.rows.cpu().numpy(), X)
    for f in flags:
        grp.communicate()
        X = O.decen_round(X, topo.neighbors_info, f, topo.neighbor_weight)
    got = grp.rows.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


# ------------------------------------------------------------------------------------ choco
@pytest.mark.parametrize("case", ["c0", "c1", "c2"])
def test_choco_vs_reference_golden(pkg, case):
    c = golden_npz("choco")
    m = {x["name"]: x for x in golden_json("choco")}[case]
    topo = Topo(c[case + "_partner"], m["alpha"], c[case + "_flags"])
    grp = pkg.ChocoWorkerGroup(topo, numel=m["P"], ratio=m["ratio"], consensus_lr=m["consensus_lr"])
    assert grp.k == m["k"]
    grp.rows.copy_(torch.from_numpy(c[case + "_X0"]))
    for r in range(m["rounds"]):
        grp.rows.add_(torch.from_numpy(c[case + "_D"][r]).cuda())
        assert np.array_equal(grp.rows.cpu().numpy(), c[case + "_Xin"][r])
        grp.communicate()
        got = grp.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), c[case + "_Y"][r].view(np.uint32)), f"round {r}"
    assert np.array_equal(grp.x_hat[:, :m["P"]].cpu().numpy(), c[case + "_xhat"])
    assert np.array_equal(grp.s[:, :m["P"]].cpu().numpy(), c[case + "_s"])


def test_topk_vs_reference_golden(pkg):
    t = golden_npz("topk")
    import oracle as O
    for row in golden_json("topk"):
        key = f"P{row['P']}_r{row['ratio']}_idx"
        if key not in t:
            continue
        x = torch.from_numpy(O.synth(row["P"], row["P"])).cuda()
        v, i = pkg.get_top_k(x, row["ratio"])
        assert i.dtype == torch.int64 and i.numel() == row["k"]
        assert np.array_equal(i.cpu().numpy(), t[key])
        assert np.array_equal(v.cpu().numpy(), t[f"P{row['P']}_r{row['ratio']}_val"])


@pytest.mark.parametrize("P,ratio", [(14_774_436, 0.99), (1_000_003, 0.9), (4097, 0.5)])
def test_topk_large_and_ties_vs_oracle(pkg, O, P, ratio):
    x = O.synth(P + 1, P)
    x[::7] = np.float32(0.5)          # many exact ties at one magnitude
    x[::11] = np.float32(-0.5)
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(x, k)
    v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


def _topk_case(O, P, pattern):
    x = O.synth(P + 3, P)
    if pattern == "layers":           # parameter-tensor-like blocks of very different scales
        edges = np.linspace(0, P, 9).astype(np.int64)
        for j in range(8):
            x[edges[j]:edges[j + 1]] *= np.float32(10.0 ** (j % 4 - 2))
    elif pattern == "sampled_large":  # only the chunks the sampler reads are large: forces the
        c = np.arange(P) // 1024      # device-side fallback (candidate floor too high)
        x[(c % 16) == 0] *= np.float32(1000.0)
    elif pattern == "constant":       # every key ties
        x[:] = np.float32(-0.25)
    elif pattern == "ties":
        x[::7] = np.float32(0.5)
        x[::11] = np.float32(-0.5)
    elif pattern == "coarse":         # 1/128 grid: ~15.6k keys tie at the threshold
        x[:] = np.round(x * 128) / np.float32(128)
    elif pattern == "coarse333":      # 1/333 grid: ~6k ties, every threshold digit pass non-trivial
        x[:] = np.round(x * 333) / np.float32(333)
    elif pattern == "gap":            # 1 % of keys in [999, 1001): the threshold far above the
        x[::100] += np.float32(1000.0)    # sampled floor, 20k candidates in one 12-bit bin
    elif pattern == "spread":         # 1 % of keys spread over [2, 1002): threshold bin nearly empty
        x[::100] = np.copysign(np.float32(2) + np.float32(1000) * np.abs(x[::100]), x[::100])
    return x


@pytest.mark.parametrize("stride,pieces,blocks", [(0, 1, 1024), (1, 1, 1024), (16, 1, 1024), (0, 4, 2048),
                                                  (16, 3, 77), (0, 2, 4096)])
@pytest.mark.parametrize("pattern", ["layers", "sampled_large", "constant", "ties", "coarse", "coarse333", "gap",
                                     "spread"])
def test_topk_sampled_floor_exact(pkg, O, stride, pieces, blocks, pattern):
    """The sampled candidate floor (and its device-side fallback) never changes the result, for any
    sampling grid (pieces per wave) or persistent compaction grid."""
    P, ratio = 2_000_001, 0.99
    x = _topk_case(O, P, pattern)
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(x, k)
    saved = {key: int(pkg.lib.mx_topk_get(key)) for key in (b"sample_pieces", b"compact_blocks")}
    pkg._lib.check(pkg.lib.mx_topk_set(b"sample_stride", stride))
    pkg._lib.check(pkg.lib.mx_topk_set(b"sample_pieces", pieces))
    pkg._lib.check(pkg.lib.mx_topk_set(b"compact_blocks", blocks))
    try:
        v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
    finally:
        pkg.lib.mx_topk_set(b"sample_stride", 0)
        for key, val in saved.items():
            pkg.lib.mx_topk_set(key, val)
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("pattern", ["layers", "ties", "gap"])
def test_topk_unaligned_input(pkg, O, pattern):
    """A tensor view 4 bytes off 16-byte alignment takes the compaction's element-load path for
    every chunk (no prefetched whole chunks): same index set and values as the oracle."""
    P, ratio = 300_001, 0.99
    x = _topk_case(O, P, pattern)
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(x, k)
    big = torch.zeros(P + 1, dtype=torch.float32, device="cuda")
    big[1:] = torch.from_numpy(x).cuda()
    xv = big[1:]
    assert xv.data_ptr() % 16 != 0
    v, i = pkg.get_top_k(xv, ratio)
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("select", [1, 0])
def test_topk_work_reuse_and_tile_bounds(pkg, O, select):
    """One zero-filled scratch serves a sequence of calls of different P / k / patterns (incl. the
    fallback pass): each call leaves its histograms and counters zero (no zeroing launch runs),
    results stay exact, and the tile bounds the message carries are the index-range starts of
    every 4096-element tile (what mx_choco_apply reads) -- with the one-launch selection and with
    the four selection passes."""
    L = pkg.lib
    big = max(int(L.mx_topk_work_bytes(P)) for P in (2_000_001, 4097, 300_000))
    work = torch.zeros(big, dtype=torch.uint8, device="cuda")
    hist_bytes = 4 * (3 * 4096 + 1024 + 512)
    saved = int(L.mx_topk_get(b"select"))
    pkg._lib.check(L.mx_topk_set(b"select", select))
    pkg._lib.check(L.mx_topk_set(b"sample_stride", 16))      # sampled_large then needs the fallback pass
    try:
        _reuse_calls(pkg, O, work, hist_bytes)
    finally:
        L.mx_topk_set(b"sample_stride", 0)
        L.mx_topk_set(b"select", saved)


def _reuse_calls(pkg, O, work, hist_bytes):
    L = pkg.lib
    for P, ratio, pattern in [(2_000_001, 0.99, "sampled_large"), (4097, 0.5, "ties"), (300_000, 0.9, "layers"),
                              (2_000_001, 0.99, "constant"), (2_000_001, 0.99, "coarse"), (2_000_001, 0.99, "gap"),
                              (2_000_001, 0.99, "coarse333"), (2_000_001, 0.99, "spread"),
                              (2_000_001, 0.99, "sampled_large")]:
        x = _topk_case(O, P, pattern)
        k = O.topk_k(P, ratio)
        ov, oi = O.topk_abs(x, k)
        kpad = (k + 1) // 2 * 2
        nb = int(L.mx_choco_msg_bytes(P, k))
        out = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        xd = torch.from_numpy(x).cuda()
        pkg._lib.check(L.mx_topk_abs_diff_rows(xd.data_ptr(), None, P, 1, P, k, out.data_ptr(), 0, 4 * kpad,
                                               4 * kpad + 8 * k, work.data_ptr(), 0, None), "topk rows")
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        assert np.array_equal(o[:4 * k].view(np.float32).view(np.uint32), ov.view(np.uint32)), (P, pattern)
        idx = o[4 * kpad:4 * kpad + 8 * k].view(np.int64)
        assert np.array_equal(idx, oi), (P, pattern)
        nt = (P + 4095) // 4096
        bnd = o[4 * kpad + 8 * k:nb].view(np.int32)
        assert np.array_equal(bnd, np.searchsorted(oi, np.arange(nt + 1) * 4096).astype(np.int32)), (P, pattern)
        w = work.cpu().numpy()
        assert not w[:hist_bytes].any(), "histograms not re-zeroed"
        state = w[hist_bytes:hist_bytes + 24].view(np.uint64)     # b0|T, need, cand_n
        assert state[2] == 0, "candidate total not reset"
        assert w[hist_bytes + 28:hist_bytes + 32].view(np.uint32)[0] == 0, "a row barrier's wait expired"


# ------------------------------------------------------------------------------------ helpers
def test_flatten_unflatten_scatter(pkg):
    ts = [torch.randn(s, device="cuda") for s in ((3, 5), (7,), (0,), (64, 33), (1,))]
    flat = pkg.flatten_tensors(ts)
    assert torch.equal(flat, torch.cat([t.reshape(-1) for t in ts]))
    one = pkg.flatten_tensors([ts[0]])
    assert torch.equal(one, ts[0].reshape(-1)) and one.data_ptr() != ts[0].data_ptr()
    views = pkg.unflatten_tensors(flat, ts)
    assert all(torch.equal(a, b) for a, b in zip(views, ts))
    dst = [torch.zeros_like(t) for t in ts]
    pkg.scatter_tensors(flat * 2, dst)
    assert all(torch.equal(a, 2 * b) for a, b in zip(dst, ts))


# ------------------------------------------------------------------------------------ tuning variants
VARIANTS = [(bpc, u, nt, pf, rg, ch) for bpc in (1, 5) for u in (1, 2, 4) for nt in (0, 1) for pf in (0, 1)
            for rg in (0, 1) for ch in (0, 1) if not (u == 4 and not rg) and not (u > 1 and pf)]


@pytest.mark.parametrize("bpc,u,nt,pf,rg,ch", VARIANTS)
def test_mix_every_tuning_variant(pkg, O, bpc, u, nt, pf, rg, ch):
    """Each kernel variant for <= 8 slots besides the default row kernel (LDS-column /
    register-indexed, unroll, non-temporal, prefetch, grid, chunked vs tile-strided) is bit-exact on
    a flat arena, ragged multi-segment layouts and a 16-slot graph (row kernel)."""
    saved = pkg.engine.mix_tuning()
    try:
        pkg.engine.set_mix_tuning(blocks_per_cu=bpc, unroll=u, nontemporal=nt, prefetch=pf, regidx=rg,
                                  chunked=ch, rows=1)
        _layouts_bit_exact(pkg, O)
    finally:
        pkg.engine.set_mix_tuning(**saved)


@pytest.mark.parametrize("bpc,nt,u,sp", [(1, 0, 1, 0), (2, 1, 1, 0), (5, 1, 1, 0), (4, 0, 1, 0), (2, 1, 2, 0),
                                         (1, 0, 2, 0), (2, 1, 1, 1), (2, 1, 1, 2), (2, 1, 1, 4), (1, 0, 1, 4)])
def test_mix_row_kernel_for_eight_slots(pkg, O, bpc, nt, u, sp):
    """rows = 2 routes <= 8 slots through the row-per-wave kernel too: bit-exact on the same
    layouts (flat, ragged multi-segment, unaligned) as every other variant, with the layout tile
    worked whole or as 2 / 4 sub-tiles (split)."""
    saved = pkg.engine.mix_tuning()
    try:
        pkg.engine.set_mix_tuning(blocks_per_cu=bpc, nontemporal=nt, rows=2, unroll=u, split=sp)
        _layouts_bit_exact(pkg, O)
    finally:
        pkg.engine.set_mix_tuning(**saved)


@pytest.mark.parametrize("flat,bpc,mid", [(0, 2, 4), (0, 1, 4), (128, 2, 0), (128, 2, 4), (256, 2, 2), (256, 2, 8)])
def test_mix_persistent_and_flat_grids(pkg, O, flat, bpc, mid):
    """The row kernel's grid: persistent workgroups striding over the tiles (flat_small = 0, several
    tiles per workgroup), one workgroup per work item (mid_bpc = 0), and the 8-slot mid-size
    persistent grid of mid_bpc workgroups per CU -- bit-exact on the same layouts."""
    saved = pkg.engine.mix_tuning()
    try:
        pkg.engine.set_mix_tuning(flat_small=flat, blocks_per_cu=bpc, rows=2, mid_bpc=mid)
        _layouts_bit_exact(pkg, O)
    finally:
        pkg.engine.set_mix_tuning(**saved)


def _layouts_bit_exact(pkg, O):
    """flat arena, ragged multi-segment layouts (graph 0) and an unaligned 16-slot graph, 3 rounds"""
    for gid, lens in ((0, [1, 3, 1024, 1027, 5, 4096 + 3, 0, 77, 10_000]), (2, [1, 3, 1027, 5, 9000]),
                      (0, [300_001])):
        n = pkg.GRAPH_SIZES[gid]
        gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
        M = len(gp.neighbors_info)
        flags = np.ones((3, M), np.uint8)
        flags[1, 1::2] = 0
        flags[2, ::3] = 0
        topo = Topo(gp.neighbors_info, 0.21, flags)
        eng = pkg.GossipEngine(topo)
        P = sum(lens)
        X = np.stack([O.synth(300 + i, P) for i in range(n)])
        big = torch.from_numpy(np.concatenate([X, X[:, :4]], axis=1)).cuda()
        base = 1 if gid == 2 else 0
        cuts = np.cumsum([0] + lens)
        ptrs = [[big[i].data_ptr() + 4 * (base + int(cuts[s])) for s in range(len(lens))] for i in range(n)]
        big[:, base:base + P] = torch.from_numpy(X).cuda()
        lay = pkg.Layout(lens, ptrs, eng.n_slots)
        for it, f in enumerate(flags):
            eng.mix(it, lay)
            X = O.decen_round(X, topo.neighbors_info, f, 0.21)
        torch.cuda.synchronize()
        got = big[:, base:base + P].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"graph {gid} lens {lens}"


@pytest.mark.parametrize("knobs", [{"rows": 1}, {"rows": 0, "readlane_min": 32}, {"rows": 0, "readlane_min": 16},
                                   {"rows": 0, "readlane_min": 128}, {"rows": 1, "nontemporal": 0, "blocks_per_cu": 1},
                                   {"rows": 1, "split": 1}, {"rows": 1, "split": 2}, {"rows": 1, "split": 4}],
                         ids=["rows", "lds-rl32", "lds-rl16", "lds-rl128", "rows-t-bpc1", "rows-s1", "rows-s2",
                              "rows-s4"])
@pytest.mark.parametrize("n,p,seed,P", [(32, 0.2, 7, 70_001), (64, 0.1, 1234, 50_003), (24, 0.3, 3, 9_999),
                                        (16, 0.4, 5, 1024 * 7), (64, 0.1, 1234, 256 * 9), (48, 0.15, 11, 333),
                                        (12, 0.5, 2, 100_003)])
def test_mix_er_graphs_wide_configs(pkg, O, n, p, seed, P, knobs):
    """Random ER topologies decomposed by the host path: 12-64 slots exercise the NS 16 / 32 / 64
    kernels -- the row-per-wave kernel (default) and the LDS-column kernel with both edge-step
    forms (per-row lookups, one read + v_readlane); MATCHA-like random flags, 4 rounds, ragged,
    sub-tile and whole-tile widths, bit-exact."""
    import random as pyrandom
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(**knobs)
    pyrandom.seed(0)
    gp = pkg.GraphProcessor(pkg.erdos_renyi(n, p, seed), 1.0, 0, n, 4, False)
    M = len(gp.neighbors_info)
    assert M <= 32
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(4, M)) < 0.5).astype(np.uint8)
    flags[0] = 1
    topo = Topo(gp.neighbors_info, 0.05, flags)
    try:
        grp = pkg.VirtualWorkerGroup(topo, numel=P)
        X = np.stack([O.synth(11 * seed + i, P) for i in range(n)])
        grp.rows.copy_(torch.from_numpy(X))
        for f in flags:
            grp.communicate()
            X = O.decen_round(X, topo.neighbors_info, f, 0.05)
        got = grp.rows.cpu().numpy()
    finally:
        pkg.engine.set_mix_tuning(**saved)
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


@pytest.mark.parametrize("P,ratio,apply_nt", [(14_774_436 // 16, 0.99, -1), (545_930, 0.9, -1),
                                              (14_774_436 // 16, 0.99, 0), (545_930, 0.9, 1)])
def test_choco_vs_oracle_larger(pkg, O, P, ratio, apply_nt):
    """Choco on 8 workers at VGG-16 / ResNet-50(10) scale slices, 3 rounds, x / x_hat / s bit-exact
    vs oracle; the apply pass with its access hints as chosen (-1: by row count) or forced either
    way.  Both P leave a partial last tile."""
    saved = int(pkg.lib.mx_topk_get(b"apply_nt"))
    pkg._lib.check(pkg.lib.mx_topk_set(b"apply_nt", apply_nt))
    try:
        _choco_vs_oracle_larger(pkg, O, P, ratio)
    finally:
        pkg.lib.mx_topk_set(b"apply_nt", saved)


@pytest.mark.parametrize("knobs", [{"compact_store": 0}, {"compact_store": 1}, {"compact_store": 0, "apply_nt": 0},
                                   {"apply_pf": 0}, {"apply_pf": 0, "apply_nt": 1}, {"select": 0},
                                   {"select": 1, "select_blocks": 3}, {"select": 0, "compact_store": 0}])
def test_choco_knob_variants(pkg, O, knobs):
    """Every Choco kernel variant selected by mx_topk_set (compaction stores looped over the kept
    elements or one masked store pair per element; apply access hints; apply with or without the
    message entries prefetched under the tile stream; the selection as four passes or one launch)
    is bit-exact: the 8-row round (x / x_hat / s, 3 rounds) and the one-row top-k on the tie /
    far-threshold / sampled-fallback patterns."""
    saved = {k: int(pkg.lib.mx_topk_get(k.encode())) for k in knobs}
    for k, v in knobs.items():
        pkg._lib.check(pkg.lib.mx_topk_set(k.encode(), v))
    try:
        _choco_vs_oracle_larger(pkg, O, 545_930, 0.9)
        P, ratio = 2_000_001, 0.99
        k = O.topk_k(P, ratio)
        for stride, pattern in [(0, "layers"), (16, "sampled_large"), (0, "ties"), (0, "gap"), (0, "spread"),
                                (1, "coarse333")]:
            x = _topk_case(O, P, pattern)
            ov, oi = O.topk_abs(x, k)
            pkg._lib.check(pkg.lib.mx_topk_set(b"sample_stride", stride))
            try:
                v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
            finally:
                pkg.lib.mx_topk_set(b"sample_stride", 0)
            assert np.array_equal(i.cpu().numpy(), oi), pattern
            assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32)), pattern
    finally:
        for k, v in saved.items():
            pkg.lib.mx_topk_set(k.encode(), v)


@pytest.mark.parametrize("apply_pf", [1, 0])
@pytest.mark.parametrize("case", ["concentrated", "high_degree"])
def test_choco_apply_message_shapes(pkg, O, case, apply_pf):
    """The apply pass on message shapes the synthetic rows never make: tiles where a message holds
    thousands of entries (a contiguous block of large updates -> whole tiles selected, more than
    the kTPB entries the prefetching kernel loads up front) and rows with more partners than it
    prefetches (ER(12, 0.9): up to 11 partners + the own message).  3 rounds, x / x_hat / s bit-exact,
    with and without the prefetching kernel; both P leave a partial last tile."""
    import random as pyrandom
    if case == "concentrated":
        n, P, ratio = 8, 300_001, 0.9
        gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    else:
        pyrandom.seed(0)
        n, P, ratio = 12, 70_001, 0.95
        gp = pkg.GraphProcessor(pkg.erdos_renyi(n, 0.9, 3), 1.0, 0, n, 4, False)
    M = len(gp.neighbors_info)
    deg = (np.asarray(gp.neighbors_info) >= 0).sum(0)
    if case == "high_degree":
        assert deg.max() + 1 > 8
    flags = np.ones((3, M), np.uint8)
    flags[1, ::2] = 0
    alpha = 1.0 / (deg.max() + 1)
    topo = Topo(gp.neighbors_info, alpha, flags)
    saved = int(pkg.lib.mx_topk_get(b"apply_pf"))
    pkg._lib.check(pkg.lib.mx_topk_set(b"apply_pf", apply_pf))
    try:
        grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
        X = np.stack([O.synth(700 + i, P) for i in range(n)])
        if case == "concentrated":
            X[:, 50_000:90_000] *= np.float32(1000.0)
        XH, S = np.zeros_like(X), np.zeros_like(X)
        grp.rows.copy_(torch.from_numpy(X))
        k = O.topk_k(P, ratio)
        for t, f in enumerate(flags):
            if t:
                D = np.stack([np.float32(0.01) * O.synth(9100 + 31 * t + i, P) for i in range(n)])
                X += D
                grp.rows.add_(torch.from_numpy(D).cuda())
            grp.communicate()
            O.choco_round(X, XH, S, topo.neighbors_info, f, alpha, k, 0.1)
            assert np.array_equal(grp.rows.cpu().numpy().view(np.uint32), X.view(np.uint32)), f"round {t}"
            assert np.array_equal(grp.x_hat[:, :P].cpu().numpy().view(np.uint32), XH.view(np.uint32)), t
            assert np.array_equal(grp.s[:, :P].cpu().numpy().view(np.uint32), S.view(np.uint32)), t
    finally:
        pkg.lib.mx_topk_set(b"apply_pf", saved)


def _choco_vs_oracle_larger(pkg, O, P, ratio):
    n = 8
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 1, 0, 1], [0, 1, 1, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
    X = np.stack([O.synth(500 + i, P) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X))
    k = O.topk_k(P, ratio)
    for t, f in enumerate(flags):
        if t:
            D = np.stack([np.float32(0.01) * O.synth(9000 + 31 * t + i, P) for i in range(n)])
            X += D
            grp.rows.add_(torch.from_numpy(D).cuda())
        grp.communicate()
        O.choco_round(X, XH, S, topo.neighbors_info, f, 2 / 7, k, 0.1)
        got = grp.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"round {t}"
        assert np.array_equal(grp.x_hat[:, :P].cpu().numpy().view(np.uint32), XH.view(np.uint32)), f"x_hat {t}"
        assert np.array_equal(grp.s[:, :P].cpu().numpy().view(np.uint32), S.view(np.uint32)), f"s {t}"


@pytest.mark.parametrize("gid,nranks,chunk", [(0, 2, None), (0, 4, None), (0, 8, None), (2, 4, None),
                                               (3, 3, None), (0, 8, 4096), (2, 4, 7000), (0, 2, 20_000)])
def test_multirank_pipeline_loopback(pkg, O, gid, nranks, chunk):
    """N ranks' engines on one GPU with the loopback transport: owner tables, receive-slab slot
    numbering, native exchange order and the mixing kernel over local + slab rows, end to end,
    bit-exact vs the single-process oracle (the RCCL call itself is the only piece not run)."""
    from conftest import LoopbackHub
    n = pkg.GRAPH_SIZES[gid]
    P = 20_011
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    rng = np.random.RandomState(gid + nranks)
    flags = (rng.uniform(size=(6, M)) < 0.6).astype(np.uint8)
    flags[0] = 1
    flags[3] = 0
    topo = Topo(gp.neighbors_info, 0.17, flags)
    hub = LoopbackHub(nranks)
    groups = [pkg.VirtualWorkerGroup(topo, numel=P, rank=r, nranks=nranks, comm=hub.comm(r), chunk_cols=chunk)
              for r in range(nranks)]
    assert all(g.chunked == bool(chunk and chunk < P and g.engine.max_remote) for g in groups)
    X = np.stack([O.synth(700 + i, P) for i in range(n)])
    for g in groups:
        g.rows.copy_(torch.from_numpy(X[g.row_base:g.row_base + g.n_local]))
        hub.register(g.row_base, g._row_ptrs)
    for it, f in enumerate(flags):
        for g in groups:                       # ranks one after another: exchange + mix each
            g.step(it)
        torch.cuda.synchronize()
        X = O.decen_round(X, topo.neighbors_info, f, 0.17)
    got = np.concatenate([g.rows.cpu().numpy() for g in groups])
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32))


@pytest.mark.parametrize("piece", [7, 100, 1 << 22])
def test_host_staging_pieces(pkg, piece):
    """Host-resident models' staging (communicator._Staging): pieces of the flat row that split
    parameters, an empty and a non-contiguous parameter; load() gives torch.cat's layout
    (comm_helpers.py:27-30), store() writes the row back into the same tensors (identity and
    storage kept, communicator.py:124-131)."""
    from importlib import import_module
    C = import_module(pkg.__name__ + ".communicator")
    torch.manual_seed(5)
    ps = [torch.nn.Parameter(torch.randn(*sh)) for sh in ((13, 7), (0,), (5,), (64, 33), (1,))]
    ps.append(torch.nn.Parameter(torch.randn(9, 6).t()))          # non-contiguous
    n = sum(p.numel() for p in ps)
    row = torch.zeros(n, device="cuda")
    st = C._Staging(ps, row)
    st.PIECE_FLOATS = piece
    ids, ptrs = [id(p) for p in ps], [p.data_ptr() for p in ps]
    st.load()
    torch.cuda.synchronize()
    assert torch.equal(row.cpu(), torch.cat([p.detach().reshape(-1) for p in ps]))
    new = torch.randn(n, device="cuda")
    row.copy_(new)
    st.store()
    assert torch.equal(torch.cat([p.detach().reshape(-1) for p in ps]), new.cpu())
    assert [id(p) for p in ps] == ids and [p.data_ptr() for p in ps] == ptrs
    assert not ps[-1].is_contiguous()


@pytest.mark.parametrize("on_gpu", [True, False])
def test_dropin_decen_communicators_per_rank(pkg, O, on_gpu):
    """The reference API one process per worker -- here 8 decenCommunicator(rank, 8, GP) objects
    in one process on one GPU over the loopback transport -- with nn.Module workers on the GPU
    (adopted into arenas) or on the CPU (staged, as the reference's train_mpi.py keeps them).
    communicate() return values, skipped rounds and parameter identity as in the reference."""
    from conftest import LoopbackHub
    n = 8
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, 12, True)
    dev = "cuda" if on_gpu else "cpu"
    torch.manual_seed(3)
    models = [torch.nn.Sequential(torch.nn.Linear(20, 31), torch.nn.Tanh(), torch.nn.Linear(31, 3)).to(dev)
              for _ in range(n)]
    ids = [[id(p) for p in m.parameters()] for m in models]
    X = np.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy() for m in models])
    hub = LoopbackHub(n)
    comms = [pkg.decenCommunicator(r, n, GP, transport=hub.comm(r)) for r in range(n)]
    for r in range(n):                         # bind + stage every rank before round 0
        comms[r]._bind(models[r])
        comms[r]._stage.load()
        hub.register(r, [comms[r]._group.rows[0].data_ptr()])
    partner = np.asarray(GP.neighbors_info, np.int32)
    for it in range(12):
        f = np.asarray(GP.active_flags[it], np.uint8)
        times = [comms[r].communicate(models[r]) for r in range(n)]
        if not f.any():
            assert times == [0] * n
        else:
            assert all(t > 0 for t in times)
            X = O.decen_round(X, partner, f, GP.neighbor_weight)
        got = np.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy() for m in models])
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"iteration {it}"
    assert all(c.iter == 12 for c in comms)
    assert ids == [[id(p) for p in m.parameters()] for m in models]
    assert all(p.device.type == dev for m in models for p in m.parameters())


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_choco_multirank_loopback(pkg, O, nranks):
    """ChocoWorkerGroups of N ranks on one GPU: every rank compresses, then each receives its
    partners' messages (loopback transport, native exchange order) and averages; bit-exact vs the
    single-process oracle over 4 rounds with parameter drift between rounds."""
    from conftest import LoopbackHub
    n, P, ratio = 8, 30_011, 0.95
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 1, 0, 1], [0, 0, 0, 0, 0], [0, 1, 1, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    hub = LoopbackHub(nranks)
    groups = [pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.3, rank=r, nranks=nranks,
                                   comm=hub.comm(r)) for r in range(nranks)]
    X = np.stack([O.synth(40 + i, P) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    k = O.topk_k(P, ratio)
    for g in groups:
        g.rows.copy_(torch.from_numpy(X[g.row_base:g.row_base + g.n_local]))
    for t, f in enumerate(flags):
        if t:
            D = np.stack([np.float32(0.02) * O.synth(77 * t + i, P) for i in range(n)])
            X += D
            for g in groups:
                g.rows.add_(torch.from_numpy(D[g.row_base:g.row_base + g.n_local]).cuda())
        if f.any():
            for g in groups:
                g.compress(t)
                hub.register(g.row_base, [g.msgs.data_ptr() + r * g.msg_ld for r in range(g.n_local)])
            for g in groups:
                g.average(t)
            torch.cuda.synchronize()
        O.choco_round(X, XH, S, topo.neighbors_info, f, 2 / 7, k, 0.3)
        got = np.concatenate([g.rows.cpu().numpy() for g in groups])
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"round {t}"


@pytest.mark.parametrize("gid,nranks,placement", [(0, 2, "auto"), (0, 4, "auto"), (2, 4, "auto"),
                                                  (4, 3, "auto"), (0, 2, [7, 2, 5, 0, 1, 6, 3, 4])])
def test_multirank_placement_loopback(pkg, O, gid, nranks, placement):
    """Groups built with a worker placement (placement.py): each rank holds the workers listed in
    `workers`, the exchange moves the rows the relabeled plan names, and every worker ends each
    round bit-identical to the single-process oracle on the original numbering."""
    from conftest import LoopbackHub
    n = pkg.GRAPH_SIZES[gid]
    P = 9_001
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    rng = np.random.RandomState(gid * 10 + nranks)
    flags = (rng.uniform(size=(5, M)) < 0.7).astype(np.uint8)
    flags[0] = 1
    topo = Topo(gp.neighbors_info, 0.21, flags)
    hub = LoopbackHub(nranks)
    groups = [pkg.VirtualWorkerGroup(topo, numel=P, rank=r, nranks=nranks, comm=hub.comm(r), placement=placement)
              for r in range(nranks)]
    held = [w for g in groups for w in g.workers]
    assert sorted(held) == list(range(n))
    if placement == "auto":
        assert held == pkg.best_placement(np.asarray(gp.neighbors_info), nranks) or held == list(range(n))
    else:
        assert held == placement
    X = np.stack([O.synth(900 + i, P) for i in range(n)])
    for g in groups:
        g.rows.copy_(torch.from_numpy(X[g.workers]))
        hub.register(g.row_base, g._row_ptrs)
    for it, f in enumerate(flags):
        for g in groups:
            g.step(it)
        torch.cuda.synchronize()
        X = O.decen_round(X, topo.neighbors_info, f, 0.21)
        got = np.empty_like(X)
        for g in groups:
            got[g.workers] = g.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"round {it}"
    st = groups[0].state_dict()
    assert st["workers"] == groups[0].workers
    groups[0].load_state_dict(st)


def test_choco_placement_loopback(pkg, O):
    """ChocoWorkerGroups over 2 ranks with the searched placement: bit-exact vs the oracle."""
    from conftest import LoopbackHub
    n, P, ratio, nranks = 8, 20_011, 0.95, 2
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 1, 0, 1], [0, 1, 1, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    hub = LoopbackHub(nranks)
    groups = [pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.3, rank=r, nranks=nranks,
                                   comm=hub.comm(r), placement="auto") for r in range(nranks)]
    assert [w for g in groups for w in g.workers] != list(range(n))
    X = np.stack([O.synth(60 + i, P) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    k = O.topk_k(P, ratio)
    for g in groups:
        g.rows.copy_(torch.from_numpy(X[g.workers]))
    for t, f in enumerate(flags):
        for g in groups:
            g.compress(t)
            hub.register(g.row_base, [g.msgs.data_ptr() + r * g.msg_ld for r in range(g.n_local)])
        for g in groups:
            g.average(t)
        torch.cuda.synchronize()
        O.choco_round(X, XH, S, topo.neighbors_info, f, 2 / 7, k, 0.3)
        got = np.empty_like(X)
        for g in groups:
            got[g.workers] = g.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"round {t}"


@pytest.mark.parametrize("knob", [("compact_pf2", 1), ("compact_wave", 1), ("compact_wave", 3)])
@pytest.mark.parametrize("pattern", ["layers", "sampled_large", "ties", "gap", "coarse333"])
@pytest.mark.parametrize("P", [2_000_001, 14_774_436])
def test_topk_compaction_variants(pkg, O, P, pattern, knob):
    """The compaction variants -- two whole chunks in flight per wave ("compact_pf2" 1), wave-owned
    chunks ("compact_wave" c: about c chunks per wave) -- one row and (through ChocoWorkerGroup's
    batched rows) several: index sets and values equal the oracle's, the sampled-fallback pattern
    among them."""
    ratio = 0.99
    x = _topk_case(O, P, pattern)
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(x, k)
    key, val = knob[0].encode(), knob[1]
    saved = int(pkg.lib.mx_topk_get(key))
    pkg._lib.check(pkg.lib.mx_topk_set(key, val))
    try:
        v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
        assert np.array_equal(i.cpu().numpy(), oi)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))
        if P < 3_000_000:                         # several rows in one launch
            gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
            topo = Topo(gp.neighbors_info, 2 / 7, np.ones((2, 5), np.uint8))
            grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
            X = np.stack([x * np.float32(1 + r) for r in range(8)])
            grp.rows.copy_(torch.from_numpy(X))
            grp.compress(0)
            torch.cuda.synchronize()
            for r in range(8):
                gv, gi = grp.message(r)
                rv, ri = O.topk_abs(X[r], k)
                assert np.array_equal(gi.cpu().numpy(), ri), r
                assert np.array_equal(gv.cpu().numpy().view(np.uint32), rv.view(np.uint32)), r
    finally:
        pkg.lib.mx_topk_set(key, saved)


@pytest.mark.parametrize("blocks", [0, 1, 5, 32])
@pytest.mark.parametrize("pattern,stride", [("layers", 0), ("sampled_large", 16), ("ties", 0), ("gap", 0),
                                            ("coarse333", 1), ("constant", 0), ("spread", 0)])
@pytest.mark.parametrize("P", [2_000_001, 14_774_436])
def test_topk_select_kernel(pkg, O, P, pattern, stride, blocks):
    """The one-launch selection (select_kernel: 10- and 9-bit passes, exact threshold, output placed
    from the per-block slots, behind two row barriers) for any number of blocks per row -- one
    (no other block to wait for), an odd count, the maximum -- on one row and on 8 rows of one
    launch batch (ChocoWorkerGroup): index sets, values and tile bounds equal the oracle's, the
    sampled fallback (stride 16: fewer than k candidates kept, every key re-compacted inside the
    launch) among them; the rows' barrier error word stays clear."""
    ratio = 0.99
    x = _topk_case(O, P, pattern)
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(x, k)
    L = pkg.lib
    saved = {key: int(L.mx_topk_get(key)) for key in (b"select", b"select_blocks")}
    pkg._lib.check(L.mx_topk_set(b"select", 1))
    pkg._lib.check(L.mx_topk_set(b"select_blocks", blocks))
    pkg._lib.check(L.mx_topk_set(b"sample_stride", stride))
    try:
        v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
        assert np.array_equal(i.cpu().numpy(), oi)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))
        if P < 3_000_000:
            kpad = (k + 1) // 2 * 2
            nb = int(L.mx_choco_msg_bytes(P, k))
            nt = (P + 4095) // 4096
            wb = int(L.mx_topk_work_bytes(P))
            wld = (wb + 255) // 256 * 256
            X = np.stack([x * np.float32(1 + r) for r in range(8)])
            xd = torch.from_numpy(X).cuda()
            out = torch.zeros(8 * nb + 8 * 8, dtype=torch.uint8, device="cuda")
            old = (nb + 7) // 8 * 8
            work = torch.zeros(8 * wld, dtype=torch.uint8, device="cuda")
            pkg._lib.check(L.mx_topk_abs_diff_rows(xd.data_ptr(), None, P, 8, P, k, out.data_ptr(), old, 4 * kpad,
                                                   4 * kpad + 8 * k, work.data_ptr(), wld, None), "topk rows")
            torch.cuda.synchronize()
            o = out.cpu().numpy()
            w = work.cpu().numpy()
            for r in range(8):
                rv, ri = O.topk_abs(X[r], k)
                m = o[r * old:r * old + nb]
                assert np.array_equal(m[:4 * k].view(np.uint32), rv.view(np.uint32)), r
                assert np.array_equal(m[4 * kpad:4 * kpad + 8 * k].view(np.int64), ri), r
                bnd = m[4 * kpad + 8 * k:nb].view(np.int32)
                assert np.array_equal(bnd, np.searchsorted(ri, np.arange(nt + 1) * 4096).astype(np.int32)), r
                hb = r * wld + 4 * (3 * 4096 + 1024 + 512)
                assert not w[r * wld:hb].any(), "histograms not re-zeroed"
                assert w[hb + 28:hb + 32].view(np.uint32)[0] == 0, "a row barrier's wait expired"
    finally:
        L.mx_topk_set(b"sample_stride", 0)
        for key, val in saved.items():
            L.mx_topk_set(key, val)
