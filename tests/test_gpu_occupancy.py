"""GPU: the round-6 occupancy-capped streaming forms, each against the oracle (uint32).

  * mix_kernel_rows' SPEC form (mx_mix_set "spec" / "spec_wgpc" / "spec_glds"): an 8-slot round of
    large rows whose active local rows the caller passes (mx_mix_call.need_host, the engine's host
    mask) loads their first tile before the plan record arrives -- through registers or by LDS-DMA
    (a wave whose columns pass the row end falls back to registers) -- at a capped number of
    workgroups per CU.  The
    hint steers loads only: the plan record decides what is mixed, so a wrong mask -- bits missing,
    extra, all, none -- gives the same bits (decenCommunicator.averaging, communicator.py:92-122);
  * the centralized mean at mean_wgpc workgroups per CU (centralizedCommunicator, communicator.py:
    46-76): the same bits as the uncapped launch and the oracle's reference-order mean.

The SPEC cases use rows of 10.5M params (8 rows: > 320 MB per round, where the row kernel streams
with non-temporal hints and the SPEC form applies; the launches are counted) and the mean cases
2.5M (> 64 MB)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

P_BIG = 2_500_003            # 8 x P x 4 > 64 MB, ragged last tile
P_SPEC = 10_500_001          # 8 x P x 4 > 320 MB (non-temporal row kernel), ragged last tile


def _spec_launches(pkg):
    return int(pkg.lib.mx_mix_get(b"spec_launches"))


def _u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _run(pkg, O, GP, P, rounds, idle_rows="skip", scramble=None):
    g = pkg.VirtualWorkerGroup(GP, numel=P, idle_rows=idle_rows)
    X = np.stack([O.synth(4100 + i, P) for i in range(g.n_local)])
    g.rows[:, :P] = torch.from_numpy(X).cuda()
    eng = g.engine
    if scramble is not None:
        eng.need_host[:] = scramble(eng.need_host.copy())
    partner = np.asarray(GP.neighbors_info, np.int32)
    flags = np.asarray(GP.active_flags, np.uint8)
    for it in range(rounds):
        g.step(it)
        if flags[it].any():
            X = O.decen_round(X, partner, flags[it], GP.neighbor_weight)
            if idle_rows == "canonical":
                # the reference rewrites an idle row as 0 + 1.0 * x (communicator.py:113-117)
                deg = (partner[flags[it].astype(bool)] >= 0).sum(axis=0)
                X[deg == 0] = X[deg == 0] + np.float32(0.0)
    torch.cuda.synchronize()
    got = g.rows[:, :P].cpu().numpy()
    g.close()
    return got, X


@pytest.mark.parametrize("spec,wgpc,budget,glds", [(1, 5, 1.0, 1), (1, 5, 0.5, 1), (1, 5, 1.0, 0), (1, 5, 0.5, 0),
                                                   (1, 0, 0.5, 1), (0, 5, 0.5, 1), (1, 3, 0.3, 1)])
def test_spec_rounds_match_oracle(pkg, O, spec, wgpc, budget, glds):
    """Full and MATCHA rounds of 8 x 10.5M through the SPEC form (and with it off), every round vs the
    oracle's decen rounds; the engine's host mask equals the rows plan_kernel marks."""
    E = pkg.engine
    saved = E.mix_tuning()
    try:
        E.set_mix_tuning(spec=spec, spec_wgpc=wgpc, spec_glds=glds)
        np.random.seed(1234)
        GP = pkg.MatchaProcessor(pkg.select_graph(0), budget, 0, 8, 6, True)
        n0 = _spec_launches(pkg)
        got, want = _run(pkg, O, GP, P_SPEC, 6)
        assert np.array_equal(_u32(got), _u32(want))
        active = int(np.asarray(GP.active_flags, np.uint8)[:6].any(axis=1).sum())
        assert _spec_launches(pkg) - n0 == (active if spec else 0)
    finally:
        E.set_mix_tuning(**saved)


def test_need_mask_is_the_plan_row_set(pkg):
    """need_host[t] bit r <=> the plan record gives local row r a degree > 0 (every row of an active
    round with idle_rows = "canonical"), for every schedule round and an adhoc round."""
    np.random.seed(7)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, 8, 40, True)
    for idle in ("skip", "canonical"):
        eng = pkg.GossipEngine(GP, idle_rows=idle)
        W = eng.plan_words
        plan = eng.plan.cpu().numpy().reshape(eng.T + 1, W)
        for t in range(eng.T):
            deg = plan[t, 4:4 + eng.n_local]
            rows = (deg > 0) | (idle == "canonical" and bool(eng.flags_host[t].any()))
            want = sum(1 << r for r in range(eng.n_local) if rows[r] and plan[t, 0])
            assert int(eng.need_host[t]) == want, (idle, t)
        t = eng.adhoc([1, 0, 0, 1, 0])
        torch.cuda.synchronize()
        deg = eng.plan.cpu().numpy().reshape(eng.T + 1, W)[t, 4:4 + eng.n_local]
        rows = (deg > 0) | (idle == "canonical")
        assert int(eng.need_host[t]) == sum(1 << r for r in range(eng.n_local) if rows[r])


@pytest.mark.parametrize("how,glds", [("none", 1), ("all", 1), ("flip", 1), ("random", 1), ("flip", 0), ("random", 0)])
def test_wrong_hint_same_bits(pkg, O, how, glds):
    """The hint steers loads only: a mask with rows missing, extra, all or none gives the oracle's
    bits (missing rows are loaded after the plan record, extra ones are dropped unparked)."""
    rng = np.random.RandomState(3)
    scramble = {"none": lambda m: np.zeros_like(m),
                "all": lambda m: np.full_like(m, 0xFF),
                "flip": lambda m: m ^ np.uint64(0xFF),
                "random": lambda m: rng.randint(0, 256, size=m.shape).astype(np.uint64)}[how]
    E = pkg.engine
    saved = E.mix_tuning()
    try:
        E.set_mix_tuning(spec=1, spec_wgpc=5, spec_glds=glds)
        np.random.seed(99)
        GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, 8, 5, True)
        got, want = _run(pkg, O, GP, P_SPEC, 5, scramble=scramble)
        assert np.array_equal(_u32(got), _u32(want))
    finally:
        E.set_mix_tuning(**saved)


def test_spec_canonical_idle_rows(pkg, O):
    """idle_rows = "canonical" (every row of an active round streamed, -0.0 -> +0.0 like the
    reference) through the SPEC form."""
    E = pkg.engine
    saved = E.mix_tuning()
    try:
        E.set_mix_tuning(spec=1, spec_wgpc=5)
        np.random.seed(5)
        GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.4, 0, 8, 5, True)
        n0 = _spec_launches(pkg)
        got, want = _run(pkg, O, GP, P_SPEC, 5, idle_rows="canonical")
        assert _spec_launches(pkg) > n0
        assert np.array_equal(_u32(got), _u32(want))
    finally:
        E.set_mix_tuning(**saved)


@pytest.mark.parametrize("order", ["tree", "sequential"])
def test_mean_capped_matches_oracle(pkg, O, order):
    """mx_mean_rows_to on 8 x 2.5M in place (> 64 MB: the capped launch) at mean_wgpc 0 / 2 / 3 / 5:
    every destination row equals the oracle's reference-order mean."""
    L = pkg.lib
    E = pkg.engine
    saved = E.mix_tuning()
    n, P = 8, P_BIG
    ld = (P + 63) // 64 * 64
    X = np.stack([O.synth(500 + i, P) * np.float32(1 + i % 3) for i in range(n)])
    want = O.central_mean(X, order)
    code = {"tree": 0, "sequential": 1}[order]
    try:
        for w in (0, 2, 3, 5):
            E.set_mix_tuning(mean_wgpc=w)
            rows = torch.zeros((n, ld), dtype=torch.float32, device="cuda")
            rows[:, :P] = torch.from_numpy(X).cuda()
            pkg._lib.check(L.mx_mean_rows_to(rows.data_ptr(), n, ld, P, code, rows.data_ptr(), n, ld,
                                             pkg._lib.stream_ptr()), "mx_mean_rows_to")
            torch.cuda.synchronize()
            got = rows[:, :P].cpu().numpy()
            for d in range(n):
                assert np.array_equal(_u32(got[d]), _u32(want)), (w, d)
    finally:
        E.set_mix_tuning(**saved)


def test_occupancy_knobs_roundtrip(pkg):
    """spec / spec_wgpc / mean_wgpc are readable, settable and range-checked."""
    L = pkg.lib
    E = pkg.engine
    saved = E.mix_tuning()
    try:
        for k, v in (("spec", 0), ("spec", 1), ("spec_wgpc", 0), ("spec_wgpc", 7), ("spec_glds", 0), ("spec_glds", 1),
                     ("mean_wgpc", 4)):
            assert L.mx_mix_set(k.encode(), v) == 0 and L.mx_mix_get(k.encode()) == v
        assert L.mx_mix_set(b"spec_wgpc", 33) != 0 and L.mx_mix_set(b"mean_wgpc", -1) != 0
    finally:
        E.set_mix_tuning(**saved)


def test_spec_not_with_receive_slots(pkg, O):
    """A group with receive slots (N > 1: partners on another rank, here 2 ranks' engines on one GPU
    over the loopback transport) keeps the uncapped launch -- no SPEC launch -- and the oracle's bits."""
    from conftest import LoopbackHub, Topo
    E = pkg.engine
    saved = E.mix_tuning()
    n, P = 8, 12_000_001
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    flags = np.ones((2, M), np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    try:
        E.set_mix_tuning(spec=1, spec_wgpc=5)
        hub = LoopbackHub(2)
        groups = [pkg.VirtualWorkerGroup(topo, numel=P, rank=r, nranks=2, comm=hub.comm(r)) for r in range(2)]
        assert all(g.engine.n_slots > g.n_local for g in groups)
        X = np.stack([O.synth(900 + i, P) for i in range(n)])
        for g in groups:
            g.rows.copy_(torch.from_numpy(X[g.row_base:g.row_base + g.n_local]))
            hub.register(g.row_base, g._row_ptrs)
        n0 = _spec_launches(pkg)
        for it, f in enumerate(flags):
            for g in groups:
                g.step(it)
            torch.cuda.synchronize()
            X = O.decen_round(X, topo.neighbors_info, f, 2 / 7)
        assert _spec_launches(pkg) == n0
        got = np.concatenate([g.rows.cpu().numpy() for g in groups])
        assert np.array_equal(_u32(got), _u32(X))
    finally:
        E.set_mix_tuning(**saved)


@pytest.mark.parametrize("base,glds", [(0, 1), (1, 1), (0, 0)])
def test_spec_multisegment_layouts(pkg, O, base, glds):
    """The SPEC form on a pointer-table layout of ragged tensors (adopted models: one segment per
    tensor), > 320 MB per round: segment starts 16-byte aligned (LDS-DMA except the waves past each
    segment's end) or all shifted by 4 bytes (every slot through registers), 3 rounds of graph 0 with
    partial flags vs the oracle."""
    E = pkg.engine
    saved = E.mix_tuning()
    n = 8
    lens = [4, 5_000_000, 1028, 12, 5_499_992, 64]          # multiples of 4: aligned starts at base 0
    P = sum(lens)
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    flags = np.ones((3, M), np.uint8)
    flags[1, 1::2] = 0
    flags[2, ::3] = 0
    from conftest import Topo
    topo = Topo(gp.neighbors_info, 0.21, flags)
    try:
        E.set_mix_tuning(spec=1, spec_wgpc=5, spec_glds=glds)
        eng = pkg.GossipEngine(topo)
        X = np.stack([O.synth(800 + i, P) for i in range(n)])
        big = torch.zeros((n, P + 8), dtype=torch.float32, device="cuda")
        big[:, base:base + P] = torch.from_numpy(X).cuda()
        cuts = np.cumsum([0] + lens)
        ptrs = [[big[i].data_ptr() + 4 * (base + int(cuts[s])) for s in range(len(lens))] for i in range(n)]
        lay = pkg.Layout(lens, ptrs, eng.n_slots)
        n0 = _spec_launches(pkg)
        for it, f in enumerate(flags):
            eng.mix(it, lay)
            X = O.decen_round(X, topo.neighbors_info, f, 0.21)
        torch.cuda.synchronize()
        assert _spec_launches(pkg) - n0 == len(flags)
        got = big[:, base:base + P].cpu().numpy()
        assert np.array_equal(_u32(got), _u32(X))
    finally:
        E.set_mix_tuning(**saved)
