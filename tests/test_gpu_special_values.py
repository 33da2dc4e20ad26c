"""GPU: non-finite and edge values (quiet NaNs of both signs and two payloads, +-Inf, +-0,
denormals, +-FLT_MAX; tests/conftest.special_values) through the product kernels, against the
oracle -- whose top-k semantics for them are pinned to torch.topk / torch.max, the calls
compressors.get_top_k makes (tests/test_special_values_cpu.py).  Equality is bitwise except that
a NaN only has to meet a NaN (the payload an IEEE operation returns for NaN inputs is not
specified the same way on the host and the GPU).

Reference: compressors.py:3-19 (top-k), communicator.py:92-122 (mixing), :200-230 (Choco)."""
import numpy as np
import pytest

from conftest import Topo, special_values

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return a.shape == b.shape and np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.mark.parametrize("P,ratio,with_hat", [(20_000, 0.99, False), (4_099, 0.99, True), (2_000_003, 0.99, True),
                                              (1_000_000, 0.5, False)])
def test_topk_special_values_vs_oracle(pkg, O, P, ratio, with_hat):
    """The one-row top-k (sampling, compaction, candidate passes) with NaN / Inf keys at the top of
    every histogram; x_hat (when given) finite, so x - x_hat keeps the planted values."""
    x = special_values(P, P)
    xh = (np.random.default_rng(P).standard_normal(P).astype(np.float32) * np.float32(0.1)) if with_hat else None
    d = x - xh if with_hat else x
    k = O.topk_k(P, ratio)
    ov, oi = O.topk_abs(d, k)
    L = pkg.lib
    xd = torch.from_numpy(x).cuda()
    hd = torch.from_numpy(xh).cuda() if with_hat else None
    vals = torch.empty(k, dtype=torch.float32, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    work = torch.zeros(int(L.mx_topk_work_bytes(P)), dtype=torch.uint8, device="cuda")
    pkg._lib.check(L.mx_topk_abs_diff(xd.data_ptr(), hd.data_ptr() if with_hat else None, P, k, vals.data_ptr(),
                                      idx.data_ptr(), work.data_ptr(), None), "mx_topk_abs_diff")
    assert L.mx_topk_check(work.data_ptr(), 0, 1, P, None) == 0, L.mx_last_error()
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert _same(vals.cpu().numpy(), ov)
    assert np.isnan(d[oi]).sum() == 5 and np.isinf(d[oi]).sum() == 4


def test_get_top_k_special_values_k1(pkg, O):
    """k = 1 (torch.max in the reference): the single NaN wins over +-Inf and FLT_MAX."""
    x = special_values(50_000, 21, n_nan=1, n_inf=2)
    v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), 1 - 1.5 / 50_000)
    _, oi = O.topk_abs(x, 1)
    assert np.array_equal(i.cpu().numpy(), oi) and np.isnan(v.cpu().numpy()[0])


def test_mix_special_values_vs_oracle(pkg, O):
    """Three full / partial rounds of graph 0 over rows holding NaN / Inf / denormal / FLT_MAX
    entries: the FMA chain spreads them to partners exactly as the oracle's does (Inf - Inf and
    0 * Inf give NaN in both)."""
    n, P = 8, 70_001
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    flags = np.ones((3, M), np.uint8)
    flags[1, ::2] = 0
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    X = np.stack([special_values(P, 300 + i) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X))
    for f in flags:
        grp.communicate()
        X = O.decen_round(X, topo.neighbors_info, f, 2 / 7)
        assert _same(grp.rows.cpu().numpy(), X)
    assert np.isnan(X).any() and np.isinf(X).any()


def test_choco_special_values_vs_oracle(pkg, O):
    """Three Choco rounds (top-1 %, 8 workers) with non-finite entries in x: x / x_hat / s equal to
    the oracle's, NaN-for-NaN, as the NaNs are selected, compressed, exchanged and applied."""
    n, P, ratio = 8, 200_003, 0.99
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 1, 0, 1], [0, 1, 1, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
    X = np.stack([special_values(P, 700 + i) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X))
    k = O.topk_k(P, ratio)
    for t, f in enumerate(flags):
        grp.communicate()
        O.choco_round(X, XH, S, topo.neighbors_info, f, 2 / 7, k, 0.1)
        assert _same(grp.rows.cpu().numpy(), X), f"x, round {t}"
        assert _same(grp.x_hat[:, :P].cpu().numpy(), XH), f"x_hat, round {t}"
        assert _same(grp.s[:, :P].cpu().numpy(), S), f"s, round {t}"
    assert np.isnan(X).any()


def test_get_top_k_special_values_vs_reference_fixture(pkg):
    """get_top_k (the product path, compressors.py's API) on the reference's own special-value
    cases (tests/golden/topk_special.npz): the same index sets, values x[idx] bit for bit."""
    from conftest import golden_json, golden_npz
    g = golden_npz("topk_special")
    for c, m in enumerate(golden_json("topk_special")):
        x = g[f"case{c}_x"]
        v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), m["ratio"])
        assert np.array_equal(i.cpu().numpy(), g[f"case{c}_idx"]), m
        assert np.array_equal(v.cpu().numpy().view(np.uint32), x[g[f"case{c}_idx"]].view(np.uint32)), m
