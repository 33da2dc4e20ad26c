"""Signed zeros and NaN payloads through a gossip round (VERDICT r01 "-0.0 deviation").

The reference's averaging (communicator.py:113-117) starts every worker's receive buffer at
+0.0 and adds fma(alpha, x_j, recv) per active partner, then fma(1 - d*alpha, x_i, recv).  Two
observable consequences:
  * a worker WITH partners: -0.0 inputs come out as the FMA chain gives them (alpha * -0.0 +
    0.0 = +0.0, ...) -- the kernel starts its chain from +0.0 too, so it is bit-exact;
  * a worker with NO active partner in an active round still runs the chain with d = 0:
    0 + 1.0 * x, which is x except that -0.0 -> +0.0 (and a signalling NaN is quieted).
    idle_rows="skip" (default) leaves such rows untouched (no HBM traffic; equal under IEEE ==);
    idle_rows="canonical" rewrites them and is bit-identical to the reference.
NaN inputs stay NaN; their payload bits are not compared (CPU libm fmaf and the GPU's v_fma_f32
need not agree on the payload of a propagated NaN).
"""
import numpy as np
import pytest

from conftest import Topo

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

QNAN = np.array([0x7FC01234], np.uint32).view(np.float32)[0]
SNAN = np.array([0x7F805678], np.uint32).view(np.float32)[0]


def _inputs(O, n, P, X=None):
    """synthetic rows (or X) with signed zeros and NaN payloads written in"""
    X = np.stack([O.synth(4321 + i, P) for i in range(n)]) if X is None else X.copy()
    X[:, ::5] = np.float32(-0.0)
    X[:, 1::7] = np.float32(0.0)
    X[:, 3::1001] = QNAN
    X[:, 4::997] = SNAN
    X[2, 10:20] = np.float32(-0.0)
    return X


def _flags_with_idle(partner):
    """rounds: every matching; one matching (leaves idle workers); two matchings."""
    M, n = partner.shape
    single = min(range(M), key=lambda g: int((partner[g] >= 0).sum()))
    f1 = np.zeros(M, np.uint8)
    f1[single] = 1
    f2 = np.zeros(M, np.uint8)
    f2[[0, M - 1]] = 1
    return np.stack([np.ones(M, np.uint8), f1, f2]), single


def _same(a, b):
    """bit-equal where neither is NaN, NaN where either is"""
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32)))


@pytest.mark.parametrize("idle_rows", ["skip", "canonical"])
def test_signed_zero_and_nan_rounds(pkg, O, idle_rows):
    n, P = 8, 70_001
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    partner = np.asarray(gp.neighbors_info, np.int32)
    flags, single = _flags_with_idle(partner)
    idle = [i for i in range(n) if partner[single, i] < 0]
    assert idle, "the one-matching round must leave some worker idle"
    topo = Topo(partner, 0.2857142857142856, flags)
    X = _inputs(O, n, P)
    grp = pkg.VirtualWorkerGroup(topo, numel=P, idle_rows=idle_rows)
    for t, f in enumerate(flags):
        X = _inputs(O, n, P, X)                       # fresh -0.0 / NaN inputs every round
        grp.rows.copy_(torch.from_numpy(X))
        grp.communicate()
        got = grp.rows.cpu().numpy()
        want = O.decen_round(X, partner, f, topo.neighbor_weight)
        deg = (partner[f.astype(bool)] >= 0).sum(axis=0)
        for i in range(n):
            if deg[i] > 0 or idle_rows == "canonical":
                assert _same(got[i], want[i]), f"round {t} worker {i}"
            else:                                     # skipped: the input bits, untouched
                assert np.array_equal(got[i].view(np.uint32), X[i].view(np.uint32)), f"round {t} worker {i}"
                # ... and the reference differs exactly at the -0.0 (and signalling NaN) inputs
                negz = (X[i].view(np.uint32) == 0x80000000)
                assert np.all(want[i][negz].view(np.uint32) == 0)
                keep = ~negz & ~np.isnan(X[i])
                assert np.array_equal(want[i][keep].view(np.uint32), X[i][keep].view(np.uint32))
        if t == 1:
            assert (deg == 0).any()
            if idle_rows == "canonical":
                for i in idle:                        # -0.0 inputs of idle workers are now +0.0
                    negz = (X[i].view(np.uint32) == 0x80000000)
                    assert negz.any() and np.all(got[i][negz].view(np.uint32) == 0)
        X = got.copy()


def test_signed_zero_choco_round(pkg, O):
    """ChocoSGD with -0.0 / +0.0 in x (and an idle worker, which the reference still updates with
    its own message): x, x_hat, s bit-exact vs the oracle (no NaNs: top-k of NaN magnitudes is
    undefined in torch.topk)."""
    n, P, ratio = 8, 50_003, 0.9
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    partner = np.asarray(gp.neighbors_info, np.int32)
    flags, _ = _flags_with_idle(partner)
    topo = Topo(partner, 2 / 7, flags)
    X = np.stack([O.synth(99 + i, P) for i in range(n)])
    X[:, ::3] = np.float32(-0.0)
    X[:, 1::4] = np.float32(0.0)
    XH, S = np.zeros_like(X), np.zeros_like(X)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.2)
    grp.rows.copy_(torch.from_numpy(X))
    k = O.topk_k(P, ratio)
    for t, f in enumerate(flags):
        grp.communicate()
        O.choco_round(X, XH, S, partner, f, 2 / 7, k, 0.2)
        assert np.array_equal(grp.rows.cpu().numpy().view(np.uint32), X.view(np.uint32)), f"x round {t}"
        assert np.array_equal(grp.x_hat[:, :P].cpu().numpy().view(np.uint32), XH.view(np.uint32))
        assert np.array_equal(grp.s[:, :P].cpu().numpy().view(np.uint32), S.view(np.uint32))


def test_idle_rows_mode_validation(pkg):
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
    topo = Topo(gp.neighbors_info, 0.25, np.ones((2, 5), np.uint8))
    with pytest.raises(ValueError):
        pkg.VirtualWorkerGroup(topo, numel=100, idle_rows="zero")
