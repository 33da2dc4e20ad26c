"""GPU: the reference communicators' sub-steps driven directly -- prepare_comm_buffer(),
averaging(active_flags), reset_model() (communicator.py:87-131, 175-240) -- as a caller that
does not go through communicate() would: a `tensor_list` of `param.data` aliases (copied into the
arena row, and back), flags rows from the schedule and rows the schedule never drew (a scratch
plan record, GossipEngine.adhoc), 8 ranks in one process over the loopback transport.  Bit-exact
against the oracle's rounds.

Reference: communicator.py:79-268."""
import numpy as np
import pytest

from conftest import LoopbackHub

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _models(n, dev, seed=3):
    torch.manual_seed(seed)
    return [torch.nn.Sequential(torch.nn.Linear(20, 31), torch.nn.Tanh(), torch.nn.Linear(31, 3)).to(dev)
            for _ in range(n)]


def _flat(models):
    return np.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy() for m in models])


def _rows(GP, seed, rounds):
    """schedule rows and rows the schedule did not draw (random, all-ones, all-zero: the
    reference's averaging() with no active matching still applies the worker's own terms --
    Choco's own q -- where communicate() would have skipped the round)."""
    rng = np.random.RandomState(seed)
    M = len(GP.neighbors_info)
    out = []
    for t in range(rounds):
        if t % 4 == 0:
            out.append(("schedule", t, np.asarray(GP.active_flags[t], np.uint8)))
        elif t % 4 == 1:
            out.append(("adhoc", t, (rng.uniform(size=M) < 0.5).astype(np.uint8)))
        elif t % 4 == 2:
            out.append(("adhoc", t, np.ones(M, np.uint8)))
        else:
            out.append(("adhoc", t, np.zeros(M, np.uint8)))
    return out


@pytest.mark.parametrize("dev", ["cuda", "cpu"])
def test_decen_substeps_tensor_list(pkg, O, dev):
    n = 8
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, 12, True)
    models = _models(n, dev)
    X = _flat(models)
    hub = LoopbackHub(n)
    comms = [pkg.decenCommunicator(r, n, GP, transport=hub.comm(r)) for r in range(n)]
    partner = np.asarray(GP.neighbors_info, np.int32)
    for kind, t, f in _rows(GP, 5, 10):
        for r in range(n):
            if kind == "schedule":
                comms[r].iter = t + 1                  # as communicate() leaves it before averaging
            comms[r].tensor_list = [p.data for p in models[r].parameters()]
            comms[r].prepare_comm_buffer()
            sb = comms[r].send_buffer
            assert sb.device.type == "cuda" and sb.numel() == X.shape[1]
            assert np.array_equal(sb.cpu().numpy().view(np.uint32), X[r].view(np.uint32))
            hub.register(r, [comms[r]._group.rows[0].data_ptr()])
        hub.snap.clear()                               # adhoc rounds share one plan index (T)
        for r in range(n):
            assert comms[r].averaging(f) >= 0
            assert comms[r].recv_buffer is comms[r].send_buffer
            comms[r].reset_model()
        if f.any():
            X = O.decen_round(X, partner, f, GP.neighbor_weight)
        assert np.array_equal(_flat(models).view(np.uint32), X.view(np.uint32)), (kind, t)
    assert all(p.device.type == dev for m in models for p in m.parameters())


def test_decen_substeps_after_communicate_in_place(pkg, O):
    """After communicate(model) adopted the parameters into the row, a tensor_list of their
    .data aliases the row: prepare / reset copy nothing and the round still matches."""
    n = 8
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, 6, True)
    models = _models(n, "cuda", 4)
    X = _flat(models)
    hub = LoopbackHub(n)
    comms = [pkg.decenCommunicator(r, n, GP, transport=hub.comm(r)) for r in range(n)]
    for r in range(n):
        comms[r]._bind(models[r])
        comms[r]._stage.load()
        hub.register(r, [comms[r]._group.rows[0].data_ptr()])
    partner = np.asarray(GP.neighbors_info, np.int32)
    for r in range(n):
        comms[r].communicate(models[r])
    X = O.decen_round(X, partner, np.asarray(GP.active_flags[0], np.uint8), GP.neighbor_weight)
    f = np.zeros(len(GP.neighbors_info), np.uint8)
    f[1] = 1
    hub.snap.clear()
    for r in range(n):
        comms[r].tensor_list = [p.data for p in models[r].parameters()]
        comms[r].prepare_comm_buffer()
        assert comms[r]._list_stage.adopted()          # in place: the aliases live in the row
    for r in range(n):
        comms[r].averaging(f)
        comms[r].reset_model()
    X = O.decen_round(X, partner, f, GP.neighbor_weight)
    assert np.array_equal(_flat(models).view(np.uint32), X.view(np.uint32))


def test_choco_substeps_tensor_list(pkg, O):
    """Choco: prepare_comm_buffer() returns the encode seconds and exposes `compressed` (the
    oracle's top-k of x - x_hat), averaging(flags) with schedule / undrawn / all-ones rows, x_hat
    and s persisting between calls."""
    n, ratio, lr = 8, 0.9, 0.3
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, 12, True)
    models = _models(n, "cuda", 5)
    X = _flat(models)
    P = X.shape[1]
    XH, S = np.zeros_like(X), np.zeros_like(X)
    k = O.topk_k(P, ratio)
    hub = LoopbackHub(n)
    comms = [pkg.ChocoCommunicator(r, n, GP, ratio, lr, transport=hub.comm(r)) for r in range(n)]
    partner = np.asarray(GP.neighbors_info, np.int32)
    for kind, t, f in _rows(GP, 6, 8):
        for r in range(n):
            if kind == "schedule":
                comms[r].iter = t + 1
            comms[r].tensor_list = [p.data for p in models[r].parameters()]
            assert comms[r].prepare_comm_buffer() >= 0
            ov, oi = O.topk_abs(X[r] - XH[r], k)
            c = comms[r].compressed
            assert np.array_equal(c["indices"].cpu().numpy(), oi)
            assert np.array_equal(c["values"].cpu().numpy().view(np.uint32), ov.view(np.uint32))
            hub.register(r, [comms[r]._group.msgs.data_ptr()])
        hub.snap.clear()
        for r in range(n):
            assert comms[r].averaging(f) >= 0
            comms[r].reset_model()
        O.choco_round(X, XH, S, partner, f, GP.neighbor_weight, k, lr, skip_empty=False)
        assert np.array_equal(_flat(models).view(np.uint32), X.view(np.uint32)), (kind, t)
        for r in range(n):
            assert np.array_equal(comms[r].x_hat.cpu().numpy().view(np.uint32), XH[r].view(np.uint32))
            assert np.array_equal(comms[r].s.cpu().numpy().view(np.uint32), S[r].view(np.uint32))


@pytest.mark.parametrize("kind", ["decen", "choco"])
def test_substeps_vs_reference_fixture(pkg, kind):
    """The reference's own sub-step run (tests/golden/substeps.npz: tensor_list, prepare_comm_buffer,
    averaging(flags), reset_model per given flags row, incl. an all-zero row) replayed through the
    drop-in communicators with the reference's CPU models (staged to the GPU and back), 8 ranks
    over the loopback transport: every round's parameters, and Choco's final x_hat / s, bit-exact."""
    from conftest import golden_json, golden_npz
    g, m = golden_npz("substeps"), golden_json("substeps")
    n, shapes = m["size"], [tuple(s) for s in m["shapes"]]
    np.random.seed(1234)
    GP = pkg.FixedProcessor(pkg.select_graph(0), 0.5, 0, n, 10, True)
    assert np.array_equal(np.asarray(GP.neighbors_info, np.int32), g["partner"])
    X0 = g[f"{kind}_X0"]
    models = []
    for r in range(n):
        ps, off = [], 0
        for s in shapes:
            k = int(np.prod(s))
            ps.append(torch.nn.Parameter(torch.from_numpy(X0[r, off:off + k].copy()).view(*s)))
            off += k
        mod = torch.nn.Module()
        mod.ps = torch.nn.ParameterList(ps)
        models.append(mod)
    hub = LoopbackHub(n)
    if kind == "decen":
        comms = [pkg.decenCommunicator(r, n, GP, transport=hub.comm(r)) for r in range(n)]
    else:
        comms = [pkg.ChocoCommunicator(r, n, GP, m["ratio"], m["consensus_lr"], transport=hub.comm(r))
                 for r in range(n)]
    for t, f in enumerate(g["flags"]):
        for r in range(n):
            comms[r].tensor_list = [p.data for p in models[r].parameters()]
            comms[r].prepare_comm_buffer()
            hub.register(r, [comms[r]._group.rows[0].data_ptr() if kind == "decen" else comms[r]._group.msgs.data_ptr()])
        hub.snap.clear()
        for r in range(n):
            comms[r].averaging(f)
            comms[r].reset_model()
        got = _flat(models)
        assert np.array_equal(got.view(np.uint32), g[f"{kind}_Y"][t].view(np.uint32)), t
    if kind == "choco":
        xh = np.stack([c.x_hat.cpu().numpy() for c in comms])
        s = np.stack([c.s.cpu().numpy() for c in comms])
        assert np.array_equal(xh.view(np.uint32), g["choco_xhat"].view(np.uint32))
        assert np.array_equal(s.view(np.uint32), g["choco_s"].view(np.uint32))


def test_decen_substeps_fixed_schedule_rows(pkg, O):
    """FixedProcessor's rows have two entries (graph_manager.py:208-225): averaging() takes them as
    the reference does (matchings 0 and 1), from the schedule and as given rows alike."""
    n = 8
    np.random.seed(7)
    GP = pkg.FixedProcessor(pkg.select_graph(0), 0.5, 0, n, 6, True)
    assert len(GP.active_flags[0]) == 2 and len(GP.neighbors_info) > 2
    models = _models(n, "cuda", 6)
    X = _flat(models)
    hub = LoopbackHub(n)
    comms = [pkg.decenCommunicator(r, n, GP, transport=hub.comm(r)) for r in range(n)]
    partner = np.asarray(GP.neighbors_info, np.int32)
    for t in range(4):
        f = list(GP.active_flags[t]) if t % 2 == 0 else [1, 1]
        for r in range(n):
            comms[r].iter = t + 1
            comms[r].tensor_list = [p.data for p in models[r].parameters()]
            comms[r].prepare_comm_buffer()
            hub.register(r, [comms[r]._group.rows[0].data_ptr()])
        hub.snap.clear()
        for r in range(n):
            comms[r].averaging(f)
            comms[r].reset_model()
        full = np.zeros(len(partner), np.uint8)
        full[:2] = f
        X = O.decen_round(X, partner, full, GP.neighbor_weight)
        assert np.array_equal(_flat(models).view(np.uint32), X.view(np.uint32)), t
