"""GPU: the training harness drives the gossip path exactly (every round vs the oracle), and
checkpoints resume on the same schedule."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _args(pkg, **kw):
    base = dict(size=8, epoch=2, bs=16, budget=0.5, graphid=0, lr=0.1)
    base.update(kw)
    return pkg.harness.HarnessArgs(**base)


@pytest.mark.parametrize("matcha,batched", [(True, False), (False, False), (True, True)])
def test_virtual_trainer_rounds_match_oracle(pkg, O, matcha, batched):
    """Every communicate() of the harness is one reference gossip round of the post-step rows."""
    H = pkg.harness
    args = _args(pkg, matcha=matcha)
    tr = H.VirtualTrainer(args, H.model_factory(args), n_batches=3, batched=batched)
    GP = tr.GP
    partner = np.asarray(GP.neighbors_info, np.int32)
    seen = {"rounds": 0}
    rows0 = tr.group.rows.cpu().numpy()
    assert all(np.array_equal(rows0[0], rows0[r]) for r in range(8))      # sync_allreduce
    state = {}

    def hook(when, t):
        if when == "before":
            state["X"] = t.group.rows.cpu().numpy().copy()
            state["it"] = t.group.iter
            return
        it = state["it"]
        flags = np.asarray(GP.active_flags[it], np.uint8)
        M = len(flags)
        want = O.decen_round(state["X"], partner[:M], flags, GP.neighbor_weight) if flags.any() else state["X"]
        got = t.group.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"round {it}"
        seen["rounds"] += 1

    for _ in range(args.epoch):
        stats = tr.train_epoch(on_round=hook)
        assert len(stats) == 8 and all(np.isfinite(s["loss"]) for s in stats)
    assert seen["rounds"] == 6 and tr.group.iter == 6
    # parameters are views into the arena: the models see the mixed values
    p0 = next(tr.models[3].parameters())
    assert p0.data.data_ptr() >= tr.group.arena.data_ptr()


def test_virtual_trainer_choco_rounds_match_oracle(pkg, O):
    H = pkg.harness
    args = _args(pkg, compress=True, budget=1.0, ratio=0.9)
    tr = H.VirtualTrainer(args, H.model_factory(args), n_batches=2)
    GP = tr.GP
    partner = np.asarray(GP.neighbors_info, np.int32)
    P = tr.group.numel
    XH = np.zeros((8, P), np.float32)
    S = np.zeros((8, P), np.float32)
    st = {}

    def hook(when, t):
        if when == "before":
            st["X"] = t.group.rows.cpu().numpy().copy()
            st["it"] = t.group.iter
            return
        flags = np.asarray(GP.active_flags[st["it"]], np.uint8)
        X = st["X"]
        O.choco_round(X, XH, S, partner[:len(flags)], flags, GP.neighbor_weight, t.group.k, args.consensus_lr)
        assert np.array_equal(t.group.rows.cpu().numpy().view(np.uint32), X.view(np.uint32))

    for _ in range(args.epoch):
        tr.train_epoch(on_round=hook)
    assert np.array_equal(tr.group.x_hat[:, :P].cpu().numpy(), XH)
    assert np.array_equal(tr.group.s[:, :P].cpu().numpy(), S)


@pytest.mark.parametrize("compress", [False, True])
def test_checkpoint_resume_same_schedule(pkg, tmp_path, compress):
    H = pkg.harness
    args = _args(pkg, compress=compress, epoch=2, budget=0.5)
    a = H.VirtualTrainer(args, H.model_factory(args), n_batches=3)
    a.train_epoch()
    path = str(tmp_path / "ckpt.pt")
    a.save(path)
    a.train_epoch()
    b = H.VirtualTrainer(args, H.model_factory(args), n_batches=3)
    b.load(path)
    assert b.group.iter == 3 and b.epoch == 1
    b.train_epoch()
    assert b.group.iter == a.group.iter == 6
    ra, rb = a.group.rows, b.group.rows
    assert torch.allclose(ra, rb, rtol=0, atol=1e-6), float((ra - rb).abs().max())
    with pytest.raises(ValueError):
        wrong = H.HarnessArgs(size=8, epoch=1, bs=16, graphid=0, compress=compress, num_classes=10)
        c = H.VirtualTrainer(wrong, H.model_factory(wrong), n_batches=1)
        c.load(path)


def test_recorder_through_trainer(pkg, tmp_path):
    H = pkg.harness
    args = _args(pkg, save=True, savePath=str(tmp_path) + "/", epoch=1)
    tr = H.VirtualTrainer(args, H.model_factory(args), n_batches=2)
    tr.train_epoch()
    tr.finish()
    import os
    files = os.listdir(str(tmp_path / (args.name + "_mlp")))
    assert len([f for f in files if f.endswith(".log")]) == 7 * 8


@pytest.mark.parametrize("momentum,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_batched_step_matches_per_worker_sgd(pkg, momentum, nesterov):
    """The vmap'd all-worker step gives each worker what its own torch.optim.SGD step gives
    (gradients via one batched backward: equal to fp32 rounding of the GEMM reductions)."""
    H = pkg.harness
    args = _args(pkg, momentum=momentum, nesterov=nesterov, epoch=2, lr=0.05)
    seq = H.VirtualTrainer(args, H.model_factory(args), n_batches=2)
    bat = H.VirtualTrainer(args, H.model_factory(args), n_batches=2, batched=True)
    assert torch.equal(seq.group.rows, bat.group.rows)
    for _ in range(2):
        seq.train_epoch()
        bat.train_epoch()
    assert torch.allclose(seq.group.rows, bat.group.rows, rtol=1e-4, atol=1e-6), \
        float((seq.group.rows - bat.group.rows).abs().max())


@pytest.mark.parametrize("momentum,nesterov,matcha,compress", [(0.0, False, True, False), (0.9, False, True, False),
                                                               (0.9, True, False, False), (0.0, False, True, True),
                                                               (0.9, False, True, True)])
def test_graph_mode_identical_to_batched(pkg, momentum, nesterov, matcha, compress):
    """graph=True replays one captured HIP graph per learning rate (forward / backward / SGD +
    the gossip round at the device counter): rows, per-worker losses / accuracies and the
    iteration counter equal the eager batched trainer's exactly."""
    H = pkg.harness
    args = _args(pkg, momentum=momentum, nesterov=nesterov, epoch=3, lr=0.05, matcha=matcha, compress=compress,
                 ratio=0.9, budget=0.3 if compress else 0.5)
    eag = H.VirtualTrainer(args, H.model_factory(args), n_batches=4, batched=True)
    gra = H.VirtualTrainer(args, H.model_factory(args), n_batches=4, batched=True, graph=True)
    for e in range(3):
        se = eag.train_epoch()
        sg = gra.train_epoch()
        assert torch.equal(eag.group.rows, gra.group.rows), f"epoch {e}"
        if compress:
            assert torch.equal(eag.group.x_hat, gra.group.x_hat) and torch.equal(eag.group.s, gra.group.s)
        assert [s["loss"] for s in se] == [s["loss"] for s in sg]
        assert [s["train_acc"] for s in se] == [s["train_acc"] for s in sg]
    assert eag.group.iter == gra.group.iter == 12
    assert len(gra._graphs) == 1


@pytest.mark.parametrize("compress", [False, True])
def test_graph_mode_checkpoint_reload(pkg, compress):
    """Loading a checkpoint into a graph-mode trainer whose graphs are already captured: the
    replays continue from the loaded iteration counter and momentum (loaded in place into the
    captured buffers), so the next epoch equals the eager batched trainer's from the same state."""
    H = pkg.harness
    args = _args(pkg, momentum=0.9, epoch=4, lr=0.05, compress=compress, ratio=0.9, budget=0.5)
    eag = H.VirtualTrainer(args, H.model_factory(args), n_batches=3, batched=True)
    gra = H.VirtualTrainer(args, H.model_factory(args), n_batches=3, batched=True, graph=True)
    for _ in range(2):
        eag.train_epoch()
        gra.train_epoch()
    ckpt = {k: v for k, v in gra.state_dict().items()}
    gra.train_epoch()                       # moves iter / momentum / rows past the checkpoint
    gra.load_state_dict(ckpt)
    assert gra.group.iter == 6 and gra.epoch == 2
    se = eag.train_epoch()
    sg = gra.train_epoch()
    assert torch.equal(eag.group.rows, gra.group.rows)
    if compress:
        assert torch.equal(eag.group.x_hat, gra.group.x_hat) and torch.equal(eag.group.s, gra.group.s)
    assert [s["loss"] for s in se] == [s["loss"] for s in sg]
    assert len(gra._graphs) == 1            # reused, not recaptured


@pytest.mark.parametrize("order", [0, 1])
def test_sync_rows_reference_order_mean(pkg, order):
    """sync_allreduce for arena rows: every row = (tree / rank-order sum) / n via mx_mean_rows."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from reforder import mpi4py_sum
    arena = torch.zeros((5, 1088), dtype=torch.float32, device="cuda")
    rows = arena[:, :1000]
    host = [np.random.RandomState(r).standard_normal(1000).astype(np.float32) * np.float32(10.0 ** r)
            for r in range(5)]
    rows.copy_(torch.from_numpy(np.stack(host)))
    pkg.harness.sync_rows(rows, order=order)
    want = mpi4py_sum(host, "tree" if order == 0 else "sequential") / np.float32(5)
    got = rows.cpu().numpy()
    for r in range(5):
        assert np.array_equal(got[r].view(np.uint32), want.view(np.uint32))
