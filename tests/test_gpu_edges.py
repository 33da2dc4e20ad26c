"""GPU edge shapes: rows far shorter than a tile (1 .. 4097 params; every sub-tile split), top-k
at k = 1 (the reference's torch.max path, compressors.py:12-14) and k = P, and Choco rounds on
tiny rows -- bit-exact vs the oracle."""
import numpy as np
import pytest
import torch

from conftest import Topo

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 1023, 1025, 4097]


@pytest.mark.parametrize("split", [0, 4])
@pytest.mark.parametrize("gid", [0, 2])
def test_mix_tiny_rows(pkg, O, gid, split):
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(split=split)
    try:
        n = pkg.GRAPH_SIZES[gid]
        gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
        M = len(gp.neighbors_info)
        rng = np.random.RandomState(gid + 7)
        flags = (rng.uniform(size=(3, M)) < 0.6).astype(np.uint8)
        flags[0] = 1
        topo = Topo(gp.neighbors_info, 0.19, flags)
        for P in SIZES:
            grp = pkg.VirtualWorkerGroup(topo, numel=P)
            X = np.stack([O.synth(P * 31 + i, P) for i in range(n)])
            grp.rows.copy_(torch.from_numpy(X))
            for f in flags:
                grp.communicate()
                X = O.decen_round(X, topo.neighbors_info, f, 0.19)
            got = grp.rows.cpu().numpy()
            assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"P={P}"
    finally:
        pkg.engine.set_mix_tuning(**saved)


@pytest.mark.parametrize("P", [1, 2, 3, 7, 100, 4096, 4097])
@pytest.mark.parametrize("ratio", [0.0, 0.5, 0.999999])
def test_topk_extreme_k(pkg, O, P, ratio):
    x = O.synth(P + 11, P)
    k = O.topk_k(P, ratio)
    assert 1 <= k <= P
    ov, oi = O.topk_abs(x, k)
    v, i = pkg.get_top_k(torch.from_numpy(x).cuda(), ratio)
    assert i.numel() == k
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("P", [1, 5, 257, 4099])
@pytest.mark.parametrize("ratio", [0.0, 0.5, 0.99])
def test_choco_tiny_rows(pkg, O, P, ratio):
    n = 8
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    flags = np.array([[1, 1, 1, 1, 1], [1, 0, 1, 0, 1], [0, 1, 1, 1, 0]], np.uint8)
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.2)
    X = np.stack([O.synth(70 + i, P) for i in range(n)])
    XH, S = np.zeros_like(X), np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X))
    k = O.topk_k(P, ratio)
    for t, f in enumerate(flags):
        if t:
            D = np.stack([np.float32(0.05) * O.synth(600 + 13 * t + i, P) for i in range(n)])
            X += D
            grp.rows.add_(torch.from_numpy(D).cuda())
        grp.communicate()
        O.choco_round(X, XH, S, topo.neighbors_info, f, 2 / 7, k, 0.2)
        got = grp.rows.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"round {t}"


def test_iteration_outside_schedule_raises(pkg):
    """The kernels index the plan table by iteration: the host refuses one outside the schedule
    instead of launching a read past the table."""
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
    topo = Topo(gp.neighbors_info, 0.2, np.ones((3, 5), np.uint8))
    grp = pkg.VirtualWorkerGroup(topo, numel=1000)
    for bad in (3, 4, -1):
        with pytest.raises(IndexError):
            grp.engine.mix(bad, grp.layout)
    ch = pkg.ChocoWorkerGroup(topo, numel=1000, ratio=0.9, consensus_lr=0.1)
    with pytest.raises(IndexError):
        ch.average(3)


@pytest.mark.parametrize("P,split", [(181_668, 0), (50_003, 1), (1_000_000, 0)])
def test_device_round_graph_replay(pkg, O, P, split):
    """device_round (mx_gossip_mix_at + mx_iter_advance) captured once in a HIP graph
    (torch.cuda.graph) and replayed: every replay is the next MATCHA round of the schedule --
    skipped rounds included -- bit-exact vs the oracle; past the schedule's end a replay is a no-op."""
    saved = pkg.engine.mix_tuning()
    pkg.engine.set_mix_tuning(split=split)
    try:
        n, T = 8, 12
        np.random.seed(77)
        GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.4, 0, n, T, True)
        grp = pkg.VirtualWorkerGroup(GP, numel=P)
        X = np.stack([O.synth(4000 + i, P) for i in range(n)])
        grp.rows.copy_(torch.from_numpy(X))
        partner = np.asarray(GP.neighbors_info, np.int32)
        grp.iter_dev.fill_(0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                grp.device_round()
                grp.device_round()                   # two rounds per replay
        torch.cuda.synchronize()
        assert int(grp.iter_dev.item()) == 0 and np.array_equal(grp.rows.cpu().numpy(), X)  # capture ran nothing
        rows = len(GP.active_flags)                 # T + 1 rows (graph_manager.py:298-309)
        for it in range(0, rows + 4, 2):             # the last replays run past the schedule
            g.replay()
            for j in (it, it + 1):
                if j < rows:
                    X = O.decen_round(X, partner, np.asarray(GP.active_flags[j], np.uint8), GP.neighbor_weight)
            torch.cuda.synchronize()
            got = grp.rows.cpu().numpy()
            assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), f"rounds {it}, {it + 1}"
        assert int(grp.iter_dev.item()) == len(range(0, rows + 4, 2)) * 2
    finally:
        pkg.engine.set_mix_tuning(**saved)


@pytest.mark.parametrize("K", [1, 5])
def test_device_rounds_unrolled_graph(pkg, O, K):
    """device_rounds(K) (one mx_iter_expand + K mx_gossip_mix_at launches) captured once: each
    replay is the next K rounds of a MATCHA schedule, bit-exact vs the oracle, past the end no-ops,
    and it mixes with device_round() on the same counter."""
    n, T, P = 8, 13, 181_668
    np.random.seed(91)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, T, True)
    grp = pkg.VirtualWorkerGroup(GP, numel=P)
    X = np.stack([O.synth(7000 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X))
    partner = np.asarray(GP.neighbors_info, np.int32)
    grp.iter_dev.fill_(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            grp.device_rounds(K)
            grp.device_round()                       # K + 1 rounds per replay
    torch.cuda.synchronize()
    assert int(grp.iter_dev.item()) == 0 and np.array_equal(grp.rows.cpu().numpy(), X)
    rows = len(GP.active_flags)
    done = 0
    while done < rows + K + 1:
        g.replay()
        for j in range(done, done + K + 1):
            if j < rows:
                X = O.decen_round(X, partner, np.asarray(GP.active_flags[j], np.uint8), GP.neighbor_weight)
        done += K + 1
        torch.cuda.synchronize()
        assert np.array_equal(grp.rows.cpu().numpy().view(np.uint32), X.view(np.uint32)), f"after {done} rounds"
    assert int(grp.iter_dev.item()) == done


def test_cpu_inputs_staged_through_the_gpu(pkg, O):
    """The reference keeps models on the CPU (train_mpi.py:92 has .cuda() commented out):
    flatten_tensors / get_top_k take CPU tensors, compute on the GPU and answer on the CPU."""
    ts = [torch.from_numpy(O.synth(60 + i, n)).reshape(shape) for i, (n, shape) in
          enumerate(((15, (3, 5)), (7, (7,)), (2112, (64, 33))))]
    flat = pkg.flatten_tensors(ts)
    assert flat.device.type == "cpu" and torch.equal(flat, torch.cat([t.reshape(-1) for t in ts]))
    x = O.synth(91, 50_001)
    v, i = pkg.get_top_k(torch.from_numpy(x), 0.99)
    ov, oi = O.topk_abs(x, O.topk_k(50_001, 0.99))
    assert v.device.type == "cpu" and i.device.type == "cpu" and i.dtype == torch.int64
    assert np.array_equal(i.numpy(), oi) and np.array_equal(v.numpy().view(np.uint32), ov.view(np.uint32))
    with pytest.raises(TypeError):
        pkg.flatten_tensors([ts[0], ts[1].cuda()])


@pytest.mark.parametrize("nrows", [1, 2, 3, 5, 7, 8, 9, 16, 33, 64, 65, 100, 129, 300])
@pytest.mark.parametrize("order", ["tree", "sequential"])
def test_mean_rows_reference_order(pkg, O, nrows, order):
    """mx_mean_rows (the division step of centralizedCommunicator / sync_allreduce) sums in
    mpi4py's binomial-tree order (default) or rank order, then divides: bit-exact vs numpy fp32.
    Above 64 rows the tree runs as a binary counter of partial sums (any world size)."""
    from reforder import mpi4py_sum as _mpi4py_sum
    count, ld = (100_003, 100_032) if nrows <= 64 else (20_011, 20_032)
    rows = [O.synth(31 * r + nrows, count) * np.float32(10.0 ** (r % 4 - 1)) for r in range(nrows)]
    dev = torch.zeros((nrows, ld), dtype=torch.float32, device="cuda")
    dev[:, :count] = torch.from_numpy(np.stack(rows))
    out = torch.empty(count, dtype=torch.float32, device="cuda")
    code = {"tree": 0, "sequential": 1}[order]
    pkg._lib.check(pkg.lib.mx_mean_rows(dev.data_ptr(), nrows, ld, count, code, out.data_ptr(), None))
    want = _mpi4py_sum(rows, order) / np.float32(nrows)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    # in place into row 0 (out aliases rows[0])
    pkg._lib.check(pkg.lib.mx_mean_rows(dev.data_ptr(), nrows, ld, count, code, dev.data_ptr(), None))
    assert np.array_equal(dev[0, :count].cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert pkg.lib.mx_mean_rows(dev.data_ptr(), 0, ld, count, code, out.data_ptr(), None) != 0
