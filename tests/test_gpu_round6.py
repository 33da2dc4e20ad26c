"""GPU: the round-6 changes, each against an exact expectation.

  * the IPC export probe: the allocation sequence of the one recorded export
    refusal (profiles/r05zz2_suite_ipc_failure.log -- bench.py's 2-rank no-RCCL run, --params
    100000), run in one process with mx_ipc_alloc's rounding OFF, between torch
    caching-allocator traffic of the same sizes, then again with the 2 MiB rounding; every export
    is counted (mx_ipc_stats) and the result is recorded in gpurun_out/ipc_probe.json;
  * mx_snapshot_publish_rows copies exactly the rows a peer reads in the round (an active partner
    in another block) and leaves every other row untouched.

Reference: communicator.py:99-112 (only active partners exchange), 214."""
import ctypes
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stats(L):
    ex, ref = ctypes.c_int(0), ctypes.c_int(0)
    assert L.mx_ipc_stats(ctypes.byref(ex), ctypes.byref(ref)) == 0
    return ex.value, ref.value


def _failing_run_sizes():
    """Snapshot-buffer sizes bench.py's 2-rank run (--params 100000 --choco-params 100000
    --wrn-params 50000 --resnet-params 20000 --er-params 20000) asked mx_ipc_alloc for, in order,
    unrounded: 256 + 2 * n_local * row bytes."""
    def dec(P, n_local=4):
        ld = (P + 63) // 64 * 64
        return 256 + 2 * n_local * ld * 4

    def choco(P, ratio=0.99, n_local=4):
        k = max(1, int(P * (1 - ratio)))
        kpad = (k + 1) // 2 * 2
        msg = 4 * kpad + 8 * k + 4 * ((P + 4095) // 4096 + 1)
        return 256 + 2 * n_local * ((msg + 255) // 256 * 256)

    return [dec(100_000), dec(100_000), choco(100_000), choco(100_000), dec(50_000), dec(50_000), dec(20_000),
            dec(20_000, 32), dec(20_000, 32)]


def _probe(pkg, sizes, rounds, rng):
    """mx_ipc_alloc every size `rounds` times between torch allocations of similar sizes; returns
    (exports, refusals) counted by the library over the probe."""
    L = pkg.lib
    hb = int(L.mx_ipc_handle_bytes())
    ex0, ref0 = _stats(L)
    held = []
    for _ in range(rounds):
        for nbytes in sizes:
            # torch caching-allocator traffic around each export, as in a bench process
            held.append(torch.empty(int(rng.integers(1, 2 * nbytes // 4 + 2)), dtype=torch.float32, device="cuda"))
            if len(held) > 12:
                held.pop(int(rng.integers(0, len(held))))
            p = ctypes.c_void_p()
            h = (ctypes.c_char * hb)()
            rc = L.mx_ipc_alloc(int(nbytes), ctypes.byref(p), ctypes.cast(h, ctypes.c_void_p))
            if rc == 0:
                assert L.mx_ipc_free(p) == 0
        torch.cuda.synchronize()
    del held
    torch.cuda.empty_cache()
    ex1, ref1 = _stats(L)
    return ex1 - ex0, ref1 - ref0


def test_ipc_export_probe_unrounded_and_rounded(pkg):
    L = pkg.lib
    saved = int(L.mx_ipc_get(b"granule"))
    assert saved == 2 << 20, saved
    rng = np.random.default_rng(6)
    sizes = _failing_run_sizes()
    small = [int(x) for x in rng.integers(4096, 4 << 20, 40)]       # unaligned small sizes as well
    try:
        assert L.mx_ipc_set(b"granule", 1) == 0
        unrounded = _probe(pkg, sizes + small, 6, rng)
    finally:
        assert L.mx_ipc_set(b"granule", saved) == 0
    rounded = _probe(pkg, sizes + small, 6, rng)
    rec = {"sizes": sizes, "small_sizes": len(small), "rounds": 6,
           "unrounded": {"exports": unrounded[0], "refused": unrounded[1]},
           "rounded_2MiB": {"exports": rounded[0], "refused": rounded[1]}}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ipc_probe.json"), "w") as f:
        json.dump(rec, f)
    print(json.dumps(rec))
    n = 6 * (len(sizes) + len(small))
    assert unrounded[0] == n and rounded[0] == n, rec
    # the pin: neither form is refused in a process of this shape (DESIGN.md "IPC exports")
    assert unrounded[1] == 0 and rounded[1] == 0, rec


def _publish_reference(src, dst0, flags, partner, row_base, n_local, ncols):
    """What mx_snapshot_publish_rows leaves in dst: the read rows copied, the others untouched."""
    out = dst0.copy()
    for r in range(n_local):
        w = row_base + r
        read = any(flags[g] and partner[g, w] >= 0 and not (row_base <= partner[g, w] < row_base + n_local)
                   for g in range(len(flags)))
        if read:
            out[r, :ncols] = src[r, :ncols]
    return out


@pytest.mark.parametrize("gid,nranks,rank", [(0, 2, 0), (0, 2, 1), (0, 4, 2), (2, 4, 1), (0, 8, 5), (0, 1, 0)])
def test_snapshot_publish_rows_copies_only_read_rows(pkg, O, gid, nranks, rank):
    L = pkg.lib
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    partner = np.asarray(gp.neighbors_info, np.int32)
    M = partner.shape[0]
    row_base, n_local = pkg.partition(n, nranks)[rank]
    ld, ncols = 1088, 1028
    rng = np.random.RandomState(gid * 100 + nranks * 10 + rank)
    src = rng.uniform(-1, 1, (n_local, ld)).astype(np.float32)
    dst0 = rng.uniform(5, 6, (n_local, ld)).astype(np.float32)
    part_dev = torch.from_numpy(partner).cuda()
    src_dev = torch.from_numpy(src).cuda()
    copies = 0
    for trial in range(12):
        flags = (rng.uniform(size=M) < 0.5).astype(np.uint8)
        if trial == 0:
            flags[:] = 1
        dst_dev = torch.from_numpy(dst0).cuda()
        fl_dev = torch.from_numpy(flags).cuda()
        pkg._lib.check(L.mx_snapshot_publish_rows(src_dev.data_ptr(), ld, dst_dev.data_ptr(), ld, ncols, n_local,
                                                  fl_dev.data_ptr(), M, part_dev.data_ptr(), n, row_base, None),
                       "mx_snapshot_publish_rows")
        want = _publish_reference(src, dst0, flags, partner, row_base, n_local, ncols)
        got = dst_dev.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (trial, flags)
        copies += int((got != dst0).any(axis=1).sum())
    if nranks == 1:
        assert copies == 0                         # one block: nobody outside reads a row
    else:
        assert copies > 0


def test_snapshot_publish_rows_refuses_bad_shapes(pkg):
    L = pkg.lib
    a = torch.zeros(64, device="cuda")
    f = torch.ones(5, dtype=torch.uint8, device="cuda")
    p = torch.zeros(40, dtype=torch.int32, device="cuda")
    assert L.mx_snapshot_publish_rows(a.data_ptr(), 8, a.data_ptr(), 8, 6, 2, f.data_ptr(), 5, p.data_ptr(), 8, 0,
                                      None) != 0                                 # n % 4
    assert L.mx_snapshot_publish_rows(a.data_ptr(), 8, a.data_ptr(), 8, 8, 2, f.data_ptr(), 5, p.data_ptr(), 8, 7,
                                      None) != 0                                 # block past n_global
    assert L.mx_snapshot_publish_rows(a.data_ptr(), 4, a.data_ptr(), 8, 8, 2, f.data_ptr(), 5, p.data_ptr(), 8, 0,
                                      None) != 0                                 # src_ld < n


def test_packed_mix_call_equals_unpacked(pkg, O):
    """mx_gossip_mix_packed (the group's arguments packed once in an mx_mix_call: engine.mix's
    path) launches the same rounds as mx_gossip_mix with the 13 arguments -- both equal the
    oracle's decen rounds, uint32 (communicator.py:92-122)."""
    n, P, T = 8, 70_001, 6
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, T, True)
    a = pkg.VirtualWorkerGroup(GP, numel=P)
    b = pkg.VirtualWorkerGroup(GP, numel=P)
    X = np.stack([O.synth(600 + i, P) for i in range(n)])
    for g in (a, b):
        g.rows.copy_(torch.from_numpy(X))
    partner = np.asarray(GP.neighbors_info, np.int32)
    flags = np.asarray(GP.active_flags, np.uint8)
    L, sp = pkg.lib, pkg._lib.stream_ptr
    for it in range(T):
        a.engine.mix(it, a.layout)                                   # packed
        e = b.engine
        pkg._lib.check(L.mx_gossip_mix(*b.layout._args, e._plan_ptr, it, e.n_local, e.M, e.alpha32, sp()))
        if flags[it].any():
            X = O.decen_round(X, partner, flags[it], GP.neighbor_weight)
    torch.cuda.synchronize()
    ga, gb = a.rows.cpu().numpy(), b.rows.cpu().numpy()
    assert np.array_equal(ga.view(np.uint32), gb.view(np.uint32))
    assert np.array_equal(ga.view(np.uint32), X.view(np.uint32))
    assert pkg.lib.mx_gossip_mix_packed(None, 0, None) != 0              # a null record is refused


def test_layout_call_cache_follows_the_engine(pkg, O):
    """A layout's packed-call cache is keyed by the engine object (weakly), not by its plan's
    device address: an engine built after another was freed -- its plan most likely at the same
    caching-allocator address -- gets its own alpha / M / need_host, so its rounds equal the
    oracle's under its own schedule (communicator.py:92-122)."""
    import gc
    n, P, T = 8, 70_001, 5
    np.random.seed(77)
    GP1 = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, T, True)
    GP2 = pkg.MatchaProcessor(pkg.select_graph(0), 0.25, 0, n, T, True)
    assert np.float32(GP1.neighbor_weight) != np.float32(GP2.neighbor_weight)
    g = pkg.VirtualWorkerGroup(GP1, numel=P)
    X = np.stack([O.synth(900 + i, P) for i in range(n)])
    g.rows.copy_(torch.from_numpy(X))
    e1 = pkg.GossipEngine(GP1)
    e1.mix(0, g.layout)                                   # caches e1's call in g.layout
    torch.cuda.synchronize()
    flags1 = np.asarray(GP1.active_flags, np.uint8)
    if flags1[0].any():
        X = O.decen_round(X, np.asarray(GP1.neighbors_info, np.int32), flags1[0], GP1.neighbor_weight)
    old_ptr = e1._plan_ptr
    del e1
    gc.collect()
    e2 = pkg.GossipEngine(GP2)
    reused = e2._plan_ptr == old_ptr
    partner, flags2 = np.asarray(GP2.neighbors_info, np.int32), np.asarray(GP2.active_flags, np.uint8)
    for it in range(T):
        e2.mix(it, g.layout)
        if flags2[it].any():
            X = O.decen_round(X, partner, flags2[it], GP2.neighbor_weight)
    torch.cuda.synchronize()
    got = g.rows.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), X.view(np.uint32)), {"plan_address_reused": reused}
    assert len(g.layout._calls) <= 2 and e2 in g.layout._calls
