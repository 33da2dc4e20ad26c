"""GPU regression test for the Choco apply pass's clamps (a probe build once let
write_cand store past k and the apply pass then faulted the GPU).  Since then mx_choco_apply
trusts nothing in a received message: every message's tile range [bnd[t], bnd[t+1]) is clamped to
[0, k) and entries whose index falls outside the tile are skipped.

Here the apply pass gets messages with entry indices >= P, negative and far out of range, tile
bounds past k (a count running past the slot), a negative first bound and a bound past k in the
middle of the row.  The state it writes must equal the state written from the same messages with
the dropped entries' values zeroed instead (a zero update leaves s / x_hat as they are), and the
guard regions around x, x_hat and s -- before the buffers, the row padding between P and ld, and
after the buffers -- must keep their sentinel.  Both apply kernels, both access hints.
Reference semantics: ChocoCommunicator.averaging, communicator.py:200-230."""
import numpy as np
import pytest

from conftest import Topo

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SENT = -12345.5


@pytest.mark.parametrize("apply_pf", [1, 0])
@pytest.mark.parametrize("apply_nt", [0, 1])
def test_choco_apply_clamps_untrusted_messages(pkg, O, apply_pf, apply_nt):
    n, P, k = 2, 3 * 4096 + 1000, 300               # partial last tile
    ratio = 1.0 - (k + 0.5) / P
    topo = Topo([[1, 0]], 0.25, np.array([[1]], np.uint8))
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
    assert grp.k == k
    X = np.stack([O.synth(4242 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X))
    grp.compress(0)
    torch.cuda.synchronize()
    ld, kpad, msg_ld = grp.ld, grp.kpad, grp.msg_ld
    ntiles = (P + 4095) // 4096

    def views(buf, slot):
        b = buf[slot * msg_ld:(slot + 1) * msg_ld]
        v = b[:4 * k].view(torch.float32)
        ix = b[4 * kpad:4 * kpad + 8 * k].view(torch.int64)
        bnd = b[4 * kpad + 8 * k:4 * kpad + 8 * k + 4 * (ntiles + 1)].view(torch.int32)
        return v, ix, bnd

    good = grp.msgs.clone()
    bad = grp.msgs.clone()
    # slot 0: three entries in tile 1 get indices >= P, negative and 2^40; the last bound runs past
    # the slot (2^31 - 1: an unclamped pass would read far beyond the message)
    v0g, ix0g, bnd0g = views(good, 0)
    v0b, ix0b, bnd0b = views(bad, 0)
    b1, b2 = int(bnd0g[1]), int(bnd0g[2])
    assert b2 - b1 >= 3, "tile 1 of message 0 needs entries"
    for e, val in zip(range(b1, b1 + 3), (P + 5, -3, 1 << 40)):
        ix0b[e] = val
        v0g[e] = 0.0                                 # the same entries as a zero update
    bnd0b[ntiles] = 2 ** 31 - 1
    # slot 1: first bound negative (clamped to 0: no change); the bound of tile 2 past k, so tile 2's
    # range is empty and tile 1's runs to k (its extra entries lie outside tile 1: skipped)
    v1g, ix1g, bnd1g = views(good, 1)
    v1b, ix1b, bnd1b = views(bad, 1)
    c2, c3 = int(bnd1g[2]), int(bnd1g[3])
    assert c3 > c2, "tile 2 of message 1 needs entries"
    bnd1b[0] = -50
    bnd1b[2] = k + 7
    v1g[c2:c3] = 0.0

    G = 8192                                         # guard floats before and after every buffer

    def state():
        bufs = []
        for init in (X, np.zeros_like(X), np.zeros_like(X)):     # x, x_hat, s
            t = torch.full((G + n * ld + G,), SENT, dtype=torch.float32, device="cuda")
            t[G:G + n * ld].view(n, ld)[:, :P].copy_(torch.from_numpy(init))
            bufs.append(t)
        return bufs

    saved = {key: int(pkg.lib.mx_topk_get(key)) for key in (b"apply_pf", b"apply_nt")}
    pkg._lib.check(pkg.lib.mx_topk_set(b"apply_pf", apply_pf))
    pkg._lib.check(pkg.lib.mx_topk_set(b"apply_nt", apply_nt))
    try:
        results = []
        for msgs in (good, bad):
            x, xh, s = state()
            pkg._lib.check(pkg.lib.mx_choco_apply(x.data_ptr() + 4 * G, xh.data_ptr() + 4 * G, s.data_ptr() + 4 * G,
                                                  ld, P, k, msgs.data_ptr(), msg_ld, grp.engine.n_slots,
                                                  grp.engine.plan.data_ptr(), 0, n, grp.engine.M,
                                                  grp.engine.alpha32, grp.gamma32, grp.apply_work.data_ptr(),
                                                  None), "mx_choco_apply")
            torch.cuda.synchronize()
            results.append([b.cpu().numpy() for b in (x, xh, s)])
    finally:
        for key, v in saved.items():
            pkg.lib.mx_topk_set(key, v)
    for name, a, b in zip(("x", "x_hat", "s"), results[0], results[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), name
        body = b[G:G + n * ld].reshape(n, ld)
        assert (b[:G] == SENT).all() and (b[G + n * ld:] == SENT).all(), f"{name}: guard around the buffer"
        assert (body[:, P:] == SENT).all(), f"{name}: row padding between P and ld"
    # the messages did update the state (the test is not vacuous): s holds the applied entries
    assert np.count_nonzero(results[1][2][G:G + n * ld].reshape(n, ld)[:, :P]) > k
