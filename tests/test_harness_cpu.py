"""Host-side pieces of the training harness (train_mpi.py / util.py restatements), no GPU."""
import os

import numpy as np
import pytest
import torch


def test_mlp_parameter_count_matches_reference(pkg):
    # SURVEY.md §2 row 10 [verified against models/MLP.py]: MNIST_MLP(47) has 666,547 params in 6 tensors
    m = pkg.harness.MNIST_MLP(47)
    ps = list(m.parameters())
    assert len(ps) == 6 and sum(p.numel() for p in ps) == 666_547
    assert m(torch.zeros(3, 1, 28, 28)).shape == (3, 47)


@pytest.mark.parametrize("epoch,itr,lr,warmup,expect", [
    (0, 0, 0.8, True, 0.1 + 0.7 * (1 / 50)),       # train_mpi.py:186-190, 10 itr per epoch
    (4, 9, 0.8, True, 0.8),                         # end of warmup
    (0, 3, 0.05, True, 0.05),                       # target <= base: no ramp
    (7, 0, 0.8, True, 0.8),
    (120, 0, 0.8, True, 0.8 * 0.1),                 # lr_schedule [100, 150]
    (160, 0, 0.8, True, 0.8 * 0.1 * 0.1),
    (2, 0, 0.8, False, 0.8),
])
def test_update_learning_rate(pkg, epoch, itr, lr, warmup, expect):
    H = pkg.harness
    args = H.HarnessArgs(lr=lr, warmup=warmup)
    opt = torch.optim.SGD([torch.zeros(2, requires_grad=True)], lr=123.0)
    got = H.update_learning_rate(opt, epoch, args, itr=itr, itr_per_epoch=10)
    assert got == pytest.approx(expect, rel=0, abs=1e-15)
    assert opt.param_groups[0]["lr"] == got


def test_meter_and_accuracy(pkg):
    H = pkg.harness
    m = H.AverageMeter()
    m.update(2.0, 3)
    m.update(4.0, 1)
    assert m.avg == pytest.approx(2.5) and m.count == 4 and m.val == 4.0
    out = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7], [0.6, 0.4]])
    tgt = torch.tensor([1, 0, 0, 0])
    assert H.comp_accuracy(out, tgt)[0].item() == pytest.approx(75.0)


def test_recorder_files_like_reference(pkg, tmp_path):
    """util.py:398-419: seven per-rank logs named dsgd-lr<lr>-budget<b>-r<rank>-<what>.log +
    ExpDescription, in <savePath><name>_<model>."""
    H = pkg.harness
    args = H.HarnessArgs(savePath=str(tmp_path) + "/", name="exp", model="mlp", lr=0.8, budget=0.5, save=True)
    rec = H.Recorder(args, 0)
    rec.add_new(1.5, 1.0, 0.25, 1.25, 80.0, 0.7, 79.0)
    rec.add_new(2.5, 2.0, 0.5, 2.5, 90.0, 0.5, 88.0)
    rec.save_to_file()
    folder = os.path.join(str(tmp_path), "exp_mlp")
    names = sorted(os.listdir(folder))
    want = sorted(["dsgd-lr0.8-budget0.5-r0-%s.log" % w for w in
                   ("recordtime", "time", "comptime", "commtime", "acc", "losses", "tacc")] + ["ExpDescription"])
    assert names == want
    np.testing.assert_array_equal(np.loadtxt(os.path.join(folder, "dsgd-lr0.8-budget0.5-r0-acc.log")), [79.0, 88.0])
    np.testing.assert_array_equal(np.loadtxt(os.path.join(folder, "dsgd-lr0.8-budget0.5-r0-commtime.log")),
                                  [0.25, 0.5])
    assert open(os.path.join(folder, "ExpDescription")).read().splitlines()[1] == args.description


def test_synthetic_batches_deterministic(pkg):
    H = pkg.harness
    a = H.synthetic_batches(3, 2, 5, device="cpu")
    b = H.synthetic_batches(3, 2, 5, device="cpu")
    c = H.synthetic_batches(4, 2, 5, device="cpu")
    assert all(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) for x, y in zip(a, b))
    assert not torch.equal(a[0][0], c[0][0])
    assert a[0][0].shape == (5, 1, 28, 28) and int(a[0][1].max()) < 100


def test_rendezvous_port_from_job_id(pkg):
    """MASTER_PORT: the launcher's if set, else derived from the job id (mpirun / slurm), so two
    jobs on one node get different ports and all ranks of a job the same one."""
    rp = pkg.communicator.rendezvous_port
    assert rp({"MASTER_PORT": "4711"}) == 4711
    a = rp({"PMIX_NAMESPACE": "prterun-node-1234@1"})
    b = rp({"PMIX_NAMESPACE": "prterun-node-1235@1"})
    assert a != b and 20000 <= a < 50000 and a == rp({"PMIX_NAMESPACE": "prterun-node-1234@1"})
    assert rp({"SLURM_JOB_ID": "77"}) == rp({"SLURM_JOB_ID": "77"})
    assert rp({}) == 29533


def test_pull_transport_refused_where_it_cannot_carry(pkg):
    """The pull transport serves gossip rounds (whole rows and, from round 5, Choco messages): the
    centralized communicator refuses it at construction with a clear TypeError, not
    with a null-handle error at the first round (the Choco communicator takes it: -m gpu tests).
    No GPU: the refusal comes first."""
    import pytest as _pytest
    t = pkg.PullTransport.__new__(pkg.PullTransport)
    with _pytest.raises(TypeError, match="PullTransport"):
        pkg.centralizedCommunicator(0, 2, transport=t)


def test_rccl_deadline_api_declared(pkg):
    """The non-blocking RCCL communicator with a deadline is part of the C ABI (checked without a
    GPU: argument validation only)."""
    import ctypes
    h = ctypes.c_void_p()
    assert pkg.lib.mx_rccl_init_timeout(None, 2, 0, 1000, ctypes.byref(h), None) == -1
    uid = (ctypes.c_char * 128)()
    assert pkg.lib.mx_rccl_init_timeout(ctypes.cast(uid, ctypes.c_void_p), 2, 5, 1000, ctypes.byref(h), None) == -1
    assert pkg.lib.mx_rccl_init_timeout(ctypes.cast(uid, ctypes.c_void_p), 2, 0, 0, ctypes.byref(h), None) == -1
    assert pkg.lib.mx_rccl_abort(None) == 0 and pkg.lib.mx_rccl_destroy(None) == 0
