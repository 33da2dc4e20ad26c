"""CPU: bench.py's self-launch and the oracle's centralized restatement.

`python bench.py --gpus N` (N > 1) without a launcher must run N ranks -- a child
`torch.distributed.run` -- relay rank 0's line, and never initialise HIP in the parent (an exec or
a GPU context in the parent would be fatal on the GPU pool); with too few GPUs it must fail with a
message instead of timing N = 1."""
import io
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)


class _FakeProc:
    """Stands in for the child launcher: prints a rank-0 line and a stray log line."""

    def __init__(self, cmd, **kw):
        self.cmd, self.kw, self.pid = cmd, kw, os.getpid()
        line = {"metric": "m", "value": 1.0, "n_gpus": 2}
        self.stdout = io.StringIO("torchrun banner\n" + json.dumps(line) + "\n")

    def wait(self):
        return 0


def test_self_launch_spawns_child_and_never_touches_hip(monkeypatch, capsys):
    import torch
    import bench

    def no_hip(*a, **k):
        raise AssertionError("the launching parent initialised HIP")

    monkeypatch.setattr(torch.cuda, "_lazy_init", no_hip)
    monkeypatch.setattr(torch.cuda, "init", no_hip)
    seen = {}

    def popen(cmd, **kw):
        seen["p"] = _FakeProc(cmd, **kw)
        return seen["p"]

    argv = ["--gpus", "2", "--transport", "gloo", "--steps", "3"]
    sys.argv = ["bench.py"] + argv
    args = bench.parse()
    rc = bench.self_launch(args, argv, popen=popen)
    assert rc == 0
    assert not torch.cuda.is_initialized()
    cmd = seen["p"].cmd
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:] == argv       # the same flags, forwarded
    assert seen["p"].kw["start_new_session"] is True                          # a child, own process group
    out = capsys.readouterr()
    lines = [l for l in out.out.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["launcher"]["self_launched"] is True
    assert "torchrun banner" in out.err


def test_gpus8_without_devices_fails_with_message():
    """No torchrun, --gpus 8, the RCCL transport, and fewer GPUs than ranks (none in this
    container): a non-zero exit with a message and NO JSON line -- never a silent N = 1 line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "GPU(s) visible" in r.stderr


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 64, 70])
@pytest.mark.parametrize("order", ["tree", "sequential"])
def test_oracle_central_mean_is_mpi4py_order(O, n, order):
    """orc_central_mean (centralizedCommunicator, communicator.py:46-76) = the restated mpi4py
    object-allreduce order (tests/reforder.py) / n, uint32 -- the parity target of
    mx_mean_rows_to and the bench's all-reduce figure (mpi4py itself is absent: parity unpinned
    against it, pinned against the restatement)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from reforder import mpi4py_sum
    rng = np.random.default_rng(n)
    X = (rng.standard_normal((n, 4099)) * rng.uniform(0.1, 100, (n, 1))).astype(np.float32)
    want = mpi4py_sum(list(X), order) / np.float32(n)
    got = O.central_mean(X, order)
    assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))


_WD_SCRIPT = r"""
import os, signal, sys, time
sys.path.insert(0, {root!r})
import bench
line = bench.Line(0)
line.out["value"] = 1.0
wd = bench.Watchdog(0, line.emit)
if {mode!r} == "watchdog":
    wd.arm("figure_x", 0.5)
    time.sleep(30)
else:
    wd.arm("figure_y", 600)
    signal.signal(signal.SIGTERM, bench.term_handler(line, wd))
    print("ready", file=sys.stderr, flush=True)
    time.sleep(30)
"""


@pytest.mark.parametrize("mode", ["watchdog", "sigterm"])
def test_aborted_run_exits_nonzero_with_one_error_line(mode):
    """a figure that hangs (the watchdog's deadline) or a SIGTERM from the
    launcher prints the line so far with an "error" field ONCE and exits EXIT_ABORTED (3), never 0,
    so the driver's exit code tells an aborted N > 1 bench from a clean one."""
    import signal
    import time
    p = subprocess.Popen([sys.executable, "-c", _WD_SCRIPT.format(root=ROOT, mode=mode)], cwd=ROOT,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if mode == "sigterm":
        t0 = time.time()
        while p.stderr.readline().strip() != "ready":
            assert time.time() - t0 < 120 and p.poll() is None
        p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=120)
    import bench
    assert p.returncode == bench.EXIT_ABORTED == 3, err[-2000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["error"], d
    if mode == "watchdog":
        assert "figure_x" in d["error"] and "no progress" in d["error"]
    else:
        assert "figure_y" in d["error"] and "signal 15" in d["error"]


def test_failed_self_check_withholds_rates():
    """a figure whose oracle self-check failed reports no rate -- its rate keys move
    under "unverified", recursively (configs' entries, the ER sweep's budgets); passing ones keep
    theirs."""
    import bench
    fig = {"rounds_per_s": 5.0, "parity_ok": True,
           "a": {"rounds_per_s": 1.0, "ms_per_round": 1.0, "parity_ok": False, "budget": 0.5},
           "sweep": [{"rounds_per_s": 2.0, "parity_ok": True}, {"rounds_per_s": 3.0, "hbm_TBps_rank0": 4.0,
                                                              "parity_ok": False}]}
    assert bench.withhold_unverified(fig) is True
    assert fig["rounds_per_s"] == 5.0 and fig["sweep"][0]["rounds_per_s"] == 2.0
    assert "rounds_per_s" not in fig["a"] and fig["a"]["unverified"] == {"rounds_per_s": 1.0, "ms_per_round": 1.0}
    assert fig["a"]["budget"] == 0.5
    assert fig["sweep"][1]["unverified"] == {"rounds_per_s": 3.0, "hbm_TBps_rank0": 4.0}
    assert bench.withhold_unverified({"rounds_per_s": 1.0, "parity_ok": True}) is False
    assert bench.withhold_unverified(None) is False


def test_settle_rounds_sizes_the_burst():
    """bench.settle_rounds: about --settle-ms of streaming at the headline's settled rate for rows of
    >= 64 MB per round (the post-pause DVFS ramp, profiles/r06w_dvfs_ramp.json), none for smaller
    rows or settle_ms 0, at most SETTLE_MAX_ROUNDS; a function of the bytes alone, so ranks that pass
    the same rank-independent byte count run the same number of lockstep rounds."""
    import bench
    head = 2 * 8 * 25_600_000 * 4
    per_round_ms = head / (bench.HEADLINE_HBM_FRAC * bench.HBM_PEAK) * 1e3
    n = bench.settle_rounds(head, 50.0)
    assert (n - 1) * per_round_ms < 50.0 <= n * per_round_ms
    assert bench.settle_rounds(head, 0) == 0
    assert bench.settle_rounds(bench.SETTLE_MIN_BYTES - 1, 50.0) == 0           # launch-bound rows
    assert bench.settle_rounds(bench.SETTLE_MIN_BYTES, 1e6) == bench.SETTLE_MAX_ROUNDS
    assert bench.settle_rounds(64 * 2 * 1_000_000_000 * 4, 50.0) == 1            # one ER(64) round > 50 ms
    assert bench.settle_rounds(2 * 8 * 36_546_980 * 4, 50.0) < n                 # bigger rows, fewer rounds
