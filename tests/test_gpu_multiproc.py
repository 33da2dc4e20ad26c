"""GPU: the multi-GPU code path across real processes (2 and 4 ranks sharing GPU 0).

Partner rows cross process boundaries through the gloo test transport (tests/gloo_transport.py);
everything else -- worker partition, exchange plan, receive slab, chunked pipelining on a side
stream, Choco message exchange, centralized all-reduce mean, and bench.py's N > 1 timing path --
is the product code.  RCCL itself needs one GPU per rank and runs only in the driver's
multi-GPU bench."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _why(r):
    """the failing ranks' own error lines first (the launcher's summary hides them), then the tails"""
    err = [l for l in r.stderr.splitlines() if (l.startswith("[rank ") or l.startswith("[matcha_gossip]") or
                                                 l.startswith("[pull_clean]") or "Error" in l or "error" in l or
                                                 "Traceback" in l) and "Gloo" not in l and "error_file" not in l]
    return "\n".join(err[:80]) + "\n--- stdout ---\n" + r.stdout[-2000:] + "\n--- stderr ---\n" + r.stderr[-2000:]


def _torchrun(nproc, args, timeout=200):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="2")
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("nproc", [2, 3, 4])
def test_multiprocess_rounds_match_oracle(nproc):
    """nproc 3: uneven worker blocks (8 -> 3, 3, 2; 16 -> 6, 5, 5), so the pull transport's peers'
    snapshot buffers differ in size (per-rank n_local in the device rank table)."""
    r = _torchrun(nproc, [os.path.join(HERE, "mp_worker.py")])
    assert r.returncode == 0, _why(r)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == nproc and all(v for k, v in res.items() if k != "world"), res


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_multiprocess_path(nproc):
    """bench.py's N > 1 branch (partition, exchange, barriers, max-over-ranks timing, xgmi object)
    end to end on one GPU, with EVERY figure at reduced size: the headline, MATCHA 0.5, Choco (VGG
    config 4), the WRN / ResNet configs 2-3 and the ER(64) budget sweep (config 5) -- each one's
    oracle self-check must pass (configs 3-5 self-checking at N > 1).  nproc 8 is the
    driver's 8-GPU layout (one worker per rank; ER(64): 8 workers per rank) on one GPU."""
    r = _torchrun(nproc, ["bench.py", "--gpus", str(nproc), "--transport", "gloo", "--steps", "3", "--warmup", "1",
                          "--params", "200000", "--choco-params", "300000", "--cpu-seconds", "0",
                          "--wrn-params", "70000", "--resnet-params", "30000", "--mlp-params", "40000", "--lb-rounds", "20", "--er-params", "20000",
                          "--er-rounds", "2", "--er-budgets", "0.3,1.0"], timeout=280)
    assert r.returncode == 0, _why(r)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert "error" not in out, out["error"]
    assert out["n_gpus"] == nproc and out["value"] > 0 and out["xgmi"]["max_link_bytes_per_round"] > 0
    assert out["xgmi"]["exchange_only_ms"] > 0 and out["xgmi"]["p2p_probe"]["uni_GBps"] > 0
    ov = out["overlap"]
    assert ov["mode"] == "auto" and ov["chunks"] == 4 and ov["chosen"] in ("chunked", "unchunked")
    assert ov["calib_ms_unchunked"] > 0 and ov["calib_ms_chunked"] > 0
    assert out["choco"]["rounds_per_s"] > 0 and out["cpu_baseline"] is None
    assert out["allreduce_baseline"]["rounds_per_s"] > 0
    assert out["allreduce_baseline"]["parity_ok"] is True          # all-gather + mx_mean_rows_to, tree order
    assert out["choco"]["topk"]["calls_per_row"] > 0
    # Choco at N > 1: the RCCL-form (gloo here) and pull forms calibrated, the faster timed
    assert set(out["choco"]["calib_ms"]) == {"rccl", "pull", "pull_direct"}
    assert out["choco"]["form"] in ("rccl", "pull", "pull_direct")
    assert out["choco"]["pull_unavailable"] is None
    # every pull bind of the run succeeded with no refused IPC export
    for obj in (out["overlap"], out["choco"], out["pull_transport"]):
        assert obj["ipc_refused"] == 0 and obj["bind_failures"] == 0, obj
    assert out["pull_transport"]["binds"] >= out["choco"]["binds"] > 0
    cp = out["choco"]["predicted"]
    for f in ("rccl", "pull"):
        assert cp[f]["busiest_link_bytes"] > 0 and cp[f]["local_ms"] > 0 and cp[f]["round_ms"] > 0, cp[f]
    assert cp["timed_form"] == out["choco"]["form"] and cp["achieved_over_predicted"] > 0
    # every self-check is the oracle's (checker) on the same inputs
    assert out["parity_ok"] is True and "oracle" in out["parity"]
    assert out["choco"]["parity_ok"] is True
    assert out["matcha_schedule"]["parity_ok"] is True
    cf = out["configs"]
    assert all(cf[k]["parity_ok"] is True and cf[k]["rounds_per_s"] > 0
               for k in ("wrn28_10_matcha0.5", "wrn28_10_full", "resnet18_100_matcha0.5", "mlp_fixed")), cf
    er = out["er64_sweep"]
    assert er["parity_ok"] is True and er["params_per_worker"] == 20000 and er["rows_per_gpu"] == 64 // nproc
    assert len(er["sweep"]) == 2 and all(len(b["slots_per_rank"]) == nproc for b in er["sweep"])
    full = er["sweep"][-1]
    assert full["budget"] == 1.0 and full["max_link_bytes_per_round"] > 0 and full["rounds_per_s"] > 0
    assert (full["exchange_only_ms"] or 0) > 0 or er["form"] != "rccl"
    assert set(er["calib_ms"]) == {"rccl", "rccl_chunked", "pull"}
    assert er["calib_parity_ok"] == {"rccl": True, "rccl_chunked": True, "pull": True}, er["calib_parity_ok"]
    assert len(out["xgmi"]["exchange_only_ms_per_rank"]) == nproc
    # the expected round of every form from its parts: present and positive
    pr = out["predicted"]
    for f in ("rccl", "rccl_chunked", "pull"):
        assert pr[f]["busiest_link_bytes"] > 0 and pr[f]["link_bound_ms"] > 0 and pr[f]["mix_ms"] > 0, pr[f]
        assert pr[f]["fixed_ms"] > 0 and pr[f]["rounds_per_s"] > 0 and 0 < pr[f]["xgmi_frac"] < 1, pr[f]
    assert pr["achieved_over_predicted"] > 0
    assert all(b["predicted"]["rounds_per_s"] > 0 for b in er["sweep"] if b["predicted"]), er["sweep"]


def test_bench_watchdog_line_on_hang():
    """A rank that skips a figure's collectives (--debug-skip allreduce:1) desynchronises the job:
    its peer waits in the figure (then the watchdog fires), or the mismatched collectives abort a
    rank and the launcher SIGTERMs the others.  Either way rank 0 prints the line measured so far
    -- the headline intact -- with an "error" field, and the job ends instead of hanging, with a
    NON-zero exit status (the driver's rc must tell an aborted run from a
    clean one)."""
    r = _torchrun(2, ["bench.py", "--gpus", "2", "--transport", "gloo", "--steps", "3", "--warmup", "1",
                      "--params", "100000", "--cpu-seconds", "0", "--configs", "0", "--er", "0",
                      "--figure-timeout", "15", "--debug-skip", "allreduce:1"], timeout=240)
    assert r.returncode != 0, _why(r)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, _why(r)
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["parity_ok"] is True
    assert out.get("error"), out


@pytest.mark.parametrize("nproc,overlap,pull", [(2, "on", "off"), (4, "off", "off"), (2, "off", "on"),
                                               (4, "auto", "auto")])
def test_bench_multiprocess_overlap_forms(nproc, overlap, pull):
    """bench.py's N > 1 branch with the exchange form forced (column-pipelined / plain / pull) or
    calibrated among all three; the timed form passes the self-check.  With --pull on the Choco
    figure runs too, forced onto the pull form (messages read from the owners' snapshots)."""
    choco = ["--choco", "1", "--choco-params", "100000"] if pull == "on" else ["--choco", "0"]
    r = _torchrun(nproc, ["bench.py", "--gpus", str(nproc), "--transport", "gloo", "--steps", "3", "--warmup", "1",
                          "--params", "100000", "--cpu-seconds", "0", "--overlap", overlap,
                          "--pull", pull, "--configs", "0", "--er", "0", "--allreduce", "0"] + choco)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["value"] > 0 and out["parity_ok"] is True
    if overlap == "on":
        assert out["overlap"]["chosen_form"] == "rccl_chunked" and "rccl_chunked" in out["config"]["parallelism"]
    elif pull == "on":
        # the pull form's two snapshot buffers each reused >= 3 times within the rounds parity covers
        # (a stale line of round r - 2 would break parity_ok)
        assert out["overlap"]["chosen_form"] == "pull" and out["overlap"]["pull_unavailable"] is None
        assert out["overlap"]["pull_rounds"] >= 6, out["overlap"]
        assert out["overlap"]["pull_gate_error"] is None, out["overlap"]
        ch = out["choco"]
        assert ch["form"] in ("pull", "pull_direct") and ch["pull_rounds"] >= 6 and ch["pull_gate_error"] is None, ch
        assert ch["parity_ok"] is True, ch
        assert ch["ipc_refused"] == 0 and ch["bind_failures"] == 0 and ch["binds"] > 0, ch
    elif overlap == "off" and pull == "off":
        assert out["overlap"] is None
    else:
        assert set(out["overlap"]["calib_ms"]) == {"rccl", "rccl_chunked", "pull"}
    if out["overlap"] is not None and out["overlap"].get("calib_ms"):
        # every calibrated form's rounds passed the oracle before one was chosen
        assert out["overlap"]["calib_parity_ok"] == {k: True for k in out["overlap"]["calib_ms"]}, out["overlap"]
    if pull != "off":                     # every pull bind succeeded, no refused export
        ov = out["overlap"]
        assert ov["ipc_refused"] == 0 and ov["bind_failures"] == 0 and ov["binds"] > 0, ov


def test_bench_falls_back_to_pull_without_rccl():
    """N > 1 when the library's RCCL communicator cannot be created (--debug-no-rccl: as if it
    failed on every rank): the gossip runs over the pull transport alone -- headline, MATCHA,
    Choco (both pull reads calibrated) and the configs each pass the oracle self-check, the line
    says why (rccl_unavailable) and the RCCL-only figures are skipped, not failed."""
    r = _torchrun(2, ["bench.py", "--gpus", "2", "--transport", "gloo", "--debug-no-rccl", "--steps", "3",
                      "--warmup", "1", "--params", "100000", "--choco-params", "100000", "--cpu-seconds", "0",
                      "--wrn-params", "50000", "--resnet-params", "20000", "--mlp-params", "30000", "--lb-rounds", "20", "--er-params", "20000",
                      "--er-rounds", "1", "--er-budgets", "1.0"], timeout=280)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert "error" not in out, out["error"]
    assert out["rccl_unavailable"] and out["overlap"]["chosen_form"] == "pull" and out["parity_ok"] is True
    assert out["overlap"]["pull_rounds"] >= 6 and out["overlap"]["pull_gate_error"] is None
    assert out["matcha_schedule"]["parity_ok"] is True
    assert set(out["choco"]["calib_ms"]) == {"pull", "pull_direct"} and out["choco"]["parity_ok"] is True
    cf = out["configs"]
    assert "error" not in cf and "skipped" not in cf, cf
    assert all(v["parity_ok"] is True for k, v in cf.items() if k != "parity"), cf
    assert out["er64_sweep"]["form"] == "pull" and out["er64_sweep"]["parity_ok"] is True
    assert "skipped" in out["allreduce_baseline"] and out["xgmi"]["exchange_only_ms"] is None
    pt = out["pull_transport"]
    assert pt["binds"] > 0 and pt["ipc_refused"] == 0 and pt["bind_failures"] == 0, pt


def test_bench_real_rccl_refusal_falls_back_to_pull():
    """the same fallback driven by a REAL RCCL failure, not the test hook -- the rccl
    transport with both ranks on GPU 0 (--debug-share-gpu), so ncclCommInitRankConfig refuses
    ("invalid usage": RCCL takes no two ranks on one device).  The bench's own collectives run on
    its gloo process group, so nothing else depends on RCCL: every rank continues over the pull
    transport, every figure's oracle self-check passes and the run exits 0."""
    r = _torchrun(2, ["bench.py", "--gpus", "2", "--debug-share-gpu", "--steps", "3", "--warmup", "1",
                      "--params", "100000", "--choco-params", "100000", "--cpu-seconds", "0", "--wrn-params", "50000",
                      "--resnet-params", "20000", "--mlp-params", "30000", "--lb-rounds", "20", "--er-params", "20000", "--er-rounds", "1",
                      "--er-budgets", "1.0", "--figure-timeout", "60"], timeout=280)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert "error" not in out, out["error"]
    assert "ncclCommInitRank" in out["rccl_unavailable"] and out["rccl_ranks"] is None, out["rccl_unavailable"]
    assert out["overlap"]["chosen_form"] == "pull" and out["parity_ok"] is True
    assert out["matcha_schedule"]["parity_ok"] is True and out["choco"]["parity_ok"] is True
    assert all(v["parity_ok"] is True for k, v in out["configs"].items() if k != "parity"), out["configs"]
    assert out["er64_sweep"]["parity_ok"] is True
    pt = out["pull_transport"]
    assert pt["binds"] > 0 and pt["ipc_refused"] == 0 and pt["bind_failures"] == 0, pt


def test_pull_gate_stalled_peer_raises():
    """PullTransport without a host barrier: a rank whose peer stops publishing is held by the
    device gate's BOUNDED wait (mx_pull_gate, 2 s deadline here) and communicate() raises MXError
    naming the peer -- no hang; the error is sticky (the next step raises at once); the stalled
    peer's own round completes once it resumes."""
    r = _torchrun(2, [os.path.join(HERE, "mp_pull_stall.py")], timeout=150)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["first_rounds_ok"] and out["raised"] and out["sticky"] and out["peer_round_ok"], out
    assert out["pull_ipc_clean"], out
    assert "rank 1 did not publish" in out["message"], out
    assert 1.5 <= out["seconds"] < 30, out


@pytest.mark.parametrize("nproc", [4, 8])
def test_pull_rounds_with_drifting_ranks(nproc):
    """The pull transport's device gate under drift: rounds enqueued back to back while every rank
    sleeps a random 0-3 ms before some of them (ranks several rounds apart, gates really waiting),
    whole rows (graph 2) and Choco messages (fetch and direct reads) -- every worker bit-exact vs the
    oracle at the end."""
    r = _torchrun(nproc, [os.path.join(HERE, "mp_pull_stress.py")], timeout=280)
    assert r.returncode == 0, _why(r)
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["world"] == nproc and all(v for k, v in res.items() if k != "world"), res


def test_bench_self_launch_gloo():
    """`python bench.py --gpus 2` WITHOUT torchrun: the parent starts the ranks
    as a child torch.distributed.run and relays rank 0's line -- n_gpus 2, the oracle self-check
    true, the launcher recorded (gloo transport: both ranks share this box's one GPU)."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--transport", "gloo", "--steps", "3",
                        "--warmup", "1", "--params", "100000", "--choco", "0", "--cpu-seconds", "0", "--configs",
                        "0", "--er", "0", "--allreduce", "1"], cwd=ROOT, capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, _why(r)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["parity_ok"] is True and out["launcher"]["self_launched"] is True
    assert out["rccl_ranks"] is None                       # gloo transport: no RCCL communicator
    assert out["allreduce_baseline"]["parity_ok"] is True


def test_dropin_communicators_one_process_per_worker():
    """train_mpi.py's deployment: 8 processes, one worker each, decenCommunicator /
    ChocoCommunicator(rank, 8, GP, ...).communicate(model) with GPU- and CPU-resident models,
    bit-exact vs the oracle every round (8 ranks share GPU 0; gloo transport)."""
    r = _torchrun(8, [os.path.join(HERE, "mp_dropin.py")], timeout=280)
    assert r.returncode == 0, _why(r)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == 8 and all(v for k, v in res.items() if k != "world"), res


def test_rank_trainer_matches_virtual_trainer():
    """train_mpi.py's per-rank loop (harness.RankTrainer: sync_allreduce, then per batch SGD step +
    communicate(model)) over 8 processes -- gossip through the gloo test transport and through the
    pull transport (decen and Choco) -- ends with every worker's parameters bit-identical to the
    single-process VirtualTrainer's (2 epochs, MATCHA 0.5, momentum 0.9)."""
    r = _torchrun(8, [os.path.join(HERE, "mp_trainer.py")], timeout=280)
    assert r.returncode == 0, _why(r)
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["world"] == 8 and all(v for k, v in res.items() if k != "world"), res


def test_rccl_single_rank_linkage():
    """The library's own RCCL communicator (unique id over torch.distributed, ncclCommInitRank,
    all-reduce mean, an exchange round with nothing to move, destroy) under torchrun with the nccl
    backend -- the N > 1 transport's linkage against the RCCL torch loaded."""
    r = _torchrun(1, [os.path.join(HERE, "rccl_single.py")], timeout=150)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out == {"rank": 0, "nranks": 1, "nonblocking": True, "allreduce_identity": True, "decen_bit_exact": True,
                   "post_self_exchange": True, "post_validates": True, "post_validates_peer": True,
                   "allreduce_ordered_identity": True, "count": 1, "wait_deadline": True,
                   "wait_deadline_s_ok": True}, out


def test_bench_watchdog_line_on_stall():
    """A rank that hangs inside a figure (--debug-stall choco:1): its peer waits in the figure's
    collectives until the watchdog's deadline, rank 0 prints the line measured so far with ONE error
    naming the figure (its own watchdog's, or -- when rank 1's watchdog fired first and the launcher
    stopped rank 0 -- the SIGTERM handler's), and the job exits NON-zero (bench.EXIT_ABORTED per
    rank)."""
    r = _torchrun(2, ["bench.py", "--gpus", "2", "--transport", "gloo", "--steps", "3", "--warmup", "1",
                      "--params", "100000", "--choco-params", "100000", "--cpu-seconds", "0", "--configs", "0",
                      "--er", "0", "--figure-timeout", "15", "--debug-stall", "choco:1"], timeout=240)
    assert r.returncode != 0, _why(r)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, _why(r)
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["parity_ok"] is True
    assert "choco" in out["error"] and ("no progress" in out["error"] or "signal 15" in out["error"]), out["error"]
    assert out["allreduce_baseline"]["rounds_per_s"] > 0 and out.get("choco") is None


def test_rccl_init_deadline():
    """A 2-rank RCCL communicator whose second rank never joins: mx_rccl_init_timeout returns
    MX_ERR_RCCL ("timed out") after its 4 s deadline instead of hanging, and the process exits."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_deadline.py")], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["rc"] == -3 and out["handle_null"] and "never joined" in out["message"], out
    assert 3.5 <= out["seconds"] < 60, out


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (one RCCL rank each)")
def test_rccl_peer_skips_exchange():
    """Two ranks on two GPUs: after a first all-gather connected them, rank 1 skips the second.
    Rank 0's bounded wait (RcclComm.wait -> mx_rccl_wait) raises MXError within ~3 s and aborts
    the communicator instead of hanging.  Skipped on a one-GPU box: RCCL
    refuses two ranks on one device."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "rccl_skip.py")],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["first_ok"] and out["aborted"] and "did not drain" in (out["error"] or ""), out
    assert 2.5 <= out["seconds"] < 30, out


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (one RCCL rank each)")
def test_cross_gpu_transports_match_oracle():
    """One rank per GPU (2-4 GPUs): RCCL plain / pipelined exchange, Choco messages, the ordered
    all-reduce, and the pull transport's device gate with snapshots on other GPUs (the cross-L2
    coherence protocol), every worker's row bit-exact vs the oracle.  Skipped on a one-GPU box."""
    n = min(4, torch.cuda.device_count())
    r = _torchrun(n, [os.path.join(HERE, "mp_gpus.py")], timeout=280)
    assert r.returncode == 0, _why(r)
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["world"] == n and all(v for k, v in res.items() if k != "world"), res


def test_bench_single_gpu_line():
    """bench.py at N = 1 (headline shape, few rounds): the line's contract fields, the self-check,
    the per-round event statistics, the config and host-model figures and the CPU baseline legs."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "2",
                        "--choco-params", "200000", "--cpu-seconds", "1", "--er-params", "3e6",
                        "--er-budgets", "0.2,1.0"], cwd=ROOT, capture_output=True,
                       text=True, timeout=280, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["steps"] == 4 and out["warmup"] == 2 and out["value"] > 0
    assert "error" not in out and out["parity_ok"] is True and "oracle" in out["parity"]
    assert out["choco"]["parity_ok"] is True and out["matcha_schedule"]["parity_ok"] is True
    assert out["er64_sweep"]["parity_ok"] is True and out["er64_sweep"]["params_per_worker"] == 3_000_000
    assert all(out["configs"][k]["parity_ok"] for k in ("wrn28_10_matcha0.5", "wrn28_10_full",
                                                         "resnet18_100_matcha0.5", "mlp_fixed"))
    ru = out["round_us"]
    assert 0 < ru["events_min"] <= ru["events_median"]
    assert out["roofline"]["frac"] > 0 and out["roofline"]["min_launch_ms"] > 0
    assert out["cpu_resident_models"]["rounds_per_s"] > 0
    cfg = {k: v for k, v in out["configs"].items() if k != "parity"}
    assert set(cfg) == {"wrn28_10_matcha0.5", "wrn28_10_full", "resnet18_100_matcha0.5", "mlp_fixed"}
    # config 1 (FixedProcessor D-PSGD, MNIST MLP): GPU rounds and the reference's pickled CPU sequence
    assert cfg["mlp_fixed"]["cpu_pickle"]["rounds_per_s"] > 0 and cfg["mlp_fixed"]["graph_rounds_per_s"] > 0
    assert all(v["rounds_per_s"] > 0 and v["hbm_TBps"] > 0 for v in cfg.values())
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["pickle"]["value"] > 0 and cb["pickle"]["cores"] >= 1
    ar = out["allreduce_baseline"]
    assert ar["parity_ok"] is True and 0 < ar["roofline"]["frac"] < 1 and out["rccl_ranks"] is None
    assert ar["roofline"]["kernel"].startswith("mean_tile"), ar["roofline"]    # named from the dispatch
    assert out["choco"]["topk"]["fallback_compactions"] >= 0 and out["choco"]["topk"]["floor"] == "fine sampled"


def test_ipc_export_after_closing_imports():
    """The sequence behind the recorded export refusals: a block allocated right after this process
    closed a peer's IPC import can land on that import's address range, whose export the runtime
    refuses (tools/ipc_reuse_probe.py).  With mx_ipc_alloc's hold-and-reallocate (default) every
    re-export of the probe's close-then-allocate loop succeeds, 2 ranks x 3 sizes x 2 x 10 rounds."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tools", "ipc_reuse_probe.py")]
    env = dict(os.environ, OMP_NUM_THREADS="2", ITERS="10", MODES="safe_hold")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, _why(r)
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["safe_hold"] and all(v == 0 for v in out["safe_hold"].values()), out
