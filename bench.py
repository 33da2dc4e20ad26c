"""Gossip-round benchmark (BASELINE.json metric): rounds/s of one MATCHA gossip round over
8 workers x 25.6M fp32 params on graph 0 (util.py:281-285), with HBM / xGMI rooflines.

    python bench.py [--gpus N] [--steps K] [--warmup W]            # N = 1: all 8 workers on 1 GPU
    torchrun --nproc-per-node N ... bench.py --gpus N               # workers split over N GPUs

A "step" is one gossip round of the whole 8-worker job (flatten + partner exchange + FMA-chain
mixing + unflatten, fused: communicator.py:133-158).  Workload: full rounds (every matching
active -- the worst case, 2 * 8 * P * 4 bytes of HBM traffic per round on one GPU); inputs are
synthetic (splitmix64 uniform[-1,1)) and resident in HBM before timing starts.  Rank 0 prints
one JSON line.

Parity: after the timed region every figure is checked against the CPU oracle (oracle/, the
restatement pinned to the reference's own outputs) -- the oracle is the checker only, loaded
after the measurements, never timed and never on the measured path.

Secondary figures (MATCHA C_b = 0.5, all-reduce, ChocoSGD, host-resident models, the WRN-28-10 /
CIFAR-ResNet configs, the ER(64) budget sweep) each run under a watchdog deadline
(--figure-timeout) and a total budget (--figures-budget): a figure that hangs (e.g. a peer rank
gone) makes rank 0 print the line measured so far with an "error" field and every rank exit with
status 3 (EXIT_ABORTED), instead of losing the headline or hanging.
"""
import argparse
import json
import os
import random
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG_NAME = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"

HBM_PEAK = 8.0e12          # bytes/s, MI355X spec (MI355X_MICROARCH.md)
XGMI_LINK_PEAK = 153e9     # bytes/s per direction per link
METRIC = "gossip rounds/sec (8 workers x 25.6M fp32 params, graph 0, full MATCHA round)"
# Fixed per-round cost of each N > 1 exchange form (seconds), for the `predicted` object.  pull:
# measured with tools/form_overhead.py at P = 100k, N processes sharing one GPU (profiles/
# r05b_pull_overhead_after_n*.log: snapshot publish + gate + mix launches, device gate).  RCCL:
# a cross-GPU group cannot run on a one-GPU box (RCCL refuses two ranks on one device); its floor
# is measured with a one-rank self send + receive in one group, back to back (tools/
# rccl_overhead.py, profiles/r05m_rccl_overhead.log: 7.3 us for 4 KB - 1.8 MB) -- a LOWER bound of a
# cross-GPU group's cost, one per exchange (one per chunk for the pipelined form).
PULL_FIXED_S = {2: 26e-6, 4: 31e-6, 8: 62e-6}
# the same for a ChocoSGD round under the pull transport, fetch form (message publish + gate + the
# fetch of the partners' messages, minus compress + apply with a transport that moves nothing;
# P = 100k, top-1 %: profiles/r05z_overhead_fetch_n*.log; the direct form measured 10.6 / 12.0 /
# 41.8 us, profiles/r05p_overhead_n*.log)
PULL_CHOCO_FIXED_S = {2: 11.9e-6, 4: 13.5e-6, 8: 47.5e-6}
PULL_TIMEOUT_S = 20.0      # the pull gate's deadline in the bench (lockstep rounds of at most a few ms)
RCCL_FIXED_S = 7.3e-6
PEER_GONE = ("Connection closed by peer", "Connection reset by peer", "Broken pipe")   # gloo / c10d errors
RCCL_WARMUP_WAIT_S = 60.0  # N > 1: deadline of the headline's first RCCL exchanges (then: pull transport)
LAUNCH_BOUND_ROUNDS = 400  # rounds per measurement of a launch-bound config (P < 1e6: ~6 us rounds), --lb-rounds
WARM_BURST = 10            # untimed warm-burst rounds before them, per measured round (N = 1; N > 1: 1)
EXIT_PARITY = 4            # exit status when the headline's oracle self-check failed (its value withheld)
EXIT_ABORTED = 3           # exit status of a rank whose run was cut short (watchdog, peer gone, SIGTERM)
HEADLINE_HBM_FRAC = 0.79   # the mixing kernel's measured fraction of 8 TB/s (round 6: profiles/r06u_bench.json)
SETTLE_MIN_BYTES = 64 << 20  # rounds streaming at least this much from HBM get a settle burst (settle_rounds)
SETTLE_MAX_ROUNDS = 400


def settle_rounds(bytes_per_round, settle_ms):
    """Untimed rounds to run before a figure's timed region so its rounds stream at the settled
    clock, as the headline's settle blocks do: after a pause (a figure's allocation and fill) the
    mixing kernel runs ~278 us, then 305-320 us, and settles at 255-258 us only after ~50 launches,
    ~14 ms of streaming (DVFS give-back, MI355X_MICROARCH.md; profiles/r06w_dvfs_ramp.json).  About
    `settle_ms` of streaming at HEADLINE_HBM_FRAC of the peak; 0 below SETTLE_MIN_BYTES per round
    (launch-bound rows have their own warm burst).  `bytes_per_round` must be the same on every
    rank (the N > 1 rounds exchange in lockstep)."""
    if settle_ms <= 0 or bytes_per_round < SETTLE_MIN_BYTES:
        return 0
    per_round_s = bytes_per_round / (HEADLINE_HBM_FRAC * HBM_PEAK)
    return int(min(SETTLE_MAX_ROUNDS, -(-settle_ms * 1e-3 // per_round_s)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--params", type=int, default=25_600_000)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--budget", type=float, default=1.0, help="1.0 = full rounds (headline)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--choco", type=int, default=1, help="also time ChocoSGD rounds (VGG-16 size, top-1%%)")
    ap.add_argument("--choco-params", type=int, default=14_774_436, help="Choco figure row size (VGG-16)")
    ap.add_argument("--transport", choices=("rccl", "gloo"), default="rccl",
                    help="N > 1 partner exchange: rccl (the product path, one GPU per rank) or gloo "
                         "(tests/gloo_transport.py: host staging, lets N ranks share one GPU to test "
                         "the multi-process path; never a performance number)")
    ap.add_argument("--settle-ms", type=float, default=50.0, help="diagnostic rounds (per-round HIP events) "
                    "run for at least this long between the warmup and the timed region")
    ap.add_argument("--configs", type=int, default=1, help="also time the WRN-28-10 and CIFAR-ResNet configs' "
                    "rounds (BASELINE configs 2-3) on the same GPUs")
    ap.add_argument("--wrn-params", type=int, default=36_546_980, help="config 3 row size (WRN-28-10)")
    ap.add_argument("--resnet-params", type=int, default=181_668, help="config 2 row size (ResNet(18,100))")
    ap.add_argument("--mlp-params", type=int, default=666_547, help="config 1 row size (MNIST_MLP(47))")
    ap.add_argument("--lb-rounds", type=int, default=LAUNCH_BOUND_ROUNDS, help="rounds per measurement of a "
                    "launch-bound config (P < 1e6), after a warm burst of 10x as many (N = 1; N > 1: as many)")
    ap.add_argument("--er", type=int, default=1, help="also run config 5: the ER(64, 0.1, 1234) MATCHA budget "
                    "sweep 0.1 .. 1.0 (1e9 params per worker where memory allows)")
    ap.add_argument("--er-params", type=float, default=1e9, help="config 5 row size (reduced to what fits, "
                    "recorded in the line)")
    ap.add_argument("--er-rounds", type=int, default=3, help="timed rounds per budget of the ER sweep")
    ap.add_argument("--er-budgets", default="0.1,0.2,0.3,0.4,0.5,0.6,0.7,0.8,0.9,1.0")
    ap.add_argument("--staged", type=int, default=1, help="N = 1: also time host-resident models (the drop-in "
                    "communicators' staging path for CPU models)")
    ap.add_argument("--allreduce", type=int, default=1, help="also time all-reduce averaging (the paper's "
                    "centralized baseline) on the same rows")
    ap.add_argument("--overlap", choices=("auto", "on", "off"), default="auto",
                    help="N > 1: column-pipelined exchange (RCCL on a side stream overlapped with mixing; "
                         "VirtualWorkerGroup chunk_cols) -- auto: time both forms over a few untimed rounds and "
                         "use the faster for the timed region; on / off: force")
    ap.add_argument("--pull", choices=("auto", "on", "off"), default="auto",
                    help="N > 1: also calibrate the pull transport (partner rows read from the peers' IPC-mapped "
                         "HBM by the mixing kernel) and time it if fastest (auto), force it (on) or skip it (off)")
    ap.add_argument("--chunk-cols", type=int, default=0, help="pipelined chunk width (0: a quarter of the row)")
    ap.add_argument("--placement", choices=("auto", "contiguous"), default="auto",
                    help="N > 1: which workers share a GPU -- auto (placement.best_placement, fewest rows "
                         "over the busiest xGMI pair) or contiguous id blocks")
    ap.add_argument("--figure-timeout", type=float, default=240.0, help="watchdog deadline per secondary "
                    "figure (s): past it rank 0 prints the line so far with an error and every rank exits")
    ap.add_argument("--figures-budget", type=float, default=600.0, help="total wall time for the secondary "
                    "figures (s); the ones left when it is spent are skipped")
    ap.add_argument("--headline-timeout", type=float, default=300.0, help="watchdog deadline of the headline "
                    "measurement (s)")
    ap.add_argument("--pg-timeout", type=float, default=1800.0, help="torch.distributed timeout (s), above "
                    "the watchdog's")
    ap.add_argument("--debug-skip", default="", help="test hook FIGURE:RANK -- that rank skips that figure "
                    "(its peers then wait in the figure's collectives: exercises the watchdog)")
    ap.add_argument("--debug-no-rccl", action="store_true", help="test hook: behave as if the library's RCCL "
                    "communicator could not be created on any rank (the gossip then runs over the pull transport "
                    "alone)")
    ap.add_argument("--debug-share-gpu", action="store_true", help="test hook: with the rccl transport, ranks "
                    "share the visible GPUs (local rank modulo their count), so creating the library's RCCL "
                    "communicator fails for real (RCCL refuses two ranks on one device) and the gossip falls back "
                    "to the pull transport")
    ap.add_argument("--debug-stall", default="", help="test hook FIGURE:RANK -- that rank stalls inside that "
                    "figure (a hung peer: exercises the watchdog)")
    return ap.parse_args()


# ----------------------------------------------------------------------------------- the checker
def _oracle():
    """The CPU oracle (oracle/oracle.py over liboracle.so) -- the checker.  Loaded only by the
    parity checks and the CPU baseline, after the GPU measurements."""
    p = os.path.join(ROOT, "oracle")
    if p not in sys.path:
        sys.path.insert(0, p)
    import oracle as O
    return O


def synth_columns(workers, cols, seed0=1234):
    """{worker: its synthetic row (mx_synth_fill(seed0 + worker)) at `cols`} from the oracle's
    counter-based generator -- the columns before any round, without a device read."""
    O = _oracle()
    return {int(w): O.synth_at(seed0 + int(w), cols) for w in workers}


def oracle_column_parity(topology, init, final, applied):
    """Every worker's sampled columns after the rounds `applied` (iterations, in order) vs the
    oracle's decenCommunicator round (communicator.py:92-122) run on the same columns from the
    same initial values.  A gossip round mixes each column on its own, so the columns alone are
    a complete check of those columns.  uint32 compare."""
    O = _oracle()
    n = int(topology.size)
    flags = np.asarray(topology.active_flags, np.uint8)
    partner = np.asarray(topology.neighbors_info, np.int32).reshape(-1, n)[:flags.shape[1]]
    X = np.ascontiguousarray(np.stack([init[w] for w in range(n)]).astype(np.float32))
    for it in applied:
        if flags[it].any():
            X = O.decen_round(X, partner, flags[it], topology.neighbor_weight)
    got = np.stack([final[w] for w in range(n)])
    return bool(np.array_equal(got.view(np.uint32), X.view(np.uint32)))


# ----------------------------------------------------------------------------------- watchdog
class Watchdog:
    """Deadline on a phase of the run.  When the armed deadline passes (a collective whose peer
    never arrives, a hang), rank 0 prints the line built so far with an "error" field and every
    rank leaves with os._exit(EXIT_ABORTED) -- an exit, never an exec, and a NON-zero status, so the
    launcher's (and the driver's) exit code tells an aborted run from a clean one.  A rank that
    leaves first makes the launcher SIGTERM the others: rank 0 then prints from on_term (main)."""

    def __init__(self, rank, emit):
        self.rank, self.emit = rank, emit
        self.lock = threading.Lock()
        self.name = self.deadline = self.seconds = None
        self.armed_at = time.monotonic()
        t = threading.Thread(target=self._run, daemon=True)
        t.start()

    HEARTBEAT_S = 60.0          # rank 0: one stderr line per minute naming the running phase

    def arm(self, name, seconds):
        with self.lock:
            self.name, self.seconds, self.deadline = name, seconds, time.monotonic() + seconds
            self.armed_at = time.monotonic()

    def disarm(self):
        with self.lock:
            self.deadline = None

    def _run(self):
        beat = time.monotonic()
        while True:
            time.sleep(0.25)
            with self.lock:
                fire = self.deadline is not None and time.monotonic() > self.deadline
                name, secs = self.name, self.seconds
                running = self.deadline is not None
            if self.rank == 0 and running and time.monotonic() - beat > self.HEARTBEAT_S:
                beat = time.monotonic()
                sys.stderr.write(f"[bench] {name}: running for {beat - self.armed_at:.0f} s\n")
                sys.stderr.flush()
            if fire:
                msg = (f"{name}: no progress within {secs:.0f} s on rank {self.rank} (a peer rank did not take "
                       f"part or hung); the figures after it were not run")
                sys.stderr.write(f"[bench watchdog] {msg}\n")
                sys.stderr.flush()
                if self.rank == 0:
                    self.emit(msg)
                os._exit(EXIT_ABORTED)


class Line:
    """The one JSON line rank 0 prints (once: normally at the end, or by the watchdog)."""

    def __init__(self, rank):
        self.rank = rank
        self.out = {"metric": METRIC, "value": None, "unit": "rounds/s"}
        self.lock = threading.Lock()
        self.printed = False

    def emit(self, error=None):
        with self.lock:
            if self.printed or self.rank != 0:
                return
            out = dict(self.out)
            if error:
                out["error"] = error
            try:
                s = json.dumps(out)
            except (TypeError, ValueError) as e:          # a figure mid-update: keep the headline
                s = json.dumps({k: out[k] for k in out if isinstance(out[k], (int, float, str, type(None)))}
                               | {"error": f"{error}; line not serialisable: {e}"})
            print(s, flush=True)
            self.printed = True


# ----------------------------------------------------------------------------------- helpers
def pickle_leg(partner, alpha, P, seconds):
    """The reference's per-rank sequence with its pickled transport (oracle/pickle_ranks.py): one
    process per worker pinned to its own core, torch.cat flatten, pickle.dumps -> pipe ->
    pickle.loads per active edge, add_(alpha), copy_ back -- what mpirun's 8 ranks spend per
    round (pickling dominates).  Full rounds; bounded by `seconds`."""
    _oracle()
    import pickle_ranks as PR
    flags1 = np.ones((1, partner.shape[0]), np.uint8)
    one, cores, _ = PR.run(partner, flags1, alpha, P)
    rounds = max(1, min(20, int(seconds / max(one, 1e-6))))
    el, cores, _ = PR.run(partner, np.ones((rounds, partner.shape[0]), np.uint8), alpha, P)
    return {"value": rounds / el, "unit": "rounds/s", "cores": cores, "kind": "port",
            "sample": f"{rounds} full rounds, graph 0, {partner.shape[1]} worker processes x {P} fp32 in "
                      f"{PR.TENSOR_SPLIT} tensors, {el:.1f} s; oracle/pickle_ranks.py: torch.cat flatten, "
                      f"pickled tensor per active edge over OS pipes, add_ chain, copy_ back, one process "
                      f"pinned per core (nproc {os.cpu_count()})"}


MLP_TENSORS = 6            # MNIST_MLP(47) (models/MLP.py): 666,547 params in 6 tensors


def mlp_pickle_leg(GP, P, seconds):
    """Config 1 on the host as the reference runs it: the FixedProcessor schedule's rounds through
    oracle/pickle_ranks.py (torch.cat flatten of the 6 MLP tensors, pickled sendrecv per active
    edge over OS pipes, add_ chain, copy_ back; one process per worker pinned to its own core),
    bounded by `seconds`."""
    _oracle()
    import pickle_ranks as PR
    flags = np.asarray(GP.active_flags, np.uint8)
    partner = np.asarray(GP.neighbors_info, np.int32).reshape(-1, int(GP.size))[:flags.shape[1]]
    one, _, _ = PR.run(partner, flags[:2], GP.neighbor_weight, P, nseg=MLP_TENSORS)
    rounds = max(2, min(400, int(seconds / max(one / 2, 1e-6))))
    reps = np.resize(flags[:2], (rounds, flags.shape[1]))                 # the alternating schedule
    el, cores, _ = PR.run(partner, reps, GP.neighbor_weight, P, nseg=MLP_TENSORS)
    return {"rounds_per_s": rounds / el, "cores": cores, "kind": "port",
            "sample": f"{rounds} rounds of the FixedProcessor schedule, {partner.shape[1]} worker processes x "
                      f"{P} fp32 in {MLP_TENSORS} tensors, {el:.1f} s (oracle/pickle_ranks.py)"}


def cpu_baseline(partner, alpha, n, P, seconds):
    """The oracle's port of the reference per-rank sequence (cat-flatten, sendrecv copy, add_
    FMA chain, copy_ back), one OpenMP thread per worker, on this box's host cores; beside it the
    same sequence with the reference's pickled transport, one process per worker."""
    O = _oracle()
    threads = min(n, os.cpu_count() or 1)
    rows = [[O.synth(1234 + i, P)] for i in range(n)]
    flags = np.ones((1, partner.shape[0]), np.uint8)
    t = time.time()
    O.baseline_rounds(rows, partner, flags, alpha, threads=threads)
    one = time.time() - t
    rounds = max(1, min(200, int(seconds / max(one, 1e-6))))
    flags = np.ones((rounds, partner.shape[0]), np.uint8)
    t = time.time()
    O.baseline_rounds(rows, partner, flags, alpha, threads=threads)
    el = time.time() - t
    # single-process variant: every worker's sequence on one core
    t = time.time()
    O.baseline_rounds(rows, partner, flags[:1], alpha, threads=1)
    el1 = time.time() - t
    return {"value": rounds / el, "unit": "rounds/s", "cores": threads, "kind": "port",
            "sample": f"{rounds} full rounds, graph {0}, {n} workers x {P} fp32 (same workload), "
                      f"{el:.1f} s; oracle/matcha_oracle.c orc_baseline_rounds, {threads} OpenMP threads "
                      f"(one per worker, like the mpirun ranks) of {os.cpu_count()} host CPUs",
            "single_core": {"value": 1.0 / el1, "unit": "rounds/s", "cores": 1,
                            "sample": f"1 full round, all {n} workers on one thread, {el1:.1f} s"},
            "pickle": pickle_leg(partner, alpha, P, seconds)}


def pmc_traffic(kernel_prefix="mix_kernel"):
    """HBM bytes per launch of the mixing kernel from the newest committed rocprofv3 PMC summary
    (tools/profile_round.sh -> profiles/rocprof_<round>.json; FETCH_SIZE x2 + WRITE_SIZE)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "rocprof_r[0-9]*.json")))   # headline summaries only
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    vals = [v.get("hbm_bytes_per_launch") for k, v in d.get("mix_pmc", {}).items() if kernel_prefix in k]
    vals = [v for v in vals if v]
    return (max(vals) if vals else None), os.path.relpath(files[-1], ROOT)


RATE_KEYS = ("value", "ms_per_step", "rounds_per_s", "ms_per_round", "graph_rounds_per_s", "graph_us_per_round",
             "hbm_TBps", "hbm_TBps_rank0", "roofline", "busiest_link_GBps")


def withhold_unverified(obj):
    """A figure whose oracle self-check failed reports no rate: its rate keys move under
    "unverified" (recursively: configs' entries, the ER sweep's budgets) -- a fast wrong result is
    not a number (the pull forms' cross-GPU coherence is pinned only by this check
    until tests/mp_gpus.py runs on >= 2 GPUs).  Returns True if anything was withheld."""
    hit = False
    if isinstance(obj, dict):
        if obj.get("parity_ok") is False:
            moved = {k: obj.pop(k) for k in list(obj) if k in RATE_KEYS}
            if moved:
                obj["unverified"] = moved
            hit = True
        for v in list(obj.values()):
            hit |= withhold_unverified(v)
    elif isinstance(obj, list):
        for v in obj:
            hit |= withhold_unverified(v)
    return hit


def guarded(name, fn):
    """A secondary figure: an exception is reported in the line as {"error": ...} instead of
    losing the headline line; traceback to stderr."""
    try:
        return fn()
    except Exception as e:                       # noqa: BLE001 -- reported, not swallowed
        import traceback
        traceback.print_exc()
        return {"error": f"{name}: {type(e).__name__}: {e}"}


def max_over_ranks(x, world, dev="cpu"):
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([float(x)], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pull_counts(pkg, world):
    """The pull transport's bind accounting so far, summed over ranks (collective at N > 1):
    binds, failed binds, IPC exports, allocations left without an export (refused) and refused
    blocks a second allocation recovered (engine.pull_stats) -- both show here and in the
    multi-process tests' checks, never silently."""
    st = pkg.pull_stats()
    keys = ("binds", "bind_failures", "ipc_exports", "ipc_refused", "ipc_recovered")
    v = [float(st[k]) for k in keys]
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor(v)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        v = t.tolist()
    return {k: int(x) for k, x in zip(keys, v)}


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def timed_loop(fn, first, K, world, dev):
    """K calls fn(first + j) between synchronize + barrier on both sides; seconds, max over ranks."""
    torch.cuda.synchronize()
    barrier(world)
    t = time.perf_counter()
    for j in range(K):
        fn(first + j)
    torch.cuda.synchronize()
    barrier(world)
    return max_over_ranks(time.perf_counter() - t, world, dev)


def exchange_only(group, first, K, world, dev):
    """N > 1 diagnostic: the RCCL exchange of K rounds alone (no mixing; rows do not change):
    (max over ranks, [per rank]) of the back-to-back wall time per round."""
    import torch.distributed as dist
    eng = group.engine
    slab = group.slab.data_ptr() if group.slab is not None else None
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter()
    for j in range(K):
        eng.exchange(first + j, group._row_ptrs, slab, group.ld * 4, group.numel * 4)
    torch.cuda.synchronize()
    mine = (time.perf_counter() - t) / K
    per = [None] * world
    dist.all_gather_object(per, mine)
    dist.barrier()
    return max(per), per


def sample_columns(P):
    """64 columns spread over a row, including both ends and a 1024-column tile edge"""
    c = np.linspace(0, P - 1, 64).astype(np.int64)
    if P > 1025:
        c[1], c[2] = 1023, 1024
    return np.unique(c)


def gather_columns(g, cols_dev, world, dev):
    """{worker id: its row at the sampled columns} from every rank, on every rank"""
    import torch.distributed as dist
    loc = g.rows.index_select(1, cols_dev).cpu().numpy()
    mine = (list(g.workers), loc)
    objs = [mine]
    if world > 1:
        objs = [None] * world
        dist.all_gather_object(objs, mine)
    out = {}
    for ws, blk in objs:
        for i, w in enumerate(ws):
            out[int(w)] = blk[i]
    return out


def fill_synth(pkg, g, seed0=1234):
    for r in range(g.n_local):
        pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[r].data_ptr(), g.numel, seed0 + g.workers[r], None))


def round_bytes(partner, owner, flags_rows, rank, row_base, n_local, P):
    """Per round: (this GPU's algorithmic HBM bytes of the mixing kernel, busiest directed link
    bytes, busiest GPU pair both directions, all link bytes).  HBM: every local row with degree > 0
    read and written once, every received slab row read once; links: a row crosses to a GPU at
    most once per round (mx_exchange_plan)."""
    n = partner.shape[1]
    hbm, link, pair_b, total = [], [], [], []
    for f in flags_rows:
        deg = np.zeros(n, int)
        for g in range(len(f)):
            if f[g]:
                deg += partner[g] >= 0
        act = sum(1 for i in range(row_base, row_base + n_local) if deg[i] > 0)
        moved = set()
        for g in range(len(f)):
            if not f[g]:
                continue
            for p in range(n):
                q = partner[g, p]
                if q >= 0 and owner[p] != owner[q]:
                    moved.add((p, int(owner[q])))
        links = {}
        for p, b in moved:
            a = int(owner[p])
            links[(a, b)] = links.get((a, b), 0) + P * 4
        remote = sum(1 for p, b in moved if b == rank)
        hbm.append(2 * act * P * 4 + remote * P * 4)
        link.append(max(links.values()) if links else 0)
        total.append(sum(links.values()))
        pr = {}
        for (a, b), v in links.items():
            k = (min(a, b), max(a, b))
            pr[k] = pr.get(k, 0) + v
        pair_b.append(max(pr.values()) if pr else 0)
    return hbm, link, pair_b, total


def published_rows(partner, flags_rows, row_base, n_local):
    """Mean over rounds of the local rows a pull round publishes (mx_snapshot_publish_rows): rows
    with an active partner outside [row_base, row_base + n_local)."""
    cnt = []
    for f in flags_rows:
        c = 0
        for r in range(row_base, row_base + n_local):
            c += any(f[g] and partner[g, r] >= 0 and not (row_base <= partner[g, r] < row_base + n_local)
                     for g in range(len(f)))
        cnt.append(c)
    return float(np.mean(cnt)) if cnt else 0.0


def predict_round(form, world, link_bytes, mix_s, publish_bytes, chunks=4, mix_source="measured"):
    """What a round of `form` should cost at N = world, from its parts: the busiest
    xGMI link's bytes at 153 GB/s, the mixing kernel on this GPU (mix_s), the form's fixed cost
    (PULL_FIXED_S measured / RCCL_FIXED_S a measured lower bound) and, for pull, the snapshot copy at the headline's
    HBM fraction (publish_bytes: read + write of the rows a peer reads, published_rows).  plain RCCL:
    exchange, then mix (one stream); pipelined: the longer of the two plus one chunk of the shorter;
    pull: publish, then the mix reading partners over xGMI."""
    t_link = link_bytes / XGMI_LINK_PEAK
    if form == "pull":
        fixed = PULL_FIXED_S.get(world, max(PULL_FIXED_S.values()))
        src = "measured (tools/form_overhead.py, N processes sharing one GPU)"
        t_pub = publish_bytes / (HEADLINE_HBM_FRAC * HBM_PEAK)
        t = t_pub + max(t_link, mix_s) + fixed
    elif form == "rccl_chunked":
        fixed, src, t_pub = chunks * RCCL_FIXED_S, "lower bound: one-rank RCCL self-exchange (tools/rccl_overhead.py)", 0.0
        t = max(t_link, mix_s) + min(t_link, mix_s) / chunks + fixed
    else:
        fixed, src, t_pub = RCCL_FIXED_S, "lower bound: one-rank RCCL self-exchange (tools/rccl_overhead.py)", 0.0
        t = t_link + mix_s + fixed
    return {"busiest_link_bytes": float(link_bytes), "link_bound_ms": 1e3 * t_link, "mix_ms": 1e3 * mix_s,
            "mix_source": mix_source, "publish_ms": 1e3 * t_pub, "fixed_ms": 1e3 * fixed, "fixed_source": src,
            "round_ms": 1e3 * t, "rounds_per_s": 1.0 / t if t > 0 else None,
            "xgmi_frac": (link_bytes / t / XGMI_LINK_PEAK) if t > 0 else None}


def predict_choco(form, world, link_bytes, local_s, publish_bytes):
    """What a ChocoSGD round of `form` should cost at N = world: this rank's compress
    + apply with a transport that moves nothing (local_s, measured in the same run, max over ranks),
    plus the busiest link's message bytes at 153 GB/s, plus the form's fixed cost (RCCL: the
    one-rank self-exchange floor, a lower bound; pull: PULL_CHOCO_FIXED_S measured, and the message
    snapshot copy at the headline's HBM fraction).  Serial sum: the messages cross before the apply."""
    t_link = link_bytes / XGMI_LINK_PEAK
    if form == "pull":
        fixed = PULL_CHOCO_FIXED_S.get(world, max(PULL_CHOCO_FIXED_S.values()))
        src = "measured (tools/form_overhead.py, N processes sharing one GPU)"
        t_pub = publish_bytes / (HEADLINE_HBM_FRAC * HBM_PEAK)
    else:
        fixed, src, t_pub = RCCL_FIXED_S, "lower bound: one-rank RCCL self-exchange (tools/rccl_overhead.py)", 0.0
    t = local_s + t_pub + t_link + fixed
    return {"busiest_link_bytes": float(link_bytes), "link_bound_ms": 1e3 * t_link, "local_ms": 1e3 * local_s,
            "publish_ms": 1e3 * t_pub, "fixed_ms": 1e3 * fixed, "fixed_source": src, "round_ms": 1e3 * t,
            "rounds_per_s": 1.0 / t if t > 0 else None}


def p2p_probe(rank, world, nbytes, dev, reps=5, rccl=True):
    """N > 1: one xGMI link through RCCL (torch.distributed send/recv on an nccl group created for
    this figure -- the job's own process group is gloo), ranks 0 and 1 only: unidirectional 0 -> 1
    and bidirectional 0 <-> 1, seconds per transfer (max over the two ranks).  rccl=False (the gloo
    test transport): host buffers over the gloo group."""
    import torch.distributed as dist
    grp = dist.new_group(backend="nccl") if rccl else None       # collective: every rank
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda" if rccl else "cpu")
    rbuf = torch.empty_like(buf)
    res = {}
    for mode in ("uni", "bi"):
        for rep in range(reps + 1):                 # first transfer: connection setup, untimed
            torch.cuda.synchronize()
            dist.barrier()
            t = time.perf_counter()
            if rank in (0, 1):
                peer = 1 - rank
                ops = []
                if mode == "bi" or rank == 0:
                    ops.append(dist.P2POp(dist.isend, buf, peer, group=grp))
                if mode == "bi" or rank == 1:
                    ops.append(dist.P2POp(dist.irecv, rbuf, peer, group=grp))
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            torch.cuda.synchronize()
            el = time.perf_counter() - t
            if rep == 1:
                res[mode] = []
            if rep >= 1:
                res[mode].append(el if rank in (0, 1) else 0.0)
        res[mode] = max_over_ranks(float(np.median(res[mode])), world, dev)
    del buf, rbuf
    return res


# ----------------------------------------------------------------------------------- figures
def matcha_figure(pkg, args, rank, world, n, P, K, W, comm, dev):
    """The headline shape under a MATCHA C_b = 0.5 schedule (random matching subsets per round);
    oracle column parity over every round run."""
    warm = settle_rounds(2 * -(-n // world) * P * 4, args.settle_ms)     # same count on every rank
    W += warm
    np.random.seed(1234)
    GPm = pkg.MatchaProcessor(pkg.select_graph(args.graph), 0.5, rank, n, W + K, True)
    gm = pkg.VirtualWorkerGroup(GPm, numel=P, rank=rank, nranks=world, comm=comm, placement=args.placement)
    fill_synth(pkg, gm)
    for it in range(W):                          # warmup + settle burst (untimed)
        gm.step(it)
    el = timed_loop(gm.step, W, K, world, dev)
    fl = np.asarray(GPm.active_flags[W:W + K])
    cols = sample_columns(P)
    final = gather_columns(gm, torch.from_numpy(cols).cuda(), world, dev)
    gm.close()
    del gm
    torch.cuda.empty_cache()
    out = {"budget": 0.5, "rounds_per_s": K / el, "rounds": K, "warm_rounds": W,
           "probabilities": [round(float(x), 6) for x in GPm.probabilities],
           "alpha": GPm.neighbor_weight, "mean_active_matchings": float(fl.sum(1).mean()),
           "skipped_rounds": int((fl.sum(1) == 0).sum())}
    if rank == 0:
        out["parity_ok"] = oracle_column_parity(GPm, synth_columns(range(n), cols), final, range(W + K))
    return out


def allreduce_figure(pkg, args, rank, world, n, P, K, W, comm, dev, arena=None):
    """The centralized all-reduce averaging the paper compares gossip against
    (centralizedCommunicator.communicate, communicator.py:46-76; sync_allreduce, train_mpi.py:34-56):
    every worker's row becomes the fp32 sum of all workers' rows in the reference's order (mpi4py's
    binomial tree) divided by n -- through the product kernels:
      N = 1: mx_mean_rows_to over the n arena rows, in place (harness.sync_rows): ONE pass,
             2 * n * P * 4 bytes of HBM per round -> an HBM roofline like the headline's;
      N > 1: mx_allgather of each rank's rows (RCCL; the gloo test transport stages through the
             host) + mx_mean_rows_to into the rank's own rows (centralizedCommunicator._average /
             mx_allreduce_mean_ordered's kernels).
    Workers sit in contiguous id blocks (the tree order is by worker id).  Parity: every worker's
    64 sampled columns after the W + K rounds vs the oracle's central_mean applied W + K times."""
    from importlib import import_module
    E = import_module(PKG_NAME + ".engine")
    L = pkg.lib
    row_base, n_local = E.partition(n, world)[rank]
    if n % world:
        raise RuntimeError(f"allreduce figure: {n} workers do not split evenly over {world} ranks")
    W += settle_rounds(2 * (n // world) * P * 4, args.settle_ms)            # warmup + settle burst
    ld = (P + 63) // 64 * 64
    rows = arena if arena is not None and tuple(arena.shape) == (n_local, ld) else \
        torch.empty((n_local, ld), dtype=torch.float32, device="cuda")
    for r in range(n_local):
        pkg._lib.check(L.mx_synth_fill(rows[r].data_ptr(), P, 1234 + row_base + r, None))
    gather = torch.empty((n, ld), dtype=torch.float32, device="cuda") if world > 1 else None
    sp = pkg._lib.stream_ptr
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    timing = [False]

    def one(j):
        if world == 1:
            if timing[0] and j == 0:
                ev[0].record()
            pkg._lib.check(L.mx_mean_rows_to(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld, sp()),
                           "mx_mean_rows_to")
            if timing[0] and j == K - 1:
                ev[1].record()
            return
        flat = rows.view(-1)
        if hasattr(comm, "allgather"):                # gloo test transport
            comm.allgather(flat, gather.view(-1))
        else:
            pkg._lib.check(L.mx_allgather(comm.handle, flat.data_ptr(), flat.numel(), gather.data_ptr(), sp()),
                           "mx_allgather")
        pkg._lib.check(L.mx_mean_rows_to(gather.data_ptr(), n, ld, P, 0, rows.data_ptr(), n_local, ld, sp()),
                       "mx_mean_rows_to")

    for j in range(W):
        one(j)
    torch.cuda.synchronize()
    timing[0] = True
    el = timed_loop(one, 0, K, world, dev)
    cols = sample_columns(P)
    loc = rows[:, :P].index_select(1, torch.from_numpy(cols).cuda()).cpu().numpy()
    objs = [(row_base, loc)]
    if world > 1:
        import torch.distributed as dist
        objs = [None] * world
        dist.all_gather_object(objs, (row_base, loc))
    del gather
    if arena is None:
        del rows
    torch.cuda.empty_cache()
    out = {"rounds_per_s": K / el, "ms_per_round": 1e3 * el / K, "rounds": K, "warm_rounds": W,
           "order": "tree (mpi4py default)",
           "how": ("mx_mean_rows_to in place over the arena rows: one pass (harness.sync_rows)" if world == 1 else
                   "mx_allgather (RCCL) of every rank's rows + mx_mean_rows_to into this rank's rows")}
    if world == 1:
        alg = 2 * n * P * 4
        kern_ms = ev[0].elapsed_time(ev[1]) / K
        kname = L.mx_mean_kernel_name(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld).decode()   # its dispatch
        out["roofline"] = {"bound": "hbm", "kernel": f"{kname} (mx_mean_rows_to, tree order)", "bytes_per_launch": alg,
                           "avg_launch_ms": kern_ms, "achieved": alg / (kern_ms * 1e-3) / 1e9,
                           "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": alg / (kern_ms * 1e-3) / HBM_PEAK,
                           "note": "algorithmic bytes 2 x n x P x 4 (every row read once, the mean written to "
                                   "every row) / HIP events over the K timed launches"}
    if rank == 0:
        O = _oracle()
        got = np.zeros((n, len(cols)), np.float32)
        for base, blk in objs:
            got[base:base + blk.shape[0]] = blk
        X = np.stack([O.synth_at(1234 + w, cols) for w in range(n)])
        for _ in range(W + K):
            X = np.ascontiguousarray(np.broadcast_to(O.central_mean(X, "tree"), X.shape))
        out["parity_ok"] = bool(np.array_equal(got.view(np.uint32), X.view(np.uint32)))
        out["parity"] = (f"every worker's {len(cols)} sampled columns after {W + K} rounds vs the oracle's "
                         f"centralizedCommunicator round (orc_central_mean, mpi4py tree order) from the same "
                         f"synthetic rows, uint32")
    return out


def _choco_state(grp):
    P = grp.numel
    return {int(w): (grp.x[i, :P].cpu().numpy(), grp.x_hat[i, :P].cpu().numpy(), grp.s[i, :P].cpu().numpy())
            for i, w in enumerate(grp.workers)}


def choco_oracle_round(pkg, grp, GP, it, ratio, gamma, rank, world):
    """One more Choco round (iteration `it`, untimed) checked against the oracle's
    ChocoCommunicator round (communicator.py:175-268, compressors.py:3-19) from the same state:
    x, x_hat and s of every worker gathered before and after, uint32 compare on rank 0."""
    import torch.distributed as dist
    before = _choco_state(grp)
    grp.step(it)
    torch.cuda.synchronize()
    after = _choco_state(grp)
    if world > 1:
        objs = [None] * world if rank == 0 else None
        dist.gather_object((before, after), objs, dst=0)
        if rank == 0:
            before, after = {}, {}
            for b, a in objs:
                before.update(b)
                after.update(a)
    if rank != 0:
        return None
    O = _oracle()
    n = int(GP.size)
    X = np.ascontiguousarray(np.stack([before[w][0] for w in range(n)]))
    XH = np.ascontiguousarray(np.stack([before[w][1] for w in range(n)]))
    S = np.ascontiguousarray(np.stack([before[w][2] for w in range(n)]))
    flags = np.asarray(GP.active_flags, np.uint8)
    partner = np.asarray(GP.neighbors_info, np.int32).reshape(-1, n)[:flags.shape[1]]
    if flags[it].any():
        O.choco_round(X, XH, S, partner, flags[it], GP.neighbor_weight, grp.k, gamma)
    ok = True
    for w in range(n):
        for a, b in zip(after[w], (X[w], XH[w], S[w])):
            ok &= bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))
    return ok


def choco_figure(pkg, GP, rank, world, K, W, comm, dev, P=14_774_436, ratio=0.99, gamma=0.1, placement=None,
                 pull="auto"):
    """Secondary figure: ChocoSGD rounds (BASELINE config 4: VGG-16 size, top-1 %, graph 0, every
    matching active) on the same GPUs -- top-k compress + [N > 1] message exchange + fused apply.
    N > 1: the messages travel over RCCL (mx_exchange_round) or, under the pull transport, are taken
    from the owners' IPC-mapped snapshot buffers behind the device gate -- fetched into the receive
    slots (mx_pull_fetch, form "pull") or read in place by the apply (mx_choco_apply_slots, form
    "pull_direct"); every form runs R untimed rounds and the fastest (max over ranks) is timed
    (--pull on: the faster pull form; --pull off: RCCL only).  Parity: one more round after the timed ones, x / x_hat / s of every
    worker vs the oracle's round from the same state (choco_oracle_round)."""
    R = 4
    grp = pkg.ChocoWorkerGroup(GP, numel=P, ratio=ratio, consensus_lr=gamma, rank=rank, nranks=world,
                               comm=comm, placement=placement)
    fill_synth(pkg, grp)
    for it in range(W):
        grp.step(it)
    pull_only = isinstance(comm, pkg.PullTransport)          # the RCCL communicator was unavailable
    forms, calib, pull_err = {"pull" if pull_only else "rccl": grp}, None, None
    any_remote = world > 1 and max_over_ranks(float(grp.engine.max_remote), world, dev) > 0   # collective
    # the pull forms: "pull" fetches the partner messages into the receive slots, "pull_direct" lets
    # the apply read them in place (ChocoWorkerGroup pull_read); one alive at a time while warming up
    for name, mode in (("pull", "fetch"), ("pull_direct", "direct")):
        if name in forms:
            continue
        if not (any_remote and pull != "off") or pull_err is not None:
            break
        gp, err = None, None
        try:
            gp = pkg.ChocoWorkerGroup(GP, numel=P, ratio=ratio, consensus_lr=gamma, rank=rank, nranks=world,
                                      comm=pkg.PullTransport(timeout_s=PULL_TIMEOUT_S), placement=placement,
                                      pull_read=mode)
            fill_synth(pkg, gp)
            for it in range(W):
                gp.step(it)
            gp.wait_round()                      # a gate that expired in the warmup raises here
        except pkg.MXError as e:
            err = str(e)
        if gp is None:                           # bind failed: on every rank (all-or-nothing)
            pull_err = f"{name}: {err}"
        elif max_over_ranks(float(err is not None), world, dev) > 0:
            pull_err = f"{name}: {err or 'a peer warmup failed'}"
            gp.close()
        else:
            forms[name] = gp
    if len(forms) > 1:
        calib = {name: 1e3 * timed_loop(g.step, W, R, world, dev) / R for name, g in forms.items()}
        if pull == "on":
            chosen = min((n for n in calib if n != "rccl"), key=calib.get)
        else:
            chosen = min(calib, key=calib.get)
        for name in list(forms):
            if name != chosen:
                forms.pop(name).close()
        grp = forms[chosen]
        W += R
    else:
        chosen = next(iter(forms)) if world > 1 else None
    el = timed_loop(grp.step, W, K, world, dev)
    st = np.zeros(5 * grp.n_local, np.int64)
    pkg._lib.check(pkg.lib.mx_topk_stats(grp.work.data_ptr(), grp.work_ld, grp.n_local, grp.numel, st.ctypes.data,
                                         None), "mx_topk_stats")
    grp.check_topk()                              # no bounded row-barrier wait expired
    st = st.reshape(-1, 5)
    out = {"config": f"P={P} (VGG-16 size by default), ratio {ratio} (k={grp.k}), gamma {gamma}, graph 0 full rounds",
           "rounds_per_s": K / el, "ms_per_round": 1e3 * el / K, "rows_per_gpu": grp.n_local, "rounds": K,
           "warm_rounds": W,
           "topk": {"calls_per_row": int(st[:, 0].max()), "fallback_compactions": int(st[:, 1].sum()),
                    "candidates_per_k_last": [round(int(c) / grp.k, 2) for c in st[:, 4]],
                    "floor": "fine sampled" if pkg.lib.mx_topk_get(b"fine_floor") == 1 else "sampled digit"}}
    if world > 1:
        out["form"] = chosen
        out["calib_ms"] = calib
        out["pull_unavailable"] = pull_err
        if grp.pulls:
            out["pull_rounds"] = int(grp._pull.round)
            out["pull_gate_error"] = grp._pull.error()
        # the expected round of each form from its parts: this rank's compress + apply alone (a
        # transport that moves nothing, K rounds, max over ranks) + the busiest link's messages
        eng = grp.engine
        flags = np.asarray(GP.active_flags[W:W + K], np.uint8)
        _, link_b, _, _ = round_bytes(eng.partner, eng.owner, flags, rank, grp.row_base, grp.n_local,
                                      grp.msg_bytes / 4)
        loc = pkg.ChocoWorkerGroup(GP, numel=P, ratio=ratio, consensus_lr=gamma, rank=rank, nranks=world,
                                   comm=_NullComm(rank, world), placement=placement)
        fill_synth(pkg, loc)
        for it in range(W):
            loc.step(it)
        local_s = timed_loop(loc.step, W, K, world, dev) / K
        del loc
        lb = float(np.mean(link_b))
        pub = 2 * published_rows(eng.partner, flags, grp.row_base, grp.n_local) * grp.publish_cols * 4
        out["predicted"] = {f: predict_choco(f, world, lb, local_s, pub) for f in ("rccl", "pull")}
        out["predicted"]["pull_direct"] = out["predicted"]["pull"]
        pr = out["predicted"][chosen]
        out["predicted"]["timed_form"] = chosen
        out["predicted"]["note"] = ("pull and pull_direct share one prediction (the fixed cost measured for the "
                                    "fetch form); the calibration ranks them")
        out["predicted"]["achieved_over_predicted"] = pr["round_ms"] / (1e3 * el / K)
        out["message_bytes"] = int(grp.msg_bytes)
        out.update(pull_counts(pkg, world))                  # collective: binds / failures / refused exports
    out["parity_ok"] = choco_oracle_round(pkg, grp, GP, W + K, ratio, gamma, rank, world)
    out["parity"] = (f"round {W + K} (after the {W} warmup / calibration + {K} timed rounds) of every worker: x, "
                     f"x_hat, s vs the oracle's Choco round from the same state, uint32")
    if world == 1:
        # ~6 P 4 B per worker (top-k reads x, x_hat; apply reads x, s, x_hat, writes x)
        alg = 24 * P * grp.n_local
        out["roofline"] = {"bound": "hbm", "alg_bytes_per_round": alg, "achieved_GBps": alg / (el / K) / 1e9,
                           "frac_of_8TBps": alg / (el / K) / HBM_PEAK,
                           "note": "algorithmic bytes; the passes also move the dirty 64-B granules of s / x_hat "
                                   "and the candidate / message bytes (~3.2 GB per 8-row round by PMC, r02)"}
    grp.close()
    del grp, forms
    torch.cuda.empty_cache()
    if world == 1:
        out["one_row_share_n8"] = choco_row_share(pkg, GP, P, ratio, gamma, K, W)
    return out


class _NullComm:
    """Transport that moves nothing (the received message slots hold valid stand-ins)."""

    def __init__(self, rank, nranks):
        self.rank, self.nranks, self.handle = rank, nranks, None

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        return int(sum(1 for op in engine.exchange_plan(it) if op[0] == 1))


def choco_row_share(pkg, GP, P, ratio, gamma, K, W):
    """Config 4's per-GPU work at N = 8 measured on this GPU: rank 0's single row (placement
    "auto") with a null transport -- top-k, then the apply pass over its own and its partners'
    messages.  The partners' messages are stand-ins: the top-k messages of other synthetic rows
    (distinct index sets, so the apply dirties as many s granules as real partner messages do;
    until round 3 they were copies of the row's own message, which collide in the same granules).
    What every GPU adds to the message exchange in a real 8-GPU Choco round; per-round HIP events."""
    c = pkg.ChocoWorkerGroup(GP, numel=P, ratio=ratio, consensus_lr=gamma, rank=0, nranks=8,
                             comm=_NullComm(0, 8), placement="auto")
    for s in range(c.n_local, c.engine.n_slots):            # a distinct synthetic row per partner slot
        pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[0].data_ptr(), P, 7000 + s, None))
        c.compress(0)
        torch.cuda.synchronize()
        c.msgs[s * c.msg_ld:(s + 1) * c.msg_ld].copy_(c.msgs[:c.msg_ld])
    pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[0].data_ptr(), P, 1234 + c.workers[0], None))
    c.work.zero_()                                          # a fresh top-k scratch for the row itself
    torch.cuda.synchronize()
    for it in range(W):
        c.step(it)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j, (a, b) in enumerate(ev):
        a.record()
        c.step(W + j)
        b.record()
    torch.cuda.synchronize()
    us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
    out = {"rows": 1, "partners": int(c.engine.n_slots - c.n_local), "round_us_median": float(np.median(us)),
           "round_us_min": float(us.min()), "rounds": K,
           "hbm_GBps_alg": 24 * P / (np.median(us) * 1e-6) / 1e9,
           "how": "rank 0's row of an 8-GPU layout, null transport, partner messages = top-k of other synthetic "
                  "rows, per-round HIP events"}
    del c
    torch.cuda.empty_cache()
    return out


def config_figures(pkg, args, rank, world, n, K, W, comm, dev):
    """Secondary figures: the other BASELINE configs' gossip rounds on the same GPUs -- WRN-28-10
    (36,546,980 params per worker) under MATCHA C_b = 0.5 and full rounds, the repo's CIFAR
    ResNet (181,668 params, launch-bound) under MATCHA C_b = 0.5, and config 1's MNIST MLP
    (666,547 params) under the FixedProcessor schedule (D-PSGD; at N = 1 also through the reference's
    pickled CPU sequence, `cpu_pickle`); rounds/s, at N = 1 HBM bytes / s
    over the algorithmic bytes of the rounds run, and oracle parity of every worker's 64 sampled
    columns over every round the group ran (eager and graph-replayed).

    Every config also carries per-round HIP events (kernel time, `round_us_events`) beside the
    host-clocked rate.  A launch-bound config (P < 1e6) runs a warm burst of untimed rounds first
    (an idle GPU's clocks ramp over ~10 ms of work: profiles/r02_clock_ramp.log) and at least
    --lb-rounds (LAUNCH_BOUND_ROUNDS) rounds per measurement, so the fixed cost of the two host barriers and
    synchronizes around the timed region is not spread over a handful of 6-us rounds, and one host
    hiccup cannot double the figure: on one box 20 rounds measured 6.5 / 12.3 us per round (idle /
    warm), 400 rounds 5.5 us (tools/latency_bound.py, profiles/r06_latency_bound.json) -- the
    driver's r05 8.14 us was a 20-round sample."""
    out = {}
    for name, P, budget in (("wrn28_10_matcha0.5", args.wrn_params, 0.5), ("wrn28_10_full", args.wrn_params, 1.0),
                            ("resnet18_100_matcha0.5", args.resnet_params, 0.5),
                            ("mlp_fixed", args.mlp_params, None)):
        lb = P < 1_000_000
        Kc = max(K, args.lb_rounds) if lb else K
        warm = ((WARM_BURST * args.lb_rounds if world == 1 else args.lb_rounds) if lb else
                settle_rounds(2 * -(-n // world) * P * 4, args.settle_ms))
        np.random.seed(1234)
        if budget is None:
            # config 1: D-PSGD, FixedProcessor (graph_manager.py:183-225: the alternating matchings
            # 0 / 1 after the discarded draws; issubgraph=True as README.md:53 builds it)
            GPc = pkg.FixedProcessor(pkg.select_graph(0), 0.5, rank, n, W + warm + 3 * Kc, True)
        else:
            GPc = pkg.MatchaProcessor(pkg.select_graph(0), budget, rank, n, W + warm + 3 * Kc, True)
        g = pkg.VirtualWorkerGroup(GPc, numel=P, rank=rank, nranks=world, comm=comm, placement=args.placement)
        fill_synth(pkg, g)
        applied = list(range(W + warm + 3 * Kc))
        for it in range(W + warm):                # warmup + warm burst (untimed)
            g.step(it)
        torch.cuda.synchronize()
        ev = timed_rounds(lambda grp, it: grp.step(it), g, W + warm, Kc)    # per-round events
        torch.cuda.synchronize()
        us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
        blk = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        blk[0].record()                           # one event pair around Kc back-to-back rounds
        for it in range(W + warm + Kc, W + warm + 2 * Kc):
            g.step(it)
        blk[1].record()
        torch.cuda.synchronize()
        blk_us = 1e3 * blk[0].elapsed_time(blk[1]) / Kc
        first = W + warm + 2 * Kc
        el = timed_loop(g.step, first, Kc, world, dev)
        partner = np.asarray(GPc.neighbors_info, np.int32)
        byts = 0
        for f in np.asarray(GPc.active_flags[first:first + Kc], np.uint8):
            deg = (partner[:len(f)][f.astype(bool)] >= 0).sum(axis=0) if f.any() else np.zeros(n, int)
            byts += 2 * int((deg > 0).sum()) * P * 4
        out[name] = {"params_per_worker": P, "budget": budget, "rounds_per_s": Kc / el, "ms_per_round": 1e3 * el / Kc,
                     "schedule": "FixedProcessor (alternating matchings 0 / 1)" if budget is None else
                                 f"MatchaProcessor C_b = {budget}",
                     "rounds": Kc, "warm_rounds": warm,
                     "round_us_events": {"median": float(np.median(us)), "min": float(us.min()),
                                         "mean": float(us.mean()), "block_per_round": blk_us,
                                         "note": f"this rank's GPU time per round, no host barrier / synchronize: "
                                                 f"median / min / mean of per-round HIP event pairs over {Kc} "
                                                 f"rounds (each pair adds its own records between launches), "
                                                 f"block_per_round = one event pair around {Kc} back-to-back "
                                                 f"rounds / {Kc}"},
                     "hbm_TBps": byts / el / 1e12 if world == 1 else None}
        if world == 1 and lb:
            # launch-bound rows: the timed rounds replayed from one captured HIP graph
            # (device_rounds: the rounds read their iteration from a device counter)
            gr = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream()
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                with torch.cuda.graph(gr):
                    g.device_rounds(Kc)
            torch.cuda.synchronize()
            g.iter_dev.fill_(first)
            gr.replay()                           # warm replay of the same rounds' shapes
            g.iter_dev.fill_(first)
            torch.cuda.synchronize()
            t = time.perf_counter()
            gr.replay()
            torch.cuda.synchronize()
            elg = time.perf_counter() - t
            applied += list(range(first, first + Kc)) * 2
            out[name]["graph_rounds_per_s"] = Kc / elg
            out[name]["graph_us_per_round"] = 1e6 * elg / Kc
            out[name]["graph_note"] = f"{Kc} rounds (iterations {first}..{first + Kc - 1}) replayed from one HIP graph"
            del gr
        cols = sample_columns(P)
        final = gather_columns(g, torch.from_numpy(cols).cuda(), world, dev)
        g.close()
        del g
        torch.cuda.empty_cache()
        if rank == 0:
            out[name]["parity_ok"] = oracle_column_parity(GPc, synth_columns(range(n), cols), final, applied)
        if budget is None and world == 1 and rank == 0 and args.cpu_seconds > 0:
            # BASELINE config 1 is the reference's own CPU plumbing run (8 ranks via mpirun): the same
            # schedule through the pickled-transport port, 8 processes pinned one per core
            out[name]["cpu_pickle"] = mlp_pickle_leg(GPc, P, args.cpu_seconds)
    if rank == 0:
        out["parity"] = ("every worker's 64 sampled columns after every round the group ran vs the oracle's "
                         "decen rounds on the same columns, uint32")
    return out


def er_figure(pkg, args, rank, world, comm, dev):
    """BASELINE config 5: a 64-worker Erdos-Renyi(0.1, seed 1234) topology decomposed on the host,
    P params per worker (1e9 by default, reduced to what fits this GPU -- the P run is recorded),
    MATCHA budget sweep.  At N > 1 the workers are placed over the GPUs ("auto") and every exchange
    form that fits at that P (plain / column-pipelined RCCL, pull) is calibrated ONE AT A TIME at
    budget 1.0 (only one form's buffers are alive at once); the fastest runs the sweep.  Per
    budget: rounds/s (max over ranks), per-rank slot count, busiest-link bytes per round, the
    exchange alone (RCCL forms), and oracle parity of every worker's 64 sampled columns."""
    from importlib import import_module
    E = import_module(PKG_NAME + ".engine")
    PL = import_module(PKG_NAME + ".placement")
    n, seed = 64, 1234
    budgets = [float(b) for b in args.er_budgets.split(",") if b]
    Ker, Wer, R = max(1, args.er_rounds), 1, 1
    T = Wer + Ker + 2 * R + 2
    random.seed(0)
    base = pkg.erdos_renyi(n, 0.1, seed)
    np.random.seed(seed)
    GP0 = pkg.MatchaProcessor(base, 1.0, rank, n, T, False)
    sub = GP0.subGraphs
    topo0, perm = PL.place(GP0, world, args.placement if world > 1 else None)
    row_base, n_local = E.partition(n, world)[rank]
    part0 = np.asarray(topo0.neighbors_info, np.int32).reshape(-1, n)
    max_remote = E.max_incoming_remote(part0, row_base, n_local)
    # bytes per parameter column on this GPU for each exchange form
    forms = {"local": n_local} if world == 1 else {}
    if world > 1:
        if not isinstance(comm, pkg.PullTransport):          # else: the RCCL communicator was unavailable
            forms["rccl"] = n_local + max_remote
            forms["rccl_chunked"] = n_local + 2 * max_remote / 4.0 if max_remote else n_local
        if args.pull != "off" or not forms:
            forms["pull"] = 3 * n_local
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info()
    reserve = 4 << 30
    P_req = int(args.er_params)
    fit = {k: int((free - reserve) / (4 * v)) // 64 * 64 for k, v in forms.items()}
    P = min(P_req, max(fit.values()))
    P = int(-max_over_ranks(-float(P), world, dev))            # every rank runs the same P
    if P < 1024:
        raise RuntimeError(f"ER(64) leg: only {free / 2**30:.1f} GiB free on rank {rank}")
    # forms that fit at P on EVERY rank (free memory differs per GPU: agree, or the ranks would
    # calibrate different forms and their collectives would not pair up)
    cand = [k for k in forms if max_over_ranks(float(fit[k] < P), world, dev) == 0]
    cols = sample_columns(P)
    cols_dev = torch.from_numpy(cols).cuda()
    init = synth_columns(range(n), cols)

    def make(GPb, form):
        kw = dict(numel=P, rank=rank, nranks=world, placement=perm if world > 1 else None)
        if form == "rccl":
            g = pkg.VirtualWorkerGroup(GPb, comm=comm, **kw)
        elif form == "rccl_chunked":
            g = pkg.VirtualWorkerGroup(GPb, comm=comm, chunk_cols=((P + 3) // 4 + 63) // 64 * 64, **kw)
        elif form == "pull":
            g = pkg.VirtualWorkerGroup(GPb, comm=pkg.PullTransport(timeout_s=PULL_TIMEOUT_S), **kw)
        else:
            g = pkg.VirtualWorkerGroup(GPb, **kw)
        fill_synth(pkg, g)
        return g

    calib, calib_ok = {}, {}
    chosen = cand[0]
    if len(cand) > 1:
        for form in cand:                         # one form alive at a time
            try:
                g = make(GP0, form)
            except pkg.MXError as e:
                calib[form] = f"unavailable: {e}"
                continue
            g.step(0)
            calib[form] = 1e3 * timed_loop(g.step, 1, R, world, dev) / R
            got = gather_columns(g, cols_dev, world, dev)
            ok = oracle_column_parity(GP0, init, got, range(R + 1)) if rank == 0 else True
            calib_ok[form] = max_over_ranks(float(not ok), world, dev) == 0      # rank 0's verdict, shared
            g.close()
            del g
            torch.cuda.empty_cache()
        timed = {k: v for k, v in calib.items() if isinstance(v, float)}
        # only a form whose calibration rounds passed the oracle is eligible (as the headline's)
        timed = {k: v for k, v in timed.items() if calib_ok.get(k)} or timed
        chosen = min(timed, key=timed.get)
    sweep = []
    for b in budgets:
        np.random.seed(seed)
        GPb = pkg.MatchaProcessor(sub, b, rank, n, T, True)       # same matchings, budget b
        g = make(GPb, chosen)
        applied = list(range(Wer))
        for it in range(Wer):
            g.step(it)
        el = timed_loop(g.step, Wer, Ker, world, dev)
        applied += list(range(Wer, Wer + Ker))
        flags = np.asarray(GPb.active_flags, np.uint8)[Wer:Wer + Ker]
        eng = g.engine
        g_row_base = g.row_base
        hbm, link, _, _ = round_bytes(eng.partner, eng.owner, flags, rank, g.row_base, g.n_local, P)
        xo = None
        if world > 1 and chosen == "rccl" and flags.any():        # whole rows into the slab: plain form only
            xo = exchange_only(g, Wer, Ker, world, dev)[0]
        slots = [None] * world
        if world > 1:
            import torch.distributed as dist
            dist.all_gather_object(slots, int(eng.n_slots))
        else:
            slots = [int(eng.n_slots)]
        final = gather_columns(g, cols_dev, world, dev)
        g.close()
        del g
        torch.cuda.empty_cache()
        pred = None
        if world > 1:
            mix_est = float(np.mean(hbm)) / (HEADLINE_HBM_FRAC * HBM_PEAK)
            pub = 2 * published_rows(eng.partner, flags, g_row_base, n_local) * P * 4
            pred = predict_round(chosen, world, float(np.mean(link)), mix_est, pub,
                                 mix_source="this GPU's algorithmic HBM bytes at the headline kernel's 0.75 of 8 TB/s")
            pred["achieved_over_predicted"] = pred["round_ms"] / (1e3 * el / Ker)
        row = {"budget": b, "rounds_per_s": Ker / el, "ms_per_round": 1e3 * el / Ker, "predicted": pred,
               "mean_active_matchings": float(flags.sum(1).mean()), "skipped_rounds": int((flags.sum(1) == 0).sum()),
               "alpha": GPb.neighbor_weight, "slots_per_rank": slots,
               "hbm_TBps_rank0": (float(np.sum(hbm)) / el / 1e12) if world == 1 else None,
               "max_link_bytes_per_round": float(np.mean(link)) if world > 1 else None,
               "busiest_link_GBps": (float(np.mean(link)) / (el / Ker) / 1e9) if world > 1 else None,
               "exchange_only_ms": 1e3 * xo if xo else None}
        if rank == 0:
            row["parity_ok"] = oracle_column_parity(GPb, init, final, applied)
        sweep.append(row)
    out = {"graph": f"ER({n}, 0.1, seed {seed})", "matchings": len(sub), "edges": int(sum(len(m) for m in sub)),
           "params_per_worker": P, "params_requested": P_req, "rows_per_gpu": n_local,
           "max_remote_partners_rank0": max_remote, "form": chosen, "calib_ms": calib or None,
           "calib_parity_ok": calib_ok or None,
           "rounds_per_budget": Ker, "sweep": sweep}
    if rank == 0:
        out["parity_ok"] = all(r.get("parity_ok") for r in sweep)
        out["parity"] = ("every worker's 64 sampled columns after every round of each budget vs the oracle's "
                         "decen rounds on the same columns (initial values from the oracle's generator), uint32")
    return out


def staged_figure(pkg, GP, n, P, K, first):
    """Secondary figure (N = 1): workers whose models stay on the host, as the reference's
    train_mpi.py keeps them -- each round the drop-in communicator's staging (communicator.py
    _Staging: torch.cat + H2D copy, round, D2H copy + copy_ into the model's tensors) for every
    worker around the same mixing launch."""
    from importlib import import_module
    C = import_module(PKG_NAME + ".communicator")
    grp = pkg.VirtualWorkerGroup(GP, numel=P)
    host = []
    for r in range(n):
        pkg._lib.check(pkg.lib.mx_synth_fill(grp.rows[r].data_ptr(), P, 1234 + r, None))
        row = grp.rows[r].cpu()
        cuts = np.linspace(0, P, 55).astype(np.int64)          # VGG-16's 54 parameter tensors
        ps = [torch.nn.Parameter(row[a:b].clone()) for a, b in zip(cuts[:-1], cuts[1:])]
        host.append(C._Staging(ps, grp.rows[r]))
    for st in host:                      # untimed first round: pinned buffers and staging plans
        st.load()
    torch.cuda.synchronize()
    for st in host:
        st.store()
    t = time.perf_counter()
    for j in range(K):
        for st in host:
            st.load()
        grp.step(first + j)
        torch.cuda.synchronize()
        for st in host:
            st.store()
    el = time.perf_counter() - t
    del grp, host
    torch.cuda.empty_cache()
    return {"rounds_per_s": K / el, "ms_per_round": 1e3 * el / K, "rounds": K,
            "how": "8 host-resident models (54 pageable tensors each): stage in (flatten into pinned 16 MB "
                   "pieces, each DMA'd as soon as filled), mixing launch, stage out (DMA per piece, each "
                   "scattered into the tensors as it lands) per round, after one untimed round -- the "
                   "drop-in communicators' path for CPU models"}


def timed_rounds(run, group, first, K):
    """K rounds from iteration `first` with per-round HIP events on the launch stream."""
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j in range(K):
        ev[j][0].record(stream)
        run(group, first + j)
        ev[j][1].record(stream)
    return ev


# ----------------------------------------------------------------------------------- main
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv, popen=None):
    """`bench.py --gpus N` (N > 1) started WITHOUT a launcher (no WORLD_SIZE): run the N ranks
    as a child `python -m torch.distributed.run --nproc-per-node N bench.py ...` and relay rank 0's
    JSON line; returns the exit status for the parent to exit with.

    The parent never initialises HIP: it counts devices with torch.cuda.device_count() (which on
    this image does not initialise the GPU) and starts the launcher as a CHILD process -- never an
    exec from this process.  With the RCCL transport it refuses (non-zero, with a message) when
    fewer than N GPUs are visible, instead of silently timing N = 1.  SIGTERM / SIGINT to the
    parent are forwarded to the child's process group (each rank then prints its line so far)."""
    import signal
    import subprocess
    n = int(args.gpus)
    if args.transport == "rccl":
        have = torch.cuda.device_count()
        if have < n:
            sys.stderr.write(f"bench.py --gpus {n}: only {have} GPU(s) visible -- the RCCL transport needs one GPU "
                             f"per rank (run the N = {n} scaling bench on a node with {n} GPUs, or --transport gloo "
                             f"to exercise the multi-process path on fewer)\n")
            return 2
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    popen = popen or subprocess.Popen
    proc = popen(cmd, stdout=subprocess.PIPE, env=env, start_new_session=True, text=True, bufsize=1)

    def forward(signum, _frame):
        try:
            os.killpg(proc.pid, signum)
        except (ProcessLookupError, PermissionError, OSError):
            pass

    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    printed = False
    try:
        for raw in proc.stdout:
            s = raw.strip()
            if s.startswith("{") and not printed:
                try:
                    d = json.loads(s)
                except ValueError:
                    d = None
                if isinstance(d, dict) and "metric" in d:
                    d["launcher"] = {"self_launched": True, "nproc_per_node": n,
                                     "how": "bench.py (no WORLD_SIZE) started torch.distributed.run as a child "
                                            "process; this is rank 0's line"}
                    print(json.dumps(d), flush=True)
                    printed = True
                    continue
            sys.stderr.write(raw)
        rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if not printed and rc == 0:
        sys.stderr.write("bench.py self-launch: the ranks exited without a JSON line\n")
        return 1
    return rc


def term_handler(line, wd):
    """SIGTERM (the launcher stops every rank when one fails or leaves): rank 0 prints the line so
    far with an "error" naming the running phase, and the rank exits EXIT_ABORTED."""
    def on_term(signum, _frame):
        line.emit(f"terminated by signal {signum} during {wd.name or 'the run'} (the launcher stops every rank "
                  f"when one rank fails or leaves)")
        os._exit(EXIT_ABORTED)
    return on_term


def main():
    """The run happens on a worker thread; the main thread only waits, so it stays free to take
    SIGTERM -- what the launcher (torchrun) sends every rank when one rank dies -- and rank 0
    then prints the line measured so far with an "error" field before leaving."""
    import signal
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    line = Line(rank)
    wd = Watchdog(rank, line.emit)
    failed = []
    signal.signal(signal.SIGTERM, term_handler(line, wd))

    status = [0]

    def body():
        try:
            run(args, world, rank, line, wd, status)
        except BaseException as e:                   # noqa: BLE001 -- reported in the line, then re-raised
            import traceback
            traceback.print_exc()
            failed.append(e)
            line.emit(f"{wd.name or 'run'}: {type(e).__name__}: {e}")

    t = threading.Thread(target=body, name="bench")
    t.start()
    while t.is_alive():
        t.join(0.5)
    if failed:
        sys.exit(1)
    if status[0]:
        sys.exit(status[0])


def run(args, world, rank, line, wd, status=None):
    """The whole run; status[0] is set to EXIT_PARITY (rank 0) when the headline's self-check fails."""
    status = status if status is not None else [0]
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wd.arm("startup (process group / RCCL communicator)", args.headline_timeout)
    import datetime
    import torch.distributed as dist
    gloo = args.transport == "gloo"
    if gloo or args.debug_share_gpu:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    pg_timeout = datetime.timedelta(seconds=args.pg_timeout)
    if world > 1:
        # the job's own agreement, timing barriers, max-over-ranks and result gathers run over gloo
        # (host tensors) whatever the gossip transport: none of them depends on RCCL, so the no-RCCL
        # fallback below really does without it and a collective never queues behind an
        # RCCL kernel on the GPU stream.  RCCL itself is the library's communicator (RcclComm,
        # bootstrapped over this group) and torch's nccl group of the p2p probe figure.
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout)
    dev = "cpu"
    import importlib
    pkg = importlib.import_module(PKG_NAME)
    comm = None
    rccl_err = None
    if world > 1:
        try:
            if args.debug_no_rccl:
                raise pkg.MXError("--debug-no-rccl")
            if gloo:
                sys.path.insert(0, os.path.join(ROOT, "tests"))
                from gloo_transport import GlooTransport
                comm = GlooTransport(pkg)
            else:
                comm = pkg.engine.RcclComm(timeout_s=min(args.figure_timeout, args.headline_timeout) * 0.8)
        except pkg.MXError as e:
            rccl_err = str(e)
        if max_over_ranks(float(rccl_err is not None), world, dev) > 0:
            # the library's RCCL communicator is unusable on some rank: every rank drops it and the
            # gossip runs over the pull transport alone (the line says why; the RCCL-only figures
            # -- exchange alone, the centralized all-gather -- then report errors)
            if isinstance(comm, pkg.engine.RcclComm):
                comm.abort()
            comm = pkg.PullTransport(timeout_s=PULL_TIMEOUT_S)
            rccl_err = rccl_err or "a peer rank's RCCL communicator failed"
    pull_only = isinstance(comm, pkg.PullTransport)
    # the ranks RCCL itself holds (ncclCommCount on the library's communicator): proof that the
    # exchange really spans N processes / GPUs
    rccl_ranks = comm.count() if isinstance(comm, pkg.engine.RcclComm) else None
    wd.arm("headline", args.headline_timeout)

    n, P = args.workers, args.params
    K, W = args.steps, args.warmup
    R = 4                                        # N > 1: untimed calibration rounds per exchange form
    DMAX = max(K, 4000)                          # most diagnostic (settling) rounds
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(args.graph), args.budget, rank, n,
                             W + DMAX + 2 * K + (R + 1 if world > 1 else 0), True)
    group = pkg.VirtualWorkerGroup(GP, numel=P, rank=rank, nranks=world, comm=comm, placement=args.placement)
    fill_synth(pkg, group)
    torch.cuda.synchronize()
    cols = sample_columns(P)
    cols_dev = torch.from_numpy(cols).cuda()
    applied = {}                                             # group -> iterations it ran, in order

    def run(g, it):
        g.step(it)
        applied.setdefault(id(g), []).append(it)

    for it in range(W):
        run(group, it)
    if isinstance(comm, pkg.engine.RcclComm):
        # the first cross-GPU exchanges, waited for with a deadline (an exchange that never completes
        # aborts the communicator instead of hanging the stream), before any torch collective queues
        # behind them; on expiry on any rank every rank continues over the pull transport
        try:
            comm.wait(timeout_s=RCCL_WARMUP_WAIT_S)
        except pkg.MXError as e:
            rccl_err = f"warmup exchange: {e}"
        if max_over_ranks(float(rccl_err is not None), world, dev) > 0:
            rccl_err = rccl_err or "a peer rank's warmup exchange did not complete"
            comm.abort()
            comm, pull_only = pkg.PullTransport(timeout_s=PULL_TIMEOUT_S), True
            group = pkg.VirtualWorkerGroup(GP, numel=P, rank=rank, nranks=world, comm=comm, placement=args.placement)
            fill_synth(pkg, group)
            for it in range(W):
                run(group, it)
    torch.cuda.synchronize()
    timed, overlap = group, None
    any_remote = world > 1 and max_over_ranks(float(group.engine.max_remote), world, dev) > 0   # collective
    base_it = W + DMAX + 2 * K
    forms = {"pull" if pull_only else "rccl": group}
    C = None
    if any_remote and args.overlap != "off" and not pull_only:
        # column pipelining: chunk c+1 of every exchanged row travels on a side stream while chunk c
        # is mixed (bit-identical results)
        C = args.chunk_cols or ((P + 3) // 4 + 63) // 64 * 64
        gchunk = pkg.VirtualWorkerGroup(GP, numel=P, rank=rank, nranks=world, comm=comm, placement=args.placement,
                                        chunk_cols=C)
        fill_synth(pkg, gchunk)
        for it in range(W):
            run(gchunk, it)
        run(gchunk, base_it)                     # first chunked round (side stream, events) untimed
        forms["rccl_chunked"] = gchunk
    pull_err = None
    if any_remote and args.pull != "off" and not pull_only:
        # the pull transport: partner rows read straight from the peers' HBM (IPC-mapped
        # snapshots) by the mixing kernel -- no RCCL copies; collective setup, all ranks agree
        # (bench rounds run in lockstep: a device gate that waits PULL_TIMEOUT_S has met a fault,
        # not a slow peer -- the form is then dropped on EVERY rank, so the forms stay in step)
        gpull = None
        try:
            gpull = pkg.VirtualWorkerGroup(GP, numel=P, rank=rank, nranks=world,
                                           comm=pkg.PullTransport(timeout_s=PULL_TIMEOUT_S), placement=args.placement)
            fill_synth(pkg, gpull)
            for it in range(W):
                run(gpull, it)
            gpull.wait_round()                   # a gate that expired in the warmup raises here
        except pkg.MXError as e:
            pull_err = str(e)
        if gpull is not None:                    # bound on every rank (bind is all-or-nothing)
            if max_over_ranks(float(pull_err is not None), world, dev) > 0:
                pull_err = pull_err or "a peer's pull warmup failed"
                gpull.close()
            else:
                forms["pull"] = gpull
    if len(forms) > 1:
        # every form runs R untimed rounds; the fastest (max over ranks, so every rank picks the
        # same) is the one timed -- unless one is forced (--overlap on / --pull on)
        calib_ms = {name: 1e3 * timed_loop(lambda it, g=g: run(g, it), base_it + 1, R, world, dev) / R
                    for name, g in forms.items()}
        # a form is eligible only if every round it ran so far matches the oracle (rank 0's verdict,
        # shared): a transport that returns wrong bits -- e.g. a cross-GPU coherence fault of the pull
        # form, whose cross-L2 case no one-GPU test can reach -- is never the one timed
        init_cols = synth_columns(range(n), cols) if rank == 0 else None
        calib_ok = {}
        for name, g in forms.items():
            got = gather_columns(g, cols_dev, world, dev)
            ok = oracle_column_parity(GP, init_cols, got, applied[id(g)]) if rank == 0 else True
            calib_ok[name] = max_over_ranks(float(not ok), world, dev) == 0
        eligible = {k: v for k, v in calib_ms.items() if calib_ok[k]} or calib_ms
        if args.pull == "on" and "pull" in eligible:
            chosen = "pull"
        elif args.overlap == "on" and "rccl_chunked" in eligible:
            chosen = "rccl_chunked"
        else:
            chosen = min(eligible, key=eligible.get)
        timed = forms[chosen]
        overlap = {"mode": args.overlap, "pull": args.pull, "chunk_cols": C if "rccl_chunked" in forms else None,
                   "chunks": len(forms["rccl_chunked"].chunks) if "rccl_chunked" in forms else None,
                   "calib_ms": calib_ms, "calib_parity_ok": calib_ok, "calib_ms_unchunked": calib_ms.get("rccl"),
                   "calib_ms_chunked": calib_ms.get("rccl_chunked"), "chosen_form": chosen,
                   "chosen": "chunked" if chosen == "rccl_chunked" else "unchunked",
                   "pull_unavailable": pull_err,
                   "note": f"{R} untimed rounds per exchange form before the timed region, max over ranks; "
                           f"only a form whose rounds so far pass the oracle self-check (calib_parity_ok) is "
                           f"eligible for the timed region"}
        for name in list(forms):
            if forms[name] is not timed and forms[name] is not group:
                forms[name].close()
                del forms[name]
    elif pull_err is not None:
        overlap = {"pull_unavailable": pull_err}
    if pull_only:
        overlap = {"mode": args.overlap, "pull": args.pull, "chosen_form": "pull", "calib_ms": None,
                   "note": "the library's RCCL communicator was unavailable (rccl_unavailable): pull transport only"}
    if world > 1:
        ipc = pull_counts(pkg, world)                       # collective
        if overlap is not None:
            overlap.update(ipc)
    # per-round HIP events of the whole round (diagnostic): real rounds run BEFORE the timed region,
    # in blocks of K, for at least --settle-ms (an idle MI355X takes ~10 ms of streaming to reach
    # its steady clocks: profiles/r02_clock_ramp.log), so the timed rounds measure the steady state of the loop
    step_ms = []
    it = W
    t_settle = time.perf_counter()
    while True:
        ev = timed_rounds(run, timed, it, K)
        torch.cuda.synchronize()
        step_ms += [a.elapsed_time(b) for a, b in ev]
        it += K
        done = (time.perf_counter() - t_settle) * 1e3 >= args.settle_ms or it - W + K > DMAX
        if world > 1:                            # every rank leaves after the same block
            done = max_over_ranks(float(done), world, dev) > 0
        if done:
            break
    diag_rounds = it - W
    step_ms = np.array(step_ms)
    barrier(world)
    torch.cuda.synchronize()
    tev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    tev[0].record()                              # HIP events on the launch stream over the timed region
    for j in range(K):                           # the timed rounds: back to back, nothing else
        run(timed, it + j)
    tev[1].record()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed_events_ms = tev[0].elapsed_time(tev[1]) / K
    elapsed = max_over_ranks(elapsed, world, dev)
    timed_first = it
    if overlap is not None and getattr(timed, "pulls", False):
        # rounds the pull group ran on its two alternating snapshot buffers (each reused >= 3 times
        # when this is >= 6); parity_ok below covers every one of them
        overlap["pull_rounds"] = int(timed._pull.round)
        overlap["pull_gate_error"] = timed._pull.error()   # an expired device wait (None: every gate passed)
    final_cols = gather_columns(timed, cols_dev, world, dev)
    # mixing kernel alone (N > 1: without the RCCL exchange, so rows go stale) -> its HBM roofline
    stream = torch.cuda.current_stream()
    mev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j in range(K):
        mev[j][0].record(stream)
        group.engine.mix(timed_first + K + j, group.layout)
        mev[j][1].record(stream)
    torch.cuda.synchronize()
    mix_ms = np.array([a.elapsed_time(b) for a, b in mev])
    # same-box context for the roofline fraction: torch's copy_ of the same bytes (read + write of
    # the active rows), timed the same way right after the mixing launches
    ref_copy_ms = None
    if world == 1:
        nbytes = group.n_local * P * 4
        src_t = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
        dst_t = torch.empty_like(src_t)
        dst_t.copy_(src_t)
        cev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in cev:
            a.record(stream)
            dst_t.copy_(src_t)
            b.record(stream)
        torch.cuda.synchronize()
        ref_copy_ms = float(np.mean([a.elapsed_time(b) for a, b in cev]))
        del src_t, dst_t
    flags = np.asarray(GP.active_flags[timed_first:timed_first + K], np.uint8)
    eng = group.engine
    partner = eng.partner
    hbm_bytes, link_bytes, pair_bytes, total_bytes = round_bytes(partner, eng.owner, flags, rank, group.row_base,
                                                                 group.n_local, P)
    avg_ms = float(step_ms.mean())
    # the mixing kernel's average launch duration: at N = 1 the timed region IS the K mixing
    # launches back to back (HIP events bracketing it on the launch stream, 0 us between launches
    # by kernel trace); at N > 1 the timed rounds also hold the exchange, so the K separate
    # mixing-alone launches (per-launch events) stand in
    mix_avg_ms = float(timed_events_ms) if world == 1 else float(mix_ms.mean())
    mix_bytes = float(np.mean(hbm_bytes))
    achieved = mix_bytes / (mix_avg_ms * 1e-3)
    traffic, traffic_src = pmc_traffic()
    # the headline line (filled in further as the figures complete)
    out = line.out
    out.update({
        "metric": METRIC,
        "value": K / elapsed,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": 1e3 * elapsed / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 uniform[-1,1), resident in HBM)",
        "config": {"workload": f"graph {args.graph} ({n} workers), P={P} fp32 per worker, "
                               f"budget {args.budget} ({'every matching active' if args.budget >= 1 else 'MATCHA schedule'})",
                   "workers": n, "params_per_worker": P, "graph": args.graph, "budget": args.budget,
                   "parallelism": f"{n} workers over {world} GPU(s)" +
                                  (f", placement {args.placement}" if world > 1 else "") +
                                  (f", exchange form {overlap['chosen_form']}" if overlap and
                                   overlap.get("chosen_form") else ""),
                   "placement": group.placement if world > 1 else None,
                   "transport": args.transport if world > 1 else None},
        "rccl_ranks": rccl_ranks,
        "rccl_unavailable": rccl_err,
        "parity_ok": None,
        "round_us": {"events_min": 1e3 * float(step_ms.min()), "events_median": 1e3 * float(np.median(step_ms)),
                     "events_mean": 1e3 * avg_ms, "events_last_block_mean": 1e3 * float(step_ms[-K:].mean()),
                     "events_first_block_mean": 1e3 * float(step_ms[:K].mean()),
                     "diag_rounds": int(diag_rounds), "timed_mean": 1e6 * elapsed / K,
                     "note": f"per-round HIP events of {diag_rounds} untimed rounds (blocks of K, >= "
                             f"{args.settle_ms} ms) run between the warmup and the timed region (rank 0)"},
        "roofline": {"bound": "hbm", "kernel": f"{pkg.engine.mix_kernel_name(eng.n_slots)} (mx_gossip_mix)",
                     "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic,
                     "traffic_source": traffic_src, "bytes_per_launch": mix_bytes,
                     "avg_launch_ms": mix_avg_ms,
                     "avg_launch_source": ("HIP events over the K timed rounds (the mixing launches back to back)"
                                           if world == 1 else "K mixing-alone launches after the timed region, "
                                                              "per-launch HIP events"),
                     "mixing_alone_events_ms": {"mean": float(mix_ms.mean()), "min": float(mix_ms.min()),
                                                "median": float(np.median(mix_ms))},
                     "min_launch_ms": float(mix_ms.min()), "median_launch_ms": float(np.median(mix_ms)),
                     "frac_timed_region": (mix_bytes / (elapsed / K)) / HBM_PEAK if world == 1 else None,
                     "same_box_torch_copy_ms": ref_copy_ms,
                     "vs_same_box_copy": (ref_copy_ms / mix_avg_ms) if ref_copy_ms else None,
                     "tuning": pkg.engine.mix_tuning(),
                     "note": "achieved = algorithmic bytes (2 x active rows x P x 4 [+ slab rows]) / "
                             "average launch duration (avg_launch_source), HIP events on the launch stream"},
        "overlap": overlap,
    })
    if world > 1:
        lb = float(np.mean(link_bytes))
        pb = float(np.mean(pair_bytes))
        round_s = elapsed / K
        out["xgmi"] = {"max_link_bytes_per_round": lb, "achieved": lb / round_s / 1e9,
                       "peak": XGMI_LINK_PEAK / 1e9, "unit": "GB/s",
                       "frac": lb / round_s / XGMI_LINK_PEAK,
                       "max_pair_bytes_both_directions": pb,
                       "achieved_both_directions": pb / round_s / 1e9,
                       "frac_both_directions": pb / round_s / XGMI_LINK_PEAK,
                       "aggregate_bytes_per_round": float(np.mean(total_bytes)),
                       "aggregate_achieved": float(np.mean(total_bytes)) / round_s / 1e9,
                       "round_ms": 1e3 * round_s, "round_ms_events_rank0": avg_ms,
                       "exchange_only_ms": None, "exchange_only_ms_per_rank": None, "p2p_probe": None,
                       "note": "busiest GPU pair: bytes that cross it per round (one direction, and "
                               "both directions summed) / whole-job round time (exchange + mix), "
                               "against the 153 GB/s per-link figure of SURVEY.md §8d"}
        # the expected round of every form, from its parts (achieved / predicted names the term that is off)
        mix_s = float(np.median(mix_ms)) * 1e-3
        mix_s = max_over_ranks(mix_s, world, dev)
        pub = 2 * published_rows(partner, flags, group.row_base, group.n_local) * P * 4   # read + write
        chunks = overlap.get("chunks") if overlap and overlap.get("chunks") else 4
        out["predicted"] = {f: predict_round(f, world, lb, mix_s, pub, chunks,
                                             "mixing-alone launches of this run (max over ranks)")
                            for f in ("rccl", "rccl_chunked", "pull")}
        chosen_form = overlap.get("chosen_form") if overlap else "rccl"
        pr = out["predicted"].get(chosen_form or "rccl")
        out["predicted"]["timed_form"] = chosen_form or "rccl"
        out["predicted"]["achieved_over_predicted"] = (pr["round_ms"] / (1e3 * round_s)) if pr else None
    wd.disarm()
    # self-check: every worker's sampled columns after every round the timed group ran vs the
    # oracle's rounds on the same columns from the synthetic initial values (checker, untimed)
    if rank == 0:
        out["parity_ok"] = oracle_column_parity(GP, synth_columns(range(n), cols), final_cols, applied[id(timed)])
        out["parity"] = (f"every worker's {len(cols)} sampled columns after all {len(applied[id(timed)])} rounds "
                         f"this run applied, vs the CPU oracle's decen rounds (oracle/matcha_oracle.c) on the "
                         f"same columns from the same synthetic initial values (uint32 compare)")
        if not out["parity_ok"]:
            # a wrong result is not a throughput: the headline value is withheld and the run fails
            out["unverified"] = {"value": out.pop("value"), "ms_per_step": out.pop("ms_per_step")}
            out["value"], out["ms_per_step"] = None, None
            out["error"] = "headline: the oracle self-check failed -- value withheld (unverified)"
            status[0] = EXIT_PARITY

    # ------------------------------------------------------------------ secondary figures
    t_fig = time.monotonic()
    skip, stall = {}, {}
    if args.debug_skip:
        nm, rk = args.debug_skip.split(":")
        skip = {nm: int(rk)}
    if args.debug_stall:
        nm, rk = args.debug_stall.split(":")
        stall = {nm: int(rk)}

    def figure(name, fn, enabled=True):
        if not enabled:
            return None
        over = time.monotonic() - t_fig > args.figures_budget
        if world > 1:
            wd.arm(f"{name} (budget check)", args.figure_timeout)
            over = max_over_ranks(float(over), world, dev) > 0
            wd.disarm()
        if over:
            return {"skipped": f"figures budget of {args.figures_budget:.0f} s spent"}
        if skip.get(name) == rank:
            return {"skipped": "--debug-skip"}
        wd.arm(name, args.figure_timeout)
        if stall.get(name) == rank:
            time.sleep(10 * args.figure_timeout)
        res = guarded(name, fn)
        wd.disarm()
        if rank == 0 and withhold_unverified(res):
            sys.stderr.write(f"[bench] {name}: oracle self-check FAILED -- its rates are withheld (unverified)\n")
        if world > 1 and isinstance(res, dict) and any(m in str(res.get("error", "")) for m in PEER_GONE):
            # a peer rank left the job (its watchdog fired first, or it died): no later collective
            # can complete -- as the watchdog does, rank 0 prints the line so far and every rank leaves
            line.emit(f"{name}: no progress -- a peer rank left the job ({res['error']}); the figures after it "
                      f"were not run")
            os._exit(EXIT_ABORTED)
        return res

    if world > 1 and not pull_only:
        def _xo():
            s, per = exchange_only(group, timed_first, K, world, dev)
            out["xgmi"].update({"exchange_only_ms": 1e3 * s, "exchange_only_ms_per_rank": [1e3 * x for x in per],
                                "exchange_only_busiest_link_GBps": float(np.mean(link_bytes)) / s / 1e9,
                                "exchange_only_busiest_pair_both_directions_GBps":
                                    float(np.mean(pair_bytes)) / s / 1e9})
            return True
        xo = figure("exchange_only", _xo)
        if isinstance(xo, dict):
            out["xgmi"]["exchange_only_error"] = xo
        probe = figure("p2p_probe", lambda: p2p_probe(rank, world, P * 4, dev, rccl=not gloo))
        if probe and "uni" in probe:
            out["xgmi"]["p2p_probe"] = {"bytes": P * 4, "uni_ms": 1e3 * probe["uni"],
                                        "uni_GBps": P * 4 / probe["uni"] / 1e9, "bi_ms": 1e3 * probe["bi"],
                                        "bi_GBps_both_directions": 2 * P * 4 / probe["bi"] / 1e9,
                                        "how": "torch.distributed batch_isend_irecv (RCCL), ranks 0 and 1, "
                                               "median of 5 after one untimed transfer"}
        elif probe:
            out["xgmi"]["p2p_probe"] = probe
    out["cpu_baseline"] = None
    if world == 1 and args.cpu_seconds > 0 and rank == 0:
        out["cpu_baseline"] = guarded("cpu_baseline", lambda: cpu_baseline(partner, GP.neighbor_weight, n, P,
                                                                           args.cpu_seconds))
    out["matcha_schedule"] = figure("matcha", lambda: matcha_figure(pkg, args, rank, world, n, P, K, W, comm, dev),
                                    args.budget >= 1.0)
    out["allreduce_baseline"] = figure("allreduce", lambda: allreduce_figure(
        pkg, args, rank, world, n, P, max(5, K), 2, comm, dev,
        arena=group.arena if world == 1 else None), bool(args.allreduce) and not pull_only)
    if pull_only and args.allreduce:
        out["allreduce_baseline"] = {"skipped": "the all-gather needs the RCCL communicator (rccl_unavailable)"}
    # the headline groups are done: release them before the large figures
    for g in {id(g): g for g in (timed, group)}.values():
        g.close()
    forms.clear()
    del timed, group
    torch.cuda.empty_cache()
    choco_warm = 3 + settle_rounds(24 * args.choco_params * -(-n // world), args.settle_ms)
    out["choco"] = figure("choco", lambda: choco_figure(pkg, GP, rank, world, max(20, K), choco_warm, comm, dev,
                                                        P=args.choco_params, placement=args.placement,
                                                        pull=args.pull),
                          bool(args.choco))
    out["cpu_resident_models"] = figure("staged", lambda: staged_figure(pkg, GP, n, P, 3, W),
                                        world == 1 and bool(args.staged))
    out["configs"] = figure("configs", lambda: config_figures(pkg, args, rank, world, n, max(10, K), 3, comm, dev),
                            bool(args.configs))
    out["er64_sweep"] = figure("er64", lambda: er_figure(pkg, args, rank, world, comm, dev), bool(args.er))
    out["figures_s"] = time.monotonic() - t_fig
    if world > 1:
        out["pull_transport"] = pull_counts(pkg, world)     # the whole run's binds, summed over ranks
    line.emit()
    if world > 1:
        wd.arm("teardown", args.figure_timeout)
        dist.barrier()
        if isinstance(comm, pkg.engine.RcclComm):
            comm.close()
        dist.destroy_process_group()
        wd.disarm()


if __name__ == "__main__":
    main()
