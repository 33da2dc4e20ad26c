"""Gossip engine: the device-resident schedule, round plans, worker layout and transport.

One process drives one GPU and a contiguous block of the topology's workers
(rows [row_base, row_base + n_local)).  With one process (the "virtual worker" mode) the
block is every worker; with N processes (torch.distributed, one per GPU) the workers are split
into N contiguous blocks and edges that cross blocks go over RCCL (xGMI).

Per round (reference: decenCommunicator.communicate, communicator.py:133-158):
    1. [N > 1] mx_exchange_round: one ncclGroupStart/End with a send of every local row whose
       active partner is remote and a receive of every remote partner row into the slab;
    2. mx_gossip_mix: the in-place FMA-chain mixing kernel over local rows + slab rows, driven
       by the precomputed plan record of this iteration.
Everything is enqueued on one HIP stream; nothing is copied to or from the host per round.
"""
import ctypes
import sys
import time
import weakref

import numpy as np
import torch

from ._lib import MX_ERR_RCCL, MXError, check, lib, require_device, stream_ptr

ROW_ALIGN = 64  # arena rows padded to 256 B

TUNE_KEYS = ("blocks_per_cu", "unroll", "nontemporal", "prefetch", "regidx", "chunked", "grid", "readlane_min",
             "rows", "split", "flat_small", "ns48", "rows_pf2", "wide_lds_kb", "wide_plan_lds", "wide_per_cu", "wide_tpb", "rows_tpb", "mid_bpc", "mid_tiles", "wide_pf2", "spec", "spec_wgpc", "spec_glds", "mean_wgpc")


def mix_tuning():
    """Current mixing-kernel knobs (include/matcha_gossip.h, mx_mix_set)."""
    return {k: int(lib.mx_mix_get(k.encode())) for k in TUNE_KEYS}


def mix_kernel_name(n_slots):
    """The kernel mx_gossip_mix launches for n_slots under the current knobs."""
    return lib.mx_mix_kernel_name(int(n_slots)).decode()


_TUNE_GEN = [0]     # bumped on every knob change: layouts re-check their tile size only then
_mix_packed = lib.mx_gossip_mix_packed


def set_mix_tuning(**knobs):
    _TUNE_GEN[0] += 1
    for k, v in knobs.items():
        check(lib.mx_mix_set(k.encode(), int(v)), "mx_mix_set")


def partition(n, nranks):
    """Contiguous worker blocks [(row_base, n_local)] per rank (sizes differ by at most 1)."""
    base, extra = divmod(n, nranks)
    out, start = [], 0
    for r in range(nranks):
        cnt = base + (1 if r < extra else 0)
        out.append((start, cnt))
        start += cnt
    return out


def owner_table(n, nranks):
    own = np.empty(n, np.int32)
    for r, (b, c) in enumerate(partition(n, nranks)):
        own[b:b + c] = r
    return own


def validate_partner(partner):
    """The drawer's table must describe matchings: symmetric, in range (graph_manager.py:157-180)."""
    M, n = partner.shape
    for g in range(M):
        for i in range(n):
            j = int(partner[g, i])
            if j == -1:
                continue
            if not (0 <= j < n) or j == i or int(partner[g, j]) != i:
                raise ValueError(f"neighbors_info[{g}] is not a matching at worker {i} -> {j}")


def max_incoming_remote(partner, row_base, n_local):
    """Receive-slab rows needed when every matching is active (upper bound over all rounds): the
    distinct remote workers that partner a local worker in some matching -- each is received
    once per round however many local partners it has (mx_exchange_plan / plan_kernel)."""
    M, n = partner.shape
    remote = set()
    for g in range(M):
        for p in range(n):
            q = int(partner[g, p])
            if q < 0:
                continue
            if row_base <= q < row_base + n_local and not (row_base <= p < row_base + n_local):
                remote.add(p)
    return len(remote)


class RcclComm:
    """An RCCL communicator owned by the C library (one per process), bootstrapped through
    torch.distributed (which must be initialised; any backend) for the unique-id broadcast.

    The communicator is non-blocking with a deadline (mx_rccl_init_timeout): if a peer never
    joins the init, or the connection setup of a later exchange / all-reduce, the call raises
    MXError ("timed out") after `timeout_s` (default $MX_RCCL_TIMEOUT_S or 300 s) instead of
    hanging; abort() then releases the communicator.  A peer that dies or skips an exchange
    AFTER the connections exist leaves the RCCL kernel waiting on the GPU: wait() is the stream
    synchronisation with the same deadline (mx_rccl_wait: on expiry the communicator is aborted
    and MXError raised) -- use it instead of torch.cuda.synchronize() where a peer may be gone."""

    def __init__(self, group=None, timeout_s=None):
        import os
        import torch.distributed as dist
        require_device()
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        if timeout_s is None:
            timeout_s = float(os.environ.get("MX_RCCL_TIMEOUT_S") or 300.0)
        self.timeout_s = float(timeout_s)
        uid = (ctypes.c_char * 128)()
        if self.rank == 0:
            check(lib.mx_rccl_unique_id(ctypes.cast(uid, ctypes.c_void_p)), "mx_rccl_unique_id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=group)
        buf = (ctypes.c_char * 128).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        nb = ctypes.c_int(0)
        check(lib.mx_rccl_init_timeout(ctypes.cast(buf, ctypes.c_void_p), self.nranks, self.rank,
                                       int(self.timeout_s * 1000), ctypes.byref(h), ctypes.byref(nb)),
              "mx_rccl_init_timeout")
        self.handle = h
        self.nonblocking = bool(nb.value)

    def count(self):
        """ncclCommCount: the ranks RCCL holds in this communicator."""
        n = ctypes.c_int(0)
        check(lib.mx_rccl_count(self.handle, ctypes.byref(n)), "mx_rccl_count")
        return int(n.value)

    def wait(self, stream=None, timeout_s=None):
        """Block until everything enqueued on `stream` (default: the current stream) has run, or
        raise MXError after timeout_s (default: the communicator's deadline) -- the communicator is
        then aborted (mx_rccl_wait)."""
        if not self.handle:
            raise MXError("RcclComm.wait: communicator closed or aborted")
        ms = int(1000 * (self.timeout_s if timeout_s is None else float(timeout_s)))
        rc = lib.mx_rccl_wait(self.handle, stream_ptr(stream), max(1, ms))
        if rc:
            if rc == MX_ERR_RCCL:
                self.handle = None              # only the timeout path aborts the communicator
            check(rc, "mx_rccl_wait")

    def abort(self):
        """Release a communicator whose peers are gone (ncclCommAbort; after a timed-out call)."""
        if self.handle:
            lib.mx_rccl_abort(self.handle)
            self.handle = None

    def close(self):
        if self.handle:
            rc = lib.mx_rccl_destroy(self.handle)
            self.handle = None
            check(rc, "mx_rccl_destroy")


class PullTransport:
    """Cross-GPU partner rows without RCCL: every rank publishes a snapshot of its rows in an
    IPC-shared device buffer (mx_ipc_alloc); its peers map it (mx_ipc_open) and their mixing
    kernel reads the partner rows straight from this GPU's HBM over xGMI (communicator.py:110's
    sendrecv becomes a remote load inside the FMA chain).  A round is three launches on one
    stream and nothing on the host (VirtualWorkerGroup._step_pull):
        1. mx_snapshot_publish_rows: the local rows a peer reads this round (an active partner in
           another block) into snapshot `round % 2` of the buffer, every workgroup ending with a
           system-scope release (the bytes reach HBM, not only this GPU's write-back L2);
        2. mx_pull_gate (one wave): this rank's epoch = round + 1 (system-scope release), then a
           bounded wait for the epochs of the ranks owning this round's and the previous round's
           remote partners, then the receive slots pointed at their snapshot rows (csrc/pull.hip);
        3. the mixing kernel; the plan records carry the peer-reads bit
           (mx_plan_set_peer_reads), so every workgroup first acquires at system scope: lines of
           the same snapshot buffer cached on THIS GPU in round r - 2 are not served.
    Snapshots alternate between two buffers; a rank overwrites snapshot r % 2 in round r + 2 only
    after its gate of round r + 1 saw every reader of round r past its mix.  A
    peer that stops publishing makes the gate expire after `timeout_s` (default
    $MX_PULL_TIMEOUT_S or 300 s): sticky error words, MXError at the end of the round
    (VirtualWorkerGroup.wait_round) or at the next step.  Needs one process per GPU of ONE node
    (the peers' HBM must be mappable) -- or, for tests, several processes sharing a GPU.
    Bootstrap uses torch.distributed (any backend).  VirtualWorkerGroup.close() is collective
    under this transport (a barrier before the buffers are freed)."""

    handle = None

    def __init__(self, group=None, timeout_s=None):
        import os
        import torch.distributed as dist
        require_device()
        self.group = group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        if self.nranks > 64:
            raise ValueError("PullTransport: at most 64 ranks")
        if timeout_s is None:
            timeout_s = float(os.environ.get("MX_PULL_TIMEOUT_S") or 300.0)
        if not timeout_s > 0:
            raise ValueError("PullTransport: timeout_s must be > 0")
        self.timeout_s = float(timeout_s)

    def bind(self, vwg, row_bytes=None):
        """Collective: allocate vwg's snapshot buffer, exchange handles, map the peers'.  Every
        rank takes part in every exchange even when its own step failed, and all ranks raise
        together (MXError naming the first failing rank) if any failed, so a refusal on one GPU
        cannot leave the others waiting.  No retry: a refused export is counted by the library
        (mx_ipc_stats -> pull_stats()) and reported, never absorbed (DESIGN.md "IPC exports").
        row_bytes: the stride of one worker's snapshot (default: a whole row, vwg.ld floats; a
        ChocoWorkerGroup passes its message stride)."""
        import torch.distributed as dist
        hb = int(lib.mx_ipc_handle_bytes())
        half = vwg.n_local * (int(row_bytes) if row_bytes is not None else vwg.ld * 4)
        _BIND_STATS["binds"] += 1
        own = ctypes.c_void_p()
        handle = (ctypes.c_char * hb)()
        err = None
        try:
            check(lib.mx_ipc_alloc(PULL_HEADER + 2 * half, ctypes.byref(own), ctypes.cast(handle, ctypes.c_void_p)),
                  "mx_ipc_alloc")
        except MXError as e:
            err = str(e)
        objs = [None] * self.nranks
        dist.all_gather_object(objs, (self.rank, None if err else bytes(handle)), group=self.group)
        peers = [0] * self.nranks
        opened = []
        if err is None and all(h is not None for _, h in objs):
            try:
                for r, h in objs:
                    if r == self.rank:
                        peers[r] = own.value
                        continue
                    buf = (ctypes.c_char * hb).from_buffer_copy(h)
                    p = ctypes.c_void_p()
                    check(lib.mx_ipc_open(ctypes.cast(buf, ctypes.c_void_p), ctypes.byref(p)), "mx_ipc_open")
                    peers[r] = p.value
                    opened.append(p.value)
            except MXError as e:
                err = str(e)
        elif err is None:
            err = "a peer could not allocate its snapshot buffer"
        oks = [None] * self.nranks
        dist.all_gather_object(oks, err, group=self.group)
        bad = [(r, e) for r, e in enumerate(oks) if e is not None]
        if bad:
            for p in opened:
                lib.mx_ipc_close(p)
            if own.value:
                lib.mx_ipc_free(own.value)
            _BIND_STATS["failed"] += 1
            sys.stderr.write(f"[matcha_gossip] PullTransport.bind: rank {self.rank}: failed: {bad}\n")
            raise MXError(f"pull transport unavailable: rank {bad[0][0]}: {bad[0][1]}")
        return _PullState(self, vwg, own.value, peers, opened, half)


PULL_HEADER = 256          # MX_PULL_HEADER_BYTES: the epoch word ahead of the two snapshots

# this process's pull-transport binds: how many, how many failed (on any rank of the group)
# (with mx_ipc_stats' refused exports, reported by bench.py's line and checked
# to be zero by the multi-process tests -- never absorbed silently)
_BIND_STATS = {"binds": 0, "failed": 0}


def ipc_stats():
    """(hipIpcGetMemHandle calls, refusals) of this process so far (mx_ipc_stats)."""
    ex, ref = ctypes.c_int(0), ctypes.c_int(0)
    check(lib.mx_ipc_stats(ctypes.byref(ex), ctypes.byref(ref)), "mx_ipc_stats")
    return int(ex.value), int(ref.value)


def pull_stats():
    """{"binds", "bind_failures", "ipc_exports", "ipc_refused", "ipc_recovered"} of this process so
    far: every PullTransport.bind, every hipIpcGetMemHandle call, every mx_ipc_alloc that returned no
    exported block, and every refused block a second allocation recovered (the address range of a
    just-closed import reused: mx_ipc_alloc, tools/ipc_reuse_probe.py)."""
    ex, ref = ipc_stats()
    return {"binds": _BIND_STATS["binds"], "bind_failures": _BIND_STATS["failed"], "ipc_exports": ex,
            "ipc_refused": ref, "ipc_recovered": int(lib.mx_ipc_get(b"recovered"))}


class _PullState:
    """One group's bound pull buffers: the device table of every rank's snapshot buffer
    (mx_pull_rank), the previous round's flags row, and the gate's sticky error words."""

    def __init__(self, transport, vwg, own, peers, opened, half):
        self.transport, self.own, self.peers, self.opened, self.half = transport, own, peers, opened, half
        self.round = 0
        blocks = partition(int(vwg.topology.size), transport.nranks)
        tab = np.zeros((transport.nranks, 2), np.int64)
        for r, (b, c) in enumerate(blocks):
            tab[r, 0] = peers[r]
            tab[r, 1] = (int(b) & 0xFFFFFFFF) | (int(c) << 32)      # int32 row_base, int32 n_local
        self.ranks_dev = torch.from_numpy(tab).to("cuda")
        self.owner_dev = torch.from_numpy(np.ascontiguousarray(vwg.engine.owner)).to("cuda")
        self.prev_row = torch.zeros(vwg.engine.M, dtype=torch.uint8, device="cuda")
        host, dev = ctypes.POINTER(ctypes.c_int32)(), ctypes.c_void_p()
        check(lib.mx_host_words(4, ctypes.byref(host), ctypes.byref(dev)), "mx_host_words")
        self.err_host, self.err_dev = host, dev.value

    def error(self):
        """None, or the gate's message once one of its waits expired (sticky)."""
        if not self.err_host or self.err_host[0] == 0:
            return None
        e = [int(self.err_host[i]) for i in range(4)]
        if e[0] == 2:
            return "pull gate: more distinct remote partners than receive slots"
        return (f"pull gate: rank {e[1]} did not publish round epoch {e[2]} within "
                f"{self.transport.timeout_s:g} s (last seen {e[3]}); the round's result is undefined")

    def close(self):
        for p in self.opened:
            lib.mx_ipc_close(p)
        self.opened = []
        if self.own:
            lib.mx_ipc_free(self.own)
            self.own = 0
        if self.err_host:
            lib.mx_host_words_free(ctypes.cast(self.err_host, ctypes.c_void_p))
            self.err_host = None


def wait_round(comm, stream=None):
    """The end-of-round synchronisation of communicate(): with the library's RCCL communicator a
    deadline-bounded wait (RcclComm.wait -- a peer gone mid-exchange raises instead of hanging),
    otherwise torch.cuda.synchronize().  An RcclComm that was aborted raises: its kernels may
    still be queued, and an unbounded synchronize could hang on them."""
    if isinstance(comm, RcclComm):
        if not comm.handle:
            raise MXError("the RCCL communicator was aborted or closed (an earlier exchange timed out)")
        comm.wait(stream)
    else:
        torch.cuda.synchronize()


_DEFAULT_COMM = None


def default_comm():
    """Process-wide RCCL communicator over the default torch.distributed group."""
    global _DEFAULT_COMM
    if _DEFAULT_COMM is None:
        _DEFAULT_COMM = RcclComm()
    return _DEFAULT_COMM


def topology_flags(topology):
    """Device flag table uint8 [T][M] of a processor, consistent with its host active_flags."""
    host = np.asarray(topology.active_flags, dtype=np.uint8)
    if host.ndim != 2:
        raise ValueError("active_flags must be a rectangular [iterations][matchings] table")
    dev = getattr(topology, "flags_dev", None)
    if dev is not None and tuple(dev.shape) == host.shape:
        if np.array_equal(dev.cpu().numpy(), host):
            return dev, host
    return torch.from_numpy(np.ascontiguousarray(host)).to("cuda"), host


def flags_row(active_flags, M):
    """A flags row as uint8[M]: a shorter row (FixedProcessor's two columns) names the first
    matchings only, like the reference's enumerate(active_flags) walk (communicator.py:99-110); a
    longer one names matchings that do not exist (neighbors_info[graph_id] would fail there too)."""
    f = np.asarray(active_flags)
    if f.ndim != 1 or f.shape[0] > M:
        raise IndexError(f"active_flags must hold at most one entry per matching ({M}), got shape {f.shape}")
    row = np.zeros(M, np.uint8)
    row[:f.shape[0]] = f != 0
    return row


class MixCall(ctypes.Structure):
    """mx_mix_call (include/matcha_gossip.h): a group's mixing arguments packed once, so an eager
    round converts 3 ctypes arguments instead of 13 (mx_gossip_mix_packed)."""
    _fields_ = [("seg_ptrs_dev", ctypes.c_void_p), ("seg_len_dev", ctypes.c_void_p),
                ("tile_off_dev", ctypes.c_void_p), ("seg_vec_dev", ctypes.c_void_p),
                ("plan_dev", ctypes.c_void_p), ("total_tiles", ctypes.c_int64), ("nseg", ctypes.c_int32),
                ("n_slots", ctypes.c_int32), ("n_local", ctypes.c_int32), ("M", ctypes.c_int32),
                ("alpha", ctypes.c_float), ("pad_", ctypes.c_int32), ("need_host", ctypes.c_void_p),
                ("n_iters", ctypes.c_int64)]


class Layout:
    """Pointer table of the mixing kernel: slot k's copy of segment s (include/matcha_gossip.h)."""

    def __init__(self, seg_lens, slot_ptrs, n_slots):
        nseg = len(seg_lens)
        seg_len = np.asarray(seg_lens, dtype=np.int64)
        table = np.zeros((nseg, n_slots), dtype=np.int64)
        vec = np.ones(nseg, dtype=np.uint8)
        for k, ptrs in enumerate(slot_ptrs):
            for s in range(nseg):
                table[s, k] = ptrs[s]
                if ptrs[s] % 16:
                    vec[s] = 0
        tile_off = np.zeros(nseg + 1, dtype=np.int64)
        check(lib.mx_mix_layout(seg_len.ctypes.data, nseg, n_slots, tile_off.ctypes.data), "mx_mix_layout")
        self.nseg = nseg
        self.n_slots = n_slots
        self.tile = int(lib.mx_mix_tile(n_slots))
        self.total_tiles = int(tile_off[-1])
        self.seg_ptrs = torch.from_numpy(table).to("cuda")
        self.seg_len = torch.from_numpy(seg_len).to("cuda")
        self.tile_off = torch.from_numpy(tile_off).to("cuda")
        self.seg_vec = torch.from_numpy(vec).to("cuda")
        self.tune_gen = _TUNE_GEN[0]
        self._args = (self.seg_ptrs.data_ptr(), self.seg_len.data_ptr(), self.tile_off.data_ptr(),
                      self.seg_vec.data_ptr(), nseg, self.total_tiles, n_slots)
        # engine -> (MixCall, its address).  Keyed by the engine object, weakly: a freed engine's
        # record goes with it, so a later engine whose plan tensor reuses the same device address
        # never inherits its n_local / M / alpha or its need_host pointer
        self._calls = weakref.WeakKeyDictionary()

    def call_for(self, engine):
        """The packed mx_mix_call of this layout under `engine` (built once, kept while both live)."""
        rec = self._calls.get(engine)
        if rec is None:
            need = engine.need_host
            c = MixCall(self._args[0], self._args[1], self._args[2], self._args[3], engine._plan_ptr,
                        self.total_tiles, self.nseg, self.n_slots, engine.n_local, engine.M, engine.alpha32, 0,
                        need.ctypes.data if need is not None else None, len(need) if need is not None else 0)
            rec = self._calls[engine] = (c, ctypes.addressof(c))
        return rec[1]


IDLE_MODES = {"skip": 0, "canonical": 1}


class GossipEngine:
    """Schedule + plans for one block of workers of a FixedProcessor / MatchaProcessor.

    idle_rows -- workers with no active partner in an active round: "skip" (default; not read or
    written) or "canonical" (rewritten as 0 + 1.0 * x like the reference's averaging, which turns
    -0.0 into +0.0 -- bit-identical to the reference at the cost of streaming those rows;
    mx_plan_set_idle)."""

    def __init__(self, topology, row_base=0, n_local=None, comm=None, owner=None, idle_rows="skip"):
        require_device()
        if idle_rows not in IDLE_MODES:
            raise ValueError(f"idle_rows must be one of {sorted(IDLE_MODES)}")
        self.idle_rows = idle_rows
        self.topology = topology
        self.n = int(topology.size)
        partner_all = np.asarray(topology.neighbors_info, dtype=np.int32).reshape(-1, self.n)
        self.flags_dev, self.flags_host = topology_flags(topology)
        self.T, self.M = self.flags_host.shape
        if self.M > partner_all.shape[0]:
            raise IndexError(f"active_flags has {self.M} columns but only {partner_all.shape[0]} "
                             "matchings exist (neighbors_info[graph_id] would fail)")
        if self.M < partner_all.shape[0]:
            # FixedProcessor's table has two columns (graph_manager.py:208-225) while the
            # reference's averaging(active_flags) walks whatever row it is given over
            # neighbors_info: the table is padded with zero columns, so a round over every
            # matching (adhoc) is expressible; schedule rounds are unchanged
            pad = partner_all.shape[0] - self.M
            self.flags_host = np.hstack([self.flags_host, np.zeros((self.T, pad), np.uint8)])
            self.flags_dev = torch.from_numpy(np.ascontiguousarray(self.flags_host)).to("cuda")
            self.M = partner_all.shape[0]
        self.partner = np.ascontiguousarray(partner_all[:self.M])
        validate_partner(self.partner)
        self.alpha = float(topology.neighbor_weight)
        self.alpha32 = float(np.float32(self.alpha))
        self.row_base = int(row_base)
        self.n_local = self.n if n_local is None else int(n_local)
        self.comm = comm
        self.rank = comm.rank if comm is not None else 0
        if comm is not None and owner is not None and int(owner[self.row_base]) != self.rank:
            raise ValueError("worker block does not belong to this rank")
        self.owner = (np.zeros(self.n, np.int32) if owner is None
                      else np.ascontiguousarray(owner, dtype=np.int32))
        self.max_remote = max_incoming_remote(self.partner, self.row_base, self.n_local)
        if self.max_remote and comm is None:
            raise ValueError("workers outside this block have partners inside it: an RCCL "
                             "communicator is required")
        self.n_slots = self.n_local + self.max_remote
        if lib.mx_mix_tile(self.n_slots) <= 0:   # 1-64 slots: tuned kernels; 65-156: mix_kernel_wide
            raise MXError(f"{self.n_slots} slots per GPU (local workers + distinct remote partners) exceed "
                          "the 156 a mixing tile holds in LDS: spread the workers over more GPUs")
        self.plan_words = int(lib.mx_plan_words(self.n_local, self.M))
        self.partner_dev = torch.from_numpy(self.partner).to("cuda")
        # the schedule's T records + one scratch record (index T) for a round of arbitrary flags (adhoc)
        self.plan = torch.empty((self.T + 1) * self.plan_words, dtype=torch.int32, device="cuda")
        check(lib.mx_plan_build(self.flags_dev.data_ptr(), self.T, self.M, self.partner_dev.data_ptr(),
                                self.n, None, self.rank, self.row_base, self.n_local, self.alpha,
                                self.plan.data_ptr(), stream_ptr()), "mx_plan_build")
        if IDLE_MODES[idle_rows]:
            check(lib.mx_plan_set_idle(self.plan.data_ptr(), self.T, self.n_local, self.M, IDLE_MODES[idle_rows],
                                       stream_ptr()), "mx_plan_set_idle")
        self.flags_host = np.vstack([self.flags_host, np.zeros((1, self.M), np.uint8)])
        self.any_active = self.flags_host.any(axis=1).tolist()
        # per round, the local rows the mixing kernel reads and writes (the plan record's own row
        # set, from the host's copy of the flags): mx_mix_call.need_host, the kernel's load hint
        self._has_partner = (self.partner[:, self.row_base:self.row_base + self.n_local] >= 0).astype(np.int32)
        self.need_host = None
        if self.n_local <= 64:
            self.need_host = np.zeros(self.T + 1, np.uint64)
            self.need_host[:] = self._need_bits(self.flags_host)
        self._plan_ptr = self.plan.data_ptr()
        self.peer_reads = False                  # set by a pull-transport group: applied to adhoc records too
        self._adhoc_ready = False
        self._adhoc_flags = None
        self._row_index = None                   # flags bytes -> first schedule iteration (record_for)

    def adhoc(self, active_flags):
        """A round for an arbitrary flags row -- the reference's averaging(active_flags) takes any
        row, not only the schedule's (communicator.py:92-122, 200-230): its plan record is built
        into the scratch record after the schedule's T rows (stream-ordered, on the current
        stream) and its index, T, returned; valid until the next adhoc() call.  Collective like the
        reference's sendrecv: with N > 1 every rank passes the same row."""
        f = self.flags_row(active_flags)
        self.flags_host[self.T] = f
        self.any_active[self.T] = bool(f.any())
        if self.need_host is not None:
            self.need_host[self.T] = self._need_bits(f[None, :])[0]
        self._adhoc_flags = torch.from_numpy(f.copy()).to("cuda")
        rec = self._plan_ptr + 4 * self.T * self.plan_words
        check(lib.mx_plan_build(self._adhoc_flags.data_ptr(), 1, self.M, self.partner_dev.data_ptr(), self.n, None,
                                self.rank, self.row_base, self.n_local, self.alpha, rec, stream_ptr()),
              "mx_plan_build")
        if IDLE_MODES[self.idle_rows]:
            check(lib.mx_plan_set_idle(rec, 1, self.n_local, self.M, IDLE_MODES[self.idle_rows], stream_ptr()),
                  "mx_plan_set_idle")
        if self.peer_reads:
            check(lib.mx_plan_set_peer_reads(rec, 1, self.n_local, self.M, 1, stream_ptr()), "mx_plan_set_peer_reads")
        self._adhoc_ready = True
        return self.T

    def _need_bits(self, flags):
        """uint64 row masks of rounds `flags` [t][M]: bit r = local row r has an active partner
        (every row of an active round in idle mode "canonical"), as plan_kernel decides."""
        flags = np.asarray(flags, np.int32)
        rows = (flags @ self._has_partner) > 0
        if IDLE_MODES[self.idle_rows]:
            rows = np.repeat(flags.any(axis=1)[:, None], self.n_local, axis=1)
        weights = np.left_shift(np.uint64(1), np.arange(self.n_local, dtype=np.uint64))
        return (rows.astype(np.uint64) * weights[None, :]).sum(axis=1, dtype=np.uint64)

    def record_for(self, active_flags):
        """The plan record of an arbitrary flags row without rebuilding when one exists: a record
        depends only on the row (partners and alpha are fixed), so any schedule iteration with the
        same row -- or the scratch record when it already holds this row -- serves it; otherwise
        adhoc() builds it.  (The reference's averaging(active_flags) sub-step, communicator.py:92-122,
        driven directly: at most 2^M distinct rows, so rebuilds stop after the first of each.)"""
        f = self.flags_row(active_flags)
        key = f.tobytes()
        if self._row_index is None:
            self._row_index = {}
            for t in range(self.T - 1, -1, -1):          # the first iteration holding each row
                self._row_index[self.flags_host[t].tobytes()] = t
        t = self._row_index.get(key)
        if t is not None:
            return t
        if self._adhoc_ready and self.flags_host[self.T].tobytes() == key:
            return self.T
        return self.adhoc(f)

    def flags_row(self, active_flags):
        return flags_row(active_flags, self.M)

    def round_index(self, it):
        """`it` checked against the plan table: a schedule row, or T after adhoc()."""
        it = int(it)
        if not (0 <= it < self.T or (it == self.T and self._adhoc_ready)):
            raise IndexError(f"iteration {it} outside the schedule's {self.T} rows")
        return it

    # ------------------------------------------------------------------ per round
    def exchange_plan(self, it):
        """The ordered point-to-point operations of round `it` for this block (native
        mx_exchange_plan): int32 [n_ops][4] = (0 send / 1 recv, peer, local row / slab slot,
        worker whose row travels)."""
        fr = np.ascontiguousarray(self.flags_host[it])
        cnt = ctypes.c_int(0)
        check(lib.mx_exchange_plan(fr.ctypes.data, self.M, self.partner.ctypes.data, self.n,
                                   self.owner.ctypes.data, self.rank, self.row_base, self.n_local,
                                   None, 0, ctypes.byref(cnt)), "mx_exchange_plan")
        ops = np.zeros((max(1, cnt.value), 4), np.int32)
        check(lib.mx_exchange_plan(fr.ctypes.data, self.M, self.partner.ctypes.data, self.n,
                                   self.owner.ctypes.data, self.rank, self.row_base, self.n_local,
                                   ops.ctypes.data, cnt.value, ctypes.byref(cnt)), "mx_exchange_plan")
        return ops[:cnt.value]

    def exchange(self, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes, stream=None):
        """Sends/receives of iteration `it` (no-op with one process).  The transport is the RCCL
        communicator (mx_exchange_round); an object with an ``exchange_round`` method may stand
        in for it (tests use an in-process loopback to drive N ranks on one GPU)."""
        if self.comm is None:
            return 0
        if hasattr(self.comm, "exchange_round"):
            return self.comm.exchange_round(self, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes)
        row_arr = (ctypes.c_void_p * self.n_local)(*row_ptrs)
        nrem = ctypes.c_int(0)
        fr = np.ascontiguousarray(self.flags_host[it])
        check(lib.mx_exchange_round(self.comm.handle, fr.ctypes.data, self.M, self.partner.ctypes.data,
                                    self.n, self.owner.ctypes.data, self.rank, self.row_base,
                                    self.n_local, row_arr, slab_ptr, int(slab_ld_bytes), int(row_bytes),
                                    ctypes.byref(nrem), stream_ptr(stream)), "mx_exchange_round")
        return nrem.value

    def mix(self, it, layout, stream=None):
        it = self.round_index(it)                # the kernel indexes the plan table by `it`
        if layout.tune_gen != _TUNE_GEN[0]:
            if layout.tile != lib.mx_mix_tile(layout.n_slots):
                raise MXError("layout built for another mixing tile size (the unroll knob changed it)")
            layout.tune_gen = _TUNE_GEN[0]
        # one ctypes call per round with the group's arguments packed once (small rows are
        # launch-bound: tools/launch_overhead.py)
        rc = _mix_packed(layout.call_for(self), it, stream_ptr(stream))
        if rc:
            check(rc, "mx_gossip_mix_packed")


    def mix_at(self, iter_dev, layout, stream=None):
        """Graph-replayable round: the kernel reads the iteration from the int64 device tensor
        `iter_dev` when it runs (mx_gossip_mix_at) and the counter is advanced by one on the same
        stream, so a captured launch pair serves every iteration (a counter past the schedule
        makes the launch a no-op)."""
        if layout.tune_gen != _TUNE_GEN[0]:
            if layout.tile != lib.mx_mix_tile(layout.n_slots):
                raise MXError("layout built for another mixing tile size (the unroll knob changed it)")
            layout.tune_gen = _TUNE_GEN[0]
        if iter_dev.dtype != torch.int64 or iter_dev.device.type != "cuda" or iter_dev.numel() != 1:
            raise TypeError("iter_dev must be a one-element int64 CUDA tensor")
        s = stream_ptr(stream)
        check(lib.mx_gossip_mix_at(*layout._args, self._plan_ptr, iter_dev.data_ptr(), self.T, self.n_local,
                                   self.M, self.alpha32, s), "mx_gossip_mix_at")
        check(lib.mx_iter_advance(iter_dev.data_ptr(), 1, s), "mx_iter_advance")

    def mix_rounds_at(self, iter_dev, ctrs, layout, stream=None):
        """len(ctrs) graph-replayable rounds with one bookkeeping launch (mx_iter_expand: ctrs[j] =
        *iter_dev + j, *iter_dev += K), then one mixing launch per round reading its own counter --
        the same rounds as K mix_at calls, without the K counter bumps."""
        if layout.tune_gen != _TUNE_GEN[0]:
            if layout.tile != lib.mx_mix_tile(layout.n_slots):
                raise MXError("layout built for another mixing tile size (the unroll knob changed it)")
            layout.tune_gen = _TUNE_GEN[0]
        for t in (iter_dev, ctrs):
            if t.dtype != torch.int64 or t.device.type != "cuda" or not t.is_contiguous():
                raise TypeError("iteration counters must be contiguous int64 CUDA tensors")
        K = ctrs.numel()
        s = stream_ptr(stream)
        check(lib.mx_iter_expand(iter_dev.data_ptr(), ctrs.data_ptr(), K, s), "mx_iter_expand")
        for j in range(K):
            check(lib.mx_gossip_mix_at(*layout._args, self._plan_ptr, ctrs.data_ptr() + 8 * j, self.T,
                                       self.n_local, self.M, self.alpha32, s), "mx_gossip_mix_at")


def _params(model):
    return [p for p in model.parameters()]


class VirtualWorkerGroup:
    """A block of the topology's workers resident on this process's GPU as rows of an
    [n_local, P] HBM arena (the "all virtual workers on one MI355X" mode, and each rank's share
    in the multi-GPU mode).

    models  -- optional list of n_local torch modules on the GPU (identical architectures);
               with adopt=True their parameters are re-homed into the arena as views (identity
               and shapes kept, so optimizers stay valid) and every round mixes them in place.
    numel   -- arena width when no models are given (synthetic workloads / benchmarks).
    placement -- which workers share a GPU when nranks > 1: None / "contiguous" (blocks of
               consecutive ids), "auto" (placement.best_placement: fewest rows over the busiest
               xGMI pair) or an explicit worker order.  `workers` lists the worker id of each
               local row (models are given in that order).
    idle_rows -- "skip" (default) or "canonical": see GossipEngine.
    """

    def __init__(self, topology, models=None, numel=None, *, rank=0, nranks=1, comm=None, adopt=True,
                 chunk_cols=None, placement=None, idle_rows="skip"):
        require_device()
        from .placement import block_workers, place
        n = int(topology.size)
        topology, self.placement = place(topology, nranks, placement)
        blocks = partition(n, nranks)
        self.row_base, self.n_local = blocks[rank]
        self.workers = block_workers(self.placement, self.row_base, self.n_local)
        if nranks > 1 and comm is None:
            comm = default_comm()
        self.engine = GossipEngine(topology, self.row_base, self.n_local, comm=comm,
                                   owner=owner_table(n, nranks), idle_rows=idle_rows)
        self.topology = topology
        self.iter = 0
        self.iter_dev = torch.zeros(1, dtype=torch.int64, device="cuda")   # device_round's counter
        self._round_ctrs = {}                # device_rounds(K): per-round counters, one tensor per K
        if models is not None:
            if len(models) != self.n_local:
                raise ValueError(f"{len(models)} models for {self.n_local} local workers")
            shapes = [tuple(p.shape) for p in _params(models[0])]
            for m in models[1:]:
                if [tuple(p.shape) for p in _params(m)] != shapes:
                    raise ValueError("all workers must share one architecture")
            self.numel = int(sum(p.numel() for p in _params(models[0])))
        else:
            if numel is None:
                raise ValueError("give models or numel")
            self.numel = int(numel)
        self.ld = (self.numel + ROW_ALIGN - 1) // ROW_ALIGN * ROW_ALIGN
        self.arena = torch.zeros((self.n_local, self.ld), dtype=torch.float32, device="cuda")
        # column pipelining of the cross-GPU exchange (N > 1): chunk c+1 travels over RCCL on a side
        # stream while chunk c is mixed; the receive slab is two chunk-wide buffers
        self._pull = None
        self.chunked = bool(self.engine.max_remote and chunk_cols and int(chunk_cols) < self.numel
                            and not isinstance(comm, PullTransport))
        if self.chunked:
            W = (int(chunk_cols) + ROW_ALIGN - 1) // ROW_ALIGN * ROW_ALIGN
            self.chunk_w = W
            self.chunks = [(c0, min(self.numel, c0 + W)) for c0 in range(0, self.numel, W)]
            self.slab = torch.empty((2, self.engine.max_remote, W), dtype=torch.float32, device="cuda")
            self.comm_stream = torch.cuda.Stream()
        else:
            self.slab = (torch.empty((self.engine.max_remote, self.ld), dtype=torch.float32, device="cuda")
                         if self.engine.max_remote and not isinstance(comm, PullTransport) else None)
        if models is not None:
            for r, m in enumerate(models):
                off = 0
                for p in _params(m):
                    if p.dtype != torch.float32 or p.device.type != "cuda":
                        raise TypeError("worker parameters must be float32 CUDA tensors")
                    k = p.numel()
                    view = self.arena[r, off:off + k].view(p.shape)
                    view.copy_(p.data)
                    if adopt:
                        p.data = view
                    off += k
        self._row_ptrs = [self.arena[r].data_ptr() for r in range(self.n_local)]
        if self.chunked:
            self.chunk_layouts = []
            for ci, (c0, c1) in enumerate(self.chunks):
                buf = self.slab[ci % 2]
                ptrs = [[p + 4 * c0] for p in self._row_ptrs]
                ptrs += [[buf[k].data_ptr()] for k in range(self.engine.max_remote)]
                self.chunk_layouts.append(Layout([c1 - c0], ptrs, self.engine.n_slots))
            self.layout = Layout([self.numel], [[p] for p in self._row_ptrs] +
                                 [[self.slab[0, 0].data_ptr()]] * self.engine.max_remote, self.engine.n_slots)
        elif isinstance(comm, PullTransport):
            # receive slots point at the peers' snapshot rows, set per round (_step_pull); no slab
            self._pull = comm.bind(self)
            # receive slots will be peers' memory: the mixing kernels acquire at system scope first
            check(lib.mx_plan_set_peer_reads(self.engine.plan.data_ptr(), self.engine.T + 1, self.n_local,
                                             self.engine.M, 1, stream_ptr()), "mx_plan_set_peer_reads")
            self.engine.peer_reads = True
            # receive slots start at this rank's own snapshot 0 (valid memory); every round's gate
            # points them at the partners' snapshot rows on the device (mx_pull_gate)
            slot_ptrs = [[p] for p in self._row_ptrs]
            slot_ptrs += [[self._pull.own + PULL_HEADER]] * self.engine.max_remote
            self.layout = Layout([self.numel], slot_ptrs, self.engine.n_slots)
        else:
            slot_ptrs = [[p] for p in self._row_ptrs]
            if self.slab is not None:
                slot_ptrs += [[self.slab[k].data_ptr()] for k in range(self.engine.max_remote)]
            self.layout = Layout([self.numel], slot_ptrs, self.engine.n_slots)

    @property
    def rows(self):
        """[n_local, P] view of the workers' flat parameter vectors."""
        return self.arena[:, :self.numel]

    @property
    def publish_cols(self):
        """Floats of a row the pull round publishes (the P the mixing kernel reads, rounded up to 4)."""
        return (self.numel + 3) // 4 * 4

    def step(self, it, stream=None):
        """Enqueue round `it` (exchange + mix) on `stream`; returns False for an all-zero round."""
        if not self.engine.any_active[it]:
            return False
        if self.chunked:
            return self._step_chunked(it, stream)
        if self._pull is not None:
            return self._step_pull(it, stream)
        if self.engine.comm is not None:
            self.engine.exchange(it, self._row_ptrs,
                                 self.slab.data_ptr() if self.slab is not None else None,
                                 self.ld * 4, self.numel * 4, stream)
        self.engine.mix(it, self.layout, stream)
        return True

    def _step_pull(self, it, stream=None):
        """PullTransport round, three launches on one stream and no host wait: snapshot publish,
        the gate (epoch out, bounded epoch waits, receive slots -> the partners' snapshot rows),
        mix.  A gate that expired in an earlier round raises here (sticky)."""
        st = self._pull
        msg = st.error()
        if msg:
            raise MXError(msg)
        eng = self.engine
        it = eng.round_index(it)
        par = st.round & 1
        st.round += 1
        s = stream_ptr(stream)
        frow = (eng._adhoc_flags.data_ptr() if it == eng.T else eng.flags_dev.data_ptr() + it * eng.M)
        # only the rows a peer reads this round (an active partner in another block), each ending
        # with a system-scope release per workgroup (visible to the peers' loads); a row not
        # published in round k is read by no peer in round k
        check(lib.mx_snapshot_publish_rows(self.arena.data_ptr(), self.ld, st.own + PULL_HEADER + par * st.half,
                                           self.ld, self.publish_cols, self.n_local, frow, eng.M,
                                           eng.partner_dev.data_ptr(), eng.n, self.row_base, s),
              "mx_snapshot_publish_rows")
        tr = st.transport
        check(lib.mx_pull_gate(frow, st.prev_row.data_ptr(), eng.M, eng.partner_dev.data_ptr(), eng.n,
                               st.owner_dev.data_ptr(), st.ranks_dev.data_ptr(), tr.nranks, tr.rank, self.row_base,
                               self.n_local, self.ld * 4, par, st.round, self.layout.seg_ptrs.data_ptr(),
                               eng.n_slots, tr.timeout_s, st.err_dev, s), "mx_pull_gate")
        eng.mix(it, self.layout, stream)
        return True

    def wait_round(self, stream=None):
        """The end of a round for communicate(): the transport's wait (engine.wait_round), then
        the pull gate's sticky error, if any, as MXError."""
        wait_round(self.engine.comm, stream)
        if self._pull is not None:
            msg = self._pull.error()
            if msg:
                raise MXError(msg)

    @property
    def pulls(self):
        """True when the receive slots are peers' IPC-mapped snapshots (PullTransport)."""
        return self._pull is not None

    def close(self):
        """Release the pull transport's shared buffers.  COLLECTIVE under PullTransport: every
        rank's snapshot buffer may still be read by a slower peer's last round, so all ranks first
        meet at a barrier (after their own last mix has finished), then unmap and free.  Not to be
        called from a finalizer (decenCommunicator.__del__ leaves a pull group to process exit)."""
        if self._pull is not None:
            import torch.distributed as dist
            torch.cuda.synchronize()
            dist.barrier(group=self._pull.transport.group)
            self._pull.close()
            self._pull = None

    def _step_chunked(self, it, stream=None):
        cur = stream if stream is not None else torch.cuda.current_stream()
        cs = self.comm_stream
        start = torch.cuda.Event()
        start.record(cur)
        cs.wait_event(start)                 # rows are final (previous round, optimizer) before sending
        mixed = [None, None]
        for ci, (c0, c1) in enumerate(self.chunks):
            b = ci % 2
            if mixed[b] is not None:
                cs.wait_event(mixed[b])      # slab buffer b is free once chunk ci-2 has been mixed
            self.engine.exchange(it, [p + 4 * c0 for p in self._row_ptrs], self.slab[b].data_ptr(),
                                 self.chunk_w * 4, (c1 - c0) * 4, cs)
            arrived = torch.cuda.Event()
            arrived.record(cs)
            cur.wait_event(arrived)
            self.engine.mix(it, self.chunk_layouts[ci], cur)
            mixed[b] = torch.cuda.Event()
            mixed[b].record(cur)
        return True

    def device_round(self, stream=None):
        """Enqueue the round at the device-side counter `self.iter_dev` and advance it (no host
        work depends on the round, so the pair can be captured once in a HIP graph --
        torch.cuda.graph -- and replayed every iteration).  One GPU only: a cross-GPU exchange's
        operation list depends on the round's flags on the host.  Set the counter with
        `self.iter_dev.fill_(it)`; `self.iter` (the host counter of communicate()) is not touched."""
        if self.engine.comm is not None:
            raise MXError("device_round: graph-replayable rounds need all partners on this GPU (nranks = 1)")
        if self.chunked:
            raise MXError("device_round: not with chunk_cols")
        self.engine.mix_at(self.iter_dev, self.layout, stream)

    def device_rounds(self, K, stream=None):
        """K device_round()s in K + 1 launches instead of 2 K (for capture in one HIP graph): the
        rounds at the counter `self.iter_dev` .. + K - 1, counter advanced by K."""
        if self.engine.comm is not None:
            raise MXError("device_rounds: graph-replayable rounds need all partners on this GPU (nranks = 1)")
        if self.chunked:
            raise MXError("device_rounds: not with chunk_cols")
        K = int(K)
        if K < 1:
            raise ValueError("device_rounds: K >= 1")
        ctrs = self._round_ctrs.get(K)
        if ctrs is None:
            ctrs = self._round_ctrs[K] = torch.zeros(K, dtype=torch.int64, device="cuda")
        self.engine.mix_rounds_at(self.iter_dev, ctrs, self.layout, stream)

    def state_dict(self):
        """Checkpoint: the workers' rows and the iteration counter (resume on the same schedule)."""
        return {"kind": "decen", "iter": int(self.iter), "row_base": int(self.row_base),
                "workers": list(self.workers), "rows": self.rows.detach().clone()}

    def load_state_dict(self, state):
        if state.get("kind") != "decen" or int(state["row_base"]) != self.row_base or \
                list(state.get("workers", self.workers)) != self.workers or \
                tuple(state["rows"].shape) != tuple(self.rows.shape):
            raise ValueError("checkpoint does not match this worker group")
        with torch.no_grad():
            self.rows.copy_(state["rows"])
        self.iter = int(state["iter"])

    def communicate(self):
        """One round at the group's own iteration counter; returns seconds like the reference's
        communicate() (0 for a skipped round)."""
        it = self.iter
        self.iter += 1
        if np.sum(self.topology.active_flags[it]) == 0:
            return 0
        torch.cuda.synchronize()
        tic = time.time()
        self.step(it)
        self.wait_round()
        return time.time() - tic
