"""ChocoSGD compressed gossip on the GPU (communicator.py:161-268, compressors.py:3-19).

ChocoWorkerGroup keeps, for a block of workers on this GPU, the parameter arena x and the
persistent Choco state x_hat and s (all [n_local, P] in HBM).  Per round:
    q_r = top-k(|x_r - x_hat_r|)            mx_topk_abs_diff   (prepare_comm_buffer, 175-196)
    [N > 1] RCCL exchange of the messages   mx_exchange_round  (12 k bytes per edge direction)
    s / x_hat updates + dense x update      mx_choco_apply     (averaging, 200-230; one fused pass)
Under PullTransport (N > 1, one process per GPU of a node) the messages are not sent: every rank
publishes the messages its peers read this round into its IPC-shared snapshot buffer
(mx_snapshot_publish_rows), the device
gate (mx_pull_gate) waits for the partners' epochs and points a device slot table at their
snapshots, mx_pull_fetch copies the round's partner messages from the owners' HBM into the receive
slots, and the apply pass runs as under RCCL (pull_read="fetch"; "direct": the apply reads them in
place, mx_choco_apply_slots) -- no host step per round, as VirtualWorkerGroup's pull round
(engine.PullTransport).
"""
import time

import numpy as np
import torch

from ._lib import MXError, check, lib, require_device, stream_ptr
from .engine import (PULL_HEADER, GossipEngine, PullTransport, ROW_ALIGN, default_comm, owner_table, partition,
                     wait_round)


def topk_count(P, ratio):
    """compressors.py:11 -- k = max(1, int(len * (1 - ratio)))."""
    return max(1, int(P * (1 - ratio)))


class ChocoWorkerGroup:
    def __init__(self, topology, models=None, numel=None, *, ratio, consensus_lr, rank=0, nranks=1,
                 comm=None, adopt=True, placement=None, pull_read="fetch"):
        """placement: as VirtualWorkerGroup (None / "contiguous", "auto" or a worker order);
        `workers` lists the worker id of each local row.  pull_read (PullTransport only): "fetch"
        (default) copies the round's partner messages from their owners' snapshots into the receive
        slots (mx_pull_fetch) before the apply; "direct" lets the apply read them in place
        (mx_choco_apply_slots: no copy, but a system-scope acquire per apply workgroup and a table
        load per message).  Same bits; which is faster across GPUs is measured by bench.py."""
        if pull_read not in ("fetch", "direct"):
            raise ValueError("pull_read must be 'fetch' or 'direct'")
        self.pull_read = pull_read
        require_device()
        from .placement import block_workers, place
        n = int(topology.size)
        topology, self.placement = place(topology, nranks, placement)
        self.row_base, self.n_local = partition(n, nranks)[rank]
        self.workers = block_workers(self.placement, self.row_base, self.n_local)
        if nranks > 1 and comm is None:
            comm = default_comm()
        self.engine = GossipEngine(topology, self.row_base, self.n_local, comm=comm,
                                   owner=owner_table(n, nranks))
        self.topology = topology
        self.ratio = ratio
        self.consensus_lr = consensus_lr
        self.iter = 0
        if models is not None:
            if len(models) != self.n_local:
                raise ValueError(f"{len(models)} models for {self.n_local} local workers")
            self.numel = int(sum(p.numel() for p in models[0].parameters()))
        else:
            self.numel = int(numel)
        P = self.numel
        self.ld = (P + ROW_ALIGN - 1) // ROW_ALIGN * ROW_ALIGN
        self.x = torch.zeros((self.n_local, self.ld), dtype=torch.float32, device="cuda")
        self.x_hat = torch.zeros_like(self.x)     # communicator.py:179-182 (lazy zeros)
        self.s = torch.zeros_like(self.x)
        if models is not None:
            for r, m in enumerate(models):
                off = 0
                for p in m.parameters():
                    if p.dtype != torch.float32 or p.device.type != "cuda":
                        raise TypeError("worker parameters must be float32 CUDA tensors")
                    k = p.numel()
                    view = self.x[r, off:off + k].view(p.shape)
                    view.copy_(p.data)
                    if adopt:
                        p.data = view
                    off += k
        self.k = topk_count(P, ratio)
        self.kpad = (self.k + 1) // 2 * 2
        # vals f32[kpad] | idx int64[k] | tile bounds int32[ceil(P/4096) + 1] (written by the top-k)
        self.msg_bytes = int(lib.mx_choco_msg_bytes(P, self.k))
        self.bnd_off = 4 * self.kpad + 8 * self.k
        self.msg_ld = (self.msg_bytes + 255) // 256 * 256
        self.msgs = torch.empty(self.engine.n_slots * self.msg_ld, dtype=torch.uint8, device="cuda")
        self.work_ld = int(lib.mx_topk_work_bytes(P))
        self.work = torch.zeros(self.n_local * self.work_ld, dtype=torch.uint8, device="cuda")  # zero on first use
        self.apply_work = torch.empty(int(lib.mx_choco_apply_work_bytes(P, self.engine.n_slots)),
                                      dtype=torch.uint8, device="cuda")
        self.gamma32 = float(np.float32(consensus_lr))
        self.iter_dev = torch.zeros(1, dtype=torch.int64, device="cuda")   # device_round's counter
        self._pull = None
        if isinstance(comm, PullTransport):
            # each rank's snapshot buffer holds two generations of its rows' messages; the gate
            # points the remote entries of the slot table at the round's partners' snapshots
            # (placeholder: this rank's own snapshot 0).  "fetch": mx_pull_fetch copies them into
            # the receive slots and the apply reads local memory only; "direct": the apply reads
            # every slot through the table, acquiring at system scope first (peer-reads bit)
            self._pull = comm.bind(self, row_bytes=self.msg_ld)
            ptrs = [self.msgs.data_ptr() + r * self.msg_ld for r in range(self.n_local)]
            ptrs += [self._pull.own + PULL_HEADER] * (self.engine.n_slots - self.n_local)
            self.slot_ptrs = torch.tensor(ptrs, dtype=torch.int64, device="cuda")
            if pull_read == "direct":
                check(lib.mx_plan_set_peer_reads(self.engine.plan.data_ptr(), self.engine.T + 1, self.n_local,
                                                 self.engine.M, 1, stream_ptr()), "mx_plan_set_peer_reads")
                self.engine.peer_reads = True

    @property
    def rows(self):
        return self.x[:, :self.numel]

    @property
    def publish_cols(self):
        """Floats of a message slot the pull round publishes (msg_bytes rounded up to 16 bytes: what
        mx_pull_fetch and mx_choco_apply_slots read)."""
        return (self.msg_bytes + 15) // 16 * 4

    def message(self, slot):
        """(values float32[k], indices int64[k]) views of message `slot` (index-sorted)."""
        base = slot * self.msg_ld
        vals = self.msgs[base:base + 4 * self.k].view(torch.float32)
        idx = self.msgs[base + 4 * self.kpad:base + 4 * self.kpad + 8 * self.k].view(torch.int64)
        return vals, idx

    def compress(self, it, stream=None):
        """prepare_comm_buffer (communicator.py:175-196): every local row's top-k message of
        x - x_hat into its message slot."""
        check(lib.mx_topk_abs_diff_rows(self.x.data_ptr(), self.x_hat.data_ptr(), self.ld, self.n_local,
                                        self.numel, self.k, self.msgs.data_ptr(), self.msg_ld, 4 * self.kpad,
                                        self.bnd_off, self.work.data_ptr(), self.work_ld, stream_ptr(stream)),
              "mx_topk_abs_diff_rows")

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
        """True when partner messages are read from the peers' IPC-mapped snapshots (PullTransport)."""
        return self._pull is not None

    def close(self):
        """Release the pull transport's shared buffers; COLLECTIVE under PullTransport (as
        VirtualWorkerGroup.close: a barrier after this rank's last apply, then unmap and free)."""
        if self._pull is not None:
            import torch.distributed as dist
            torch.cuda.synchronize()
            dist.barrier(group=self._pull.transport.group)
            self._pull.close()
            self._pull = None

    def check_topk(self, stream=None):
        """Synchronise and raise MXError if a top-k row barrier's bounded wait expired since the
        last check (mx_topk_check: that round's messages are undefined; never a GPU hang)."""
        check(lib.mx_topk_check(self.work.data_ptr(), self.work_ld, self.n_local, self.numel, stream_ptr(stream)),
              "mx_topk_check")

    def average(self, it, stream=None):
        """averaging (communicator.py:200-230): receive partner messages ([N > 1] over the
        transport into the message slots after the local ones), then the s / x_hat scatters and
        the dense x update."""
        it = self.engine.round_index(it)         # mx_choco_apply indexes the plan table by `it`
        if self._pull is not None:
            return self._average_pull(it, stream)
        mbase = self.msgs.data_ptr()
        if self.engine.comm is not None:
            self.engine.exchange(it, [mbase + r * self.msg_ld for r in range(self.n_local)],
                                 mbase + self.n_local * self.msg_ld, self.msg_ld, self.msg_bytes, stream)
        check(lib.mx_choco_apply(self.x.data_ptr(), self.x_hat.data_ptr(), self.s.data_ptr(), self.ld,
                                 self.numel, self.k, mbase, self.msg_ld, self.engine.n_slots,
                                 self.engine.plan.data_ptr(), int(it), self.n_local, self.engine.M,
                                 self.engine.alpha32, self.gamma32, self.apply_work.data_ptr(),
                                 stream_ptr(stream)), "mx_choco_apply")

    def _average_pull(self, it, stream=None):
        """PullTransport averaging, four launches (three with pull_read="direct") and no host wait:
        the local messages a peer reads this round into snapshot `round % 2` (system-scope release
        per workgroup), the gate
        (this rank's epoch out, bounded waits for the partners', remote slot table -> their
        snapshots), the fetch of the round's partner messages from their owners' HBM into the
        receive slots, the apply.  A gate that expired earlier raises here."""
        st = self._pull
        msg = st.error()
        if msg:
            raise MXError(msg)
        eng = self.engine
        par = st.round & 1
        st.round += 1
        s = stream_ptr(stream)
        frow = (eng._adhoc_flags.data_ptr() if it == eng.T else eng.flags_dev.data_ptr() + it * eng.M)
        # the messages of the rows a peer reads this round (an active partner in another block)
        check(lib.mx_snapshot_publish_rows(self.msgs.data_ptr(), self.msg_ld // 4, st.own + PULL_HEADER + par * st.half,
                                           self.msg_ld // 4, self.publish_cols, self.n_local, frow, eng.M,
                                           eng.partner_dev.data_ptr(), eng.n, self.row_base, s),
              "mx_snapshot_publish_rows")
        tr = st.transport
        check(lib.mx_pull_gate(frow, st.prev_row.data_ptr(), eng.M, eng.partner_dev.data_ptr(), eng.n,
                               st.owner_dev.data_ptr(), st.ranks_dev.data_ptr(), tr.nranks, tr.rank, self.row_base,
                               self.n_local, self.msg_ld, par, st.round, self.slot_ptrs.data_ptr(), eng.n_slots,
                               tr.timeout_s, st.err_dev, s), "mx_pull_gate")
        if self.pull_read == "direct":
            check(lib.mx_choco_apply_slots(self.x.data_ptr(), self.x_hat.data_ptr(), self.s.data_ptr(), self.ld,
                                           self.numel, self.k, self.slot_ptrs.data_ptr(), eng.n_slots,
                                           eng.plan.data_ptr(), int(it), self.n_local, eng.M, eng.alpha32,
                                           self.gamma32, s), "mx_choco_apply_slots")
            return
        mbase = self.msgs.data_ptr()
        rec = eng.plan.data_ptr() + 4 * int(it) * eng.plan_words
        check(lib.mx_pull_fetch(self.slot_ptrs.data_ptr(), self.n_local, eng.max_remote, rec,
                                mbase + self.n_local * self.msg_ld, self.msg_ld, self.msg_bytes, s), "mx_pull_fetch")
        check(lib.mx_choco_apply(self.x.data_ptr(), self.x_hat.data_ptr(), self.s.data_ptr(), self.ld, self.numel,
                                 self.k, mbase, self.msg_ld, eng.n_slots, eng.plan.data_ptr(), int(it), self.n_local,
                                 eng.M, eng.alpha32, self.gamma32, self.apply_work.data_ptr(), s), "mx_choco_apply")

    def device_round(self, stream=None):
        """Graph-replayable round at the device counter `self.iter_dev` (then advanced): top-k of
        every row, then mx_choco_apply_at, which reads the round on the device and leaves the state
        untouched for a round without active matchings (the reference skips those,
        communicator.py:249-250; the messages written meanwhile are scratch).  One GPU only."""
        if self.engine.comm is not None:
            raise RuntimeError("device_round: graph-replayable rounds need all partners on this GPU (nranks = 1)")
        self.compress(0, stream)
        sp = stream_ptr(stream)
        check(lib.mx_choco_apply_at(self.x.data_ptr(), self.x_hat.data_ptr(), self.s.data_ptr(), self.ld,
                                    self.numel, self.k, self.msgs.data_ptr(), self.msg_ld, self.engine.n_slots,
                                    self.engine.plan.data_ptr(), self.iter_dev.data_ptr(), self.engine.T,
                                    self.n_local, self.engine.M, self.engine.alpha32, self.gamma32,
                                    self.apply_work.data_ptr(), sp), "mx_choco_apply_at")
        check(lib.mx_iter_advance(self.iter_dev.data_ptr(), 1, sp), "mx_iter_advance")

    def step(self, it, stream=None):
        """One round at iteration `it`; False (nothing done) for an all-zero flags row."""
        if not self.engine.any_active[it]:
            return False
        self.compress(it, stream)
        self.average(it, stream)
        return True

    def state_dict(self):
        """Checkpoint: rows, the persistent Choco state x_hat / s (communicator.py:179-182) and
        the iteration counter."""
        P = self.numel
        return {"kind": "choco", "iter": int(self.iter), "row_base": int(self.row_base), "k": int(self.k),
                "workers": list(self.workers),
                "rows": self.x[:, :P].detach().clone(), "x_hat": self.x_hat[:, :P].detach().clone(),
                "s": self.s[:, :P].detach().clone()}

    def load_state_dict(self, state):
        P = self.numel
        if state.get("kind") != "choco" or int(state["row_base"]) != self.row_base or \
                list(state.get("workers", self.workers)) != self.workers or \
                int(state["k"]) != self.k or tuple(state["rows"].shape) != (self.n_local, P):
            raise ValueError("checkpoint does not match this Choco worker group")
        with torch.no_grad():
            self.x[:, :P].copy_(state["rows"])
            self.x_hat[:, :P].copy_(state["x_hat"])
            self.s[:, :P].copy_(state["s"])
        self.iter = int(state["iter"])

    def communicate(self):
        it = self.iter
        self.iter += 1
        if np.sum(self.topology.active_flags[it]) == 0:
            return 0
        torch.cuda.synchronize()
        tic = time.time()
        self.step(it)
        self.wait_round()
        toc = time.time()
        self.check_topk()
        return toc - tic
