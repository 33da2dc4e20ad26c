"""Drop-in per-rank communicators (communicator.py:10-268 of the reference).

    communicator = decenCommunicator(rank, size, GP)            # train_mpi.py:81
    communicator = ChocoCommunicator(rank, size, GP, 0.9, lr)   # train_mpi.py:79
    comm_time = communicator.communicate(model)                 # train_mpi.py:142

One process per worker, as under mpirun.  The reference's MPI COMM_WORLD is replaced by
torch.distributed (for bootstrap) plus an RCCL communicator owned by the native library; each
rank's model is a one-row VirtualWorkerGroup / ChocoWorkerGroup on its GPU and partner rows
travel over xGMI.  If torch.distributed is not initialised, it is initialised here from the
environment (torchrun's RANK/WORLD_SIZE/MASTER_*, or the (rank, size) given, with
MASTER_ADDR 127.0.0.1 and a MASTER_PORT derived from the launcher's job id -- rendezvous_port).

Model parameters on the GPU are re-homed into the group's arena on the first call (views, so
identity, shapes and optimizer references are kept) and mixed in place every round.  Models
left on the CPU -- the reference's train_mpi.py keeps them there -- are staged: copied to the
GPU row before and back after each round.  All arithmetic runs in the HIP kernels.
"""
import os
import time

import numpy as np
import torch

from ._lib import check, lib, require_device, stream_ptr
from .choco import ChocoWorkerGroup
from .comm_helpers import flatten_tensors, unflatten_tensors
from .engine import VirtualWorkerGroup, default_comm, wait_round


def _same_params(model, params):
    cur = list(model.parameters())
    return params is not None and len(cur) == len(params) and all(a is b for a, b in zip(cur, params))


_JOB_ID_VARS = ("PMIX_NAMESPACE", "OMPI_MCA_ess_base_jobid", "SLURM_JOB_ID", "PBS_JOBID", "LSB_JOBID")


def rendezvous_port(env=None):
    """MASTER_PORT for the bootstrap when the launcher did not set one (mpirun, as the reference
    is launched: README.md:62-65).  Derived from the launcher's job id, so every rank of one job
    agrees on it without talking and two jobs on one node do not collide; 29533 only when no job
    id is visible either."""
    env = os.environ if env is None else env
    if env.get("MASTER_PORT"):
        return int(env["MASTER_PORT"])
    for k in _JOB_ID_VARS:
        if env.get(k):
            import zlib
            return 20000 + zlib.crc32(env[k].encode()) % 30000
    return 29533


def _ensure_process_group(rank, size):
    import torch.distributed as dist
    require_device()
    if size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(rendezvous_port())
        dist.init_process_group("gloo", rank=rank, world_size=size)
    if size > 1:
        if dist.get_world_size() != size or dist.get_rank() != rank:
            raise RuntimeError(f"communicator rank/size ({rank}, {size}) do not match the process "
                               f"group ({dist.get_rank()}, {dist.get_world_size()}): one process per worker")
    if "LOCAL_RANK" in os.environ:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    elif size > 1:
        torch.cuda.set_device(rank % torch.cuda.device_count())


class _Staging:
    """Moves a model's parameters into / out of a group row.

    GPU models are adopted: every parameter's storage is a view of the group row, so a round
    mixes them in place and nothing is copied.  Host models (the reference's default) are staged:
    copied to the row before and back after each round.  adopt=False (a plain tensor list, e.g.
    the reference's `tensor_list` of `param.data` aliases, which cannot be re-homed): GPU tensors
    already at their place in the row are used in place, others are copied in and back out."""

    def __init__(self, params, row, adopt=True):
        self.params = params
        self.row = row
        self.may_adopt = adopt
        self.on_gpu = all(p.device.type == "cuda" for p in params)

    def adopted(self):
        """True while every parameter still lives at its place in the row (a caller may have
        reassigned p.data since, e.g. torch.nn.utils.vector_to_parameters or model.cpu())."""
        base, off = self.row.data_ptr(), 0
        for p in self.params:
            if p.data.data_ptr() != base + 4 * off and p.numel():
                return False
            off += p.numel()
        return True

    def adopt(self):
        """(Re-)home the parameters' current values into the row as views (identity kept)."""
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                view = self.row[off:off + k].view(p.shape)
                if p.data.data_ptr() != view.data_ptr():
                    view.copy_(p.data)
                    p.data = view
                off += k

    PIECE_FLOATS = 4 << 20        # staging pieces of 16 MB: the host copy of one piece overlaps
                                  # the DMA of its neighbour (both directions)

    def _pinned(self):
        n = self.row.numel()
        if getattr(self, "_pin", None) is None or self._pin.numel() != n:
            self._pin = torch.empty(n, dtype=torch.float32, pin_memory=True)
        return self._pin

    def _plan(self):
        """Pieces [a, b) of the flat row and, per piece, the parameter slices it holds:
        (param index, first, end within the parameter, offset in the row).  Non-contiguous
        parameters are copied whole, outside the pieces."""
        key = (self.PIECE_FLOATS, tuple(p.numel() for p in self.params))
        if getattr(self, "_plan_key", None) != key:
            offs = np.cumsum([0] + [p.numel() for p in self.params])
            n, step = int(offs[-1]), max(1, int(self.PIECE_FLOATS))
            pieces, i = [], 0
            for a in range(0, n, step):
                b = min(n, a + step)
                while i < len(self.params) and offs[i + 1] <= a:
                    i += 1
                parts, j = [], i
                while j < len(self.params) and offs[j] < b:
                    lo, hi = max(a, int(offs[j])), min(b, int(offs[j + 1]))
                    if hi > lo:
                        parts.append((j, lo - int(offs[j]), hi - int(offs[j]), lo))
                    j += 1
                pieces.append((a, b, parts))
            self._plan_key, self._plan_pieces, self._offs = key, pieces, offs
        return self._plan_pieces

    def load(self):
        if self.on_gpu:
            if not self.adopted():
                self.on_gpu = all(p.device.type == "cuda" for p in self.params)
                if self.on_gpu:
                    if self.may_adopt:
                        self.adopt()
                    else:
                        self._copy_in()
            if self.on_gpu:
                return
        # host model: flatten (comm_helpers.py:27-30's torch.cat) into a pinned staging buffer piece
        # by piece, each piece's DMA to the row issued as soon as it is filled
        pin = self._pinned()
        for a, b, parts in self._plan():
            for i, lo, hi, d in parts:
                t = self.params[i].data
                src = t.reshape(-1)[lo:hi] if t.is_contiguous() else t.contiguous().reshape(-1)[lo:hi]
                pin[d:d + hi - lo].copy_(src)
            self.row[a:b].copy_(pin[a:b], non_blocking=True)

    def _copy_in(self):
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.row[off:off + k].view(p.shape).copy_(p.data)
                off += k

    def store(self):
        if self.on_gpu:
            if not self.may_adopt and not self.adopted():
                off = 0
                with torch.no_grad():
                    for p in self.params:
                        k = p.numel()
                        p.data.copy_(self.row[off:off + k].view(p.shape))
                        off += k
            return
        # every piece's DMA back is queued at once; piece i is scattered into the parameters while
        # the later pieces are still in flight
        pin = self._pinned()
        pieces = self._plan()
        events = []
        for a, b, _ in pieces:
            pin[a:b].copy_(self.row[a:b], non_blocking=True)
            e = torch.cuda.Event()
            e.record()
            events.append(e)
        later = set()
        with torch.no_grad():
            for (a, b, parts), e in zip(pieces, events):
                e.synchronize()
                for i, lo, hi, d in parts:
                    t = self.params[i].data
                    if t.is_contiguous():
                        t.reshape(-1)[lo:hi].copy_(pin[d:d + hi - lo])
                    else:
                        later.add(i)
            for i in sorted(later):                 # non-contiguous: whole-tensor copy_ (view_as)
                t = self.params[i].data
                o = int(self._offs[i])
                t.copy_(pin[o:o + t.numel()].view_as(t))


def _refuse_pull(transport, who):
    """The pull transport serves gossip rounds (decenCommunicator / ChocoCommunicator): the
    centralized all-gather needs a transport that moves buffers."""
    from .engine import PullTransport
    if isinstance(transport, PullTransport):
        raise TypeError(f"{who}: PullTransport carries gossip rounds only (decenCommunicator / "
                        "ChocoCommunicator); use the RCCL transport (transport=None)")


class Communicator(object):
    """communicator.py:10-43 -- communicate(model) -> seconds spent averaging.

    `transport` (keyword-only extension, default None = the process-wide RCCL communicator
    bootstrapped over torch.distributed) may be any object GossipEngine accepts as its comm."""

    def __init__(self, rank, size, *, transport=None):
        self.comm = None
        self.rank = rank
        self.size = size
        self._transport = transport
        if transport is None:
            _ensure_process_group(rank, size)
        else:
            require_device()

    def _comm(self):
        if self.size <= 1:
            return None
        return self._transport if self._transport is not None else default_comm()

    def communicate(self, model):
        raise NotImplementedError


class decenCommunicator(Communicator):
    """communicator.py:79-158 -- decentralized averaging according to the topology's schedule."""

    def __init__(self, rank, size, topology, *, transport=None, idle_rows="skip"):
        """idle_rows="canonical": a round in which this worker has no active partner rewrites its
        parameters as 0 + 1.0 * x, as the reference does (-0.0 -> +0.0); "skip" leaves them."""
        super(decenCommunicator, self).__init__(rank, size, transport=transport)
        self.idle_rows = idle_rows
        self.topology = topology
        self.neighbor_weight = topology.neighbor_weight
        self.iter = 0
        self._group = None
        self._stage = None
        self._model_params = None

    def _bind(self, model):
        params = [p for p in model.parameters()]
        n = int(sum(p.numel() for p in params))
        if self._group is not None and self._group.numel == n:
            # same size (e.g. parameters re-created): adopt the new tensors into the same row
            self._stage = _Staging(params, self._group.rows[0])
        else:
            # a new parameter count: a new row.  The old group's transport buffers are released
            # first (under PullTransport this re-bind is collective: every rank must re-bind in the
            # same call, as every rank's model changes size together in data-parallel training)
            self.close()
            on_gpu = all(p.device.type == "cuda" for p in params)
            self._group = VirtualWorkerGroup(self.topology, [model] if on_gpu else None,
                                             numel=None if on_gpu else n, rank=self.rank,
                                             nranks=self.size, comm=self._comm(), idle_rows=self.idle_rows)
            self._stage = _Staging(params, self._group.rows[0])
        self._model_params = params

    def close(self):
        """Release the worker group (and the pull transport's shared buffers, if any)."""
        if self._group is not None:
            self._group.close()
            self._group = None
            self._stage = None
            self._model_params = None

    def __del__(self):
        # a pull group's close() is collective (a barrier): never from a finalizer -- its IPC
        # buffers go with the process
        try:
            if self._group is not None and not self._group.pulls:
                self.close()
        except Exception:                        # interpreter teardown: nothing left to release
            pass

    def communicate(self, model):
        """communicator.py:133-158: the three steps below fused, with the model's parameters
        adopted into the arena row on the first call (no flatten / unflatten afterwards)."""
        active_flags = self.topology.active_flags[self.iter]
        it = self.iter
        self.iter += 1
        if np.sum(active_flags) == 0:            # communicator.py:140-141
            return 0
        if self._group is None or not _same_params(model, self._model_params):
            self._bind(model)
        self._stage.load()
        torch.cuda.synchronize()
        tic = time.time()
        self._group.step(it)
        self._group.wait_round()
        toc = time.time()
        self._stage.store()
        return toc - tic

    # ---- the reference's sub-steps (communicator.py:87-131), for callers that drive them directly
    def _bind_list(self, tensors, make_group):
        n = int(sum(t.numel() for t in tensors))
        if self._group is None or self._group.numel != n:
            self.close()
            self._group = make_group(n)
            self._model_params = None
            self._stage = None
        self._list_stage = _Staging(tensors, self._group.rows[0], adopt=False)
        self._list_stage.load()
        return self._group.rows[0]

    def _round_of(self, active_flags):
        """The plan record of `active_flags`: the schedule's row of the current iteration when they
        are that row (the reference's communicate() passes exactly it), else any record already
        built for the same row (engine.record_for), else a scratch record."""
        eng = self._group.engine
        f = eng.flags_row(active_flags)
        i = self.iter - 1
        if 0 <= i < eng.T and np.array_equal(f, eng.flags_host[i]):
            return i
        return eng.record_for(f)

    def prepare_comm_buffer(self):
        """communicator.py:87-90.  `self.tensor_list` (set by the caller, as the reference's
        communicate() does) is copied into this rank's arena row -- or used in place when it
        already lives there (parameters adopted by an earlier communicate(model)) -- and
        `send_buffer` is that row (flat, on the GPU).  The reference's zero `recv_buffer` has no
        counterpart: the kernel accumulates in registers and writes the row in place, so after
        averaging() `recv_buffer` names the same row."""
        self.send_buffer = self._bind_list(list(self.tensor_list), lambda n: VirtualWorkerGroup(
            self.topology, None, numel=n, rank=self.rank, nranks=self.size, comm=self._comm(),
            idle_rows=self.idle_rows))
        self.recv_buffer = None

    def averaging(self, active_flags):
        """communicator.py:92-122: one gossip round of send_buffer under `active_flags` (any row;
        every rank passes the same one, as the reference's sendrecv pairs require); seconds."""
        it = self._round_of(active_flags)
        torch.cuda.synchronize()
        tic = time.time()
        self._group.step(it)
        self._group.wait_round()
        toc = time.time()
        self.recv_buffer = self.send_buffer
        return toc - tic

    def reset_model(self):
        """communicator.py:124-131: the averaged row back into tensor_list (nothing to do for
        tensors that live in the row)."""
        self._list_stage.store()


class ChocoCommunicator(Communicator):
    """communicator.py:161-268 -- top-k compressed gossip with persistent x_hat / s."""

    def __init__(self, rank, size, topology, ratio, consensus_lr, *, transport=None):
        super(ChocoCommunicator, self).__init__(rank, size, transport=transport)
        self.topology = topology
        self.neighbor_weight = topology.neighbor_weight
        self.iter = 0
        self.initialized = False
        self.consensus_lr = consensus_lr
        self.ratio = ratio
        self._group = None
        self._stage = None

    @property
    def x_hat(self):
        return self._group.x_hat[0, :self._group.numel] if self._group is not None else None

    @property
    def s(self):
        return self._group.s[0, :self._group.numel] if self._group is not None else None

    def _bind(self, model):
        params = [p for p in model.parameters()]
        n = int(sum(p.numel() for p in params))
        if self._group is not None:
            # x_hat / s persist for the communicator's life (communicator.py:179-182): new parameter
            # tensors of the same size are adopted into the same row, keeping the Choco state
            if self._group.numel != n:
                raise ValueError(f"ChocoCommunicator: the model now has {n} parameters, its x_hat / s "
                                 f"hold {self._group.numel}")
            self._stage = _Staging(params, self._group.rows[0])
        else:
            on_gpu = all(p.device.type == "cuda" for p in params)
            self._group = ChocoWorkerGroup(self.topology, [model] if on_gpu else None,
                                           numel=None if on_gpu else n, ratio=self.ratio,
                                           consensus_lr=self.consensus_lr, rank=self.rank,
                                           nranks=self.size, comm=self._comm())
            self._stage = _Staging(params, self._group.rows[0])
        self._model_params = params
        self.initialized = True

    def communicate(self, model):
        """communicator.py:242-268: the three steps below fused (compression + averaging timed
        together: the reference's encode_time + comm_time), parameters adopted into the arena."""
        active_flags = self.topology.active_flags[self.iter]
        it = self.iter
        self.iter += 1
        if np.sum(active_flags) == 0:            # communicator.py:249-250
            return 0
        if self._group is None or not _same_params(model, self._model_params):
            self._bind(model)
        self._stage.load()
        torch.cuda.synchronize()
        tic = time.time()
        self._group.step(it)
        self._group.wait_round()
        toc = time.time()
        self._group.check_topk()
        self._stage.store()
        return toc - tic

    # ---- the reference's sub-steps (communicator.py:175-240), for callers that drive them directly
    _bind_list = decenCommunicator._bind_list
    _round_of = decenCommunicator._round_of

    def prepare_comm_buffer(self):
        """communicator.py:175-196: `self.tensor_list` into this rank's x row (copied, or used in
        place when it lives there), x_hat / s created zero on first use (they persist), then the
        top-k of x - x_hat; `compressed` = {"values", "indices"} views of the message (GPU,
        index-sorted).  Returns the compression seconds (the reference's encode time)."""
        tensors = list(self.tensor_list)
        n = int(sum(t.numel() for t in tensors))
        if self._group is not None and self._group.numel != n:
            raise ValueError(f"ChocoCommunicator: tensor_list holds {n} values, its x_hat / s hold {self._group.numel}")
        self.x = self._bind_list(tensors, lambda n: ChocoWorkerGroup(
            self.topology, None, numel=n, ratio=self.ratio, consensus_lr=self.consensus_lr, rank=self.rank,
            nranks=self.size, comm=self._comm()))
        self.initialized = True
        torch.cuda.synchronize()
        tic = time.time()
        self._group.compress(self.iter)
        self._group.check_topk()
        toc = time.time()
        vals, idx = self._group.message(0)
        self.compressed = {"values": vals, "indices": idx}
        return toc - tic

    def averaging(self, active_flags):
        """communicator.py:200-230: partner messages under `active_flags` (any row; every rank the
        same), s / x_hat scatters and x += consensus_lr (s - x_hat), in place; seconds."""
        it = self._round_of(active_flags)
        torch.cuda.synchronize()
        tic = time.time()
        self._group.average(it)
        self._group.wait_round()
        toc = time.time()
        return toc - tic

    def reset_model(self):
        """communicator.py:233-240: x back into tensor_list (nothing to do for tensors in the row)."""
        self._list_stage.store()

    def close(self):
        """Release the worker group (collective under PullTransport, as decenCommunicator.close)."""
        if self._group is not None:
            self._group.close()
        self._group = None
        self._stage = None
        self._model_params = None

    def __del__(self):
        try:
            if self._group is not None and not self._group.pulls:
                self.close()
        except Exception:                        # interpreter teardown: nothing left to release
            pass


ORDERS = {"tree": 0, "sequential": 1}


class centralizedCommunicator(Communicator):
    """communicator.py:46-76 -- all-reduce averaging: x = allreduce_sum(x) / size.

    order -- how the ranks' vectors are summed:
      "tree" (default): the order of the reference's comm.allreduce(obj, op=MPI.SUM) under
          mpi4py's default object reduction (a binomial tree to rank 0, then a broadcast), as
          restated from mpi4py's published algorithm (tests/reforder.py; mpi4py is not installed
          here, so parity against mpi4py itself is unpinned): every vector is all-gathered over
          RCCL and each rank sums them in that order on its GPU (mx_allreduce_mean_ordered /
          mx_mean_rows, any world size) before the division of communicator.py:62;
      "sequential": the same with a rank-order left fold (mpi4py with rc.fast_reduce off);
      "ring": RCCL's own all-reduce + division (mx_allreduce_mean) -- less traffic and memory per
          rank, equal to the reference within fp32 reassociation only.
    Memory: "tree" / "sequential" keep a gather buffer of size x P floats per rank (the all-gather
    target; e.g. 8 ranks x 25.6M params = 819 MB), "ring" none."""

    def __init__(self, rank, size, *, transport=None, order="tree"):
        _refuse_pull(transport, "centralizedCommunicator")
        super(centralizedCommunicator, self).__init__(rank, size, transport=transport)
        if order not in ORDERS and order != "ring":
            raise ValueError(f"order must be 'tree', 'sequential' or 'ring', not {order!r}")
        self.order = order
        self._gather = None

    def _gather_buf(self, count, device):
        if self._gather is None or self._gather.numel() < self.size * count or self._gather.device != device:
            self._gather = torch.empty(self.size * count, dtype=torch.float32, device=device)
        return self._gather

    def _average(self, flat):
        comm = self._comm()
        count = flat.numel()
        if self.order == "ring":
            if hasattr(comm, "allreduce_mean"):
                comm.allreduce_mean(flat, self.size)
            else:
                check(lib.mx_allreduce_mean(comm.handle, flat.data_ptr(), count, self.size, stream_ptr()),
                      "mx_allreduce_mean")
            return
        gather = self._gather_buf(count, flat.device)
        if hasattr(comm, "allgather"):          # a test transport: gathers, then the same kernel
            comm.allgather(flat, gather[:self.size * count])
            check(lib.mx_mean_rows(gather.data_ptr(), self.size, count, count, ORDERS[self.order],
                                   flat.data_ptr(), stream_ptr()), "mx_mean_rows")
        else:
            check(lib.mx_allreduce_mean_ordered(comm.handle, flat.data_ptr(), count, gather.data_ptr(),
                                                ORDERS[self.order], stream_ptr()), "mx_allreduce_mean_ordered")

    def prepare_comm_buffer(self):
        """communicator.py:52-54: `send_buffer` = the flattened tensor_list (on the GPU)."""
        tensors = list(self.tensor_list)
        on_gpu = all(t.device.type == "cuda" for t in tensors)
        self.send_buffer = flatten_tensors([t if on_gpu else t.cuda() for t in tensors])

    def averaging(self):
        """communicator.py:56-67: the all-reduce mean of send_buffer, in place (recv_buffer names
        it); seconds."""
        torch.cuda.synchronize()
        tic = time.time()
        if self.size > 1 and self.send_buffer.numel():
            self._average(self.send_buffer)
        wait_round(self._comm())
        toc = time.time()
        self.recv_buffer = self.send_buffer
        return toc - tic

    def reset_model(self):
        """communicator.py:69-76: the averaged vector back into tensor_list."""
        with torch.no_grad():
            for f, t in zip(unflatten_tensors(self.recv_buffer, self.tensor_list), self.tensor_list):
                t.copy_(f)

    def communicate(self, model):
        """communicator.py:18-33 (the base class's sequence)."""
        self.tensor_list = [p.data for p in model.parameters()]
        self.prepare_comm_buffer()
        comm_time = self.averaging()
        self.reset_model()
        return comm_time
