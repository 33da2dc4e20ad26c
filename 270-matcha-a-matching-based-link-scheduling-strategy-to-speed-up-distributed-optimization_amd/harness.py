"""GPU training harness around the gossip hot path: train_mpi.py:34-201 with synthetic batches.

The reference's run(rank, size) (train_mpi.py:58-168) trains one model per MPI rank on the CPU
and calls communicator.communicate(model) after every optimizer step.  This harness keeps that
loop -- forward, loss, accuracy bookkeeping, backward, update_learning_rate, SGD step,
zero_grad, communicate -- with two layouts:

  * VirtualTrainer (one process, one GPU): all `size` workers' models live on the GPU and
    their parameters are re-homed into ONE VirtualWorkerGroup / ChocoWorkerGroup arena, so each
    batch runs `size` forward/backward/step sequences and then a single gossip launch for all
    workers (the "8 virtual workers on one MI355X" mode of BASELINE configs 1-2);
  * RankTrainer (torchrun, one process per worker): the drop-in decenCommunicator /
    ChocoCommunicator on this rank's model, exactly the reference's per-rank call pattern.

Data is synthetic (no dataset download on the GPU box): per worker a fixed seeded stream of
MNIST-shaped (1x28x28) or CIFAR-shaped batches with random labels.  The Recorder writes the
reference's seven per-rank logs (util.py:378-419); checkpoints hold the worker rows, the
Choco state (x_hat, s) and the iteration counter so a run resumes on the same schedule.
"""
import os
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ._lib import check, lib, stream_ptr
from .choco import ChocoWorkerGroup
from .engine import VirtualWorkerGroup
from .graph_manager import FixedProcessor, MatchaProcessor
from .topologies import select_graph


# ----------------------------------------------------------------------------- model / meters
class MNIST_MLP(nn.Module):
    """models/MLP.py:5-25: 784 -> 500 -> 500 -> num_classes, ReLU, weights in self.layers."""

    def __init__(self, num_classes):
        super(MNIST_MLP, self).__init__()
        self.layers = nn.ModuleList([nn.Linear(28 * 28, 500), nn.Linear(500, 500), nn.Linear(500, num_classes)])

    def forward(self, x):
        x = x.view(-1, 28 * 28)
        x = F.relu(self.layers[0](x))
        x = F.relu(self.layers[1](x))
        return self.layers[2](x)


def comp_accuracy(output, target, topk=(1,)):
    """util.py:342-356 -- top-k accuracy in percent."""
    with torch.no_grad():
        maxk = max(topk)
        batch_size = target.size(0)
        _, pred = output.topk(maxk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.view(1, -1).expand_as(pred))
        return [correct[:k].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / batch_size) for k in topk]


class AverageMeter(object):
    """util.py:358-373."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class Recorder(object):
    """util.py:376-419 -- per-rank timing / accuracy logs, same folder and file names."""

    def __init__(self, args, rank):
        self.record_accuracy = []
        self.record_timing = []
        self.record_comp_timing = []
        self.record_comm_timing = []
        self.record_losses = []
        self.record_trainacc = []
        self.total_record_timing = []
        self.args = args
        self.rank = rank
        self.saveFolderName = args.savePath + args.name + '_' + args.model
        if rank == 0 and not os.path.isdir(self.saveFolderName) and self.args.save:
            os.makedirs(self.saveFolderName, exist_ok=True)

    def add_new(self, record_time, comp_time, comm_time, epoch_time, top1, losses, test_acc):
        self.total_record_timing.append(record_time)
        self.record_timing.append(epoch_time)
        self.record_comp_timing.append(comp_time)
        self.record_comm_timing.append(comm_time)
        self.record_trainacc.append(top1)
        self.record_losses.append(losses)
        self.record_accuracy.append(test_acc)

    def log_path(self, suffix):
        return (self.saveFolderName + '/dsgd-lr' + str(self.args.lr) + '-budget' + str(self.args.budget) +
                '-r' + str(self.rank) + '-' + suffix + '.log')

    def save_to_file(self):
        for suffix, data in (("recordtime", self.total_record_timing), ("time", self.record_timing),
                             ("comptime", self.record_comp_timing), ("commtime", self.record_comm_timing),
                             ("acc", self.record_accuracy), ("losses", self.record_losses),
                             ("tacc", self.record_trainacc)):
            np.savetxt(self.log_path(suffix), np.asarray(data, dtype=np.float64), delimiter=',')
        with open(self.saveFolderName + '/ExpDescription', 'w') as f:
            f.write(str(self.args) + '\n')
            f.write(self.args.description + '\n')


def update_learning_rate(optimizer, epoch, args, itr=None, itr_per_epoch=None):
    """train_mpi.py:171-201: linear warmup from 0.1 over 5 epochs when lr > 0.1, then x0.1 at
    epochs 100 and 150."""
    base_lr = 0.1
    target_lr = args.lr
    lr_schedule = [100, 150]
    if args.warmup and epoch < 5:
        if target_lr <= base_lr:
            lr = target_lr
        else:
            count = epoch * itr_per_epoch + itr + 1
            lr = base_lr + (target_lr - base_lr) * (count / (5 * itr_per_epoch))
    else:
        lr = target_lr
        for e in lr_schedule:
            if epoch >= e:
                lr *= 0.1
    for group in optimizer.param_groups:
        group['lr'] = lr
    return lr


# ----------------------------------------------------------------------------- synthetic data
def synthetic_batches(worker, n_batches, bs, shape=(1, 28, 28), num_classes=100, seed=1234, device="cuda"):
    """A fixed stream of (data, target) batches for one worker (the partition_dataset stand-in:
    util.py:115-254 downloads datasets, which the GPU box cannot)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed * 1000 + worker)
    out = []
    for _ in range(n_batches):
        data = torch.randn((bs,) + tuple(shape), generator=g)
        target = torch.randint(0, num_classes, (bs,), generator=g)
        out.append((data.to(device), target.to(device)))
    return out


# ----------------------------------------------------------------------------- harness
def make_topology(args, rank, size, iterations):
    """train_mpi.py:69-75 (MatchaProcessor when args.matcha, else FixedProcessor)."""
    subGraphs = select_graph(args.graphid)
    if args.matcha:
        return MatchaProcessor(subGraphs, args.budget, rank, size, iterations, False)
    return FixedProcessor(subGraphs, args.budget, rank, size, iterations, True)


def sync_rows(rows, order=0):
    """sync_allreduce (train_mpi.py:34-56) for workers held as rows of one arena: every row
    becomes (sum over workers) / size -- mx_mean_rows, the same kernel and summation order
    (order 0: mpi4py's binomial tree, 1: rank order) as centralizedCommunicator's per-rank path.
    (The reference's buffer Allreduce sums in the MPI library's own order; either order is within
    fp32 reassociation of it.)"""
    n, count = rows.shape
    if n == 1 or count == 0:
        return
    if rows.stride(1) != 1:
        raise ValueError("sync_rows: rows must be contiguous along the parameter axis")
    # one pass: every column of every row read, then the mean written to that column of every row
    check(lib.mx_mean_rows_to(rows.data_ptr(), n, rows.stride(0), count, int(order), rows.data_ptr(), n,
                              rows.stride(0), stream_ptr()), "mx_mean_rows_to")


class VirtualTrainer:
    """All workers of the topology on this GPU; one gossip launch per batch for all of them.

    batched=False: each worker runs its own forward / backward / torch.optim.SGD step, exactly
    train_mpi.py's per-rank sequence.  batched=True: the workers' parameters are addressed as
    stacked [n, ...] views of the worker arena, one vmap'd forward / backward computes every
    worker's gradients (torch.func), and the SGD update (weight decay, momentum, Nesterov; the
    element-wise op sequence of torch.optim.SGD) runs once over the stacked views -- a training
    step for all workers is a handful of batched launches plus the gossip kernel."""

    def __init__(self, args, model_fn, n_batches, device="cuda", batched=False, graph=False):
        """graph=True (with batched=True, decentralized gossip, one GPU): once the learning rate
        is constant within an epoch, the whole training iteration -- vmap'd forward / backward,
        SGD update and the gossip round at a device-side iteration counter (device_round) -- is
        captured once per learning rate in a HIP graph and replayed, so an iteration costs one
        graph launch plus the batch copies instead of dozens of host launches.  Results are
        identical to batched=True (same kernels, same order)."""
        self.args = args
        size = args.size
        np.random.seed(args.randomSeed)                          # train_mpi.py:62
        torch.manual_seed(args.randomSeed)
        self.GP = make_topology(args, 0, size, args.epoch * n_batches)
        self.models = []
        for r in range(size):
            torch.manual_seed(args.randomSeed + r)                # train_mpi.py:61, per rank
            self.models.append(model_fn().to(device))
        if args.compress:
            self.group = ChocoWorkerGroup(self.GP, self.models, ratio=args.ratio,
                                          consensus_lr=args.consensus_lr)
        else:
            self.group = VirtualWorkerGroup(self.GP, self.models)
        sync_rows(self.group.rows)
        self.optimizers = [torch.optim.SGD(m.parameters(), lr=args.lr, momentum=args.momentum,
                                           weight_decay=5e-4, nesterov=args.nesterov, dampening=0)
                           for m in self.models]
        self.criterion = nn.CrossEntropyLoss()
        self.data = [synthetic_batches(r, n_batches, args.bs, args.shape, args.num_classes, args.randomSeed,
                                       device) for r in range(size)]
        self.n_batches = n_batches
        self.recorders = [Recorder(args, r) for r in range(size)] if args.save else None
        self.epoch = 0
        self.batched = bool(batched)
        self.graph = bool(graph)
        if self.graph and not self.batched:
            raise ValueError("graph mode needs batched=True")
        self._graphs = {}
        self._dev_iter_synced = False
        if self.batched:
            self._setup_batched()

    def communicate(self):
        return self.group.communicate()

    # ------------------------------------------------------------------ batched workers
    def _setup_batched(self):
        from torch.func import functional_call, grad_and_value, vmap
        m0 = self.models[0]
        rows = self.group.rows
        n = rows.shape[0]
        self._stack = {}
        self._stack_off = []
        off = 0
        for name, p in m0.named_parameters():          # the arena's adoption order
            k = p.numel()
            self._stack[name] = rows[:, off:off + k].view((n,) + tuple(p.shape))
            self._stack_off.append(off)
            off += k
        self._mom = {}

        def loss_fn(params, x, y):
            out = functional_call(m0, params, (x,))
            return F.cross_entropy(out, y), out

        self._grad_fn = vmap(grad_and_value(loss_fn, has_aux=True))
        self._data_stacked = [(torch.stack([self.data[r][b][0] for r in range(n)]),
                               torch.stack([self.data[r][b][1] for r in range(n)]))
                              for b in range(self.n_batches)]

    def _batched_step(self, b, lr):
        """Every worker's forward / backward / SGD step for batch b; per-worker (loss, acc)."""
        X, Y = self._data_stacked[b]
        return self._batched_update(X, Y, lr)

    def _batched_update(self, X, Y, lr):
        args = self.args
        grads, (loss, out) = self._grad_fn(self._stack, X, Y)
        wd, mom = 5e-4, args.momentum
        with torch.no_grad():
            for name, p in self._stack.items():         # torch.optim.SGD's element-wise sequence
                d_p = grads[name].add(p, alpha=wd)
                if mom != 0:
                    buf = self._mom.get(name)
                    if buf is None:
                        buf = self._mom[name] = d_p.clone()
                    else:
                        buf.mul_(mom).add_(d_p)
                    d_p = d_p.add(buf, alpha=mom) if args.nesterov else buf
                p.add_(d_p, alpha=-lr)
            acc = (out.argmax(-1) == Y).float().mean(-1) * 100.0
        return loss.detach(), acc

    # ------------------------------------------------------------------ HIP-graph iterations
    def _lr_stable(self, epoch):
        """update_learning_rate's value is constant within this epoch (no per-iteration warmup)"""
        return not (self.args.warmup and epoch < 5 and self.args.lr > 0.1)

    def _graph_for(self, lr):
        """(graph, loss, acc) of one whole iteration at learning rate lr, captured on first use:
        forward / backward / SGD on the static batch buffers, then the gossip round at the device
        counter.  Capturing runs nothing."""
        hit = self._graphs.get(lr)
        if hit is not None:
            return hit
        if not hasattr(self, "_Xs"):
            X0, Y0 = self._data_stacked[0]
            self._Xs, self._Ys = X0.clone(), Y0.clone()      # valid labels: the warm-up runs on them
            self._cap_stream = torch.cuda.Stream()
        # warm the BLAS libraries for these GEMM shapes on the capture stream first (they set up
        # handles / workspaces / heuristics lazily, which a capturing stream does not permit),
        # on a scratch copy of the arena laid out like the live one: no worker state changes
        cs = self._cap_stream
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            base = self.group.x if hasattr(self.group, "x_hat") else self.group.arena
            scratch = base.clone()
            n = scratch.shape[0]
            views = {name: scratch[:, off:off + v.shape[1:].numel()].view(v.shape)
                     for (name, v), off in zip(self._stack.items(), self._stack_off)}
            self._grad_fn(views, self._Xs, self._Ys)
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        del scratch, views
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            loss, acc = self._batched_update(self._Xs, self._Ys, lr)
            self.group.device_round()
        self._graphs[lr] = (g, loss, acc)
        return self._graphs[lr]

    def _graph_iteration(self, b, lr):
        """One training iteration + gossip round by graph replay; (loss, acc) device tensors."""
        g, loss, acc = self._graph_for(lr)
        X, Y = self._data_stacked[b]
        self._Xs.copy_(X)
        self._Ys.copy_(Y)
        if not self._dev_iter_synced:
            self.group.iter_dev.fill_(self.group.iter)
            self._dev_iter_synced = True
        g.replay()
        self.group.iter += 1
        return loss, acc

    def train_epoch(self, on_round=None):
        """One epoch of train_mpi.py:109-168 for every worker; returns per-worker stats."""
        args = self.args
        size = len(self.models)
        epoch = self.epoch
        comp = [0.0] * size
        comm_time = 0.0
        losses = [AverageMeter() for _ in range(size)]
        top1 = [AverageMeter() for _ in range(size)]
        tic = time.time()
        for m in self.models:
            m.train()
        use_graph = self.graph and self._lr_stable(epoch) and (self.args.momentum == 0 or self._mom)
        if use_graph:
            if on_round is not None:
                raise ValueError("graph mode runs the step and the gossip round as one replay: no round hooks")
            t0 = time.time()
            stat = torch.empty((self.n_batches, 2, size), dtype=torch.float32, device="cuda")
            for b in range(self.n_batches):
                lr = update_learning_rate(self.optimizers[0], epoch, args, itr=b, itr_per_epoch=self.n_batches)
                loss_b, acc_b = self._graph_iteration(b, lr)
                stat[b, 0].copy_(loss_b)
                stat[b, 1].copy_(acc_b)
            st = stat.cpu().numpy()                            # one host sync per epoch
            dt = (time.time() - t0) / size
            bs = self._data_stacked[0][1].shape[1]
            for b in range(self.n_batches):
                for r in range(size):
                    losses[r].update(float(st[b, 0, r]), bs)
                    top1[r].update(float(st[b, 1, r]), bs)
            for r in range(size):
                comp[r] += dt                                  # gossip included (one replay per iteration)
        for b in range(0 if not use_graph else self.n_batches, self.n_batches):
            if self.batched:
                t0 = time.time()
                lr = update_learning_rate(self.optimizers[0], epoch, args, itr=b, itr_per_epoch=self.n_batches)
                loss_b, acc_b = self._batched_step(b, lr)
                lb, ab = loss_b.cpu().tolist(), acc_b.cpu().tolist()
                bs = self._data_stacked[b][1].shape[1]
                dt = (time.time() - t0) / size
                for r in range(size):
                    losses[r].update(lb[r], bs)
                    top1[r].update(ab[r], bs)
                    comp[r] += dt
            else:
                for r, (m, opt) in enumerate(zip(self.models, self.optimizers)):
                    t0 = time.time()
                    data, target = self.data[r][b]
                    output = m(data)
                    loss = self.criterion(output, target)
                    acc1 = comp_accuracy(output, target)
                    losses[r].update(loss.item(), data.size(0))
                    top1[r].update(acc1[0].item(), data.size(0))
                    loss.backward()
                    update_learning_rate(opt, epoch, args, itr=b, itr_per_epoch=self.n_batches)
                    opt.step()
                    opt.zero_grad()
                    comp[r] += time.time() - t0
            if on_round is not None:
                on_round("before", self)
            comm_time += self.communicate()                  # train_mpi.py:142, all workers at once
            self._dev_iter_synced = False
            if on_round is not None:
                on_round("after", self)
        record_time = time.time() - tic
        stats = []
        for r in range(size):
            test_acc = top1[r].avg             # no test split in the synthetic stream
            stats.append({"worker": r, "loss": losses[r].avg, "train_acc": top1[r].avg,
                          "comp_time": comp[r], "comm_time": comm_time})
            if self.recorders is not None:
                self.recorders[r].add_new(record_time, comp[r], comm_time, comp[r] + comm_time, top1[r].avg,
                                          losses[r].avg, test_acc)
                if epoch % 10 == 0:
                    self.recorders[r].save_to_file()
        self.epoch += 1
        return stats

    def finish(self):
        if self.recorders is not None:
            for rec in self.recorders:
                rec.save_to_file()

    # checkpoint / resume: worker rows, Choco state, iteration and epoch counters, optimizers
    def state_dict(self):
        out = {"group": self.group.state_dict(), "epoch": self.epoch,
               "optimizers": [o.state_dict() for o in self.optimizers]}
        if self.batched:
            out["momentum"] = {k: v.detach().clone() for k, v in self._mom.items()}
        return out

    def load_state_dict(self, state):
        self.group.load_state_dict(state["group"])
        self.epoch = int(state["epoch"])
        for o, s in zip(self.optimizers, state["optimizers"]):
            o.load_state_dict(s)
        if self.batched:
            loaded = state.get("momentum", {})
            if set(loaded) == set(self._mom) and all(self._mom[k].shape == v.shape for k, v in loaded.items()):
                # captured graphs update these buffers at their captured addresses: load in place
                with torch.no_grad():
                    for k, v in loaded.items():
                        self._mom[k].copy_(v)
            else:
                self._mom = {k: v.clone() for k, v in loaded.items()}
                self._graphs = {}            # captured against the old buffers: recapture on next use
        # the device-side round counter of graph replays restarts from the loaded host counter
        self._dev_iter_synced = False

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        self.load_state_dict(torch.load(path, map_location="cuda", weights_only=True))


class RankTrainer:
    """One worker per process (torchrun): train_mpi.py's run(rank, size) with the drop-in
    communicators -- sync through RCCL all-reduce, then per batch step + communicate(model)."""

    def __init__(self, args, model_fn, n_batches, rank, size, transport=None, device="cuda",
                 sync_transport="same"):
        """transport: the communicators' (None = RCCL; "pull" = a PullTransport over the default
        process group, which the gossip rounds use while the initial sync_allreduce stays on RCCL,
        as the pull transport carries gossip rounds only).  sync_transport: the sync_allreduce's
        ("same": `transport`, or RCCL when that is the pull transport)."""
        from .communicator import ChocoCommunicator, _ensure_process_group, centralizedCommunicator, decenCommunicator
        from .engine import PullTransport
        if isinstance(transport, str):
            if transport != "pull":
                raise ValueError(f"transport {transport!r}: None, 'pull' or a transport object")
            _ensure_process_group(rank, size)
            transport = PullTransport()
        if isinstance(sync_transport, str) and sync_transport == "same":
            sync_transport = None if isinstance(transport, PullTransport) else transport
        self.args = args
        self.rank, self.size = rank, size
        torch.manual_seed(args.randomSeed + rank)                # train_mpi.py:61
        np.random.seed(args.randomSeed)                          # train_mpi.py:62
        self.GP = make_topology(args, rank, size, args.epoch * n_batches)
        if args.compress:
            self.communicator = ChocoCommunicator(rank, size, self.GP, args.ratio, args.consensus_lr,
                                                  transport=transport)
        else:
            self.communicator = decenCommunicator(rank, size, self.GP, transport=transport)
        self.model = model_fn().to(device)
        self.optimizer = torch.optim.SGD(self.model.parameters(), lr=args.lr, momentum=args.momentum,
                                         weight_decay=5e-4, nesterov=args.nesterov, dampening=0)
        self.criterion = nn.CrossEntropyLoss()
        centralizedCommunicator(rank, size, transport=sync_transport).communicate(self.model)   # sync_allreduce
        self.data = synthetic_batches(rank, n_batches, args.bs, args.shape, args.num_classes, args.randomSeed,
                                      device)
        self.n_batches = n_batches
        self.recorder = Recorder(args, rank) if args.save else None
        self.epoch = 0

    def train_epoch(self):
        args = self.args
        comp_time = comm_time = 0.0
        losses, top1 = AverageMeter(), AverageMeter()
        tic = time.time()
        self.model.train()
        for b, (data, target) in enumerate(self.data):
            t0 = time.time()
            output = self.model(data)
            loss = self.criterion(output, target)
            acc1 = comp_accuracy(output, target)
            losses.update(loss.item(), data.size(0))
            top1.update(acc1[0].item(), data.size(0))
            loss.backward()
            update_learning_rate(self.optimizer, self.epoch, args, itr=b, itr_per_epoch=self.n_batches)
            self.optimizer.step()
            self.optimizer.zero_grad()
            comp_time += time.time() - t0
            comm_time += self.communicator.communicate(self.model)          # train_mpi.py:142
        if self.recorder is not None:
            self.recorder.add_new(time.time() - tic, comp_time, comm_time, comp_time + comm_time, top1.avg,
                                  losses.avg, top1.avg)
            if self.epoch % 10 == 0:
                self.recorder.save_to_file()
        self.epoch += 1
        return [{"worker": self.rank, "loss": losses.avg, "train_acc": top1.avg, "comp_time": comp_time,
                 "comm_time": comm_time}]

    def finish(self):
        """Save the logs and release the communicator's group (collective under the pull
        transport: every rank calls finish)."""
        if self.recorder is not None:
            self.recorder.save_to_file()
        self.communicator.close()


class HarnessArgs:
    """train_mpi.py:205-231 defaults, plus the harness's own (size, shape, num_classes, ratio)."""

    def __init__(self, **kw):
        self.name = "Vanilla DecenSGD-synthetic"
        self.description = "MI355X gossip harness, synthetic batches"
        self.model = "mlp"
        self.lr = 0.8
        self.momentum = 0.0
        self.epoch = 1
        self.bs = 64
        self.warmup = True
        self.nesterov = False
        self.matcha = True
        self.budget = 1.0
        self.graphid = 0
        self.savePath = "./saveModel"
        self.save = False
        self.compress = False
        self.consensus_lr = 0.1
        self.ratio = 0.9          # train_mpi.py:79 hard-codes ChocoCommunicator(..., 0.9, ...)
        self.randomSeed = 1234
        self.size = 8
        self.shape = (1, 28, 28)
        self.num_classes = 100    # train_mpi.py:84 select_model(100, args)
        for k, v in kw.items():
            if not hasattr(self, k):
                raise TypeError(f"unknown harness argument {k!r}")
            setattr(self, k, v)

    def __str__(self):
        return "Namespace(" + ", ".join(f"{k}={v!r}" for k, v in sorted(vars(self).items())) + ")"


def model_factory(args):
    if args.model == "mlp":
        return lambda: MNIST_MLP(args.num_classes)
    raise ValueError(f"model {args.model!r}: the harness ships the MLP plumbing config; pass a "
                     "model_fn to VirtualTrainer for other architectures")


def epoch_summary(stats, epoch):
    loss = float(np.mean([s["loss"] for s in stats]))
    acc = float(np.mean([s["train_acc"] for s in stats]))
    comp = float(np.mean([s["comp_time"] for s in stats]))
    return (f"{epoch:0>3}  workers: {len(stats)}, loss: {loss:.3f}, train_acc: {acc:.3f}, "
            f"comp_time: {comp:.3f}, comm_time: {stats[0]['comm_time']:.3f}")


__all__ = ["MNIST_MLP", "comp_accuracy", "AverageMeter", "Recorder", "update_learning_rate",
           "synthetic_batches", "make_topology", "sync_rows", "VirtualTrainer", "RankTrainer", "HarnessArgs",
           "model_factory", "epoch_summary"]
