"""One rank of the per-rank training-harness test (tests/test_gpu_multiproc.py launches 8 via
torchrun, all sharing GPU 0): train_mpi.py's run(rank, size) -- harness.RankTrainer: sync_allreduce,
then per batch forward / backward / SGD step + communicate(model) (train_mpi.py:109-145) -- with the
gossip over the gloo test transport or the pull transport, against the single-process
VirtualTrainer (batched=False: the same per-worker step, itself checked round by round against the
oracle in test_gpu_harness.py) on rank 0.  Every worker's final parameters must be bit-identical.
Exit status 0 = all matched."""
import importlib
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)
from conftest import PKG_NAME, pull_clean, report_rank_errors  # noqa: E402
from gloo_transport import GlooTransport  # noqa: E402


def flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()


def case(pkg, H, compress, transport, rank, world, epochs=2, batches=5):
    args = H.HarnessArgs(epoch=epochs, bs=16, budget=0.5, compress=compress, size=world, lr=0.1, momentum=0.9)
    sync = GlooTransport(pkg)
    tr = H.RankTrainer(args, H.model_factory(args), batches, rank, world, transport=transport, sync_transport=sync)
    start = flat(tr.model)                                  # after sync_allreduce: the same on every rank
    while tr.epoch < args.epoch:
        tr.train_epoch()
    rows = [None] * world
    dist.all_gather_object(rows, flat(tr.model))
    tr.finish()
    if rank != 0:
        return True
    # the run trained: every worker moved away from the synced start, and the workers differ
    if any(np.array_equal(r, start) for r in rows) or np.array_equal(rows[0], rows[1]):
        return False
    vt = H.VirtualTrainer(args, H.model_factory(args), batches)
    while vt.epoch < args.epoch:
        vt.train_epoch()
    want = vt.group.rows.cpu().numpy()
    got = np.stack(rows)
    return bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))


def main():
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = importlib.import_module(PKG_NAME)
    H = pkg.harness
    res = {"decen_gloo": case(pkg, H, False, GlooTransport(pkg), rank, world),
           "decen_pull": case(pkg, H, False, pkg.PullTransport(), rank, world),
           "choco_pull": case(pkg, H, True, pkg.PullTransport(), rank, world)}
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=2)
    torch.cuda.synchronize()
    if rank == 0:
        print(json.dumps({"world": world, **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(res.values()) else 1)


if __name__ == "__main__":
    report_rank_errors(main)
