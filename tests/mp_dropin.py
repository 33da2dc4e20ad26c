"""One rank of the per-rank drop-in test (tests/test_gpu_multiproc.py launches 8 via torchrun).

The reference's deployment: one process per worker, each holding one model and calling
decenCommunicator / ChocoCommunicator(rank, size, GP, ...).communicate(model) after its
optimizer step (train_mpi.py:79-81, 142).  Here the 8 processes share GPU 0 and exchange rows /
messages through the gloo test transport; each round every rank's parameters are gathered and
compared bit-exactly with the single-process oracle -- and the same over the pull transport.
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
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
import oracle as O  # noqa: E402
from conftest import PKG_NAME, pull_clean, report_rank_errors  # noqa: E402
from gloo_transport import GlooTransport  # noqa: E402


def flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()


def all_rows(model):
    rows = [None] * dist.get_world_size()
    dist.all_gather_object(rows, flat(model))
    return np.stack(rows)


def make_model(rank, dev):
    torch.manual_seed(100 + rank)
    return torch.nn.Sequential(torch.nn.Linear(24, 37), torch.nn.ReLU(), torch.nn.Linear(37, 5)).to(dev)


def drift(model, t, rank):
    """stand-in for the optimizer step between rounds (train_mpi.py:134)"""
    g = torch.Generator().manual_seed(1000 * t + rank)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(0.01 * torch.randn(p.shape, generator=g).to(p.device))


def decen_case(pkg, T, dev, rounds=8):
    rank, n = dist.get_rank(), dist.get_world_size()
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, rank, n, rounds, True)
    model = make_model(rank, dev)
    ids = [id(p) for p in model.parameters()]
    comm = pkg.decenCommunicator(rank, n, GP, transport=T)
    partner = np.asarray(GP.neighbors_info, np.int32)
    ok = True
    for it in range(rounds):
        drift(model, it, rank)
        X = all_rows(model)
        t = comm.communicate(model)
        f = np.asarray(GP.active_flags[it], np.uint8)
        want = O.decen_round(X, partner, f, GP.neighbor_weight) if f.any() else X
        got = all_rows(model)
        ok &= bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        ok &= (t == 0) == (not f.any())
    ok &= ids == [id(p) for p in model.parameters()] and comm.iter == rounds
    comm.close()                         # collective under PullTransport (every rank, same call)
    return ok


def choco_case(pkg, T, dev, rounds=6, ratio=0.9, gamma=0.2):
    rank, n = dist.get_rank(), dist.get_world_size()
    np.random.seed(99)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, rank, n, rounds, True)
    model = make_model(rank, dev)
    comm = pkg.ChocoCommunicator(rank, n, GP, ratio, gamma, transport=T)
    partner = np.asarray(GP.neighbors_info, np.int32)
    P = sum(p.numel() for p in model.parameters())
    k = O.topk_k(P, ratio)
    XH = np.zeros((n, P), np.float32)
    S = np.zeros((n, P), np.float32)
    ok = True
    for it in range(rounds):
        drift(model, it, rank)
        X = np.ascontiguousarray(all_rows(model))
        comm.communicate(model)
        f = np.asarray(GP.active_flags[it], np.uint8)
        if f.any():
            O.choco_round(X, XH, S, partner, f, GP.neighbor_weight, k, gamma)
        got = all_rows(model)
        ok &= bool(np.array_equal(got.view(np.uint32), X.view(np.uint32)))
    if comm.x_hat is not None:
        xh = [None] * n
        dist.all_gather_object(xh, comm.x_hat.cpu().numpy())
        ok &= bool(np.array_equal(np.stack(xh), XH))
    comm.close()
    return ok


def main():
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    pkg = importlib.import_module(PKG_NAME)
    T = GlooTransport(pkg)
    res = {"decen_gpu_models": decen_case(pkg, T, "cuda"),
           "decen_cpu_models": decen_case(pkg, T, "cpu"),
           "choco_gpu_models": choco_case(pkg, T, "cuda"),
           "choco_cpu_models": choco_case(pkg, T, "cpu"),
           # train_mpi.py's deployment over the pull transport: rows / Choco messages read from the
           # peers' IPC-mapped snapshot buffers behind the device gate (8 processes share GPU 0 here)
           "decen_gpu_models_pull": decen_case(pkg, pkg.PullTransport(), "cuda"),
           "choco_gpu_models_pull": choco_case(pkg, pkg.PullTransport(), "cuda"),
           "choco_cpu_models_pull": choco_case(pkg, pkg.PullTransport(), "cpu")}
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=3)
    torch.cuda.synchronize()
    flags = [None] * dist.get_world_size()
    dist.all_gather_object(flags, all(res.values()))
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "all_ranks": all(flags), **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(flags) else 1)


if __name__ == "__main__":
    report_rank_errors(main)
