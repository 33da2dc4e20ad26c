"""train_mpi.py on the MI355X with synthetic batches (no dataset download on the GPU box).

    python tools/train_gpu.py --workers 8 --epoch 2 --batches 50                 # 8 virtual workers, 1 GPU
    python tools/train_gpu.py --compress --budget 0.5                           # ChocoSGD
    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/train_gpu.py     # one worker per GPU

Flags follow train_mpi.py:205-231 (same names and defaults where they apply); --workers,
--batches, --checkpoint and --resume are the harness's own.
"""
import argparse
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
H = pkg.harness


def main():
    ap = argparse.ArgumentParser(description="MI355X gossip training harness (synthetic data)")
    ap.add_argument("--name", default="Vanilla DecenSGD-synthetic")
    ap.add_argument("--description", default="MI355X gossip harness, synthetic batches")
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--lr", default=0.8, type=float)
    ap.add_argument("--momentum", default=0.0, type=float)
    ap.add_argument("--epoch", "-e", default=1, type=int)
    ap.add_argument("--bs", default=64, type=int)
    ap.add_argument("--no-warmup", dest="warmup", action="store_false")
    ap.add_argument("--nesterov", action="store_true")
    ap.add_argument("--fixed", dest="matcha", action="store_false", help="FixedProcessor (D-PSGD)")
    ap.add_argument("--budget", default=1.0, type=float)
    ap.add_argument("--graphid", default=0, type=int)
    ap.add_argument("--savePath", default="./saveModel")
    ap.add_argument("--save", action="store_true")
    ap.add_argument("--compress", action="store_true")
    ap.add_argument("--consensus_lr", default=0.1, type=float)
    ap.add_argument("--randomSeed", default=1234, type=int)
    ap.add_argument("--workers", default=8, type=int)
    ap.add_argument("--batches", default=20, type=int, help="batches per epoch")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--resume", default=None)
    ap.add_argument("--batched", action="store_true", help="one vmap'd step for all virtual workers")
    ap.add_argument("--graph", action="store_true", help="with --batched: replay each iteration (step + "
                    "gossip round) as one captured HIP graph once the learning rate is constant")
    ap.add_argument("--pull", action="store_true", help="one process per GPU: gossip rounds over the pull "
                    "transport (partner rows / Choco messages read from the peers' HBM) instead of RCCL")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    args = H.HarnessArgs(name=a.name, description=a.description, model=a.model, lr=a.lr, momentum=a.momentum,
                         epoch=a.epoch, bs=a.bs, warmup=a.warmup, nesterov=a.nesterov, matcha=a.matcha,
                         budget=a.budget, graphid=a.graphid, savePath=a.savePath, save=a.save,
                         compress=a.compress, consensus_lr=a.consensus_lr, randomSeed=a.randomSeed,
                         size=a.workers if world == 1 else world)
    import torch
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        tr = H.RankTrainer(args, H.model_factory(args), a.batches, rank, world,
                           transport="pull" if a.pull else None)
    else:
        tr = H.VirtualTrainer(args, H.model_factory(args), a.batches, batched=a.batched or a.graph, graph=a.graph)
        if a.resume:
            tr.load(a.resume)
    import time
    while tr.epoch < args.epoch:
        torch.cuda.synchronize()
        t = time.time()
        stats = tr.train_epoch()
        torch.cuda.synchronize()
        if rank == 0:
            print(H.epoch_summary(stats, tr.epoch - 1) + f", wall: {time.time() - t:.3f} s "
                  f"({a.batches / (time.time() - t):.1f} iterations/s)", flush=True)
    tr.finish()
    if a.checkpoint and world == 1:
        tr.save(a.checkpoint)


if __name__ == "__main__":
    main()
