"""One rank per GPU (tests/test_gpu_multiproc.py::test_cross_gpu_transports_match_oracle launches 2-4
via torchrun when that many GPUs are visible): the REAL cross-GPU transports -- the library's RCCL
communicator (plain and column-pipelined exchange, Choco messages, the ordered all-reduce) and the
pull transport over xGMI with its device gate (whole rows and Choco messages, back to back,
arbitrary rows, snapshot buffers on
different GPUs, so the cross-L2 release / acquire protocol is exercised) -- every worker's row vs
the single-process oracle, bit-exact.  Skipped on a one-GPU box (RCCL refuses two ranks on one
device).  Rank 0 prints one JSON line; exit status 0 = every case matched."""
import importlib
import json
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
from conftest import PKG_NAME, pull_clean, report_rank_errors  # noqa: E402
import mp_worker as W  # noqa: E402
import mp_pull_stress as ST  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    pkg = importlib.import_module(PKG_NAME)
    comm = pkg.engine.RcclComm(timeout_s=60)
    res = {
        "rccl_decen_g0": W.decen_case(pkg, comm, 0, 30_011, 5),
        "rccl_decen_g2_placed": W.decen_case(pkg, comm, 2, 9_001, 4, placement="auto"),
        "rccl_decen_g0_chunked": W.decen_case(pkg, comm, 0, 70_001, 4, chunk_cols=16_384),
        "rccl_choco_g0": W.choco_case(pkg, comm, 40_003, 0.9, 4),
        "rccl_centralized": W.centralized_case(pkg, comm),
        "pull_decen_g0_long": W.decen_case(pkg, pkg.PullTransport(timeout_s=60), 0, 30_011, 30, seed=11,
                                           back_to_back=True),
        "pull_rows_g2_placed": W.pull_rows_case(pkg, 2, 12_007, 20, placement="auto"),
        "pull_choco_g0_placed_long": W.choco_case(pkg, pkg.PullTransport(timeout_s=60), 20_011, 0.9, 12, seed=13,
                                                  placement="auto", back_to_back=True),
        "pull_choco_direct_g0": W.choco_case(pkg, pkg.PullTransport(timeout_s=60), 20_011, 0.9, 8, seed=19,
                                             back_to_back=True, pull_read="direct"),
        # the drift stress across GPUs: ranks several rounds apart, gates waiting over xGMI
        "pull_stress_decen": ST.decen(pkg, dist.get_rank(), dist.get_world_size()),
        "pull_stress_choco_fetch": ST.choco(pkg, dist.get_rank(), dist.get_world_size(), "fetch"),
        "pull_stress_choco_direct": ST.choco(pkg, dist.get_rank(), dist.get_world_size(), "direct"),
    }
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=7)
    torch.cuda.synchronize()
    flags = [None] * dist.get_world_size()
    dist.all_gather_object(flags, all(res.values()))
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "all_ranks": all(flags), **res}), flush=True)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    sys.exit(0 if all(flags) else 1)


if __name__ == "__main__":
    report_rank_errors(main)
