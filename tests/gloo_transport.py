"""Test double for the RCCL transport across REAL processes: gloo over the host.

GossipEngine accepts any object with ``exchange_round`` (and ``allgather`` / ``allreduce_mean``
for the centralized communicator) in place of the RCCL communicator.  This one moves each row the
native mx_exchange_plan names through host memory with gloo isend / irecv, in the plan's order,
so several processes can run the multi-GPU code path (partition, plan slots, receive slab,
chunked pipelining, the bench's N > 1 timing) on ONE GPU -- RCCL refuses two ranks on one
device.  Test / tool infrastructure only: the product's transport is RCCL (exchange.cpp).
Device rows are copied with the library's own mx_gather / mx_scatter (no second HIP runtime).
"""
import numpy as np
import torch
import torch.distributed as dist


class GlooTransport:
    handle = None

    def __init__(self, pkg, group=None):
        self.pkg = pkg
        self.group = group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        self._off = {}

    def _seg(self, n):
        if n not in self._off:
            self._off[n] = torch.tensor([0, n], dtype=torch.int64, device="cuda")
        return self._off[n]

    def _pull(self, ptr, n):
        """device row at raw pointer -> new device tensor"""
        out = torch.empty(n, dtype=torch.float32, device="cuda")
        ptrs = torch.tensor([int(ptr)], dtype=torch.int64, device="cuda")
        self.pkg._lib.check(self.pkg.lib.mx_gather(ptrs.data_ptr(), self._seg(n).data_ptr(), 1, n,
                                                   out.data_ptr(), self.pkg._lib.stream_ptr()), "mx_gather")
        return out

    def _push(self, t, ptr):
        """device tensor -> device row at raw pointer"""
        n = t.numel()
        ptrs = torch.tensor([int(ptr)], dtype=torch.int64, device="cuda")
        self.pkg._lib.check(self.pkg.lib.mx_scatter(ptrs.data_ptr(), self._seg(n).data_ptr(), 1, n,
                                                    t.data_ptr(), self.pkg._lib.stream_ptr()), "mx_scatter")

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        n = row_bytes // 4
        ops = engine.exchange_plan(it)
        posted, reqs = [], []
        for kind, peer, idx, _who in ops:          # plan order: per-pair FIFO matching, like RCCL
            if kind == 0:
                buf = self._pull(row_ptrs[int(idx)], n).cpu()
                reqs.append(dist.isend(buf, int(peer), group=self.group))
            else:
                buf = torch.empty(n, dtype=torch.float32)
                reqs.append(dist.irecv(buf, int(peer), group=self.group))
            posted.append((int(kind), int(idx), buf))
        for r in reqs:
            r.wait()
        nrem = 0
        for kind, idx, buf in posted:
            if kind == 1:
                self._push(buf.cuda(), slab_ptr + idx * slab_ld_bytes)
                nrem += 1
        torch.cuda.synchronize()
        return nrem

    def allgather(self, flat, gather):
        """every rank's `flat` into gather[rank * n : (rank + 1) * n] (device), rank order"""
        host = [torch.empty(flat.numel(), dtype=torch.float32) for _ in range(self.nranks)]
        dist.all_gather(host, flat.cpu(), group=self.group)
        gather.copy_(torch.cat(host).to(gather.device))

    def allreduce_mean(self, flat, size):
        host = flat.cpu()
        dist.all_reduce(host, group=self.group)
        flat.copy_((host / float(size)).to(flat.device))


def gather_rows(rows_local, row_base, n_total, group=None):
    """All workers' rows on every rank (host numpy), for comparing with the oracle."""
    world = dist.get_world_size(group)
    host = rows_local.detach().cpu().numpy()
    meta = [None] * world
    dist.all_gather_object(meta, (int(row_base), host), group=group)
    P = host.shape[1]
    out = np.zeros((n_total, P), np.float32)
    for base, blk in meta:
        out[base:base + blk.shape[0]] = blk
    return out
