import importlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG_NAME = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def O():
    import oracle
    return oracle


def golden_npz(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def golden_json(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


class Topo:
    """Minimal stand-in for a processor: the attributes the communicators read."""

    def __init__(self, partner, alpha, flags):
        partner = np.asarray(partner, dtype=np.int32)
        self.size = int(partner.shape[1])
        self.neighbors_info = partner.tolist()
        self.neighbor_weight = float(alpha)
        self.active_flags = [list(map(int, r)) for r in np.asarray(flags)]


class LoopbackHub:
    """Test double for the RCCL transport: N simulated ranks on ONE GPU in one process.

    Each rank's GossipEngine gets a LoopbackComm; a round runs in two phases driven by the test:
    every rank's exchange (the ops of the native mx_exchange_plan, executed as device copies from
    the peer rank's rows into this rank's slab, in posting order), then every rank's mix."""

    def __init__(self, nranks):
        self.nranks = nranks
        self.rows = {}          # rank -> {local row index: device pointer}
        self.row_base = {}

    def comm(self, rank):
        return LoopbackComm(self, rank)


class LoopbackComm:
    def __init__(self, hub, rank):
        self.hub, self.rank, self.nranks = hub, rank, hub.nranks
        self.handle = None

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        import ctypes
        import torch
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        torch.cuda.synchronize()
        nrem = 0
        for kind, peer, idx, who in engine.exchange_plan(it):
            if kind == 1:   # what ncclRecv delivers: the partner's pre-round row into slab slot idx
                src = self.hub.rows[int(peer)][int(who) - self.hub.row_base[int(peer)]]
                dst = slab_ptr + int(idx) * slab_ld_bytes
                assert hip.hipMemcpy(dst, src, int(row_bytes), 3) == 0   # device to device
                nrem += 1
        return nrem
