"""Emit the golden fixtures under tests/golden/ by RUNNING THE REFERENCE in this container.

Test infrastructure only (see refharness.py).  Run from the repo root:

    python tests/golden/make_golden.py

It imports /root/reference's own graph_manager / communicator / compressors / comm_helpers
(stubbed mpi4py/cvxpy/torchvision, threaded fake COMM_WORLD) and records their outputs on
small seeded inputs.  The reference never travels to the GPU box; these .npz/.json files do.

Fixtures (all small):
  decomposition.json  GraphProcessor.getSubGraphs / drawer / FixedProcessor.getAlpha
                      (graph_manager.py:51-206) for util.select_graph 0..5 and a 64-node ER graph
  flags.npz           MatchaProcessor.set_flags (graph_manager.py:298-309) and
                      FixedProcessor.set_flags (208-225) for given p / budget, seed, T, plus the
                      numpy MT19937 state before and after
  decen.npz           decenCommunicator.communicate (communicator.py:79-158) over several rounds
  choco.npz           ChocoCommunicator.communicate (communicator.py:161-268) over several rounds
  topk.npz/json       compressors.get_top_k (compressors.py:3-19): k table + index sets
  substeps.npz/json   decen / Choco prepare_comm_buffer + averaging(flags) + reset_model driven
                      directly, flags rows given per call (incl. all-zero)
  topk_special.npz/json  get_top_k on rows with NaN / +-Inf / +-0 / denormals / +-FLT_MAX
                      (inputs stored with the index sets; `python tests/golden/make_golden.py topk_special`)
"""
import contextlib
import io
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refharness as H  # noqa: E402

MASK = (1 << 64) - 1


def synth(seed, n):
    """splitmix64 counter generator -> fp32 uniform[-1,1) (same definition as oracle/)."""
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    m = (z >> np.uint64(40)).astype(np.float32)
    return (m * np.float32(2.0 ** -23) - np.float32(1.0)).astype(np.float32)


class Params(torch.nn.Module):
    def __init__(self, shapes, flat):
        super().__init__()
        ps, off = [], 0
        for s in shapes:
            n = int(np.prod(s)) if len(s) else 1
            ps.append(torch.nn.Parameter(torch.from_numpy(flat[off:off + n].copy()).view(*s)))
            off += n
        self.ps = torch.nn.ParameterList(ps)


def flat_of(model):
    return torch.cat([p.data.reshape(-1) for p in model.parameters()]).numpy().copy()


def numel(shapes):
    return int(sum(int(np.prod(s)) if len(s) else 1 for s in shapes))


def quiet(fn, *a, **kw):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


# ----------------------------------------------------------------------------------------
def gen_decomposition(ns):
    gm = ns.graph_manager
    import networkx as nx
    graphs = {str(g): (ns.util.select_graph(g), 16 if g in (1, 2, 3, 4) else 8) for g in range(6)}
    er = nx.gnp_random_graph(64, 0.1, seed=1234)
    graphs["er64"] = ([sorted(tuple(sorted(e)) for e in er.edges())], 64)
    out = {}
    for name, (base, size) in graphs.items():
        ent = {"size": size, "base": [[list(e) for e in sg] for sg in base], "seeds": {}}
        # issubgraph=True: the given matchings are used as is (graph_manager.py:22-25)
        try:
            fp = quiet(gm.FixedProcessor, base, 1.0, 0, size, 4, True)
            ent["given_neighbors_info"] = fp.neighbors_info
            ent["given_alpha"] = float(fp.neighbor_weight)
        except SystemExit:            # drawer() calls exit() when a "subgraph" is no matching (172-174)
            ent["given_neighbors_info"] = None
            ent["given_alpha"] = None
        for seed in (0, 1, 2):
            random.seed(seed)
            gp = quiet(gm.GraphProcessor, base, 1.0, 0, size, 4, False)
            random.seed(seed)
            fpd = quiet(gm.FixedProcessor, base, 1.0, 0, size, 4, False)
            ent["seeds"][str(seed)] = {
                "subgraphs": [[list(map(int, e)) for e in sg] for sg in gp.subGraphs],
                "neighbors_info": gp.neighbors_info,
                "alpha": float(fpd.neighbor_weight),
                "laplacian_sum_diag": [int(v) for v in np.diag(sum(np.asarray(L) for L in gp.L_matrices))],
            }
        out[name] = ent
        print("decomposition", name, "M =", len(ent["seeds"]["0"]["subgraphs"]))
    with open(os.path.join(HERE, "decomposition.json"), "w") as f:
        json.dump(out, f)


# ----------------------------------------------------------------------------------------
def gen_flags(ns):
    gm = ns.graph_manager
    rng = np.random.RandomState(42)
    matcha_cases = [
        ([0.0, 1.0, 0.5, 0.3, 0.7], 1234, 0, 1000),
        ([0.25, 0.25, 0.25], 7, 77, 2000),
        ([1.0] * 5, 1234, 0, 50),
        ([0.0] * 5, 1234, 0, 50),
        ([0.999999, 1e-9, 0.5000001, 0.4999999], 99, 5, 3000),
        ([float("nan"), -0.1, 0.6], 3, 0, 100),
        (list(rng.uniform(0, 1, 10)), 1234, 0, 19600),
        (list(rng.uniform(0, 1, 5)), 2024, 623, 700),
    ]
    fixed_cases = [(0.5, 1234, 0, 100), (1.0, 5, 0, 10), (0.37, 11, 300, 999)]
    arrs = {}
    meta = {"matcha": [], "fixed": []}
    for ci, (p, seed, pre, T) in enumerate(matcha_cases):
        mp = object.__new__(gm.MatchaProcessor)
        mp.L_matrices = [None] * len(p)
        mp.probabilities = np.array(p, dtype=np.float64)
        np.random.seed(seed)
        if pre:
            np.random.random(pre)
        st0 = np.random.get_state()
        flags = mp.set_flags(T + 1)
        st1 = np.random.get_state()
        arrs[f"matcha{ci}_flags"] = np.asarray(flags, dtype=np.uint8)
        arrs[f"matcha{ci}_key0"] = np.asarray(st0[1], dtype=np.uint32)
        arrs[f"matcha{ci}_key1"] = np.asarray(st1[1], dtype=np.uint32)
        arrs[f"matcha{ci}_psan"] = np.asarray(mp.probabilities, dtype=np.float64)
        meta["matcha"].append({"p": [float(x) for x in p], "seed": seed, "pre_draws": pre, "T": T,
                               "pos0": int(st0[2]), "pos1": int(st1[2])})
    for ci, (b, seed, pre, T) in enumerate(fixed_cases):
        fp = object.__new__(gm.FixedProcessor)
        fp.probabilities = b
        np.random.seed(seed)
        if pre:
            np.random.random(pre)
        st0 = np.random.get_state()
        flags = fp.set_flags(T + 1)
        st1 = np.random.get_state()
        arrs[f"fixed{ci}_flags"] = np.asarray(flags, dtype=np.uint8)
        arrs[f"fixed{ci}_key0"] = np.asarray(st0[1], dtype=np.uint32)
        arrs[f"fixed{ci}_key1"] = np.asarray(st1[1], dtype=np.uint32)
        meta["fixed"].append({"budget": b, "seed": seed, "pre_draws": pre, "T": T,
                              "pos0": int(st0[2]), "pos1": int(st1[2])})
    np.savez_compressed(os.path.join(HERE, "flags.npz"), **arrs)
    with open(os.path.join(HERE, "flags.json"), "w") as f:
        json.dump(meta, f)
    print("flags", len(matcha_cases), "matcha +", len(fixed_cases), "fixed cases")


# ----------------------------------------------------------------------------------------
DECEN_CASES = [
    # name, graph id, shapes, flags rows (None -> the processor's own), seed base
    ("g0", 0, [(17, 3), (5,), (64, 33), (1,), (7, 7, 2)],
     [[1, 1, 1, 1, 1], [0, 0, 0, 0, 0], [1, 0, 1, 1, 0], [0, 1, 0, 0, 1], [1, 0, 0, 0, 0], [0, 0, 0, 1, 1]], 1234),
    ("g5", 5, [(1000,)], None, 77),
    ("g2", 2, [(0,), (31, 29), (3,), (2, 2, 2, 2)], "matcha", 4321),
]


def gen_decen(ns):
    gm, cm = ns.graph_manager, ns.communicator
    arrs, meta = {}, []
    for name, gid, shapes, flags, sb in DECEN_CASES:
        base = ns.util.select_graph(gid)
        size = 16 if gid in (1, 2, 3, 4) else 8
        GP = quiet(gm.FixedProcessor, base, 0.5, 0, size, 10, True)
        M = len(GP.neighbors_info)
        if flags == "matcha":
            mp = object.__new__(gm.MatchaProcessor)
            mp.L_matrices = [None] * M
            mp.probabilities = np.linspace(0.15, 0.9, M)
            np.random.seed(sb)
            flags = mp.set_flags(6)
        if flags is not None:
            GP.active_flags = [list(map(int, r)) for r in flags]
        R = len(GP.active_flags) if flags is not None else 5
        P = numel(shapes)
        X0 = np.stack([synth(sb + r, P) for r in range(size)])
        H.new_world(size)
        models = [Params(shapes, X0[r]) for r in range(size)]
        comms = [cm.decenCommunicator(r, size, GP) for r in range(size)]

        def body(r):
            outs = []
            for _ in range(R):
                comms[r].communicate(models[r])
                outs.append(flat_of(models[r]))
            return np.stack(outs)

        res = H.run_ranks(size, body)                  # [size][R][P]
        Y = np.stack(res, axis=1)                      # [R][size][P]
        arrs[f"{name}_X0"] = X0
        arrs[f"{name}_Y"] = Y
        arrs[f"{name}_flags"] = np.asarray(GP.active_flags[:R], dtype=np.uint8)
        arrs[f"{name}_partner"] = np.asarray(GP.neighbors_info, dtype=np.int32)
        meta.append({"name": name, "graph": gid, "size": size, "shapes": [list(s) for s in shapes],
                     "alpha": float(GP.neighbor_weight), "rounds": R, "P": P})
        print("decen", name, "n =", size, "P =", P, "rounds =", R)
    np.savez_compressed(os.path.join(HERE, "decen.npz"), **arrs)
    with open(os.path.join(HERE, "decen.json"), "w") as f:
        json.dump(meta, f)


# ----------------------------------------------------------------------------------------
CHOCO_CASES = [
    ("c0", 0, [(17, 3), (5,), (64, 33), (1,), (7, 7, 2)], 0.9, 0.1, 1234),
    ("c1", 0, [(1500,)], 0.99, 0.5, 99),
    ("c2", 5, [(40, 25), (13,)], 0.9999, 0.2, 5),      # k == 1 -> torch.max path
]
CHOCO_FLAGS = [[1, 1, 1, 1, 1], [1, 0, 1, 1, 0], [0, 0, 0, 0, 0], [0, 1, 0, 0, 1], [1, 1, 0, 1, 1]]


def gen_choco(ns):
    gm, cm = ns.graph_manager, ns.communicator
    arrs, meta = {}, []
    for name, gid, shapes, ratio, clr, sb in CHOCO_CASES:
        base = ns.util.select_graph(gid)
        size = 8
        GP = quiet(gm.FixedProcessor, base, 0.5, 0, size, 10, True)
        M = len(GP.neighbors_info)
        GP.active_flags = [r[:M] for r in CHOCO_FLAGS]
        R = len(GP.active_flags)
        P = numel(shapes)
        X0 = np.stack([synth(sb + r, P) for r in range(size)])
        # per-round perturbation applied BEFORE communicate (stands in for optimizer.step)
        D = np.stack([np.stack([np.float32(0.05) * synth(10_000 * (t + 1) + sb + r, P) for r in range(size)])
                      for t in range(R)])
        H.new_world(size)
        models = [Params(shapes, X0[r]) for r in range(size)]
        comms = [cm.ChocoCommunicator(r, size, GP, ratio, clr) for r in range(size)]

        def body(r):
            outs, xin = [], []
            for t in range(R):
                with torch.no_grad():
                    off = 0
                    for p in models[r].parameters():
                        n = p.numel()
                        p.data.add_(torch.from_numpy(D[t, r, off:off + n]).view_as(p))
                        off += n
                xin.append(flat_of(models[r]))
                if comms[r].initialized:
                    d = (torch.from_numpy(xin[-1]) - comms[r].x_hat).abs()
                else:
                    d = torch.from_numpy(xin[-1]).abs()
                k = max(1, int(P * (1 - ratio)))
                srt = torch.sort(d, descending=True).values
                if k < P:
                    assert srt[k - 1] != srt[k], f"tie at top-k threshold: {name} r{r} t{t}"
                comms[r].communicate(models[r])
                outs.append(flat_of(models[r]))
            return np.stack(xin), np.stack(outs), comms[r].x_hat.numpy().copy(), comms[r].s.numpy().copy()

        res = H.run_ranks(size, body)
        arrs[f"{name}_X0"] = X0
        arrs[f"{name}_D"] = D
        arrs[f"{name}_Xin"] = np.stack([r[0] for r in res], axis=1)    # [R][n][P] input to communicate
        arrs[f"{name}_Y"] = np.stack([r[1] for r in res], axis=1)      # [R][n][P]
        arrs[f"{name}_xhat"] = np.stack([r[2] for r in res])           # final [n][P]
        arrs[f"{name}_s"] = np.stack([r[3] for r in res])
        arrs[f"{name}_flags"] = np.asarray(GP.active_flags, dtype=np.uint8)
        arrs[f"{name}_partner"] = np.asarray(GP.neighbor_info if hasattr(GP, "neighbor_info") else GP.neighbors_info, dtype=np.int32)
        meta.append({"name": name, "graph": gid, "size": size, "shapes": [list(s) for s in shapes],
                     "alpha": float(GP.neighbor_weight), "ratio": ratio, "consensus_lr": clr,
                     "rounds": R, "P": P, "k": max(1, int(P * (1 - ratio)))})
        print("choco", name, "P =", P, "k =", meta[-1]["k"])
    np.savez_compressed(os.path.join(HERE, "choco.npz"), **arrs)
    with open(os.path.join(HERE, "choco.json"), "w") as f:
        json.dump(meta, f)


# ----------------------------------------------------------------------------------------
def gen_topk(ns):
    gtk = ns.compressors.get_top_k
    arrs, ktab = {}, []
    for P in (1, 2, 10, 2267, 100_000):
        x = torch.from_numpy(synth(P, P))
        for ratio in (0.0, 0.5, 0.9, 0.99, 0.9999):
            v, idx = gtk(x.clone(), ratio)
            o = torch.argsort(idx)
            arrs[f"P{P}_r{ratio}_idx"] = idx[o].numpy().astype(np.int64)
            arrs[f"P{P}_r{ratio}_val"] = v[o].numpy()
            ktab.append({"P": P, "ratio": ratio, "k": int(idx.numel()), "dtype": str(idx.dtype)})
    for P in (181_668, 545_930, 666_547, 14_774_436, 25_600_000, 36_546_980):
        x = torch.zeros(P)
        for ratio in (0.9, 0.99):
            v, idx = gtk(x, ratio)
            ktab.append({"P": P, "ratio": ratio, "k": int(idx.numel()), "dtype": str(idx.dtype)})
    np.savez_compressed(os.path.join(HERE, "topk.npz"), **arrs)
    with open(os.path.join(HERE, "topk.json"), "w") as f:
        json.dump(ktab, f)
    print("topk", len(ktab), "k-table rows")


SUBSTEP_FLAGS = [[1, 0, 1, 0, 1], [0, 0, 0, 0, 0], [1, 1, 1, 1, 1], [0, 1, 1, 0, 0]]


def gen_substeps(ns):
    """substeps.npz/json: the communicators' sub-steps driven directly -- tensor_list set,
    prepare_comm_buffer(), averaging(active_flags), reset_model() (communicator.py:87-131, 175-240)
    -- on flags rows given per call, incl. an all-zero row (which communicate() would skip)."""
    gm, cm = ns.graph_manager, ns.communicator
    arrs, meta = {}, []
    size, shapes = 8, [(23, 7), (9,)]
    P = numel(shapes)
    base = ns.util.select_graph(0)
    GP = quiet(gm.FixedProcessor, base, 0.5, 0, size, 10, True)
    M = len(GP.neighbors_info)
    F = [r[:M] for r in SUBSTEP_FLAGS]
    for kind in ("decen", "choco"):
        X0 = np.stack([synth((77 if kind == "decen" else 88) + r, P) for r in range(size)])
        H.new_world(size)
        models = [Params(shapes, X0[r]) for r in range(size)]
        if kind == "decen":
            comms = [cm.decenCommunicator(r, size, GP) for r in range(size)]
        else:
            comms = [cm.ChocoCommunicator(r, size, GP, 0.9, 0.3) for r in range(size)]

        def body(r):
            outs = []
            for f in F:
                comms[r].tensor_list = [p.data for p in models[r].parameters()]
                comms[r].prepare_comm_buffer()
                comms[r].averaging(f)
                comms[r].reset_model()
                outs.append(flat_of(models[r]))
            extra = (comms[r].x_hat.numpy().copy(), comms[r].s.numpy().copy()) if kind == "choco" else ()
            return (np.stack(outs),) + extra

        res = H.run_ranks(size, body)
        arrs[f"{kind}_X0"] = X0
        arrs[f"{kind}_Y"] = np.stack([r[0] for r in res], axis=1)      # [R][n][P]
        if kind == "choco":
            arrs["choco_xhat"] = np.stack([r[1] for r in res])
            arrs["choco_s"] = np.stack([r[2] for r in res])
        print("substeps", kind, "P =", P, "rounds =", len(F))
    arrs["flags"] = np.asarray(F, dtype=np.uint8)
    arrs["partner"] = np.asarray(GP.neighbors_info, dtype=np.int32)
    meta = {"size": size, "shapes": [list(x) for x in shapes], "P": P, "alpha": float(GP.neighbor_weight),
            "ratio": 0.9, "consensus_lr": 0.3, "k": max(1, int(P * (1 - 0.9)))}
    np.savez_compressed(os.path.join(HERE, "substeps.npz"), **arrs)
    with open(os.path.join(HERE, "substeps.json"), "w") as f:
        json.dump(meta, f)


def special(P, seed, n_nan=5, n_inf=4):
    """A float32 row with quiet NaNs of both signs and two payloads, +-Inf, +-0, denormals and
    +-FLT_MAX planted at random positions; the rest standard normal."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(P).astype(np.float32)
    pos = rng.permutation(P)
    nan = np.array([0x7FC00000, 0xFFC00000, 0x7FC00123, 0xFFC00001], np.uint32).view(np.float32)
    vals = [nan[i % 4] for i in range(n_nan)] + [np.float32(np.inf), np.float32(-np.inf)] * (n_inf // 2) + \
        [np.float32(0.0), np.float32(-0.0), np.float32(1e-42), np.float32(-3e-41), np.float32(3.4028235e38),
         np.float32(-3.4028235e38)]
    for j, v in enumerate(vals):
        x[pos[j]] = v
    return x


def gen_topk_special(ns):
    """topk_special.npz/json: compressors.get_top_k on rows with non-finite and edge values (the
    inputs are stored with the index sets); k = 1 goes through the reference's torch.max branch."""
    gtk = ns.compressors.get_top_k
    arrs, meta = {}, []
    for P, ratio, seed, n_nan, n_inf in ((20_000, 0.99, 1, 5, 4), (4_099, 0.99, 2, 5, 4), (100_003, 0.99, 3, 5, 4),
                                         (30_000, 1 - 12.5 / 30_000, 5, 6, 6), (50_000, 1 - 1.5 / 50_000, 4, 1, 2)):
        x = special(P, seed, n_nan, n_inf)
        v, idx = gtk(torch.from_numpy(x.copy()), ratio)
        o = torch.argsort(idx)
        c = len(meta)
        arrs[f"case{c}_x"] = x
        arrs[f"case{c}_idx"] = idx.reshape(-1)[o.reshape(-1)].numpy().astype(np.int64)
        meta.append({"P": P, "ratio": ratio, "k": int(idx.numel()), "nan": n_nan, "inf": n_inf})
    np.savez_compressed(os.path.join(HERE, "topk_special.npz"), **arrs)
    with open(os.path.join(HERE, "topk_special.json"), "w") as f:
        json.dump(meta, f)
    print("topk_special", len(meta), "cases")


if __name__ == "__main__":
    torch.set_num_threads(1)
    ns = H.install(8)
    which = sys.argv[1:] or ["decomposition", "flags", "decen", "choco", "topk"]
    for w in which:
        globals()["gen_" + w](ns)
