"""The CPU oracle against the reference's own outputs (tests/golden, from make_golden.py)."""
import numpy as np
import pytest

from conftest import golden_json, golden_npz


def test_synth_c_matches_numpy(O):
    for seed, n in ((0, 1), (1234, 10_007), (2 ** 63 + 5, 4096)):
        assert np.array_equal(O.synth(seed, n), O.synth_np(seed, n))
    x = O.synth(99, 1 << 16)
    assert x.min() >= -1.0 and x.max() < 1.0


def test_mt_seed_matches_numpy(O):
    for seed in (0, 1, 1234, 2 ** 32 - 1):
        key, pos = O.mt_seed(seed)
        st = np.random.RandomState(seed).get_state()
        assert np.array_equal(key, st[1]) and pos == st[2]


@pytest.mark.parametrize("ci", range(8))
def test_matcha_flags_vs_reference(O, ci):
    g, meta = golden_npz("flags"), golden_json("flags")["matcha"][ci]
    flags, key, pos = O.matcha_flags(g[f"matcha{ci}_key0"], meta["pos0"], np.array(meta["p"]), meta["T"] + 1)
    assert np.array_equal(flags, g[f"matcha{ci}_flags"])
    assert np.array_equal(key, g[f"matcha{ci}_key1"]) and pos == meta["pos1"]


@pytest.mark.parametrize("ci", range(3))
def test_fixed_flags_vs_reference(O, ci):
    g, meta = golden_npz("flags"), golden_json("flags")["fixed"][ci]
    flags, key, pos = O.fixed_flags(g[f"fixed{ci}_key0"], meta["pos0"], meta["budget"], meta["T"] + 1)
    assert np.array_equal(flags, g[f"fixed{ci}_flags"])
    assert np.array_equal(key, g[f"fixed{ci}_key1"]) and pos == meta["pos1"]


def test_binomial_restatement_vs_numpy_random_p(O):
    """numpy itself (the third-party generator the reference calls) on random p, seeds, offsets."""
    rng = np.random.RandomState(7)
    for _ in range(40):
        M = int(rng.randint(1, 6))
        p = rng.uniform(0, 1, M)
        p[rng.uniform(size=M) < 0.2] = rng.choice([0.0, 1.0, 0.5])
        T = int(rng.randint(1, 400))
        np.random.seed(int(rng.randint(0, 2 ** 31)))
        np.random.random(int(rng.randint(0, 700)))
        st = np.random.get_state()
        ref = np.stack([np.random.binomial(1, pm, T) for pm in p], axis=1)
        st1 = np.random.get_state()
        flags, key, pos = O.matcha_flags(st[1], st[2], p, T)
        assert np.array_equal(flags, ref)
        assert np.array_equal(key, st1[1]) and pos == st1[2]


@pytest.mark.parametrize("case", ["g0", "g5", "g2"])
def test_decen_vs_reference(O, case):
    d = golden_npz("decen")
    meta = {m["name"]: m for m in golden_json("decen")}[case]
    X = d[case + "_X0"]
    for r in range(meta["rounds"]):
        X = O.decen_round(X, d[case + "_partner"], d[case + "_flags"][r], meta["alpha"])
        assert np.array_equal(X.view(np.uint32), d[case + "_Y"][r].view(np.uint32)), f"round {r}"


@pytest.mark.parametrize("case", ["c0", "c1", "c2"])
def test_choco_vs_reference(O, case):
    c = golden_npz("choco")
    m = {x["name"]: x for x in golden_json("choco")}[case]
    X = c[case + "_X0"].copy()
    XH, S = np.zeros_like(X), np.zeros_like(X)
    for r in range(m["rounds"]):
        X += c[case + "_D"][r]
        assert np.array_equal(X, c[case + "_Xin"][r])
        O.choco_round(X, XH, S, c[case + "_partner"], c[case + "_flags"][r], m["alpha"], m["k"], m["consensus_lr"])
        assert np.array_equal(X.view(np.uint32), c[case + "_Y"][r].view(np.uint32)), f"round {r}"
    assert np.array_equal(XH, c[case + "_xhat"]) and np.array_equal(S, c[case + "_s"])


def test_topk_k_table(O):
    for row in golden_json("topk"):
        assert O.topk_k(row["P"], row["ratio"]) == row["k"], row
        assert row["dtype"] == "torch.int64"


def test_topk_index_sets(O):
    t = golden_npz("topk")
    for row in golden_json("topk"):
        key = f"P{row['P']}_r{row['ratio']}_idx"
        if key not in t:
            continue
        x = O.synth(row["P"], row["P"])
        vals, idx = O.topk_abs(x, row["k"])
        assert np.array_equal(idx, t[key])
        assert np.array_equal(vals, t[f"P{row['P']}_r{row['ratio']}_val"])


def test_baseline_port_matches_round(O):
    """The timed CPU port computes the same round as the restatement (segments + threads)."""
    n, P = 8, 3001
    d = golden_npz("decen")
    partner = d["g0_partner"]
    X = np.stack([O.synth(50 + i, P) for i in range(n)])
    cuts = [0, 7, 1000, 1001, P]
    segs = [[X[i, a:b].copy() for a, b in zip(cuts[:-1], cuts[1:])] for i in range(n)]
    flags = np.array([[1, 1, 1, 1, 1], [0, 0, 0, 0, 0], [1, 0, 1, 0, 1]], np.uint8)
    O.baseline_rounds(segs, partner, flags, 2 / 7, threads=4)
    for f in flags:
        X = O.decen_round(X, partner, f, 2 / 7)
    got = np.stack([np.concatenate(s) for s in segs])
    assert np.array_equal(got, X)


@pytest.mark.parametrize("P,k,pattern", [(1, 1, "rand"), (10_007, 100, "rand"), (10_007, 10_007, "rand"),
                                         (50_000, 4_999, "ties"), (50_000, 777, "const"), (65_536, 655, "zeros"),
                                         (200_003, 2_000, "signed_zero")])
def test_topk_select_equals_sort(O, P, k, pattern):
    """The O(P) quickselect top-k equals the full-sort statement of the rule (|x| descending,
    lowest index first among equal magnitudes) on random data and on heavy ties."""
    x = O.synth(P + 17, P)
    if pattern == "ties":
        x[::3] = np.float32(0.75)
        x[1::5] = np.float32(-0.75)
    elif pattern == "const":
        x[:] = np.float32(-0.5)
    elif pattern == "zeros":
        x[:] = 0
        x[::97] = np.float32(1e-30)
    elif pattern == "signed_zero":
        x[::2] = np.float32(-0.0)
        x[1::4] = np.float32(0.0)
    v1, i1 = O.topk_abs(x, k)
    v2, i2 = O.topk_abs(x, k, sort=True)
    assert np.array_equal(i1, i2)
    assert np.array_equal(v1.view(np.uint32), v2.view(np.uint32))


def test_substeps_vs_reference(O):
    """The reference's sub-steps driven directly (tests/golden/substeps.npz): decenCommunicator and
    ChocoCommunicator prepare_comm_buffer + averaging(flags) + reset_model on given flags rows,
    incl. an all-zero row -- which the reference's averaging still applies (Choco: every worker's
    own message) though communicate() would skip it.  The oracle (decen_round; choco_round with
    skip_empty=False) reproduces every round bit for bit."""
    g, m = golden_npz("substeps"), golden_json("substeps")
    partner, flags = g["partner"], g["flags"]
    X = g["decen_X0"].copy()
    for t, f in enumerate(flags):
        if f.any():
            X = O.decen_round(X, partner, f, m["alpha"])
        assert np.array_equal(X.view(np.uint32), g["decen_Y"][t].view(np.uint32)), t
    X = np.ascontiguousarray(g["choco_X0"].copy())
    XH, S = np.zeros_like(X), np.zeros_like(X)
    for t, f in enumerate(flags):
        O.choco_round(X, XH, S, partner, f, m["alpha"], m["k"], m["consensus_lr"], skip_empty=False)
        assert np.array_equal(X.view(np.uint32), g["choco_Y"][t].view(np.uint32)), t
    assert np.array_equal(XH.view(np.uint32), g["choco_xhat"].view(np.uint32))
    assert np.array_equal(S.view(np.uint32), g["choco_s"].view(np.uint32))
