"""Non-finite and edge values through the oracle's top-k, against the library the reference calls
(compressors.get_top_k, compressors.py:3-19: torch.topk(|x|, k, largest=True, sorted=False), or
torch.max(|x|) for k = 1) -- torch on the CPU here, so these semantics are pinned, not assumed:
NaN ranks above +Inf (any sign or payload), +-Inf above every finite value, -0 equal to +0.  The
GPU kernels are held to the same oracle in tests/test_gpu_special_values.py."""
import numpy as np
import pytest

from conftest import special_values

torch = pytest.importorskip("torch")


def _ref_indices(x, k):
    a = torch.from_numpy(x).abs()
    if k == 1:
        _, i = torch.max(a, dim=0, keepdim=True)
    else:
        _, i = torch.topk(a, k, largest=True, sorted=False)
    return np.sort(i.numpy())


@pytest.mark.parametrize("P,k,seed", [(20_000, 200, 1), (4_099, 17, 2), (100_003, 1_000, 3), (64, 12, 4)])
def test_oracle_topk_special_values_vs_torch(O, P, k, seed):
    x = special_values(P, seed)
    vals, idx = O.topk_abs(x, k)
    ref = _ref_indices(x, k)
    assert np.array_equal(idx, ref)
    assert np.array_equal(vals.view(np.uint32), x[idx].view(np.uint32))        # the values are x's own bits
    assert np.isnan(x[idx]).sum() == 5 and np.isinf(x[idx]).sum() == 4          # every NaN and Inf selected


def test_oracle_topk_k1_single_nan_vs_torch_max(O):
    x = special_values(5_000, 9, n_nan=1, n_inf=2)
    _, idx = O.topk_abs(x, 1)
    assert np.array_equal(idx, _ref_indices(x, 1)) and np.isnan(x[idx[0]])


def test_oracle_topk_all_nonfinite_prefix_vs_torch(O):
    """k exactly the number of non-finite entries: the set is the NaNs and Infs, nothing else."""
    x = special_values(30_000, 11, n_nan=6, n_inf=6)
    _, idx = O.topk_abs(x, 12)
    assert np.array_equal(idx, _ref_indices(x, 12))
    assert not np.isfinite(x[idx]).any()


def test_oracle_topk_special_values_vs_reference_fixture(O):
    """The reference's own get_top_k (tests/golden/topk_special.npz, make_golden.py topk_special),
    incl. its torch.max branch at k = 1: the oracle's index sets equal it."""
    from conftest import golden_json, golden_npz
    g = golden_npz("topk_special")
    for c, m in enumerate(golden_json("topk_special")):
        x = g[f"case{c}_x"]
        assert O.topk_k(m["P"], m["ratio"]) == m["k"]
        _, idx = O.topk_abs(x, m["k"])
        assert np.array_equal(idx, g[f"case{c}_idx"]), m
