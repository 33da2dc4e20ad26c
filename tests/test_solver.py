"""MATCHA probability / alpha solves (parity unpinned: CVXOPT absent; known answers only)."""
import numpy as np
import pytest


def _laps(pkg, g, n):
    return pkg.GraphProcessor(pkg.select_graph(g), 1.0, 0, n, 4, True).L_matrices


def test_budget_one_gives_all_ones_and_fixed_alpha(pkg):
    for g, n in ((0, 8), (2, 16), (5, 8)):
        Ls = _laps(pkg, g, n)
        p = pkg.solver.matcha_probabilities(Ls, 1.0)
        assert np.array_equal(p, np.ones(len(Ls)))
        w = np.linalg.eigvalsh(sum(np.asarray(L, float) for L in Ls))
        a_fixed = 2 / (w[1] + w[-1])
        assert abs(pkg.solver.matcha_alpha(Ls, p) - a_fixed) < 1e-7


@pytest.mark.parametrize("budget,rho", [(0.1, 0.94), (0.47, 0.66), (0.6, 0.58), (1.0, 0.66)])
def test_graph0_spectral_norms_fig1c(pkg, budget, rho):
    """ResearchReport.pdf Fig. 1(c) (chart readings, +-0.01)."""
    Ls = _laps(pkg, 0, 8)
    p = pkg.solver.matcha_probabilities(Ls, budget)
    a = pkg.solver.matcha_alpha(Ls, p)
    assert abs(pkg.solver.spectral_norm(Ls, p, a) - rho) < 0.011


def test_probabilities_feasible_and_optimal_vs_uniform(pkg):
    Ls = _laps(pkg, 3, 16)
    for b in (0.1, 0.3, 0.5, 0.8):
        p = pkg.solver.matcha_probabilities(Ls, b)
        assert (p >= -1e-12).all() and (p <= 1 + 1e-12).all() and p.sum() <= len(Ls) * b + 1e-7
        uni = np.full(len(Ls), b)
        lam = pkg.solver.lambda2(sum(pj * L for pj, L in zip(p, Ls)))
        lam_u = pkg.solver.lambda2(sum(pj * L for pj, L in zip(uni, Ls)))
        assert lam >= lam_u - 1e-9


def test_alpha_minimises_spectral_norm(pkg):
    Ls = _laps(pkg, 0, 8)
    p = pkg.solver.matcha_probabilities(Ls, 0.5)
    a = pkg.solver.matcha_alpha(Ls, p)
    r = pkg.solver.spectral_norm(Ls, p, a)
    for da in (-1e-3, 1e-3, -1e-2, 1e-2):
        assert pkg.solver.spectral_norm(Ls, p, a + da) >= r - 1e-9
