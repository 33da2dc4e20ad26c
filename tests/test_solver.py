"""MATCHA probability / alpha solves (CVXOPT absent, and p is not unique: the objective values are
certified instead -- independent upper bound for lambda_2, global minimum for alpha -- plus the
known answers)."""
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


def _lambda2_upper_bound(Ls, budget, tol=1e-6, iters=2000):
    """Independent certificate for getProbability's optimum (graph_manager.py:240-266): Kelley's
    cutting-plane method on the concave lambda_2(p) = lambda_min(Q^T L(p) Q).  Every eigenvector v
    of the smallest eigenvalue at an iterate gives a valid cut t <= sum_j p_j v^T A_j v, so the LP
    over the cuts and the budget polytope bounds the optimum from above; iterate until that bound
    is within tol of the best lambda_2 seen.  Returns (best, upper bound)."""
    import scipy.linalg
    from scipy.optimize import linprog
    M, n = len(Ls), Ls[0].shape[0]
    Q = scipy.linalg.null_space(np.ones((1, n)))
    A = np.stack([Q.T @ np.asarray(L, float) @ Q for L in Ls])
    cuts, p, best, ub = [], np.full(M, min(1.0, budget)), -np.inf, np.inf
    for _ in range(iters):
        w, V = np.linalg.eigh(np.tensordot(p, A, 1))
        best = max(best, w[0])
        for k in range(len(w)):
            if w[k] > w[0] + 1e-7:
                break
            cuts.append(np.einsum("i,jik,k->j", V[:, k], A, V[:, k]))
        A_ub = np.array([np.r_[-c, 1.0] for c in cuts] + [np.r_[np.ones(M), 0.0]])
        b_ub = np.r_[np.zeros(len(cuts)), M * budget]
        res = linprog(np.r_[np.zeros(M), -1.0], A_ub=A_ub, b_ub=b_ub, bounds=[(0, 1)] * M + [(None, None)],
                      method="highs")
        p, ub = res.x[:M], -res.fun
        if ub - best < tol:
            break
    return best, ub


@pytest.mark.parametrize("g", [0, 1, 2, 3, 4, 5])
def test_probabilities_certified_optimal(pkg, g):
    """The lambda_2 the solver reaches is within 1e-6 of an independently certified upper bound on
    the optimum, for every reference graph and budgets 0.1-0.8 (p itself is not unique, so the
    objective value is what can be pinned without CVXOPT)."""
    Ls = _laps(pkg, g, pkg.GRAPH_SIZES[g])
    for b in (0.1, 0.3, 0.5, 0.8):
        p = pkg.solver.matcha_probabilities(Ls, b)
        assert (p >= -1e-12).all() and (p <= 1 + 1e-12).all() and p.sum() <= len(Ls) * b + 1e-7
        lam = pkg.solver.lambda2(sum(pj * np.asarray(L, float) for pj, L in zip(p, Ls)))
        best, ub = _lambda2_upper_bound(Ls, b)
        assert ub - 1e-6 - 1e-9 <= lam <= ub + 1e-9, (g, b, lam, best, ub)


@pytest.mark.parametrize("g,budget", [(0, 0.5), (2, 0.3), (3, 0.8), (4, 0.1)])
def test_alpha_global_minimum(pkg, g, budget):
    """getAlpha (graph_manager.py:268-296) reduces to min over a of lambda_max(I - J - 2aE + a^2 F),
    convex in a: no point of a dense grid over [0, 3 a*] does better than the solver's a*."""
    Ls = _laps(pkg, g, pkg.GRAPH_SIZES[g])
    p = pkg.solver.matcha_probabilities(Ls, budget)
    a = pkg.solver.matcha_alpha(Ls, p)
    r = pkg.solver.spectral_norm(Ls, p, a)
    grid = min(pkg.solver.spectral_norm(Ls, p, x) for x in np.linspace(0.0, 3 * a, 3001))
    assert r <= grid + 1e-12
