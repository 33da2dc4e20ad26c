"""Host-side MATCHA solvers without cvxpy/CVXOPT (neither is installed here or on the box).

MatchaProcessor.getProbability (graph_manager.py:240-266) solves
    maximize  lambda_sum_smallest(sum_j p_j L_j, 2)   s.t.  sum p <= M*C_b,  0 <= p <= 1
and MatchaProcessor.getAlpha (graph_manager.py:268-296) solves the 3-variable SDP
    minimize s  s.t.  (1-s) I - 2a E[L] - J + b (E[L]^2 + 2 Var[L]) << 0,  a, s, b >= 0,  a^2 <= b.

Reformulations used here:
  * Every L_j is a graph Laplacian, so the smallest eigenvalue of sum p_j L_j is 0 with the
    all-ones eigenvector; the objective is lambda_2, i.e. lambda_min of Q^T L(p) Q on the
    complement of 1 (Q orthonormal) -- a small linear-matrix-inequality problem, solved by a
    log-det barrier interior-point method (Newton centering steps on the central path).
    lambda_2 is nondecreasing in every p_j, so C_b >= 1 gives p = 1 directly.
  * E[L]^2 + 2 Var[L] is PSD, so b = a^2 at the optimum and
        s*(a) = lambda_max(I - J - 2 a E + a^2 (E^2 + 2V)),
    a maximum of convex quadratics in a -> a 1-D convex minimisation (bounded Brent, then a
    golden-section polish).

Parity status: the SDP optimum p is not unique in general, so p itself cannot be
reproduced without CVXOPT -- "parity unpinned" for p.  What IS checked (tests/test_solver.py):
the objective value -- the lambda_2 reached is within 1e-6 of an independent cutting-plane upper
bound on the optimum for graphs 0-5 x budgets 0.1-0.8; alpha is the global minimiser of its
convex 1-D reduction (dense grid); C_b = 1 gives p = 1 and alpha = FixedProcessor's
2/(lambda_2 + lambda_max); the spectral norms of ResearchReport.pdf Fig. 1(c) for graph 0.
"""
import numpy as np
import scipy.linalg
import scipy.optimize


def _complement_basis(n):
    return scipy.linalg.null_space(np.ones((1, n)))  # n x (n-1), orthonormal, orthogonal to 1


def lambda2(Lsum):
    w = np.linalg.eigvalsh(np.asarray(Lsum, dtype=np.float64))
    return float(w[1]) if w.shape[0] > 1 else 0.0


def matcha_probabilities(L_matrices, budget, tol=1e-10, max_newton=400):
    """Activation probabilities p (graph_manager.py:240-266), clipped to <= 1 as line 266.

    Primal log-barrier path following on (p, t):
        maximize t  s.t.  Z = sum_j p_j A_j - t I > 0,  0 < p < 1,  sum p < M*C_b
    with A_j = Q^T L_j Q.  Each centering step is a damped Newton method on
        F_mu(p, t) = -t - mu (log det Z + sum log p + sum log(1-p) + log(cap - sum p)),
    mu shrinks 10x per step until the barrier's duality-gap bound m*mu < tol.  Like CVXOPT's
    interior-point method this ends near the analytic centre of the optimal face when the
    optimum is not unique.
    """
    Ls = [np.asarray(L, dtype=np.float64) for L in L_matrices]
    M = len(Ls)
    if M == 0:
        return np.zeros(0)
    n = Ls[0].shape[0]
    cap = M * float(budget)
    if cap >= M:
        return np.ones(M)   # lambda_2 is nondecreasing in every p_j
    if cap <= 0:
        return np.zeros(M)
    Q = _complement_basis(n)
    A = np.stack([Q.T @ L @ Q for L in Ls])  # [M, k, k]
    k = A.shape[1]
    I = np.eye(k)

    def parts(p, t):
        Z = np.tensordot(p, A, axes=1) - t * I
        try:
            C = np.linalg.cholesky(Z)
        except np.linalg.LinAlgError:
            return None
        slack = cap - p.sum()
        if np.any(p <= 0) or np.any(p >= 1) or slack <= 0:
            return None
        return Z, C, slack

    def barrier_value(p, t, mu, pr):
        Z, C, slack = pr
        logdet = 2.0 * np.sum(np.log(np.diag(C)))
        return -t - mu * (logdet + np.sum(np.log(p)) + np.sum(np.log1p(-p)) + np.log(slack))

    p = np.full(M, min(0.5, 0.5 * cap / M))
    t = float(np.linalg.eigvalsh(np.tensordot(p, A, axes=1))[0]) - 1.0
    m_constraints = k + 2 * M + 1
    mu = 1.0
    newton_steps = 0
    while True:
        for _ in range(100):                      # centering
            pr = parts(p, t)
            Z, C, slack = pr
            Ci = scipy.linalg.solve_triangular(C, I, lower=True)            # C^-1
            B = np.matmul(np.matmul(Ci, A), Ci.T)                          # C^-1 A_j C^-T
            CC = Ci @ Ci.T
            Zi_tr = float(np.sum(Ci * Ci))                                  # tr(Z^-1)
            Zi2_tr = float(np.sum(CC * CC))                                 # tr(Z^-2)
            trB = np.trace(B, axis1=1, axis2=2)                             # tr(Z^-1 A_j)
            trBt = np.sum(B * CC, axis=(1, 2))                              # tr(Z^-1 A_j Z^-1)
            Bf = B.reshape(M, -1)
            g = np.empty(M + 1)
            g[:M] = -mu * (trB + 1.0 / p - 1.0 / (1.0 - p) - 1.0 / slack)
            g[M] = -1.0 + mu * Zi_tr
            H = np.empty((M + 1, M + 1))
            H[:M, :M] = mu * (Bf @ Bf.T
                              + np.diag(1.0 / p ** 2 + 1.0 / (1.0 - p) ** 2) + 1.0 / slack ** 2)
            H[:M, M] = H[M, :M] = -mu * trBt
            H[M, M] = mu * Zi2_tr
            step = -np.linalg.solve(H, g)
            dec = float(-g @ step)
            if dec / 2.0 <= 1e-12 * max(1.0, mu):
                break
            f0 = barrier_value(p, t, mu, pr)
            s = 1.0
            while True:
                pn, tn = p + s * step[:M], t + s * step[M]
                prn = parts(pn, tn)
                if prn is not None and barrier_value(pn, tn, mu, prn) <= f0 - 0.25 * s * dec:
                    break
                s *= 0.5
                if s < 1e-16:
                    break
            if s < 1e-16:
                break
            p, t = pn, tn
            newton_steps += 1
            if newton_steps >= max_newton:
                break
        if m_constraints * mu < tol or newton_steps >= max_newton:
            break
        mu *= 0.1
    return np.minimum(p, 1.0)


def spectral_norm(L_matrices, p, alpha):
    """rho = lambda_max(E[W^T W] - J) for W = I - alpha sum_j B_j L_j, B_j ~ Bernoulli(p_j)."""
    Ls = [np.asarray(L, dtype=np.float64) for L in L_matrices]
    n = Ls[0].shape[0]
    E = sum(pj * L for pj, L in zip(p, Ls))
    V = sum(pj * (1 - pj) * L for pj, L in zip(p, Ls))
    F = E @ E + 2 * V
    J = np.ones((n, n)) / n
    G = np.eye(n) - J - 2 * alpha * E + alpha * alpha * F
    return float(np.linalg.eigvalsh((G + G.T) / 2)[-1])


def matcha_alpha(L_matrices, p, tol=1e-13):
    """Mixing weight a of graph_manager.py:268-296 (returns float, like float(a.value))."""
    Ls = [np.asarray(L, dtype=np.float64) for L in L_matrices]
    n = Ls[0].shape[0]
    p = np.asarray(p, dtype=np.float64)
    E = sum(pj * L for pj, L in zip(p, Ls))
    V = sum(pj * (1 - pj) * L for pj, L in zip(p, Ls))
    F = E @ E + 2 * V
    J = np.ones((n, n)) / n
    I = np.eye(n)

    def s_of(a):
        G = I - J - 2 * a * E + a * a * F
        return float(np.linalg.eigvalsh((G + G.T) / 2)[-1])

    wE = np.linalg.eigvalsh(E)
    lam2 = float(wE[1]) if n > 1 else 0.0
    lam_max = float(wE[-1])
    if lam_max <= 0:
        return 0.0
    a_hi = 4.0 / max(lam2, 1e-3 * lam_max)
    res = scipy.optimize.minimize_scalar(s_of, bounds=(0.0, a_hi), method="bounded",
                                         options={"xatol": 1e-14, "maxiter": 2000})
    a = float(res.x)
    # golden-section polish around the Brent answer (the optimum is usually a kink)
    lo, hi = max(0.0, a - 1e-4 * a_hi), min(a_hi, a + 1e-4 * a_hi)
    g = (np.sqrt(5.0) - 1) / 2
    x1, x2 = hi - g * (hi - lo), lo + g * (hi - lo)
    f1, f2 = s_of(x1), s_of(x2)
    for _ in range(200):
        if hi - lo <= tol * max(1.0, a):
            break
        if f1 <= f2:
            hi, x2, f2 = x2, x1, f1
            x1 = hi - g * (hi - lo)
            f1 = s_of(x1)
        else:
            lo, x1, f1 = x1, x2, f2
            x2 = lo + g * (hi - lo)
            f2 = s_of(x2)
    cand = [(s_of(a), a), (min(f1, f2), x1 if f1 <= f2 else x2)]
    return float(min(cand)[1])
