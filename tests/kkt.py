"""Solver-independent KKT certificate for the NMPC problems (numpy/scipy only).

Used by tests/ and tests/golden/make_goldens.py to pin NLP-stage results without
trusting any particular solver: given x*, it checks primal feasibility and finds
multipliers (y free, z >= 0 on the near-active rows) minimising the stationarity
residual of  grad f + A'y + J'z = 0.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import lsq_linear


def nlp_rows(N, C, nv, G, h, obs, eps, vsat):
    """Full row set of the NLP stage in the oracle/kernel order:
    [QP rows | obstacle rows k*K+j | +xdot, +ydot, -xdot, -ydot]; returns g(x), J(x), hh."""
    K = obs.shape[1]

    def g_and_J(x):
        rows = [G @ x]
        J = [G]
        go = np.zeros(N * K); Jo = np.zeros((N * K, nv))
        for k in range(N):
            for j in range(K):
                r = k * K + j
                dx = x[4 * k] - obs[k, j, 0]; dy = x[4 * k + 2] - obs[k, j, 1]
                go[r] = -(dx * dx + dy * dy) - x[-1]
                Jo[r, 4 * k] = -2 * dx; Jo[r, 4 * k + 2] = -2 * dy; Jo[r, -1] = -1
        Gv = np.zeros((4 * N, nv))
        r = 0
        for sg in (1, -1):
            for comp in (1, 3):
                for k in range(N):
                    Gv[r, 4 * k + comp] = sg; r += 1
        rows += [go, Gv @ x]; J += [Jo, Gv]
        return np.concatenate(rows), np.vstack(J)

    hh = np.concatenate([h, -np.repeat(np.asarray(eps)[None], N, 0).ravel(), vsat * np.ones(4 * N)])
    return g_and_J, hh


def certify(Pd, c, A, b, g_and_J, hh, x, act_tol=1e-3, comp_tol=1e-3):
    """KKT certificate at x.  Candidate rows: slack h - g(x) < act_tol; multipliers y (free)
    and 0 <= z_i <= comp_tol / slack_i on them (so complementarity z_i * slack_i <= comp_tol,
    the per-row size an IPM exit at mean s.z < 1e-6 over ~300 rows allows,
    holds by construction) minimise ||grad f + A'y + J'z||_2 (bounded least squares).
    Returns stat (abs residual, inf-norm), stat_rel (stat / max(1, |grad f|, |A'y|, |J'z|)),
    comp = max_i z_i * slack_i (complementarity of the certificate's own multipliers),
    prim (max row violation), eq (|Ax - b|), zmin, nact."""
    g, J = g_and_J(x)
    slack = hh - g
    viol = float(np.maximum(-slack, 0).max()) if g.size else 0.0
    eq = float(np.abs(A @ x - b).max())
    act = np.where(slack < act_tol)[0]
    grad = Pd * x + c
    M = np.hstack([A.T, J[act].T])
    lb = np.r_[-np.inf * np.ones(A.shape[0]), np.zeros(act.size)]
    ub = np.r_[np.inf * np.ones(A.shape[0]),
               np.where(slack[act] > 1e-12, comp_tol / np.maximum(slack[act], 1e-300), np.inf)]
    sol = lsq_linear(M, -grad, bounds=(lb, ub), method="bvls", tol=1e-14, max_iter=5000)
    res = M @ sol.x + grad
    y = sol.x[:A.shape[0]]; z = sol.x[A.shape[0]:]
    scale = max(1.0, float(np.abs(grad).max()), float(np.abs(A.T @ y).max()),
                float(np.abs(J[act].T @ z).max()) if act.size else 0.0)
    stat = float(np.abs(res).max())
    comp = float((z * np.maximum(slack[act], 0)).max()) if act.size else 0.0
    return dict(stat=stat, stat_rel=stat / scale, comp=comp, prim=viol, eq=eq,
                zmin=float(z.min()) if act.size else 0.0, nact=int(act.size))


def qp_exact_optimum(Pd, c, A, b, G, h, x_start, act_tol=1e-5, max_changes=20):
    """Exact optimum of the convex QP  min 0.5 x'diag(Pd)x + c'x  s.t. Ax = b, Gx <= h  by a
    primal-dual active-set iteration started from the rows within act_tol of their bound at
    x_start: the equality-constrained optimum of [A; G_act] on its null space (least squares
    where lambda is not unique, C = 4), multipliers by bounded least squares (y free, z >= 0),
    then drop / add rows until z >= 0 fits exactly and every row holds.  Returns (x*, y, z)."""
    from scipy.optimize import lsq_linear
    act = np.where(G @ x_start - h > -act_tol)[0]
    P = np.diag(Pd)
    for _ in range(max_changes):
        M = np.vstack([A, G[act]])
        r = np.r_[b, h[act]]
        _, S, Vt = np.linalg.svd(M)
        rank = int((S > 1e-10 * S[0]).sum())
        Zn = Vt[rank:].T
        xp = np.linalg.lstsq(M, r, rcond=None)[0]
        xs = xp - Zn @ np.linalg.lstsq(Zn.T @ P @ Zn, Zn.T @ (P @ xp + c), rcond=1e-13)[0]
        grad = P @ xs + c
        lb = np.r_[-np.inf * np.ones(A.shape[0]), np.zeros(act.size)]
        sol = lsq_linear(M.T, -grad, bounds=(lb, np.inf * np.ones(M.shape[0])), method="bvls", tol=1e-14)
        res = np.abs(M.T @ sol.x + grad).max()
        viol = G @ xs - h
        if res > 1e-7 * max(1.0, np.abs(grad).max()):
            m2 = np.linalg.lstsq(M.T, -grad, rcond=None)[0][A.shape[0]:]
            act = np.delete(act, np.argmin(m2))
            continue
        if viol.max() > 1e-9:
            act = np.union1d(act, np.where(viol > 1e-9)[0])
            continue
        z = np.zeros(G.shape[0])
        z[act] = sol.x[A.shape[0]:]
        return xs, sol.x[:A.shape[0]], z
    raise RuntimeError("qp_exact_optimum: active set did not settle")


def l1_merit(Pd, c, A, b, G, h, x, y, z):
    """Exact l1-penalty merit with the optimal multipliers (|y|, z): minimised by the optimum
    and >= f(x*) at every point, feasible or not -- a fair 'how optimal' measure for two
    approximate solutions with different residuals."""
    return 0.5 * Pd @ (x * x) + c @ x + np.abs(y) @ np.abs(A @ x - b) + z @ np.maximum(G @ x - h, 0)
