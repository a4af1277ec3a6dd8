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


def certify(Pd, c, A, b, g_and_J, hh, x, act_tol=1e-5):
    """Returns dict(stat=||grad L||_inf, prim=max violation, eq=||Ax-b||_inf, zmin, nact)."""
    g, J = g_and_J(x)
    viol = np.maximum(g - hh, 0).max() if g.size else 0.0
    eq = np.abs(A @ x - b).max()
    act = np.where(hh - g < act_tol)[0]
    grad = Pd * x + c
    M = np.hstack([A.T, J[act].T])
    lb = np.r_[-np.inf * np.ones(A.shape[0]), np.zeros(act.size)]
    ub = np.inf * np.ones(M.shape[1])
    sol = lsq_linear(M, -grad, bounds=(lb, ub), method="bvls", tol=1e-14, max_iter=2000)
    res = M @ sol.x + grad
    return dict(stat=float(np.abs(res).max()), prim=float(viol), eq=float(eq),
                zmin=float(sol.x[A.shape[0]:].min()) if act.size else 0.0, nact=int(act.size))
