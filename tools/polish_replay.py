"""Diagnostic: replay the active-set polish (srb_polish_kernel / oracle polish) in numpy, full space,
from the state tools/nlp_trace.py dumped for a traced config-5 agent (gpurun_out/polish_in_<a>.npy:
the exported z / proximal weights per row slot, x at the start and after each Newton step), and
print the per-step |dx| next to the GPU's.  The reference point is the oracle's polished solution
(saved by the caller as gpurun_out/oracle_x_<a>.npy).
    python tools/polish_replay.py agent [rho] [zfirst]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd"), os.path.join(ROOT, "tests")]
import oracle
from srbnmpc import workload
import srbnmpc
a = int(sys.argv[1]); rho = float(sys.argv[2]) if len(sys.argv) > 2 else 1e9
N, C, Ko, Kn = 20, 2, 3, 8
K = Ko + Kn
b = workload.make_batch(2048, N, C, seed=1234)
op = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
obs, eps = oracle.select_obstacles(op, b["x0"][a], b["obstacles"], b["nbr_state"], a)
Pd, c, Aeq, beq, G, h = oracle.build_qp(op, b["x0"][a], b["ref"][a], b["foot"][a])
n = Pd.size
p = srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn)
d = np.load(os.path.join(ROOT, "gpurun_out", f"polish_in_{a}.npy"))
zp = d[:1024]; x = d[1024:1024 + n].copy()
xg = [d[1280 + 256 * i:1280 + 256 * i + n] for i in range(3)]
xo_path = os.path.join(ROOT, "gpurun_out", f"oracle_x_{a}.npy")
if not os.path.exists(xo_path):
    r = oracle.solve_batch(op, b["x0"][a:a + 1], b["ref"][a:a + 1], b["foot"][a:a + 1], b["obstacles"], b["nbr_state"],
                           agent_offset=a, nthreads=1)
    np.save(xo_path, r["x"][0])
xo = np.load(xo_path)
NE = 2 * (N - 1); sE = n; sV = n + NE; sO = sV + 2 * N; S = sO + N * K
# slot rows: list of (func(x)->(g, grad, hess-diag-on-positions?), h, exported value)
rows = []
for sl in range(S):
    for r in range(2):
        v = zp[2 * sl + r]
        if sl < sE:
            i0 = sl; isL = 6 * N <= sl < n - 1
            if sl == n - 1: hv = (p.box, p.box)   # slack var
            hv = (1.0, 0.0) if isL else (p.box, p.box)
            if sl == n - 1: m = (0, 0)   # slack var has no box? (lin only for i0 < n-1)
            else: m = (1, 1)
            def f(x, i0=i0): e = np.zeros(n); e[i0] = 1; return x[i0], e, None
            kind = "VAR"
        elif sl < sV:
            e_ = sl - sE; i = e_ >> 1; dd = e_ & 1
            i0 = 4 * i + 2 * dd; i1 = 4 * N + 2 * (i + 1) + dd
            def f(x, i0=i0, i1=i1): e = np.zeros(n); e[i0] = 1; e[i1] = -1; return x[i0] - x[i1], e, None
            FR = p.mu * p.hcom / np.sqrt(2); hv = (FR, FR); m = (1, 1); kind = "COP"
        elif sl < sO:
            tt = sl - sV; comp = 1 if tt < N else 3; k = tt % N; i0 = 4 * k + comp
            def f(x, i0=i0): e = np.zeros(n); e[i0] = 1; return x[i0], e, None
            hv = (p.vsat, p.vsat); m = (1, 1); kind = "VEL"
        else:
            o = sl - sO; k = o // K; j = o % K
            def f(x, k=k, j=j):
                dx = x[4 * k] - obs[k, j, 0]; dy = x[4 * k + 2] - obs[k, j, 1]
                e = np.zeros(n); e[4 * k] = -2 * dx; e[4 * k + 2] = -2 * dy; e[-1] = -1
                return -(dx * dx + dy * dy) - x[-1], e, k
            hv = (-eps[j], 0); m = (1, 0); kind = "OBS"
        if not m[r]: continue
        sg = 1 if r == 0 else -1
        rows.append((f, sg, hv[r], v, kind, sl))
act = [i for i, R in enumerate(rows) if R[3] > 0]
print("active", [(rows[i][4], rows[i][5], round(rows[i][3], 3)) for i in act])
z = np.array([rows[i][3] for i in act])
om = np.array([(-R[3] if R[3] < 0 else 0.0) for R in rows])
use_om = True
for it in range(4):
    H = np.diag(Pd).astype(float); gr = Pd * x + c
    cA = np.zeros(len(act)); JA = np.zeros((len(act), n))
    for ii, i in enumerate(act):
        f, sg, hv, v, kind, sl = rows[i]
        gv, e, k = f(x)
        cA[ii] = sg * gv - hv; JA[ii] = sg * e
        if kind == "OBS": H[4 * k, 4 * k] -= 2 * z[ii]; H[4 * k + 2, 4 * k + 2] -= 2 * z[ii]
    if use_om:
        for i, R in enumerate(rows):
            if om[i] > 0:
                gv, e, k = R[0](x); H += om[i] * np.outer(e, e)
    H += rho * JA.T @ JA
    rhs = -(gr + JA.T @ (z + rho * cA))
    p_ = Aeq.shape[0]
    KK = np.block([[H, Aeq.T], [Aeq, np.zeros((p_, p_))]])
    sol = np.linalg.solve(KK, np.concatenate([rhs, beq - Aeq @ x]))
    dx = sol[:n]
    z = z + rho * (cA + JA @ dx)
    if it == 0 and "zfirst" in sys.argv:
        print(f"  z-only step: |dx| would be {np.abs(dx).max():.3e}"); continue
    x = x + dx
    print(f"numpy(gpu z) step {it}: |dx| {np.abs(dx).max():.3e}  vs oracle {np.abs(x - xo).max():.3e}  |cA| {np.abs(cA).max():.2e}")
for i in range(3):
    print(f"gpu step {i}: vs oracle {np.abs(xg[i] - xo).max():.3e}")
