"""Diagnostic: per-iteration NLP trace of chosen agents of a bench configuration's batch
(libsrbnmpc_nlpdbg.so, make -C srb-cbf-nmpc_amd nlpdbg).

    python tools/nlp_trace.py config agent [agent ...]
    NLPTRACE_SPEC="N C K_obs K_nbr agents seed" python tools/nlp_trace.py custom agent ...
    (NLPTRACE_WAVES forces the waves per agent)"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

srbnmpc.use_library("libsrbnmpc_nlpdbg.so")
if sys.argv[1] == "custom":     # NLPTRACE_SPEC="N C K_obs K_nbr agents seed" (workload.make_batch)
    N, C, Ko, Kn, A, seed = map(int, os.environ["NLPTRACE_SPEC"].split())
    cfg = dict(N=N, C=C, K_obs=Ko, K_nbr=Kn, agents=A)
    b = workload.make_batch(A, N, C, seed=seed)
else:
    c = int(sys.argv[1])
    cfg = bench.CONFIGS[c]
    A, N, C = cfg["agents"], cfg["N"], cfg["C"]
    A, b, _, _ = bench.rank_batch(c, A, 1, 0)
p = srbnmpc.default_params(N, C, K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=1)
s = srbnmpc.BatchSolver(p, A)
p_n = p.nv
s.set_waves(int(os.environ.get("NLPTRACE_WAVES", "0")))
L = srbnmpc.lib()
L.srb_debug_nlp_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
buf = np.zeros(8 * 64 + 32 * 32 + 32 + 1024 + 256 + 3 * 256)
for ag in map(int, sys.argv[2:]):
    L.srb_debug_nlp_trace(ag, None)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"] if cfg["K_nbr"] else None)
    L.srb_debug_nlp_trace(-1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    print(f"agent {ag}: status {out['status'][ag].tolist()} iters {out['iters'][ag].tolist()}")
    print("  it     |rx|        thx        |rz|       s'z/m      ap        ad        delta     sigma")
    for i in range(min(int(out["iters"][ag, 1]) + 1, 56)):
        r = buf[8 * i:8 * i + 8]
        print(f"  {i:2d} " + " ".join(f"{v:10.3e}" for v in r), flush=True)
    print("  polish pass: primal     |c_A|     -min z_A   max|z_A|   inact.viol  last|dx|   accepted   eq.resid")
    for p in range(4):
        r = buf[8 * (56 + p):8 * (56 + p) + 8]
        if r.any():
            print(f"  {p:2d}          " + " ".join(f"{v:10.3e}" for v in r[:8]), flush=True)
            print("      Newton |dx|: " + " ".join(f"{v:10.3e}" for v in buf[8 * (60 + p):8 * (60 + p) + 8] if v), flush=True)
    import oracle
    op = oracle.params(N, C, K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"])
    Ad, Bd = oracle.lip(op)
    for it in range(3):
        xs = buf[2848 + 256 * it:2848 + 256 * it + p_n]
        if not xs.any():
            continue
        X = xs[:4 * N].reshape(N, 4); U = xs[4 * N:6 * N].reshape(N, 2); Lm = xs[6 * N:6 * N + C * N].reshape(N, C)
        F = b["foot"][ag].reshape(N, 2, C)
        prev, res = b["x0"][ag], []
        for k in range(N):
            res.append(max(np.abs(X[k] - Ad @ prev - Bd @ U[k]).max(), np.abs(U[k] - F[k] @ Lm[k]).max(), abs(Lm[k].sum() - 1)))
            prev = X[k]
        print(f"  pass 0 Newton step {it}: host equality residual of x {max(res):.3e} (per grid " +
              " ".join(f"{v:.1e}" for v in res) + ")", flush=True)
    nzr = int((np.abs(buf[512 + 32 * np.arange(32) + np.arange(32)]) > 0).sum())
    if nzr:
        Hm = buf[512:512 + 1024].reshape(32, 32)[:nzr, :nzr]
        ev = np.linalg.eigvalsh(0.5 * (Hm + Hm.T))
        print(f"  polish reduced matrix (pass 0, step 0): nz {nzr}  asym {np.abs(Hm - Hm.T).max():.3e}  "
              f"eig min {ev[0]:.6e} max {ev[-1]:.6e}  diag min {np.diag(Hm).min():.3e}", flush=True)
        np.save(os.path.join("gpurun_out", f"polish_H_{ag}.npy"), np.concatenate([Hm.ravel(), buf[512 + 1024:512 + 1024 + nzr]]))
        np.save(os.path.join("gpurun_out", f"polish_in_{ag}.npy"), buf[1568:])
