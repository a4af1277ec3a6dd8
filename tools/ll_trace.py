"""Diagnostic: trace one agent's low-level CLF-QP interior-point iterations on the GPU
(srb_ll_debug_trace) next to status / iterations / x error of every agent vs the oracle."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import oracle  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import lowlevel  # noqa: E402

agent = int(sys.argv[1]) if len(sys.argv) > 1 else 2
clf = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = np.load(os.path.join(ROOT, "tests", "golden", "ll_ctrl.npz"), allow_pickle=False)
g = {k: g[k] for k in g.files}
L = srbnmpc.lib()
L.srb_ll_debug_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.srb_ll_debug_trace(agent, None)
c = srbnmpc.LowLevelCtrl(lowlevel.default_params(useCLF=clf), 64)
out = c.calc_torque(g)
tr = np.zeros(512)
L.srb_ll_debug_trace(-1, tr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
o = oracle.ll_calc_torque(oracle.ll_params(useCLF=clf), g)
print("status gpu", out["status"].tolist(), "oracle", o["status"].tolist())
print("iters  gpu", out["iters"].tolist(), "oracle", o["iters"].tolist())
print("xerr", np.abs(out["x"] - o["x"]).max(axis=1).tolist())
for k in ("tau", "QP_force", "ddq", "dq", "q", "V", "dV"):
    print(k, float(np.abs(out[k] - o[k]).max()))
tr8 = tr[:256].reshape(32, 8)
for i in range(min(26, 32)):
    r = tr8[i]
    print(i, " ".join("%.3e" % v for v in [np.sqrt(r[0]), np.sqrt(r[1]), np.sqrt(r[2]), r[3], r[4], r[5], r[6], r[7]]))
p = oracle.ll_params(useCLF=clf)
for a in range(out["x"].shape[0]):
    Pd, cc, A, b, G, h, *_ = oracle.ll_build_qp(p, g, a)
    n = Pd.size
    x = out["x"][a, :n]
    xo = o["x"][a, :n]
    print(a, "n", n, "|Ax-b| %.2e  max(Gx-h) %.2e  obj %.6f  oracle: |Ax-b| %.2e max(Gx-h) %.2e obj %.6f" % (
        np.abs(A @ x - b).max(), (G @ x - h).max(), 0.5 * x @ (Pd * x) + cc @ x,
        np.abs(A @ xo - b).max(), (G @ xo - h).max(), 0.5 * xo @ (Pd * xo) + cc @ xo))
    if out["status"][a] != o["status"][a]:
        print("   gpu x", np.round(x, 4).tolist())
        print("   orc x", np.round(xo, 4).tolist())

np.save(os.path.join(ROOT, "gpurun_out", "ll_trace_init.npy"), tr[200:250])
print("init x", np.round(tr[200:231], 5).tolist())
print("init y", np.round(tr[232:250], 5).tolist())
np.save(os.path.join(ROOT, "gpurun_out", "ll_trace_rx0.npy"), tr[300:331])
print("rx0", np.round(tr[300:331], 4).tolist())
np.save(os.path.join(ROOT, "gpurun_out", "ll_trace_all.npy"), tr)
