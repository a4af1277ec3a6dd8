"""Diagnostic: trace one agent's low-level CLF-QP interior-point iterations on the GPU
(srb_ll_debug_trace) next to status / iterations / x error of every agent vs the oracle.

    python tools/ll_trace.py CASE AGENT CLF      CASE = golden | rand:SEED | trot:SEED
Writes gpurun_out/ll_trace.npz (trace buffer + the case's inputs for offline replay)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import oracle  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import ll_workload, lowlevel  # noqa: E402


def make_case(case):
    if case == "golden":
        g = np.load(os.path.join(ROOT, "tests", "golden", "ll_ctrl.npz"), allow_pickle=False)
        return {k: g[k] for k in g.files}
    kind, seed = case.split(":")
    seed = int(seed)
    if kind == "rand":        # tests/test_ll_gpu.py::test_ll_gpu_matches_oracle_random_contacts
        rng = np.random.default_rng(1000 + seed)
        ind = rng.integers(0, 2, (96, 4)).astype(np.int32)
        ind[:6] = [[0, 0, 0, 0], [1, 1, 1, 1], [1, 0, 0, 0], [0, 1, 1, 1], [1, 0, 0, 1], [0, 1, 1, 0]]
        return ll_workload.make_batch(96, seed=200 + seed, ind=ind)
    return ll_workload.make_batch(256, seed=seed)


case = sys.argv[1] if len(sys.argv) > 1 else "golden"
agent = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dump_it = int(sys.argv[4]) if len(sys.argv) > 4 else 7
clf = int(sys.argv[3]) if len(sys.argv) > 3 else 1
g = make_case(case)
L = srbnmpc.lib()
L.srb_ll_debug_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.srb_ll_debug_trace(agent | (dump_it << 16), None)
c = srbnmpc.LowLevelCtrl(lowlevel.default_params(useCLF=clf), 512)
out = c.calc_torque(g)
tr = np.zeros(512)
L.srb_ll_debug_trace(-1, tr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
o = oracle.ll_calc_torque(oracle.ll_params(useCLF=clf), g)
bad = np.nonzero((out["status"] != o["status"]) | (out["iters"] != o["iters"]))[0]
print("mismatching agents", [(int(a), int(out["status"][a]), int(o["status"][a]), int(out["iters"][a]),
                              int(o["iters"][a])) for a in bad])
print("max xerr", float(np.abs(out["x"] - o["x"]).max()))
tr8 = tr[:256].reshape(32, 8)
for i in range(26):
    r = tr8[i]
    print(i, " ".join("%.3e" % v for v in [np.sqrt(r[0]), np.sqrt(r[1]), np.sqrt(r[2]), r[3], r[4], r[5], r[6], r[7]]))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "ll_trace.npz"), tr=tr, gx=out["x"], **{"in_" + k: v for k, v in g.items()})
