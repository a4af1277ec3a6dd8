"""Calibrate the CPU baseline (bench.py cpu_baseline, the oracle's dense-LU restatement)
against the genuine vendored iSWIFT (oracle/_ref, compiled from
/root/reference/optimization/iSWIFT/src/{Prime,Auxilary,timer}.c + ldl/src/ldl.c) on the
same QP-stage instances, one thread each ("the ratio own-CPU/iSWIFT is
recorded with the fixtures").  Runs in the build container, where oracle/_ref exists.

    python tools/calibrate_cpu.py [out.json]     (default profiles/r02_cpu_calibration.json)

iSWIFT time = its own tic/toc of QP_SETUP + QP_SOLVE (Prime.c:37-120, 128-230), i.e. the
reference solver alone, without the Eigen wrapper's dense->CCS copy and AMD ordering
(iswift_qp.cpp:164-210) that the reference pays on every call -- so the ratio is the
least favourable one for the oracle.  Oracle time = wall time of orc_qp_solve per call.
"""
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))
import oracle  # noqa: E402
from srbnmpc import workload  # noqa: E402

CASES = [(4, 4, 64), (10, 2, 64), (10, 4, 32), (20, 2, 32)]


def iswift_times(P, c, A, b, G, h):
    """(x, flag, iters, t_setup + t_solve seconds) of the genuine iSWIFT, min-degree ordering."""
    R = oracle.ref_lib()
    n, m, pp = P.shape[0], G.shape[0], A.shape[0]
    x = np.zeros(n); it = ctypes.c_int(); ts = ctypes.c_double(); tv = ctypes.c_double()
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (P, c, A, b, G, h)]
    f = R.iswift_ref_solve(n, m, pp, *[a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for a in arrs],
                           x.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(it), ctypes.byref(ts),
                           ctypes.byref(tv))
    return x, f, it.value, ts.value + tv.value


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02_cpu_calibration.json")
    if not oracle.ref_available():
        sys.exit("oracle/_ref not built (make -C oracle ref, needs /root/reference)")
    res = {"what": "QP stage, one thread: oracle (dense LU on the full-space KKT) vs the genuine iSWIFT "
                   "(sparse LDL', min-degree ordering) on identical instances; iSWIFT timed by its own "
                   "tic/toc around QP_SETUP + QP_SOLVE",
           "host": platform.processor() or platform.machine(), "cases": {}}
    for N, C, n_inst in CASES:
        b = workload.make_batch(n_inst, N, C, seed=100 + N + C)
        p = oracle.params(N, C)
        t_isw, t_orc, agree, its = [], [], 0.0, []
        for a in range(n_inst):
            Pd, c, A, bb, G, h = oracle.build_qp(p, b["x0"][a], b["ref"][a], b["foot"][a])
            P = np.diag(Pd)
            reps = 5
            best = 1e9
            for _ in range(reps):
                x_r, f_r, it_r, t = iswift_times(P, c, A, bb, G, h)
                best = min(best, t)
            t_isw.append(best)
            best = 1e9
            for _ in range(reps):
                t0 = time.perf_counter()
                x_o, f_o, it_o, _ = oracle.qp_solve(Pd, c, A, bb, G, h)
                best = min(best, time.perf_counter() - t0)
            t_orc.append(best)
            its.append((it_r, it_o))
            agree = max(agree, float(np.abs(np.r_[x_o[:6 * N], x_o[-1:]] - np.r_[x_r[:6 * N], x_r[-1:]]).max()))
        its = np.array(its)
        iu, ou = 1e6 * float(np.median(t_isw)), 1e6 * float(np.median(t_orc))
        res["cases"][f"N{N}_C{C}"] = {
            "N": N, "C": C, "instances": n_inst, "iswift_us": iu, "oracle_us": ou, "oracle_over_iswift": ou / iu,
            "iswift_iters_mean": float(its[:, 0].mean()), "oracle_iters_mean": float(its[:, 1].mean()),
            "max_abs_diff_XUs": agree}
        print(f"N={N} C={C}: iSWIFT {iu:.0f} us, oracle {ou:.0f} us, ratio {ou / iu:.2f}, "
              f"iters {its[:, 0].mean():.2f}/{its[:, 1].mean():.2f}, |dx| {agree:.1e}", flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
