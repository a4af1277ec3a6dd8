"""Generate the committed golden fixtures (run in the survey container, which has
/root/reference and oracle/_ref built from it):

    make -C oracle all ref && python tests/golden/make_goldens.py [ll | nlp]

Fixtures written (data only -- inputs and expected outputs):
  kat1.json           iSWIFT's bundled test QP (optimization/iSWIFT/include/Matrices_small.h,
                      its CCS arrays and its own KKT permutation) + the genuine iSWIFT solution
  kat2.json           the reference's logged NLP instance reconstructed from print_file.out
                      (x0, reference, footholds, closest obstacle), the reference's own logged
                      QP-stage output (SNOPT start point, print_file.out:30-54) and SNOPT's final
                      point, plus the genuine-iSWIFT QP solution and the KKT-certified NLP optimum
  qp_random.json      seeded instances (N, C in {4,10,20} x {2,4}) with genuine-iSWIFT solutions
  qp_iswift_md.npz    64 instances per (N, C) in {(4,4),(4,2),(10,2),(10,4),(20,2)}: genuine iSWIFT
                      under a minimum-degree ordering (the reference's AMD stand-in) and the
                      quasi-definite one, the oracle's point, flags / iterations / KKT quality
                      (python tests/golden/make_goldens.py qpmd)
  nlp_random.json     seeded N=10 trot instances, K_obs = 3: KKT-certified NLP optimum (oracle),
                      with SciPy SLSQP's objective from the same warm start for comparison
  ll_ctrl.npz         low-level CLF-QP (LowLevelCtrl::calcTorque) inputs for 8 agents with
                      contact sets trot / stand / three legs / flight, and the genuine-iSWIFT
                      solution of each agent's QP with and without the CLF row
                      (numpy .npz, plain arrays, loads with allow_pickle=False)
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from kkt import certify, nlp_rows  # noqa: E402
from srbnmpc import workload, ll_workload  # noqa: E402  (pure numpy generators; no GPU needed)

REF = "/root/reference"


def dump(name, obj):
    def conv(o):
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, (np.floating,)):
            return float(o)
        if isinstance(o, (np.integer,)):
            return int(o)
        raise TypeError(type(o))
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, default=conv, indent=None, separators=(",", ":"))
    print("wrote", name)


# ----------------------------------------------------------------------------- KAT-1
def kat1():
    txt = open(f"{REF}/optimization/iSWIFT/include/Matrices_small.h").read()
    arrs = {}
    for m in re.finditer(r"(realqp|idxint)\s+(\w+)\[(\d+)\]\s*=\s*\{([^}]*)\}", txt):
        typ, name, cnt, body = m.groups()
        vals = [float(v) for v in body.replace("\n", "").split(",") if v.strip()]
        assert len(vals) == int(cnt), name
        arrs[name] = np.array(vals, dtype=np.int64 if typ == "idxint" else np.float64)
    dims = {k: int(v) for k, v in re.findall(r"idxint\s+(n|m|p)\s*=\s*(\d+);", txt)}
    n, m, p = dims["n"], dims["m"], dims["p"]
    x, flag, it = oracle.iswift_ref_ccs(n, m, p, arrs["Pjc"], arrs["Pir"], arrs["Ppr"], arrs["Ajc"], arrs["Air"],
                                        arrs["Apr"], arrs["Gjc"], arrs["Gir"], arrs["Gpr"], arrs["c"], arrs["h"],
                                        arrs["b"], arrs["P"])
    out = dict(n=n, m=m, p=p, x_iswift=x, flag=flag, iters=it,
               **{k: arrs[k] for k in ("Pjc", "Pir", "Ppr", "Ajc", "Air", "Apr", "Gjc", "Gir", "Gpr", "c", "h", "b", "P")})
    dump("kat1.json", out)


# ----------------------------------------------------------------------------- KAT-2
def parse_print_file():
    lines = open(f"{REF}/print_file.out").read().splitlines()
    start = {}
    for ln in lines:
        m = re.match(r"\s+(\d+)\s+([-\d.E+]+)\s+([-\d.E+]+)\s+([-\d.E+]+)\s+([-\d.E+]+)\s+(ok|bad\?)", ln)
        if m:
            start[int(m.group(1))] = (float(m.group(2)), float(m.group(4)))
    final = {}
    rowval = {}
    states = {"BS", "SBS", "EQ", "LL", "UL", "FR", "FX", "BS"}
    for ln in lines:
        t = ln.split()
        if len(t) < 5 or t[1] not in ("r", "x") or not t[0].isdigit() or not t[2].isdigit():
            continue
        i = 3
        while t[i] not in states:      # skip single-letter flags (A, D, N)
            i += 1
        v = t[i + 1]
        val = 0.0 if v == "." else float(v)
        (rowval if t[1] == "r" else final)[int(t[2])] = val
    obj = float(re.search(r"Objective Value\s+([-\d.E+]+)", "\n".join(lines)).group(1))
    return start, final, rowval, obj


def kat2():
    start, final, rowval, snopt_obj = parse_print_file()
    xs = np.array([start[j][0] for j in range(1, 25)])
    gs = np.array([start[j][1] for j in range(1, 25)])
    N, C = 4, 4
    p = oracle.params(N, C)
    Ad, Bd = oracle.lip(p)
    Qd = np.r_[300.0 * np.ones(12), 2000.0 * np.ones(4)]
    ref = xs[:16] - gs[:16] / Qd                                  # f_j = g_j - Q_jj x_j = -Q_jj ref_j
    x0 = np.linalg.solve(Ad, xs[0:4] - Bd @ xs[16:18])            # X_0 = Ad x0 + Bd U_0
    F = np.array([[0.2188, 0.2188, -0.1472, -0.1472], [-0.1320, 0.1320, -0.1320, 0.1320]])  # default stance at origin
    xf = np.array([final[j] for j in range(1, 42)])
    # closest obstacle: least squares on the 4 logged obstacle-row values d^2 + s (rows 122-125)
    dvals = np.array([rowval[r] for r in (122, 123, 124, 125)]) - xf[40]
    P = np.array([[xf[4 * k], xf[4 * k + 2]] for k in range(4)])
    # nonlinear least squares in (o_x, o_y): |p_k - o|^2 = d_k  (4 rows, 2 unknowns)
    from scipy.optimize import least_squares
    fit = least_squares(lambda o: ((P - o) ** 2).sum(1) - dvals, x0=np.array([1.0, -0.5]), xtol=1e-15, ftol=1e-15)
    obst = fit.x
    foot = np.repeat(F[None], N, 0)
    Pd, c, A, b, G, h = oracle.build_qp(p, x0, ref, foot)
    xq_qd, fq, iq = oracle.iswift_ref(Pd, c, A, b, G, h, "qd")
    xq_md, fm, im = oracle.iswift_ref(Pd, c, A, b, G, h, "md")
    obs = np.tile(obst, (N, 1, 1)); eps = np.array([p.eps_obs])
    xn, fn, itn = oracle.nlp_solve(p, x0, foot, Pd, c, A, b, G, h, obs, eps, xq_qd)
    gJ, hh = nlp_rows(N, C, p.N * 10 + 1, G, h, obs, eps, p.vsat)
    cert = certify(Pd, c, A, b, gJ, hh, xn)
    obj_nlp = 0.5 * Pd @ (xn * xn) + c @ xn
    obj_snopt_x = 0.5 * Pd @ (xf * xf) + c @ xf
    sl = slsqp(Pd, c, A, b, gJ, hh, xq_qd)
    out = dict(N=N, C=C, x0=x0, ref=ref, F=F, obstacle=obst, obstacle_fit_residual=float(np.abs(fit.fun).max()),
               logged_qp_x=xs, logged_qp_grad=gs, logged_qp_s=start[41][0],
               snopt_final_x=xf, snopt_obj_logged=snopt_obj, snopt_obj_recomputed=obj_snopt_x,
               x_qp_iswift_qd=xq_qd, iters_qp_qd=iq, flag_qp_qd=fq, x_qp_iswift_md=xq_md, iters_qp_md=im, flag_qp_md=fm,
               x_nlp=xn, flag_nlp=fn, iters_nlp=itn, obj_nlp=obj_nlp, kkt=cert, slsqp_obj=sl[1])
    print("KAT-2: |QP - logged| =", np.abs(xq_qd[:24] - xs).max(), "NLP obj", obj_nlp, "SNOPT obj", snopt_obj, "cert", cert)
    dump("kat2.json", out)


def slsqp(Pd, c, A, b, gJ, hh, x_start):
    import scipy.optimize as so
    cons = [dict(type="eq", fun=lambda x: A @ x - b, jac=lambda x: A),
            dict(type="ineq", fun=lambda x: hh - gJ(x)[0], jac=lambda x: -gJ(x)[1])]
    r = so.minimize(lambda x: 0.5 * Pd @ (x * x) + c @ x, x_start, jac=lambda x: Pd * x + c, constraints=cons,
                    method="SLSQP", options=dict(ftol=1e-15, maxiter=3000))
    return r.x, float(r.fun)


# ----------------------------------------------------------------------------- random QP
def qp_random():
    cases = []
    for (N, C, cnt) in [(4, 4, 6), (4, 2, 6), (10, 2, 10), (10, 4, 4), (20, 2, 4)]:
        b = workload.make_batch(cnt, N, C, seed=1000 + 10 * N + C)
        p = oracle.params(N, C)
        for a in range(cnt):
            Pd, c, A, bb, G, h = oracle.build_qp(p, b["x0"][a], b["ref"][a], b["foot"][a])
            x, f, it = oracle.iswift_ref(Pd, c, A, bb, G, h, "qd")
            xm, fm, im = oracle.iswift_ref(Pd, c, A, bb, G, h, "md")
            cases.append(dict(N=N, C=C, x0=b["x0"][a], ref=b["ref"][a], foot=b["foot"][a], x=x, flag=f, iters=it,
                              x_md=xm, flag_md=fm, iters_md=im))
    dump("qp_random.json", dict(cases=cases))


# ----------------------------------------------------------------------------- QP stage vs the reference's ordering
QPMD_CASES = [(4, 4), (4, 2), (10, 2), (10, 4), (20, 2)]


def qp_point_quality(Pd, c, A, b, G, h, x):
    """KKT quality of a QP-stage point: objective, |Ax - b|_inf, max(Gx - h, 0), and the
    relative stationarity of the best multipliers on its near-active rows (tests/kkt.certify)."""
    cert = certify(Pd, c, A, b, lambda v: (G @ v, G), h, x)
    return [0.5 * Pd @ (x * x) + c @ x, cert["eq"], cert["prim"], cert["stat_rel"]]


def qp_md():
    """qp_iswift_md.npz: 64 bench-distribution instances per (N, C) solved by the genuine iSWIFT
    with a minimum-degree KKT ordering (the reference's iswift_qp.cpp:184-210 orders with Eigen's
    AMD, which is absent: a plain minimum-degree order stands in, oracle/iswift_ref_driver.c) and
    with the quasi-definite order the qp_random.json goldens use, next to the oracle's point (the
    GPU's algorithm, oracle/qp_ipm.c); flags, iterations and a KKT quality row per point."""
    out = {}
    for N, C in QPMD_CASES:
        b = workload.make_batch(64, N, C, seed=5000 + 10 * N + C)
        p = oracle.params(N, C)
        rec = {k: [] for k in ("x_md", "flag_md", "iters_md", "q_md", "x_qd", "flag_qd", "iters_qd", "q_qd",
                               "x_orc", "flag_orc", "iters_orc", "q_orc")}
        for a in range(64):
            Pd, c, A, bb, G, h = oracle.build_qp(p, b["x0"][a], b["ref"][a], b["foot"][a])
            for tag, (x, f, it) in (("md", oracle.iswift_ref(Pd, c, A, bb, G, h, "md")),
                                    ("qd", oracle.iswift_ref(Pd, c, A, bb, G, h, "qd")),
                                    ("orc", oracle.qp_solve(Pd, c, A, bb, G, h)[:3])):
                rec["x_" + tag].append(x); rec["flag_" + tag].append(f); rec["iters_" + tag].append(it)
                rec["q_" + tag].append(qp_point_quality(Pd, c, A, bb, G, h, x))
        key = f"N{N}_C{C}_"
        out[key + "x0"] = b["x0"]; out[key + "ref"] = b["ref"]; out[key + "foot"] = b["foot"]
        for k, v in rec.items():
            out[key + k] = np.asarray(v)
        d = np.abs(np.asarray(rec["x_orc"]) - np.asarray(rec["x_md"]))
        d = np.concatenate([d[:, :6 * N], d[:, -1:]], 1).max(1)
        print(f"N={N} C={C}: iters md {np.mean(rec['iters_md']):.2f} qd {np.mean(rec['iters_qd']):.2f} "
              f"oracle {np.mean(rec['iters_orc']):.2f}; |x_orc - x_md| (X,U,s) max {d.max():.2e}; "
              f"flags md {np.bincount(rec['flag_md'])}")
    np.savez_compressed(os.path.join(HERE, "qp_iswift_md.npz"), **out)
    print("wrote qp_iswift_md.npz")


# ----------------------------------------------------------------------------- random NLP
def nlp_random():
    cases = []
    N, C, K = 10, 2, 3
    b = workload.make_batch(12, N, C, seed=2024)
    p = oracle.params(N, C, K_obs=K)
    for a in range(12):
        x0, ref, foot = b["x0"][a], b["ref"][a], b["foot"][a]
        Pd, c, A, bb, G, h = oracle.build_qp(p, x0, ref, foot)
        xq, fq, iq = oracle.iswift_ref(Pd, c, A, bb, G, h, "qd")
        obs, eps = oracle.select_obstacles(p, x0, b["obstacles"])
        xn, fn, itn = oracle.nlp_solve(p, x0, foot, Pd, c, A, bb, G, h, obs, eps, xq)
        gJ, hh = nlp_rows(N, C, Pd.size, G, h, obs, eps, p.vsat)
        cert = certify(Pd, c, A, bb, gJ, hh, xn)
        xs, fs = slsqp(Pd, c, A, bb, gJ, hh, xq)
        cases.append(dict(N=N, C=C, K_obs=K, x0=x0, ref=ref, foot=foot, obstacles=b["obstacles"], obs=obs, eps=eps,
                          x_qp=xq, x=xn, flag=fn, iters=itn, obj=0.5 * Pd @ (xn * xn) + c @ xn, kkt=cert,
                          slsqp_obj=fs, slsqp_x=xs))
        print("nlp case", a, fn, itn, cert, "obj-slsqp", 0.5 * Pd @ (xn * xn) + c @ xn - fs)
    dump("nlp_random.json", dict(cases=cases))


# ----------------------------------------------------------------------------- low-level CLF-QP
LL_IND = [[1, 0, 0, 1], [0, 1, 1, 0], [1, 1, 1, 1], [1, 1, 1, 0], [0, 0, 0, 0], [1, 0, 0, 1], [0, 1, 1, 0], [1, 1, 1, 1]]


def ll_ctrl():
    b = ll_workload.make_batch(len(LL_IND), seed=77, ind=LL_IND)
    out = {k: np.asarray(v) for k, v in b.items()}
    for clf in (1, 0):
        p = oracle.ll_params(useCLF=clf)
        X = np.zeros((len(LL_IND), 32)); F = np.zeros(len(LL_IND), np.int32); IT = np.zeros(len(LL_IND), np.int32)
        for a in range(len(LL_IND)):
            Pd, c, A, bb, G, h, *_ = oracle.ll_build_qp(p, b, a)
            x, f, it = oracle.iswift_ref(Pd, c, A, bb, G, h, "md")
            X[a, :x.size] = x; F[a] = f; IT[a] = it
            print("ll case", clf, a, LL_IND[a], f, it)
        out[f"iswift_x_clf{clf}"] = X; out[f"iswift_flag_clf{clf}"] = F; out[f"iswift_iters_clf{clf}"] = IT
    np.savez_compressed(os.path.join(HERE, "ll_ctrl.npz"), **out)
    print("wrote ll_ctrl.npz")


if __name__ == "__main__":
    oracle.build()
    if sys.argv[1:] == ["ll"]:
        ll_ctrl()
        sys.exit(0)
    if sys.argv[1:] == ["qpmd"]:
        qp_md()
        sys.exit(0)
    if sys.argv[1:] == ["nlp"]:               # the NLP fixtures only (oracle NLP changes)
        kat2()
        nlp_random()
        sys.exit(0)
    ll_ctrl()
    kat1()
    kat2()
    qp_random()
    nlp_random()
