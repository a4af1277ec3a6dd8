"""CPU tests of the low-level CLF-QP oracle (oracle/ll_ctrl.c, LowLevelCtrl::calcTorque
restated from /root/reference/src/LowLevelCtrl.cpp:18-236, 446-488).

Pins:
  * QP stage: the oracle's iSWIFT restatement on the oracle's assembly reproduces the genuine
    vendored iSWIFT (tests/golden/ll_ctrl.npz, made by tests/golden/make_goldens.py with
    oracle/_ref) -- same exit flag and iteration count, x to 1e-8;
  * assembly: block structure and the CLF scalars against closed forms derived here
    independently of the oracle's explicit-matrix products;
  * epilogue (swing PD, integration, swingInvKin): restatement only (the reference needs
    Eigen, absent) -- checked here against numpy formulas of the same source lines.
"""
import os

import numpy as np
import pytest

import oracle
from srbnmpc import ll_workload

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ll_ctrl.npz")


def _gold():
    g = np.load(GOLD, allow_pickle=False)
    return {k: g[k] for k in g.files}


def _mat(batch, key, a, rows, ld, cols):
    """column-major (ld) storage -> numpy matrix (rows x cols)"""
    return np.asarray(batch[key][a]).reshape(cols, ld).T[:rows, :cols]


@pytest.mark.parametrize("clf", [1, 0])
def test_ll_qp_matches_genuine_iswift(clf):
    g = _gold()
    p = oracle.ll_params(useCLF=clf)
    out = oracle.ll_calc_torque(p, g)
    assert (out["status"] == g[f"iswift_flag_clf{clf}"]).all()
    assert (out["iters"] == g[f"iswift_iters_clf{clf}"]).all()
    assert np.abs(out["x"] - g[f"iswift_x_clf{clf}"]).max() < 1e-8


def test_ll_assembly_structure_and_clf_closed_form():
    g = _gold()
    p = oracle.ll_params()
    for a in range(g["ind"].shape[0]):
        ind = g["ind"][a]
        c_ = int((ind == 1).sum())
        con, out = 3 * c_, 6 + 3 * (4 - c_)
        Pd, c, A, b, G, h, V, Veps, LfV, LgV = oracle.ll_build_qp(p, g, a)
        n = con + 12 + out + 1
        assert Pd.size == n and A.shape == (con + out, n) and G.shape == (5 * c_ + 25, n)
        Dinv = _mat(g, "Dinv", a, 18, 18, 18)
        B = _mat(g, "B", a, 18, 18, 12)
        Jc = _mat(g, "Jc", a, con, 12, 18)
        H0 = _mat(g, "H0", a, out, 18, 18)
        Hv = g["Hv"][a]
        np.testing.assert_allclose(A[:con, :con], Jc @ Dinv @ Jc.T, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(A[con:, con:con + 12], H0 @ Dinv @ B, rtol=1e-12, atol=1e-12)
        np.testing.assert_array_equal(A[con:, con + 12:con + 12 + out], np.eye(out))
        np.testing.assert_allclose(b[:con], Jc @ Dinv @ Hv - g["dJc"][a][:con], rtol=1e-12, atol=1e-10)
        y, dy = g["y"][a][:out], g["dy"][a][:out]
        np.testing.assert_allclose(b[con:], -p.kp * y - p.kd * dy + H0 @ Dinv @ Hv - g["dH0"][a][:out], rtol=1e-12,
                                   atol=1e-9)
        # CLF scalars: PP = [[P1/e^2, Pd/e], [Pd/e, P2]] (x) I, eta = [y; dy]
        kp, kd, e = p.kp, p.kd, p.clfEps
        P1 = (kd * kd + kp * kp + kp) / (2 * kp * kd); Pdd = 1 / (2 * kp); P2 = (kp + 1) / (2 * kd * kp)
        cc = 1 / (0.5 * (P1 + P2 + np.sqrt((P1 - P2) ** 2 + 4 * Pdd ** 2)))
        Vc = np.sum(P1 / e ** 2 * y * y + 2 * Pdd / e * y * dy + P2 * dy * dy)
        v2 = -kp * y - kd * dy
        LfVc = 2 * np.sum((P1 / e ** 2 * y + Pdd / e * dy) * dy + (Pdd / e * y + P2 * dy) * v2)
        LgVc = 2 * (Pdd / e * y + P2 * dy)
        assert abs(V - Vc) < 1e-10 * max(1, abs(Vc)) and abs(LfV - LfVc) < 1e-9 * max(1, abs(LfVc))
        np.testing.assert_allclose(LgV[:out], LgVc, rtol=1e-12, atol=1e-14)
        assert abs(Veps - cc / e * Vc) < 1e-10 * max(1, abs(Vc))
        np.testing.assert_allclose(h[-1], -LfVc - cc / e * Vc, rtol=1e-10, atol=1e-10)
        # friction rows of leg l act on its 3 force variables only; torque bounds +-sat
        mus = p.mu / np.sqrt(2)
        for l in range(c_):
            blk = G[5 * l:5 * l + 5, 3 * l:3 * l + 3]
            np.testing.assert_allclose(blk, [[1, 0, -mus], [-1, 0, -mus], [0, 1, -mus], [0, -1, -mus], [0, 0, -1]])
        sat = np.tile([22.0, 50.0, 50.0], 4)
        np.testing.assert_array_equal(h[5 * c_:5 * c_ + 12], sat)
        np.testing.assert_array_equal(h[5 * c_ + 12:5 * c_ + 24], sat)


def test_ll_epilogue_matches_numpy():
    g = _gold()
    p = oracle.ll_params()
    o = oracle.ll_calc_torque(p, g)
    for a in range(g["ind"].shape[0]):
        ind = g["ind"][a]
        c_ = int((ind == 1).sum())
        con, sw = 3 * c_, 12 - 3 * c_
        Dinv = _mat(g, "Dinv", a, 18, 18, 18)
        B = _mat(g, "B", a, 18, 18, 12)
        Jtoe = _mat(g, "Jtoe", a, 12, 12, 18)
        Jhip = _mat(g, "Jhip", a, 12, 12, 18)
        Js = _mat(g, "Js", a, sw, 12, 18)
        toe = g["toePos"][a].reshape(4, 3); hip = g["hipPos"][a].reshape(4, 3)
        q, dq, hd, dhd = g["q"][a], g["dq"][a], g["hd"][a], g["dhd"][a]
        x = o["x"][a]
        F = np.zeros(12); k = 0
        for i in range(4):
            if ind[i] == 1:
                F[3 * i:3 * i + 3] = x[k:k + 3]; k += 3
        np.testing.assert_array_equal(o["QP_force"][a], F)
        tau = np.array(g["tau"][a], float)
        tau[6:] = x[con:con + 12]
        if sw:
            Delta = np.linalg.inv(Js @ Dinv @ Js.T)
            pd = np.zeros(sw); vd = np.zeros(sw); cs = 0
            for i in range(4):
                if ind[i] == 0:
                    pd[cs:cs + 3] = hd[6 + cs:9 + cs] - toe[i]
                    vd[cs:cs + 3] = dhd[6 + cs:9 + cs] - Jtoe[3 * i:3 * i + 3] @ dq
                    cs += 3
            tau += Js.T @ (1600 * np.diag(Delta) * pd + 40 * vd)
        np.testing.assert_allclose(o["tau"][a], tau, rtol=1e-10, atol=1e-9)
        ddq = Dinv @ (B @ tau[6:] + Jtoe.T @ F - g["Hv"][a])
        np.testing.assert_allclose(o["ddq"][a], ddq, rtol=1e-10, atol=1e-9)
        dqn = dq + ddq / 1000
        qn = q + dqn / 1000 + 0.5e-6 * ddq
        cs = 0
        for i in range(4):
            if ind[i] == 0:
                Jt = Jtoe[3 * i:3 * i + 3] - Jhip[3 * i:3 * i + 3]
                r = (dhd[6 + cs:9 + cs] - Jhip[cs:cs + 3] @ dq) + 20 * ((hd[6 + cs:9 + cs] - hip[i]) - (toe[i] - hip[i])) \
                    - Jt[:, 3:6] @ dq[3:6]
                v = np.linalg.solve(Jt[:, 6 + 3 * i:9 + 3 * i], r)
                dqn[6 + 3 * i:9 + 3 * i] = v
                qn[6 + 3 * i:9 + 3 * i] = q[6 + 3 * i:9 + 3 * i] + v / 1000
                cs += 3
        np.testing.assert_allclose(o["dq"][a], dqn, rtol=1e-10, atol=1e-9)
        np.testing.assert_allclose(o["q"][a], qn, rtol=1e-10, atol=1e-12)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref (genuine iSWIFT) not built")
def test_ll_oracle_vs_genuine_iswift_random():
    b = ll_workload.make_batch(24, seed=5)
    p = oracle.ll_params()
    o = oracle.ll_calc_torque(p, b)
    for a in range(24):
        Pd, c, A, bb, G, h, *_ = oracle.ll_build_qp(p, b, a)
        x, f, it = oracle.iswift_ref(Pd, c, A, bb, G, h, "md")
        assert f == o["status"][a] and it == o["iters"][a]
        assert np.abs(x - o["x"][a, :x.size]).max() < 1e-8


def test_ll_no_trap_variant_differs_from_iswift_only_when_it_traps():
    """The kernel (and the default LL oracle) drop iSWIFT's sigma <= sigma_d branch
    (Prime.c:193-196), reachable only through rounding.  On every instance where the
    iSWIFT-semantics run does not take that branch, both give the identical iterates."""
    rng = np.random.default_rng(5)
    ind = rng.integers(0, 2, (64, 4)).astype(np.int32)
    b = ll_workload.make_batch(64, seed=9, ind=ind)
    n_trap = 0
    for clf in (1, 0):
        p = oracle.ll_params(useCLF=clf)
        for a in range(64):
            Pd, c, A, bb, G, h, *_ = oracle.ll_build_qp(p, b, a)
            (x1, f1, i1, tr), (x2, f2, i2) = oracle.qp_solve_variants(Pd, c, A, bb, G, h)
            n_trap += tr
            if not tr:
                assert f1 == f2 and i1 == i2 and np.array_equal(x1, x2)
            else:
                assert f2 == 0 and np.abs(x1 - x2).max() < 1e-6
    assert n_trap <= 8
