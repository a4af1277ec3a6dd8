"""SRB-12 extension mode: the north star's 12-state single-rigid-body
CBF-NMPC.  The reference declares it (include/fast_MPC.hpp:98-103) and implements nothing, so
parity with the reference is UNPINNED; the oracle (oracle/srb12.c) is pinned by a
solver-independent KKT certificate and an independent numpy restatement of the model, and the
GPU kernel (csrc/srb12_kernels.hip, a Riccati-based interior-point method) is checked against
the oracle (dense full-space LU, the same iteration)."""
import ctypes

import numpy as np
import pytest

import oracle
from kkt import certify
from srbnmpc import srb12, workload

N = 10



def _opt(st):
    """Rows whose stages all converged: the QP stage OPTIMAL, or -- when the NLP follows it -- stopped at its
    warm-start tolerance tol_qp (status 4: that point is only the NLP's warm start, never reported OPTIMAL),
    and the NLP stage OPTIMAL."""
    st = np.asarray(st)
    return np.isin(st[:, 0], (0, 4)) & (st[:, 1] == 0)

def _batch(A, gait, seed, Kn=8):
    b = workload.make_batch12(A, N, gait, seed=seed)
    p = oracle.params12(N, K_obs=3, K_nbr=Kn)
    return b, p


def _model_numpy(p, x0, xref, foot, contact):
    """Independent restatement of the SRB-12 linearisation (srb12.c header): A_k, B_k, c_k."""
    Ib = np.array(p.Ib).reshape(3, 3)
    As, Bs, cs = [], [], []
    for k in range(p.N):
        ph = x0 if k == 0 else xref[k - 1]
        c, s = np.cos(ph[5]), np.sin(ph[5])
        Rz = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])
        Iwi = np.linalg.inv(Rz @ Ib @ Rz.T)
        A = np.eye(12)
        A[0:3, 6:9] += p.Ts * np.eye(3)
        A[3:6, 9:12] += p.Ts * Rz.T
        B = np.zeros((12, 12))
        for l in range(4):
            if contact[k, l]:
                r = foot[k, l] - ph[:3]
                S = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
                B[6:9, 3 * l:3 * l + 3] = p.Ts / p.mass * np.eye(3)
                B[9:12, 3 * l:3 * l + 3] = p.Ts * Iwi @ S
        cc = np.zeros(12)
        cc[8] = -p.Ts * p.grav
        As.append(A); Bs.append(B); cs.append(cc)
    return np.array(As), np.array(Bs), np.array(cs)


def _problem(p, x0, xref, foot, contact, obs, eps):
    """Full-space problem in numpy for the KKT certificate: Pd, c, Aeq, beq, g_and_J, h."""
    Nn = p.N
    n = 24 * Nn + 1
    A, B, cvec = _model_numpy(p, x0, xref, foot, contact)
    Pd = np.zeros(n); c = np.zeros(n)
    for k in range(Nn):
        w = np.array(p.qN if k == Nn - 1 else p.q)
        Pd[12 * k:12 * k + 12] = w; c[12 * k:12 * k + 12] = -w * xref[k]
        Pd[12 * Nn + 12 * k:12 * Nn + 12 * k + 12] = np.tile(np.array(p.r), 4)
    Pd[-1] = p.Sw
    Aeq = np.zeros((12 * Nn, n)); beq = np.zeros(12 * Nn)
    for k in range(Nn):
        Aeq[12 * k:12 * k + 12, 12 * k:12 * k + 12] = np.eye(12)
        if k > 0:
            Aeq[12 * k:12 * k + 12, 12 * (k - 1):12 * k] = -A[k]
        Aeq[12 * k:12 * k + 12, 12 * Nn + 12 * k:12 * Nn + 12 * k + 12] = -B[k]
        beq[12 * k:12 * k + 12] = cvec[k] + (A[0] @ x0 if k == 0 else 0)
    mus = p.mu / np.sqrt(2)
    gc = np.array([[1, 0, -mus], [-1, 0, -mus], [0, 1, -mus], [0, -1, -mus], [0, 0, -1], [0, 0, 1.0]])
    G, h = [], []
    for k in range(Nn):
        for l in range(4):
            if contact[k, l]:
                for q in range(6):
                    row = np.zeros(n)
                    row[12 * Nn + 12 * k + 3 * l:12 * Nn + 12 * k + 3 * l + 3] = gc[q]
                    G.append(row); h.append(p.fmax if q == 5 else 0.0)
    G = np.array(G); h = np.array(h)
    K = obs.shape[1]

    def g_and_J(x):
        go = np.zeros(Nn * K); Jo = np.zeros((Nn * K, n))
        for k in range(Nn):
            for j in range(K):
                r = k * K + j
                dx = x[12 * k] - obs[k, j, 0]; dy = x[12 * k + 1] - obs[k, j, 1]
                go[r] = -(dx * dx + dy * dy) - x[-1]
                Jo[r, 12 * k] = -2 * dx; Jo[r, 12 * k + 1] = -2 * dy; Jo[r, -1] = -1
        return np.concatenate([G @ x, go]), np.vstack([G, Jo])

    hh = np.concatenate([h, -np.repeat(np.asarray(eps)[None], Nn, 0).ravel()])
    return Pd, c, Aeq, beq, g_and_J, hh


def _obs_for(p, b, a):
    op = oracle.params(p.N, 2, K_obs=p.K_obs, K_nbr=p.K_nbr, Ts=p.Ts, eps_obs=p.eps_obs, eps_nbr=p.eps_nbr)
    x = b["x0"][a]
    return oracle.select_obstacles(op, np.array([x[0], x[6], x[1], x[7]]), b["obstacles"], b["nbr_state"], int(a))


def test_srb12_model_matches_numpy_restatement():
    b, p = _batch(6, "trot", 3)
    for a in range(6):
        A, B, c = oracle.dynamics12(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a])
        An, Bn, cn = _model_numpy(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a])
        np.testing.assert_allclose(A, An, atol=1e-14)
        np.testing.assert_allclose(B, Bn, atol=1e-12)
        np.testing.assert_allclose(c, cn, atol=1e-15)


@pytest.mark.parametrize("gait", ["trot", "stand"])
def test_srb12_oracle_kkt_certificate(gait):
    """The oracle's QP and NLP points are KKT points of the stated problem (certificate with its
    own multipliers, bounded least squares; no solver trusted)."""
    b, p = _batch(8, gait, 11)
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert _opt(r["status"]).all(), r["status"]
    for a in range(8):
        obs, eps = _obs_for(p, b, a)
        Pd, c, Aeq, beq, gJ, hh = _problem(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a], obs, eps)
        cert = certify(Pd, c, Aeq, beq, gJ, hh, r["x"][a])
        assert cert["eq"] < 1e-9 and cert["prim"] < 1e-7, cert
        assert cert["stat_rel"] < 1e-6, cert
        # the dynamics hold and the swing legs carry no force
        X, U = r["x"][a, :12 * N].reshape(N, 12), r["x"][a, 12 * N:24 * N].reshape(N, 4, 3)
        assert np.abs(U[b["contact"][a] == 0]).max(initial=0.0) < 1e-9


def test_srb12_oracle_qp_stage_is_optimal_without_obstacle_rows():
    b, p = _batch(6, "trot", 5)
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    empty = np.zeros((N, 0, 2))
    for a in range(6):
        Pd, c, Aeq, beq, gJ, hh = _problem(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a], empty, [])
        cert = certify(Pd, c, Aeq, beq, gJ, hh, r["x_qp"][a])
        assert cert["stat_rel"] < 1e-6 and cert["prim"] < 1e-7 and cert["eq"] < 1e-9, cert


def _tight(p, b, **kw):
    """Independent reference optimum: the oracle's interior point run to s'z/m < 1e-11 (dual and primal
    tests at 1e-9) without the polish; MAXIT agents (round-off floor) are left out by the callers."""
    pt = oracle.params12(p.N, K_obs=p.K_obs, K_nbr=p.K_nbr, use_nlp=p.use_nlp, tol=1e-9, tol_final=1e-11,
                         qp_maxit=80, nlp_maxit=80, polish=0, **kw)
    return oracle.solve_batch12(pt, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])


@pytest.mark.parametrize("gait,A,Nh", [("trot", 128, 10), ("stand", 128, 10), ("trot", 48, 20)])
def test_srb12_oracle_forces_within_1e4_of_certified_optimum(gait, A, Nh):
    """North-star GRF clause (|f - f*|_inf < 1e-4 N): the oracle's result (last stage to s'z/m < 1e-9,
    then the active-set polish) against the independent tight run, every agent both solve OPTIMAL;
    the polish is accepted on >= 95 % of the agents."""
    b = workload.make_batch12(A, Nh, gait, seed=17)
    p = oracle.params12(Nh, K_obs=3, K_nbr=8)
    st = (ctypes.c_int * 4).in_dll(oracle.lib(), "orc12_polish_stats")
    for i in range(4):
        st[i] = 0
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    rej, acc = st[0], st[1]
    t = _tight(p, b)
    ok = _opt(t["status"]) & _opt(r["status"])
    assert ok.mean() >= 0.95
    U, Ut = r["x"][ok, 12 * Nh:24 * Nh], t["x"][ok, 12 * Nh:24 * Nh]
    assert np.abs(U - Ut).max() < 1e-4, np.abs(U - Ut).max()
    assert np.abs(r["x"][ok, :12 * Nh] - t["x"][ok, :12 * Nh]).max() < 1e-6
    assert acc + rej == A and acc >= 0.95 * A, (acc, rej)


def _exact_active_set_optimum(p, b, a, x_start, act_tol=1e-6, iters=30):
    """Independent numpy reference for one agent: the exact KKT point of the active set read off
    x_start (rows within act_tol of their bound), by Newton steps on the UNregularised full-space
    KKT system [H_L, Aeq', J_A'; Aeq, 0, 0; J_A, 0, 0] (least squares where J_A is rank deficient,
    H_L = diag(P) - 2 sum z_obs on (p_x, p_y)), certified by kkt.certify (multipliers z >= 0 by
    bounded least squares); otherwise the row with the most negative Newton multiplier leaves and
    violated rows join.  No code of the kernel or the oracle is shared."""
    obs, eps = _obs_for(p, b, a)
    Pd, c, Aeq, beq, gJ, hh = _problem(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a], obs, eps)
    n, neq, K = Pd.size, Aeq.shape[0], obs.shape[1]
    nlin = len(hh) - p.N * K
    def certified(x):
        # |f - f*| <= stat / r (the force weights make the reduced problem strongly convex along the forces):
        # stat < 1e-9 bounds the start point's force error by 1e-7 N
        cert = certify(Pd, c, Aeq, beq, gJ, hh, x, act_tol=1e-7, comp_tol=1e-9)
        return cert["prim"] < 1e-9 and cert["eq"] < 1e-9 and (cert["stat"] < 1e-9 or cert["stat_rel"] < 1e-12)
    if certified(x_start):           # degenerate active sets (rows at zero force, multipliers 0) stop here
        return x_start.copy()
    g, _ = gJ(x_start)
    act = np.where(hh - g < act_tol)[0]
    x = x_start.copy()
    for _ in range(8):
        z = np.zeros(act.size)
        for _ in range(iters):
            g, J = gJ(x)
            H = np.diag(Pd)
            for r, zr in zip(act, z):
                if r >= nlin:
                    k = (r - nlin) // K
                    H[12 * k, 12 * k] -= 2 * zr; H[12 * k + 1, 12 * k + 1] -= 2 * zr
            JA = J[act]
            M = np.block([[H, Aeq.T, JA.T], [Aeq, np.zeros((neq, neq + act.size))],
                          [JA, np.zeros((act.size, neq + act.size))]])
            rhs = -np.r_[Pd * x + c + JA.T @ z, Aeq @ x - beq, g[act] - hh[act]]
            try:
                d = np.linalg.solve(M, rhs)
            except np.linalg.LinAlgError:
                d = np.linalg.lstsq(M, rhs, rcond=None)[0]
            x = x + d[:n]
            z = z + d[n + neq:]
            if np.abs(d[:n]).max() < 1e-12:
                break
        if certified(x):
            return x
        g, _ = gJ(x)
        viol = np.where(hh - g < -1e-9)[0]
        drop = act[np.argmin(z)] if act.size and z.min() < 0 and viol.size == 0 else -1
        act = np.union1d(act[act != drop], viol)
    raise AssertionError(f"agent {a}: no certified active set")


@pytest.mark.parametrize("gait", ["stand", "trot"])
def test_srb12_oracle_polish_equals_independent_exact_optimum(gait):
    """The oracle's polished point is the exact KKT point: equal to the independent numpy active-set solve
    started from the tight interior-point run (_exact_active_set_optimum)."""
    A = 24
    b = workload.make_batch12(A, N, gait, seed=21)
    p = oracle.params12(N, K_obs=3, K_nbr=8)
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    t = _tight(p, b)
    assert _opt(r["status"]).all()
    for a in range(A):
        xe = _exact_active_set_optimum(p, b, a, t["x"][a])
        # (the reference is exact, or the tight run's own point when that certifies: then within 1e-7 N).
        # Measured (round 6, seed 21): forces to 1.3e-8 N (trot) / 2.9e-7 N (stand), X to 6e-11 / 2.5e-10
        assert np.abs(r["x"][a, 12 * N:24 * N] - xe[12 * N:24 * N]).max() < 1e-6
        assert np.abs(r["x"][a, :12 * N] - xe[:12 * N]).max() < 1e-9


def test_srb12_oracle_polish_exact_without_obstacle_rows():
    """QP stage alone (the convex problem): every polish accepted, forces at the exact optimum (the
    tight run to 1e-5: its own residual is the bound)."""
    A, Nh = 64, 10
    b = workload.make_batch12(A, Nh, "stand", seed=23)
    p = oracle.params12(Nh, K_obs=3, K_nbr=8, use_nlp=0)
    st = (ctypes.c_int * 4).in_dll(oracle.lib(), "orc12_polish_stats")
    for i in range(4):
        st[i] = 0
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert st[1] == A and st[0] == 0
    t = _tight(p, b)
    assert (t["status"][:, 0] == 0).all()
    assert np.abs(r["x"][:, 12 * Nh:24 * Nh] - t["x"][:, 12 * Nh:24 * Nh]).max() < 1e-5


def _rejected_polish_batch():
    """QP stage alone (use_nlp = 0) stopped at tol = tol_final = 1 with force bounds of 1 N: the interior-point
    point is too loose for the polish on about a third of the agents (a rejected last-stage polish
    reads 4, whichever stage is last)."""
    b = workload.make_batch12(64, N, "stand", seed=23)
    return b, dict(tol=1.0, tol_final=1.0, fmax=1.0)


def test_srb12_oracle_qp_only_rejected_polish_reads_4():
    """with use_nlp = 0 the QP stage is the last stage; a rejected polish returns the
    interior-point result with status[0] = 4, and status[1] / iters[1] read 0 (include/srbnmpc.h srb12_batch)."""
    b, kw = _rejected_polish_batch()
    p = oracle.params12(N, K_obs=3, K_nbr=8, use_nlp=0)
    for k, v in kw.items():
        setattr(p, k, v)
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    rej = r["status"][:, 0] == 4
    assert 0 < rej.sum() < len(rej) and np.isin(r["status"][:, 0], (0, 4)).all()
    assert (r["status"][:, 1] == 0).all() and (r["iters"][:, 1] == 0).all()
    p.polish = 0      # without the polish the same agents end OPTIMAL at the interior-point result
    r0 = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert (r0["status"][:, 0] == 0).all()
    np.testing.assert_array_equal(r["x"][rej], r0["x"][rej])


@pytest.mark.gpu
def test_srb12_gpu_qp_only_rejected_polish_reads_4():
    """The kernel's counterpart: status 4 on the rejected-polish agents, their interior-point result as the
    oracle's (forces to 1e-4 N), and every other agent OPTIMAL at the oracle's polished point."""
    _gpu()
    b, kw = _rejected_polish_batch()
    A = b["x0"].shape[0]
    p = oracle.params12(N, K_obs=3, K_nbr=8, use_nlp=0)
    g = srb12.default_params(N, K_obs=3, K_nbr=8, use_nlp=0)
    for k, v in kw.items():
        setattr(p, k, v)
        setattr(g, k, v)
    s = srb12.Solver12(g, A)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    s.close()
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert (out["status"][:, 0] == 4).any() and np.isin(out["status"][:, 0], (0, 4)).all()
    assert (out["status"][:, 1] == 0).all() and (out["iters"][:, 1] == 0).all()
    same = out["status"][:, 0] == r["status"][:, 0]
    assert same.sum() >= A - 2, (out["status"][:, 0], r["status"][:, 0])   # a polish decision at its threshold
    np.testing.assert_allclose(out["x"][same][:, :12 * N], r["x"][same][:, :12 * N], atol=1e-6)
    np.testing.assert_allclose(out["x"][same][:, 12 * N:], r["x"][same][:, 12 * N:], atol=1e-4)


def test_srb12_params_defaults_match_oracle():
    """srb12_params_default (C ABI, no GPU) == the oracle's defaults; reference constants."""
    pg = srb12.default_params(N)
    po = oracle.params12(N)
    for k, _ in srb12.Params12._fields_:
        a, o = getattr(pg, k), getattr(po, k)
        if hasattr(a, "__len__"):
            assert list(a) == list(o), k
        else:
            assert a == o, k
    assert pg.mass == 12.453 and abs(pg.Ib[0] - 0.01683993) < 1e-15      # fast_MPC.cpp:40-43
    assert pg.mu == 0.7 and list(pg.q) == [1e3] * 12 and list(pg.r) == [1e-2] * 3   # Parameters.cpp:32-52
    assert 0 < srb12.lds_bytes(pg) <= 160 * 1024


# ------------------------------------------------------------------------------------------- GPU
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("gait", ["trot", "stand"])
def test_srb12_gpu_vs_oracle(gait):
    _gpu()
    A = 64
    b, p = _batch(A, gait, 21)
    s = srb12.Solver12(srb12.default_params(N, K_obs=3, K_nbr=8), A)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    s.close()
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert _opt(r["status"]).all()
    assert (out["status"] == r["status"]).all(), [(a, out["status"][a].tolist(), r["status"][a].tolist())
                                                   for a in range(A) if (out["status"][a] != r["status"][a]).any()]
    same_it = (out["iters"] == r["iters"]).all(1).mean()
    assert same_it >= 0.9, same_it
    X, Xo = out["x"][:, :12 * N], r["x"][:, :12 * N]
    U, Uo = out["x"][:, 12 * N:24 * N], r["x"][:, 12 * N:24 * N]
    ex, eu, es = np.abs(X - Xo).max(), np.abs(U - Uo).max(), np.abs(out["x"][:, -1] - r["x"][:, -1]).max()
    # the north star's GRF tolerance (|.|_inf < 1e-4 N), against the oracle and against the independent
    # tight optimum (both polished to the exact KKT point of their active sets)
    assert ex < 1e-6 and eu < 1e-4 and es < 1e-6, (ex, eu, es)
    t = _tight(p, b)
    ok = _opt(t["status"])
    assert ok.mean() >= 0.95
    eut = np.abs(U[ok] - t["x"][ok, 12 * N:24 * N]).max()
    assert eut < 1e-4, eut
    np.testing.assert_allclose(out["x_qp"][:, :12 * N], r["x_qp"][:, :12 * N], atol=1e-6)
    np.testing.assert_allclose(out["obj"], r["obj"], rtol=1e-8)
    # the selection is the LIP mode's (oracle.select_idx on the CoM position / velocity)
    op = oracle.params(N, 2, K_obs=3, K_nbr=8)
    for a in range(0, A, 7):
        x = b["x0"][a]
        want = oracle.select_idx(op, np.array([x[0], x[6], x[1], x[7]]), b["obstacles"], b["nbr_state"], a)
        np.testing.assert_array_equal(out["sel"][a], want)


@pytest.mark.gpu
def test_srb12_device_entry_equals_host_entry():
    torch = _gpu()
    A = 128
    b, _ = _batch(A, "trot", 4)
    prm = srb12.default_params(N, K_obs=3, K_nbr=8)
    s = srb12.Solver12(prm, A)
    h = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    dev = torch.device("cuda:0")
    T = lambda v, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(v), dtype=dt, device=dev)
    o = dict(x_qp=torch.zeros((A, prm.nv), dtype=torch.float64, device=dev),
             x=torch.zeros((A, prm.nv), dtype=torch.float64, device=dev),
             obj=torch.zeros(A, dtype=torch.float64, device=dev),
             status=torch.zeros((A, 2), dtype=torch.int32, device=dev),
             iters=torch.zeros((A, 2), dtype=torch.int32, device=dev))
    s.solve_device(T(b["x0"]), T(b["xref"]), T(b["foot"]), T(b["contact"], torch.int32), T(b["obstacles"]),
                   T(b["nbr_state"]), o)
    torch.cuda.synchronize()
    s.close()
    for k in ("x_qp", "x", "obj", "status", "iters"):
        np.testing.assert_array_equal(o[k].cpu().numpy(), h[k], err_msg=k)


@pytest.mark.gpu
def test_srb12_full_size_properties():
    """1024 agents (the configs[2] swarm size): statuses, dynamics, friction pyramid, force bound,
    obstacle rows, swing legs at zero -- every agent."""
    _gpu()
    A = 1024
    b, p = _batch(A, "trot", 8)
    s = srb12.Solver12(srb12.default_params(N, K_obs=3, K_nbr=8), A)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    s.close()
    assert _opt(out["status"]).mean() >= 0.99, np.bincount(out["status"][:, 1])
    X, U, sl = srb12.split(p, out["x"])
    mus = p.mu / np.sqrt(2)
    ok = _opt(out["status"])
    for a in np.where(ok)[0][:256]:
        Am, Bm, cm = oracle.dynamics12(p, b["x0"][a], b["xref"][a], b["foot"][a], b["contact"][a])
        prev = b["x0"][a]
        for k in range(N):
            assert np.abs(Am[k] @ prev + Bm[k] @ U[a, k].ravel() + cm[k] - X[a, k]).max() < 1e-8
            prev = X[a, k]
    st = b["contact"] == 1
    f = U[st]
    assert (np.abs(f[:, 0]) - mus * f[:, 2]).max() < 1e-7 and (np.abs(f[:, 1]) - mus * f[:, 2]).max() < 1e-7
    assert f[:, 2].min() > -1e-7 and f[:, 2].max() < p.fmax + 1e-7
    assert np.abs(U[~st]).max() < 1e-9


@pytest.mark.gpu
def test_srb12_shards_bit_identical_to_full_batch():
    """An 8-way sharded swarm (each block solved with agent_offset against the whole snapshot, as
    one rank of an 8-GPU run) gives bit-identical results to the single batch."""
    torch = _gpu()
    A = 256
    b, _ = _batch(A, "trot", 13)
    prm = srb12.default_params(N, K_obs=3, K_nbr=8)
    s = srb12.Solver12(prm, A)
    full = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    for lo in range(0, A, A // 8):
        hi = lo + A // 8
        part = s.solve(b["x0"][lo:hi], b["xref"][lo:hi], b["foot"][lo:hi], b["contact"][lo:hi], b["obstacles"],
                       b["nbr_state"], agent_offset=lo)
        for k in ("x", "x_qp", "status", "iters", "sel"):
            np.testing.assert_array_equal(part[k], full[k][lo:hi], err_msg=k)
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("Nh,Ko,Kn,use_nlp", [(20, 3, 8, 1), (6, 0, 0, 1), (10, 3, 8, 0)])
def test_srb12_variants_vs_oracle(Nh, Ko, Kn, use_nlp):
    """Horizon 20 (two slot trips more), no obstacle rows at all, and the QP stage alone."""
    _gpu()
    A = 32
    b = workload.make_batch12(A, Nh, "trot", seed=31)
    p = oracle.params12(Nh, K_obs=Ko, K_nbr=Kn, use_nlp=use_nlp)
    s = srb12.Solver12(srb12.default_params(Nh, K_obs=Ko, K_nbr=Kn, use_nlp=use_nlp), A)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    s.close()
    r = oracle.solve_batch12(p, b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    assert _opt(r["status"]).all() and (out["status"] == r["status"]).all()
    np.testing.assert_allclose(out["x"][:, :12 * Nh], r["x"][:, :12 * Nh], atol=1e-6)
    np.testing.assert_allclose(out["x"][:, 12 * Nh:], r["x"][:, 12 * Nh:], atol=1e-4)      # forces: 1e-4 N


@pytest.mark.gpu
@pytest.mark.parametrize("n_obs,n_all", [(2, 6), (0, 1), (1, 0), (0, 0)])
def test_srb12_tables_shorter_than_k_vs_oracle(n_obs, n_all):
    """the horizon-10, 3 + 8 row shape -- which has a compiled-in (N, K) instance --
    with fewer static obstacles than K_obs and fewer other agents than K_nbr.  The rows clamp to the
    tables ("up to K nearest"), the launch picks the instance of the clamped K (the compiled K = 11
    would read sel misaligned and carve LDS for rows the oracle does not have), and every agent
    matches the oracle, which clamps the same way."""
    _gpu()
    A = max(n_all, 4)
    b = workload.make_batch12(A, N, "trot", seed=37)
    obs = b["obstacles"][:n_obs]
    nbr = b["nbr_state"][:n_all] if n_all > 0 else None
    A = n_all if n_all > 0 else A
    args = (b["x0"][:A], b["xref"][:A], b["foot"][:A], b["contact"][:A], obs if n_obs else None, nbr)
    prm = srb12.default_params(N, K_obs=3, K_nbr=8)
    s = srb12.Solver12(prm, A)
    out = s.solve(*args)
    s.close()
    Ko, Kn = srb12.n_selected(prm, n_obs, n_all)
    assert out["sel"].shape == (A, Ko + Kn) and (Ko, Kn) == (min(3, n_obs), min(8, max(n_all - 1, 0)))
    r = oracle.solve_batch12(oracle.params12(N, K_obs=3, K_nbr=8), *args)
    assert (out["status"] == r["status"]).all(), (out["status"], r["status"])
    np.testing.assert_allclose(out["x"][:, :12 * N], r["x"][:, :12 * N], atol=1e-6)
    np.testing.assert_allclose(out["x"][:, 12 * N:], r["x"][:, 12 * N:], atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("gait,tol_final", [("stand", 1e-8), ("trot", 1e-8), ("stand", 1e-9)])
def test_srb12_gpu_forces_within_1e4_of_exact_optimum_1024(gait, tol_final):
    """VERDICT r04 item 2, the north star's GRF clause on a whole 1024-agent batch: every agent the GPU
    reports OPTIMAL has its forces within 1e-4 N of the exact optimum -- the tight interior-point run
    (s'z/m < 1e-11, no polish) where that run converges, the independent numpy active-set solve
    (_exact_active_set_optimum) where it stops at its round-off floor (~1.5 % of stand agents, up to
    1e-4 N off there) and on a sample of 48 more agents, to 1e-6 N.  A rejected polish reads
    ACCEPTABLE (4), never OPTIMAL; at most 0.5 % of the agents may end so.  VERDICT r05 item 4: at tol_final 1e-9
    (below the round-5 Riccati floor) no agent may run into MAXIT."""
    _gpu()
    A = 1024
    b = workload.make_batch12(A, N, gait, seed=21)
    p = oracle.params12(N, K_obs=3, K_nbr=8)
    g = srb12.default_params(N, K_obs=3, K_nbr=8)
    g.tol_final = tol_final
    s = srb12.Solver12(g, A)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    s.close()
    opt = _opt(out["status"])
    assert np.isin(out["status"][:, 1], (0, 4)).all() and opt.mean() >= 0.995, np.bincount(out["status"][:, 1])
    assert out["iters"][:, 1].max() < g.nlp_maxit
    U = out["x"][:, 12 * N:24 * N]
    t = _tight(p, b)
    tok = _opt(t["status"])
    assert tok.mean() >= 0.97
    e = np.abs(U - t["x"][:, 12 * N:24 * N]).max(1)
    assert e[opt & tok].max() < 1e-4, (np.argmax(np.where(opt & tok, e, 0)), e[opt & tok].max())
    sample = np.where(opt & tok)[0][::max(1, int((opt & tok).sum()) // 48)][:48]
    for a in np.r_[np.where(opt & ~tok)[0], sample]:
        xe = _exact_active_set_optimum(p, b, a, t["x"][a])
        ea = np.abs(U[a] - xe[12 * N:24 * N]).max()
        assert ea < (1e-4 if a not in sample else 1e-6), (a, ea)


def test_srb12_abi_rejects_bad_arguments():
    """Parameter validation and the struct_size check run without a GPU (no context needed)."""
    import ctypes
    L = srb12._lib()
    b = srb12.Batch12()
    b.struct_size = 4
    assert L.srb12_solve_batch_device(None, 1, ctypes.byref(b), None) == -1
    assert b"struct_size" in srbnmpc_last_error()
    p = srb12.default_params(N)
    p.N = 99
    h = ctypes.c_void_p()
    assert L.srb12_ctx_create(ctypes.byref(p), 4, 0, ctypes.byref(h)) == -3        # SRB_ERR_SIZE
    p = srb12.default_params(N)
    p.r[1] = 0.0
    assert L.srb12_ctx_create(ctypes.byref(p), 4, 0, ctypes.byref(h)) == -1        # SRB_ERR_ARG
    p = srb12.default_params(N)
    assert p.tol_qp == 1e-3
    p.tol_qp = -1e-3
    assert L.srb12_ctx_create(ctypes.byref(p), 4, 0, ctypes.byref(h)) == -1        # SRB_ERR_ARG
    assert b"tol_qp" in srbnmpc_last_error()
    assert L.srb12_ctx_set_timing(None, 0) == -1


def srbnmpc_last_error():
    import srbnmpc
    return srbnmpc.lib().srb_last_error()
