"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes front-end to the CPU restatement in this directory (liboracle.so) and, when it
was built in the survey container, to the genuine vendored iSWIFT (_ref/libiswift_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / CPU baseline.  The product library never loads it.

Reference anchors: problem assembly /root/reference/src/MPC_dist.cpp:81-321, closest
obstacle :371-396, iSWIFT /root/reference/optimization/iSWIFT/src/Prime.c:127-230,
NLP rows /root/reference/include/dec_vars_constr_cost.h:245-438, Bezier fit
MPC_dist.cpp:784-855.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_REF = os.path.join(_HERE, "_ref", "libiswift_ref.so")
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


class OrcParams(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("C", ctypes.c_int), ("K_obs", ctypes.c_int), ("K_nbr", ctypes.c_int),
                ("grav", ctypes.c_double), ("hcom", ctypes.c_double), ("Ts", ctypes.c_double), ("mu", ctypes.c_double),
                ("Qw", ctypes.c_double), ("Pw", ctypes.c_double), ("Rw", ctypes.c_double), ("Sw", ctypes.c_double),
                ("box", ctypes.c_double), ("eps_obs", ctypes.c_double), ("eps_nbr", ctypes.c_double),
                ("vsat", ctypes.c_double), ("tol", ctypes.c_double),
                ("qp_maxit", ctypes.c_int), ("nlp_maxit", ctypes.c_int), ("use_nlp", ctypes.c_int),
                ("qp_init", ctypes.c_int), ("tol_qp", ctypes.c_double), ("polish", ctypes.c_int)]


def build(force: bool = False) -> None:
    """Compile liboracle.so (always possible) and, if /root/reference exists, _ref."""
    if force or not os.path.exists(_LIB) or any(
            os.path.getmtime(os.path.join(_HERE, f)) > os.path.getmtime(_LIB)
            for f in os.listdir(_HERE) if f.endswith((".c", ".h"))):
        subprocess.run(["make", "-s", "-C", _HERE, "all"], check=True)
    if os.path.isdir("/root/reference/optimization/iSWIFT") and (force or not os.path.exists(_REF)):
        subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = ctypes.CDLL(_LIB)
        _lib.orc_params_default.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int, ctypes.c_int]
        for f in ("orc_nv", "orc_neq", "orc_mqp", "orc_mnlp"):
            getattr(_lib, f).argtypes = [ctypes.POINTER(OrcParams)]
            getattr(_lib, f).restype = ctypes.c_int
    return _lib


def ref_available() -> bool:
    return os.path.exists(_REF)


def ref_lib():
    global _ref
    if _ref is None:
        _ref = ctypes.CDLL(_REF)
        _ref.iswift_ref_solve.restype = ctypes.c_int
        _ref.iswift_ref_solve_ccs.restype = ctypes.c_int
    return _ref


def params(N: int = 4, C: int = 4, **kw) -> OrcParams:
    p = OrcParams()
    lib().orc_params_default(ctypes.byref(p), N, C)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def sizes(p: OrcParams):
    L = lib()
    return (L.orc_nv(ctypes.byref(p)), L.orc_neq(ctypes.byref(p)), L.orc_mqp(ctypes.byref(p)),
            L.orc_mnlp(ctypes.byref(p)))


def _c(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a):
    return a.ctypes.data_as(_dp if a.dtype == np.float64 else _ip)


def lip(p: OrcParams):
    Ad = np.zeros(16); Bd = np.zeros(8)
    lib().orc_lip(ctypes.byref(p), _ptr(Ad), _ptr(Bd))
    return Ad.reshape(4, 4), Bd.reshape(4, 2)


def build_qp(p: OrcParams, x0, ref, foot):
    """Dense QP of MPC_dist.cpp:135-321. foot: (N, 2, C). Returns P(diag), c, A, b, G, h."""
    nv, neq, mq, _ = sizes(p)
    x0, ref, foot = _c(x0), _c(ref), _c(foot)
    Pd = np.zeros(nv); c = np.zeros(nv); A = np.zeros((neq, nv)); b = np.zeros(neq)
    G = np.zeros((mq, nv)); h = np.zeros(mq)
    lib().orc_build_qp(ctypes.byref(p), _ptr(x0), _ptr(ref), _ptr(foot), _ptr(Pd), _ptr(c), _ptr(A), _ptr(b),
                       _ptr(G), _ptr(h))
    return Pd, c, A, b, G, h


def qp_solve(Pd, c, A, b, G, h, maxit=25, tol=1e-6):
    n = Pd.size; m = G.shape[0]; pp = A.shape[0]
    x = np.zeros(n); q = np.zeros(n); it = ctypes.c_int()
    arrs = [_c(a) for a in (Pd, c, A, b, G, h)]
    f = lib().orc_qp_solve(n, m, pp, *[_ptr(a) for a in arrs], maxit, ctypes.c_double(tol), _ptr(x), _ptr(q),
                           ctypes.byref(it))
    return x, f, it.value, q


def qp_solve_variants(Pd, c, A, b, G, h, maxit=25, tol=1e-6):
    """iSWIFT semantics (with the trapped flag of its sigma <= sigma_d branch) and the kernel's
    no-trap variant: ((x, flag, iters, trapped), (x, flag, iters))."""
    n = Pd.size; m = h.size; pp = b.size
    arrs = [_c(a) for a in (Pd, c, A, b, G, h)]
    x1 = np.zeros(n); x2 = np.zeros(n); i1 = ctypes.c_int(); i2 = ctypes.c_int(); tr = ctypes.c_int()
    f1 = lib().orc_qp_solve_trap(n, m, pp, *[_ptr(a) for a in arrs], maxit, ctypes.c_double(tol), _ptr(x1),
                                 ctypes.byref(i1), ctypes.byref(tr))
    f2 = lib().orc_qp_solve_nt(n, m, pp, *[_ptr(a) for a in arrs], maxit, ctypes.c_double(tol), _ptr(x2),
                               ctypes.byref(i2))
    return (x1, f1, i1.value, tr.value), (x2, f2, i2.value)


def qp_solve_full(P, c, A, b, G, h, maxit=25, tol=1e-6):
    """iSWIFT restatement with a general symmetric P (KAT-1, Matrices_small.h)."""
    n = P.shape[0]; m = G.shape[0]; pp = A.shape[0]
    x = np.zeros(n); it = ctypes.c_int()
    arrs = [_c(a) for a in (P, c, A, b, G, h)]
    f = lib().orc_qp_solve_full(n, m, pp, *[_ptr(a) for a in arrs], maxit, ctypes.c_double(tol), _ptr(x),
                                ctypes.byref(it))
    return x, f, it.value


def ccs_to_dense(rows, cols, jc, ir, pr):
    D = np.zeros((rows, cols))
    for j in range(cols):
        for k in range(int(jc[j]), int(jc[j + 1])):
            D[int(ir[k]), j] += pr[k]
    return D


def select_obstacles(p: OrcParams, x0, obstacles, nbr_state=None, self_idx=-1):
    K = p.K_obs + p.K_nbr
    obs = np.zeros((p.N, max(K, 1), 2)); eps = np.zeros(max(K, 1))
    ob = _c(obstacles).reshape(-1, 2)
    nb = _c(nbr_state if nbr_state is not None else np.zeros((0, 4))).reshape(-1, 4)
    lib().orc_select_obstacles(ctypes.byref(p), _ptr(_c(x0)), _ptr(ob), ob.shape[0], _ptr(nb), nb.shape[0],
                               self_idx, _ptr(obs), _ptr(eps))
    return obs[:, :K], eps[:K]


def select_idx(p: OrcParams, x0, obstacles, nbr_state=None, self_idx=-1):
    """Selected rows (K_obs static obstacle indices, then K_nbr agent indices, -1: none)
    in the reference's order (MPC_dist.cpp:371-382: sqrt distance, first index on ties,
    min_dist = 1000 sentinel with default index 0 for static obstacles)."""
    K = p.K_obs + p.K_nbr
    idx = np.zeros(max(K, 1), np.int32)
    ob = _c(obstacles).reshape(-1, 2)
    nb = _c(nbr_state if nbr_state is not None else np.zeros((0, 4))).reshape(-1, 4)
    lib().orc_select_idx(ctypes.byref(p), _ptr(_c(x0)), _ptr(ob), ob.shape[0], _ptr(nb), nb.shape[0], self_idx,
                         _ptr(idx))
    return idx[:K]


def nlp_solve(p: OrcParams, x0, foot, Pd, c, A, b, G, h, obs, eps, x_init):
    n = Pd.size
    x = np.zeros(n); it = ctypes.c_int()
    obs = _c(obs); eps = _c(eps)
    f = lib().orc_nlp_solve(ctypes.byref(p), _ptr(_c(x0)), _ptr(_c(foot)), *[_ptr(_c(a)) for a in (Pd, c, A, b, G, h)],
                            _ptr(obs), _ptr(eps), _ptr(_c(x_init)), _ptr(x), ctypes.byref(it))
    return x, f, it.value


def solve_batch(p: OrcParams, x0, ref, foot, obstacles, nbr_state=None, agent_offset=0, nthreads=1):
    """Whole run_NMPC hot path for a batch (agent-major arrays, see include/srbnmpc.h)."""
    nv = sizes(p)[0]
    x0 = _c(x0).reshape(-1, 4); A_ = x0.shape[0]
    ref = _c(ref).reshape(A_, -1); foot = _c(foot).reshape(A_, -1)
    ob = _c(obstacles).reshape(-1, 2)
    nb = _c(nbr_state if nbr_state is not None else np.zeros((0, 4))).reshape(-1, 4)
    xq = np.zeros((A_, nv)); x = np.zeros((A_, nv)); obj = np.zeros(A_)
    st = np.zeros((A_, 2), np.int32); it = np.zeros((A_, 2), np.int32)
    lib().orc_solve_batch(ctypes.byref(p), A_, _ptr(x0), _ptr(ref), _ptr(foot), _ptr(ob), ob.shape[0], _ptr(nb),
                          nb.shape[0], agent_offset, _ptr(xq), _ptr(x), _ptr(obj), _ptr(st), _ptr(it), nthreads)
    return dict(x_qp=xq, x=x, obj=obj, status=st, iters=it)


def hl_plan(Pstart, Pobs, loop=100000):
    """generateReferenceTrajectory (MPC_dist.cpp:930-1104) restated: Pr, Prd (2NA x loop/40)."""
    Ps = _c(Pstart).reshape(-1)
    NA = Ps.size // 2
    ob = _c(Pobs).reshape(-1, 2)
    T = loop // 40
    Pr = np.zeros((T, 2 * NA)); Prd = np.zeros((T, 2 * NA))
    lib().orc_hl_plan(NA, _ptr(Ps), _ptr(ob), ob.shape[0], int(loop), _ptr(Pr), _ptr(Prd))
    return Pr.T.copy(), Prd.T.copy()


def fit_bezier(buf, X):
    a = np.zeros(20)
    lib().orc_fit_bezier(_ptr(_c(buf)), _ptr(_c(X)), _ptr(a))
    return a.reshape(4, 5)


# ---------------------------------------------------------------- genuine iSWIFT (oracle/_ref)
def iswift_ref(Pd, c, A, b, G, h, order: str = "qd"):
    """Solve with the compiled vendored iSWIFT.  order='md': min-degree (like Eigen AMD,
    iswift_qp.cpp:201-205); order='qd': quasi-definite z|x|y elimination order (no zero
    pivots, so iSWIFT's +-1e-7 pivot regularisation ldl.c:320-321 never fires)."""
    import scipy.sparse as sp
    P = np.diag(Pd) if np.ndim(Pd) == 1 else Pd
    n = P.shape[0]; m = G.shape[0]; pp = A.shape[0]
    R = ref_lib()
    if order == "md":
        x = np.zeros(n); it = ctypes.c_int(); ts = ctypes.c_double(); tv = ctypes.c_double()
        arrs = [_c(a) for a in (P, c, A, b, G, h)]
        f = R.iswift_ref_solve(n, m, pp, *[_ptr(a) for a in arrs], _ptr(x), ctypes.byref(it), ctypes.byref(ts),
                               ctypes.byref(tv))
        return x, f, it.value
    perm = np.r_[np.arange(n + pp, n + pp + m), np.arange(n), np.arange(n, n + pp)].astype(np.int32)
    keep = []
    args = []
    for M in (P, A, G):
        S = sp.csc_matrix(M); S.eliminate_zeros(); S.sort_indices()
        trip = (_c(S.indptr, np.int32), _c(S.indices, np.int32), _c(S.data))
        keep.append(trip)
        args += [_ptr(trip[0]), _ptr(trip[1]), _ptr(trip[2])]
    cc, hh, bb = _c(c).copy(), _c(h).copy(), _c(b).copy()
    x = np.zeros(n); it = ctypes.c_int()
    f = R.iswift_ref_solve_ccs(n, m, pp, *args, _ptr(cc), _ptr(hh), _ptr(bb), _ptr(perm), _ptr(x), ctypes.byref(it))
    return x, f, it.value


def iswift_ref_ccs(n, m, pp, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b, perm):
    R = ref_lib()
    arrs = [_c(Pjc, np.int32), _c(Pir, np.int32), _c(Ppr), _c(Ajc, np.int32), _c(Air, np.int32), _c(Apr),
            _c(Gjc, np.int32), _c(Gir, np.int32), _c(Gpr)]
    cc, hh, bb = _c(c).copy(), _c(h).copy(), _c(b).copy()
    pr = _c(perm, np.int32)
    x = np.zeros(n); it = ctypes.c_int()
    f = R.iswift_ref_solve_ccs(n, m, pp, *[_ptr(a) for a in arrs], _ptr(cc), _ptr(hh), _ptr(bb), _ptr(pr), _ptr(x),
                               ctypes.byref(it))
    return x, f, it.value


# ---------------------------------------------------------------- low-level CLF-QP (ll_ctrl.c)
class OrcLLParams(ctypes.Structure):
    _fields_ = [("mu", ctypes.c_double), ("kp", ctypes.c_double), ("kd", ctypes.c_double), ("useCLF", ctypes.c_int),
                ("tauPen", ctypes.c_double), ("dfPen", ctypes.c_double), ("auxPen", ctypes.c_double),
                ("clfPen", ctypes.c_double), ("auxMax", ctypes.c_double), ("clfEps", ctypes.c_double),
                ("maxit", ctypes.c_int), ("tol", ctypes.c_double), ("iswift_trap", ctypes.c_int)]


class OrcLLAgent(ctypes.Structure):
    _fields_ = [("ind", ctypes.c_int * 4)] + [(k, _dp) for k in (
        "q", "dq", "Dinv", "B", "Hv", "Jc", "dJc", "Js", "Jtoe", "Jhip", "toePos", "hipPos",
        "H0", "dH0", "y", "dy", "hd", "dhd", "fDes")]


LL_IN = ("q", "dq", "Dinv", "B", "Hv", "Jc", "dJc", "Js", "Jtoe", "Jhip", "toePos", "hipPos",
         "H0", "dH0", "y", "dy", "hd", "dhd", "fDes")


def ll_params(**kw) -> OrcLLParams:
    p = OrcLLParams()
    lib().orc_ll_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def ll_build_qp(p: OrcLLParams, batch: dict, a: int = 0):
    """Dense QP of LowLevelCtrl::cost/constraints for agent a: (P diag, c, A, b, G, h, V, Veps, LfV, LgV)."""
    ag = OrcLLAgent()
    keep = {}
    for i in range(4):
        ag.ind[i] = int(batch["ind"][a][i])
    for k in LL_IN:
        keep[k] = _c(batch[k][a]).reshape(-1)
        setattr(ag, k, _ptr(keep[k]))
    Pd = np.zeros(32); c = np.zeros(32); A = np.zeros(18 * 32); b = np.zeros(18); G = np.zeros(45 * 32)
    h = np.zeros(45); clf = np.zeros(3); LgV = np.zeros(18)
    n, pp, m = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib().orc_ll_build_qp(ctypes.byref(p), ctypes.byref(ag), ctypes.byref(n), ctypes.byref(pp), ctypes.byref(m),
                          _ptr(Pd), _ptr(c), _ptr(A), _ptr(b), _ptr(G), _ptr(h), _ptr(clf), _ptr(LgV))
    n, pp, m = n.value, pp.value, m.value
    return (Pd[:n].copy(), c[:n].copy(), A[:pp * n].reshape(pp, n).copy(), b[:pp].copy(),
            G[:m * n].reshape(m, n).copy(), h[:m].copy(), clf[0], clf[1], clf[2], LgV.copy())


def ll_calc_torque(p: OrcLLParams, batch: dict, nthreads: int = 1):
    """calcTorque (LowLevelCtrl.cpp:18-113) for every agent of a ll_workload batch
    (nthreads > 1: contiguous agent ranges on pthreads)."""
    A_ = batch["ind"].shape[0]
    arrs = [_c(batch[k]).reshape(A_, -1) for k in LL_IN]
    ind = _c(batch["ind"], np.int32).reshape(A_, 4)
    tau = _c(batch["tau"]).reshape(A_, 18).copy()
    out = dict(tau=tau, QP_force=np.zeros((A_, 12)), ddq=np.zeros((A_, 18)), dq=np.zeros((A_, 18)),
               q=np.zeros((A_, 18)), V=np.zeros(A_), dV=np.zeros(A_), x=np.zeros((A_, 32)),
               status=np.zeros(A_, np.int32), iters=np.zeros(A_, np.int32))
    fn = lib().orc_ll_calc_torque_batch if nthreads <= 1 else \
        (lambda pp, *a: lib().orc_ll_calc_torque_batch_mt(pp, int(nthreads), *a))
    fn(ctypes.byref(p), A_, _ptr(ind), *[_ptr(a) for a in arrs], _ptr(tau),
                                   _ptr(out["QP_force"]), _ptr(out["ddq"]), _ptr(out["dq"]), _ptr(out["q"]),
                                   _ptr(out["V"]), _ptr(out["dV"]), _ptr(out["x"]), _ptr(out["status"]),
                                   _ptr(out["iters"]))
    return out


# ------------------------------------------------------------------ SRB-12 extension mode (srb12.c)
class Orc12Params(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("K_obs", ctypes.c_int), ("K_nbr", ctypes.c_int),
                ("Ts", ctypes.c_double), ("mass", ctypes.c_double), ("Ib", ctypes.c_double * 9),
                ("grav", ctypes.c_double), ("mu", ctypes.c_double), ("fmax", ctypes.c_double),
                ("q", ctypes.c_double * 12), ("qN", ctypes.c_double * 12), ("r", ctypes.c_double * 3),
                ("Sw", ctypes.c_double), ("eps_obs", ctypes.c_double), ("eps_nbr", ctypes.c_double),
                ("tol", ctypes.c_double), ("qp_maxit", ctypes.c_int), ("nlp_maxit", ctypes.c_int),
                ("use_nlp", ctypes.c_int), ("z0", ctypes.c_double),
                ("tol_final", ctypes.c_double), ("polish", ctypes.c_int), ("tol_qp", ctypes.c_double)]


def params12(N: int = 10, **kw) -> Orc12Params:
    """SRB-12 parameters (srb12.c header: constants of fast_MPC.cpp:40-43, Parameters.cpp:32-52)."""
    p = Orc12Params()
    lib().orc12_params_default(ctypes.byref(p), N)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def nv12(p: Orc12Params) -> int:
    return 24 * p.N + 1


def dynamics12(p: Orc12Params, x0, xref, foot, contact):
    """Per-stage A_k, B_k (N, 12, 12) and c_k (N, 12) of the SRB-12 linearisation."""
    N = p.N
    A = np.zeros((N, 12, 12)); B = np.zeros((N, 12, 12)); c = np.zeros((N, 12))
    lib().orc12_dynamics(ctypes.byref(p), _ptr(_c(x0)), _ptr(_c(xref)), _ptr(_c(foot)), _ptr(_c(contact, np.int32)),
                         _ptr(A), _ptr(B), _ptr(c))
    return A, B, c


def solve_batch12(p: Orc12Params, x0, xref, foot, contact, obstacles=None, nbr_state=None, agent_offset=0,
                  nthreads=8):
    """SRB-12 solves of a batch: x0 [A,12], xref [A,N,12], foot [A,N,4,3], contact [A,N,4] int.
    Returns x_qp, x [A, 24N+1], obj, status [A,2], iters [A,2]."""
    x0 = _c(x0); A_ = x0.shape[0]; nv = nv12(p)
    ob = _c(obstacles if obstacles is not None else np.zeros((0, 2)))
    nb = _c(nbr_state) if nbr_state is not None else None
    out = dict(x_qp=np.zeros((A_, nv)), x=np.zeros((A_, nv)), obj=np.zeros(A_),
               status=np.zeros((A_, 2), np.int32), iters=np.zeros((A_, 2), np.int32))
    lib().orc12_solve_batch(ctypes.byref(p), A_, _ptr(x0), _ptr(_c(xref)), _ptr(_c(foot)), _ptr(_c(contact, np.int32)),
                            _ptr(ob), ob.shape[0], _ptr(nb) if nb is not None else None,
                            nb.shape[0] if nb is not None else 0, int(agent_offset), _ptr(out["x_qp"]), _ptr(out["x"]),
                            _ptr(out["obj"]), _ptr(out["status"]), _ptr(out["iters"]), int(nthreads))
    return out
