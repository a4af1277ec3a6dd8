"""srbnmpc -- batched CBF-NMPC solver for MI355X, Python host side.

Thin ctypes layer over the C ABI in include/srbnmpc.h (libsrbnmpc.so, HIP kernels for
gfx950).  There is no CPU fallback: if the library is missing, or no GPU is visible,
constructing a solver raises.

    BatchSolver   -- whole agent batch per call (host numpy or device torch buffers)
    MPCDist       -- per-agent object with the reference's MPC_dist call surface
                     (/root/reference/include/MPC_dist.hpp:137-190)
    workload      -- synthetic agent batches with the SURVEY.md §8d distributions
    LowLevelCtrl  -- batched low-level CLF-QP (LowLevelCtrl::calcTorque), srbnmpc.lowlevel
    ll_workload   -- synthetic A1-sized low-level controller inputs
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# the product library; no environment variable can change it: a diagnostic A/B
# build is selected only by an explicit use_library() call (bench.py --lib, pytest --srbnmpc-lib)
LIB_PATH = os.path.join(_HERE, "libsrbnmpc.so")

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)

OPTIMAL, KKTFAIL, MAXIT, FATAL, ACCEPTABLE = 0, 1, 2, 3, 4
# status 4 means, by stage: NLP -- ACCEPTABLE (round-off floor, or a loosened exit whose polish was not
# accepted); QP stage followed by the NLP -- QP_WARM, converged at the warm-start tolerance (SRB_OPT_QP_WARM_TOL;
# x_qp is the NLP's warm start, not iSWIFT's 1e-6 point); the last stage of an SRB-12 solve -- its polish rejected
QP_WARM = 4
# srb_ctx_set_option codes (SRB_OPT_* of include/srbnmpc.h)
OPTIONS = {"polish": 1, "polish_rho": 2, "polish_waves": 3, "grid_min_rows": 4, "grid_min_rows_static": 5,
           "polish_fused": 6, "last_polish": 7, "timing": 8, "qp_warm_tol": 9, "selection": 10,
           "kkt_fp32_mu": 11, "kkt_fp32_refine": 12, "last_kkt_fp32": 13}
ABI_VERSION = 5                                               # SRB_ABI_VERSION of include/srbnmpc.h


class Params(ctypes.Structure):
    """Mirror of srb_params (include/srbnmpc.h)."""
    _fields_ = [("N", ctypes.c_int), ("C", ctypes.c_int), ("K_obs", ctypes.c_int), ("K_nbr", ctypes.c_int),
                ("grav", ctypes.c_double), ("hcom", ctypes.c_double), ("Ts", ctypes.c_double), ("mu", ctypes.c_double),
                ("Qw", ctypes.c_double), ("Pw", ctypes.c_double), ("Rw", ctypes.c_double), ("Sw", ctypes.c_double),
                ("box", ctypes.c_double), ("eps_obs", ctypes.c_double), ("eps_nbr", ctypes.c_double),
                ("vsat", ctypes.c_double), ("tol", ctypes.c_double),
                ("qp_maxit", ctypes.c_int), ("nlp_maxit", ctypes.c_int), ("use_nlp", ctypes.c_int)]

    @property
    def nv(self) -> int:
        return (6 + self.C) * self.N + 1

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Batch(ctypes.Structure):
    """Mirror of srb_batch (struct_size is filled in by the constructor)."""
    _fields_ = [("struct_size", ctypes.c_int), ("x0", _dp), ("ref", _dp), ("foot", _dp), ("obstacles", _dp), ("nbr_state", _dp),
                ("n_obs", ctypes.c_int), ("n_all", ctypes.c_int), ("agent_offset", ctypes.c_int),
                ("x_qp", _dp), ("x", _dp), ("obj", _dp), ("status", _ip), ("iters", _ip),
                ("alpha_buf", _dp), ("alpha", _dp), ("sel", _ip), ("obstacles_version", ctypes.c_int)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(Batch), *args, **kw)


class Prep(ctypes.Structure):
    """Mirror of srb_prep (input assembly on the device; struct_size filled in)."""
    _fields_ = [("struct_size", ctypes.c_int), ("Pr", _dp), ("Prd", _dp), ("n_rows", ctypes.c_int), ("T", ctypes.c_int), ("agent_offset", ctypes.c_int),
                ("agent_id", _ip), ("gait_domain", _ip), ("contact", _ip),
                ("toe", _dp), ("start", _dp), ("q", _dp), ("dq", _dp),
                ("x0", _dp), ("ref", _dp), ("foot", _dp), ("last_state", _dp), ("status", _ip)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(Prep), *args, **kw)


_lib = None


def use_library(name: str):
    """Diagnostics only: load the variant build `name` (libsrbnmpc_<tag>.so in this package
    directory) instead of the product library.  Must precede the first load."""
    global LIB_PATH
    base = os.path.basename(name)
    if base != name or not (base == "libsrbnmpc.so" or (base.startswith("libsrbnmpc_") and base.endswith(".so"))):
        raise ValueError(f"srbnmpc.use_library: expected libsrbnmpc.so or libsrbnmpc_<tag>.so, got {name!r}")
    path = os.path.join(_HERE, base)
    if _lib is not None and path != LIB_PATH:
        raise RuntimeError(f"srbnmpc.use_library: {LIB_PATH} is already loaded")
    LIB_PATH = path


def lib():
    """Load libsrbnmpc.so; raise loudly when it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"srbnmpc: {LIB_PATH} not built (run __graft_entry__.build() or make -C srb-cbf-nmpc_amd)")
        L = ctypes.CDLL(LIB_PATH)
        L.srb_params_default.argtypes = [ctypes.POINTER(Params), ctypes.c_int, ctypes.c_int]
        L.srb_nv.argtypes = [ctypes.POINTER(Params)]
        L.srb_lds_bytes.argtypes = [ctypes.POINTER(Params)]
        L.srb_ctx_create.argtypes = [ctypes.POINTER(Params), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.srb_ctx_destroy.argtypes = [ctypes.c_void_p]
        for f in ("srb_solve_batch", "srb_solve_qp"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Batch)]
        L.srb_solve_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Batch), ctypes.c_void_p]
        L.srb_select_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Batch), ctypes.c_int, ctypes.c_void_p]
        L.srb_sync.argtypes = [ctypes.c_void_p]
        L.srb_ctx_set_waves.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.srb_ctx_waves.argtypes = [ctypes.c_void_p]
        L.srb_ctx_set_qp_init.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.srb_ctx_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
        L.srb_ctx_get_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.srb_last_polish_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
        L.srb_hl_plan.argtypes = [ctypes.c_int, ctypes.c_int, _dp, _dp, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.srb_prepare_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Prep), ctypes.c_void_p]
        L.srb_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        L.srb_fit_bezier.argtypes = [_dp, _dp, _dp]
        L.srb_last_error.restype = ctypes.c_char_p
        if L.srb_abi_version() != ABI_VERSION:
            raise RuntimeError(f"srbnmpc: {LIB_PATH} has ABI {L.srb_abi_version()}, these bindings {ABI_VERSION} (rebuild)")
        _lib = L
    return _lib


def default_params(N: int = 4, C: int = 4, **overrides) -> Params:
    p = Params()
    lib().srb_params_default(ctypes.byref(p), N, C)
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def lds_bytes(p: Params) -> int:
    return lib().srb_lds_bytes(ctypes.byref(p))


def _check(rc: int):
    if rc != 0:
        raise RuntimeError(f"srbnmpc error {rc}: {lib().srb_last_error().decode()}")


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _p(a):
    if a is None:
        return None
    if a.dtype == np.float64:
        return a.ctypes.data_as(_dp)
    return a.ctypes.data_as(_ip)


class BatchSolver:
    """One HIP context solving batches of up to `max_agents` agents.

    solve(...)        host numpy in/out (srb_solve_batch, synchronous)
    solve_device(...) torch CUDA tensors in/out (srb_solve_batch_device, async on a stream)
    """

    def __init__(self, params: Params, max_agents: int, device: int = 0):
        self.params = params
        self.max_agents = int(max_agents)
        self.device = int(device)
        h = ctypes.c_void_p()
        _check(lib().srb_ctx_create(ctypes.byref(params), self.max_agents, self.device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().srb_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------- host path
    def n_selected(self, n_obs: int, n_all: int):
        """(Ko, Kn): selected static obstacles / neighbours per agent for tables of these sizes
        ("up to K nearest", the clamp the C ABI applies)."""
        p = self.params
        return min(p.K_obs, max(n_obs, 0)), (min(p.K_nbr, max(n_all - 1, 0)) if n_all > 0 else 0)

    def solve(self, x0, ref, foot, obstacles=None, nbr_state=None, agent_offset: int = 0, qp_only: bool = False,
              alpha_buf=None):
        """Host arrays in, dict of outputs back.  alpha_buf ([A][4], the Bezier buffer state)
        additionally returns alpha ([A][4][5], get_alphaCOM) from the fused fit.  With the NLP
        stage, sel ([A][Ko + Kn]) holds the selected obstacle / neighbour rows."""
        p = self.params
        x0 = _f64(x0).reshape(-1, 4)
        A = x0.shape[0]
        ref = _f64(ref).reshape(A, 4 * p.N)
        foot = _f64(foot).reshape(A, p.N * 2 * p.C)
        ob = _f64(obstacles if obstacles is not None else np.zeros((0, 2))).reshape(-1, 2)
        nb = _f64(nbr_state).reshape(-1, 4) if nbr_state is not None else None
        out = dict(x_qp=np.zeros((A, p.nv)), x=np.zeros((A, p.nv)), obj=np.zeros(A),
                   status=np.zeros((A, 2), np.int32), iters=np.zeros((A, 2), np.int32))
        ab = None
        if alpha_buf is not None:
            ab = _f64(alpha_buf).reshape(A, 4)
            out["alpha"] = np.zeros((A, 4, 5))
        Ko, Kn = self.n_selected(ob.shape[0], nb.shape[0] if nb is not None else 0)
        out["sel"] = np.full((A, Ko + Kn), -2, np.int32)
        b = Batch(_p(x0), _p(ref), _p(foot), _p(ob) if ob.size else None, _p(nb) if nb is not None else None,
                  ob.shape[0], nb.shape[0] if nb is not None else 0, int(agent_offset),
                  _p(out["x_qp"]), _p(out["x"]), _p(out["obj"]), _p(out["status"]), _p(out["iters"]),
                  _p(ab) if ab is not None else None, _p(out["alpha"]) if ab is not None else None,
                  _p(out["sel"]) if out["sel"].size and not qp_only else None)
        fn = lib().srb_solve_qp if qp_only else lib().srb_solve_batch
        _check(fn(self._h, A, ctypes.byref(b)))
        return out

    # --------------------------------------------------------------- device path
    def solve_device(self, x0, ref, foot, obstacles, nbr_state, out, agent_offset: int = 0, stream=None,
                     alpha_buf=None, obstacles_version: int = 0):
        """All arguments torch tensors on this solver's device (float64 / int32), contiguous.
        `out` is a dict with x_qp (or None), x, obj, status, iters and, with alpha_buf [A][4],
        alpha [A][20]; an optional int32 out["sel"] [A][Ko + Kn] receives the selected rows
        (otherwise the context's scratch is used: one stream per context at a time).
        obstacles_version != 0 marks the obstacle tensor as unchanged since the last call with
        that version (its selection grid is reused; the reference's obstacles are static).
        Asynchronous on `stream` (a hipStream_t handle), by default torch's current stream on
        this device, so the launch is ordered after the torch work that filled the inputs."""
        def dptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _dp)

        def iptr(t):
            return ctypes.cast(ctypes.c_void_p(t.data_ptr()), _ip)
        A = x0.shape[0]
        Ko, Kn = self.n_selected(0 if obstacles is None else obstacles.shape[0],
                                 0 if nbr_state is None else nbr_state.shape[0])
        sel = out.get("sel")
        # the kernel writes rows of stride Ko + Kn (K clamped to the table sizes): the tensor must
        # have exactly that row length, or its rows would be read misaligned
        if sel is not None and (sel.dtype != torch_int32() or tuple(sel.shape) != (A, Ko + Kn) or not sel.is_contiguous()):
            raise ValueError(f"out['sel'] must be a contiguous int32 tensor of shape ({A}, {Ko + Kn}) "
                             f"(K_obs, K_nbr clamped to the table sizes: BatchSolver.n_selected), got "
                             f"{tuple(sel.shape)} {sel.dtype}")
        b = Batch(dptr(x0), dptr(ref), dptr(foot), dptr(obstacles), dptr(nbr_state),
                  0 if obstacles is None else obstacles.shape[0], 0 if nbr_state is None else nbr_state.shape[0],
                  int(agent_offset), dptr(out.get("x_qp")), dptr(out["x"]), dptr(out["obj"]),
                  iptr(out["status"]), iptr(out["iters"]), dptr(alpha_buf),
                  dptr(out.get("alpha") if alpha_buf is not None else None),
                  iptr(out["sel"]) if out.get("sel") is not None else None, int(obstacles_version))
        _check(lib().srb_solve_batch_device(self._h, A, ctypes.byref(b), self._stream(stream)))

    def select_device(self, x0, obstacles, nbr_state, sel, tables: int = 3, agent_offset: int = 0, stream=None,
                      obstacles_version: int = 0):
        """The obstacle / neighbour selection alone (srb_select_device) into the int32 tensor sel [A][Ko + Kn]:
        tables 1 the static obstacles, 2 the neighbour snapshot, 3 both.  With the option "selection" set
        to 0, solve_device then uses out["sel"] as filled here (bench.py selects the static obstacles while
        the neighbour all-gather is in flight).  Asynchronous on `stream` like solve_device."""
        A = x0.shape[0]
        Ko, Kn = self.n_selected(0 if obstacles is None else obstacles.shape[0],
                                 0 if nbr_state is None else nbr_state.shape[0])
        if sel.dtype != torch_int32() or tuple(sel.shape) != (A, Ko + Kn) or not sel.is_contiguous():
            raise ValueError(f"sel must be a contiguous int32 tensor of shape ({A}, {Ko + Kn}), got {tuple(sel.shape)} {sel.dtype}")

        def dptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _dp)
        b = Batch(dptr(x0), None, None, dptr(obstacles), dptr(nbr_state),
                  0 if obstacles is None else obstacles.shape[0], 0 if nbr_state is None else nbr_state.shape[0],
                  int(agent_offset), None, None, None, None, None, None, None,
                  ctypes.cast(ctypes.c_void_p(sel.data_ptr()), _ip), int(obstacles_version))
        _check(lib().srb_select_device(self._h, A, ctypes.byref(b), int(tables), self._stream(stream)))

    def _stream(self, stream):
        """hipStream_t for a launch: the caller's, else torch's current stream on this device
        (the C ABI's NULL would mean the context's own stream, unordered against torch's)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(self.device).cuda_stream
        return ctypes.c_void_p(stream)

    def prepare_device(self, Pr, Prd, gait_domain, contact, toe, start, q, dq, out, agent_id=None,
                       agent_offset: int = 0, stream=None):
        """Input assembly on the device (srb_prepare_batch_device): torch tensors on this
        solver's device.  Pr, Prd: [T, 2*NA] (column-major 2*NA x T); gait_domain [A] int32;
        contact [A,4] int32; toe [A,3,4]; start [A,2]; q, dq [A,18].  `out` holds x0 [A,4],
        ref [A,4N], foot [A,N*2*C], last_state [A,4], status [A] int32.  Asynchronous."""
        def dptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _dp)

        def iptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _ip)
        A = q.shape[0]
        pr = Prep(dptr(Pr), dptr(Prd), Pr.shape[1], Pr.shape[0], int(agent_offset), iptr(agent_id),
                  iptr(gait_domain), iptr(contact), dptr(toe), dptr(start), dptr(q), dptr(dq),
                  dptr(out["x0"]), dptr(out["ref"]), dptr(out["foot"]), dptr(out["last_state"]), iptr(out["status"]))
        _check(lib().srb_prepare_batch_device(self._h, A, ctypes.byref(pr), self._stream(stream)))

    def sync(self):
        _check(lib().srb_sync(self._h))

    def set_waves(self, nw: int = 0):
        """Waves per agent (0 automatic, 1, 2, 4; srb_ctx_set_waves)."""
        _check(lib().srb_ctx_set_waves(self._h, int(nw)))

    def set_option(self, name: str, value: float):
        """Context option (srb_ctx_set_option): name one of OPTIONS ("polish", "polish_rho",
        "polish_waves", "grid_min_rows", "grid_min_rows_static", "polish_fused"; "last_polish" is read only)."""
        _check(lib().srb_ctx_set_option(self._h, OPTIONS[name], float(value)))

    def get_option(self, name: str) -> float:
        v = ctypes.c_double()
        _check(lib().srb_ctx_get_option(self._h, OPTIONS[name], ctypes.byref(v)))
        return v.value

    def polish_fused_active(self) -> bool:
        """True when the last launch ran the polish inside the solve kernel (SRB_OPT_LAST_POLISH = 2)."""
        return self.get_option("last_polish") == 2.0

    def set_qp_init(self, mode: int = 1):
        """QP-stage starting point (srb_ctx_set_qp_init): 1 scaled (default), 0 iSWIFT's kkt_initialize."""
        _check(lib().srb_ctx_set_qp_init(self._h, int(mode)))

    def waves(self) -> int:
        """Waves per agent of the last launch."""
        return lib().srb_ctx_waves(self._h)

    def last_kernel_ms(self):
        a = ctypes.c_float(); b = ctypes.c_float()
        _check(lib().srb_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_polish_ms(self) -> float:
        """HIP-event time of the last launch's polish kernel (srb_polish_kernel), ms (0 when fused)."""
        t = ctypes.c_float()
        _check(lib().srb_last_polish_ms(self._h, ctypes.byref(t)))
        return t.value


def torch_int32():
    import torch
    return torch.int32


def hl_plan(Pstart, Pobs, loop: int = 100000, device: int = 0):
    """HL reference planner on the GPU (generateReferenceTrajectory, MPC_dist.cpp:930-1104).
    Pstart [NA, 2] (or flat 2NA), Pobs [n_obs, 2].  Returns Pr, Prd as (2NA, loop // 40)."""
    Ps = _f64(Pstart).reshape(-1)
    NA = Ps.size // 2
    ob = _f64(Pobs).reshape(-1, 2)
    T = int(loop) // 40
    Pr = np.zeros((T, 2 * NA)); Prd = np.zeros((T, 2 * NA))
    _check(lib().srb_hl_plan(int(device), NA, _p(Ps), _p(ob) if ob.size else None, ob.shape[0], int(loop),
                             _p(Pr), _p(Prd)))
    return Pr.T.copy(), Prd.T.copy()


def fit_bezier(buf, X):
    """fitComTrajectory_eventbase (MPC_dist.cpp:784-855): alpha_COM (4x5)."""
    a = np.zeros(20)
    lib().srb_fit_bezier(_p(_f64(buf)), _p(_f64(X)), _p(a))
    return a.reshape(4, 5)


def split(params: Params, x):
    """Split decision vectors (..., nv) into X (...,N,4), U (...,N,2), lambda (...,N,C), s (...)."""
    N, C = params.N, params.C
    x = np.asarray(x)
    return (x[..., :4 * N].reshape(*x.shape[:-1], N, 4), x[..., 4 * N:6 * N].reshape(*x.shape[:-1], N, 2),
            x[..., 6 * N:6 * N + C * N].reshape(*x.shape[:-1], N, C), x[..., -1])


from .mpc_dist import MPCDist  # noqa: E402
from . import workload  # noqa: E402
from . import ll_workload  # noqa: E402
from .lowlevel import LowLevelCtrl  # noqa: E402
