"""SRB-12 extension mode: the north star's 12-state single-rigid-body CBF-NMPC on the GPU
(srb12_* in include/srbnmpc.h, csrc/srb12_kernels.hip).

The reference declares this solver (FastMPC::runMPC / MPC_Cost / MPC_Constraints /
getLinearDynamics, /root/reference/include/fast_MPC.hpp:98-103) without a body, so there is no
reference call surface to mirror: Solver12 follows BatchSolver's shape (host numpy solve, device
torch solve on a stream).  Problem statement: DESIGN.md section 11; checker: oracle/srb12.c.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _check, _dp, _ip, _p, lib

_p12_fields = [("N", ctypes.c_int), ("K_obs", ctypes.c_int), ("K_nbr", ctypes.c_int),
               ("Ts", ctypes.c_double), ("mass", ctypes.c_double), ("Ib", ctypes.c_double * 9),
               ("grav", ctypes.c_double), ("mu", ctypes.c_double), ("fmax", ctypes.c_double),
               ("q", ctypes.c_double * 12), ("qN", ctypes.c_double * 12), ("r", ctypes.c_double * 3),
               ("Sw", ctypes.c_double), ("eps_obs", ctypes.c_double), ("eps_nbr", ctypes.c_double),
               ("tol", ctypes.c_double), ("qp_maxit", ctypes.c_int), ("nlp_maxit", ctypes.c_int),
               ("use_nlp", ctypes.c_int), ("z0", ctypes.c_double),
               ("tol_final", ctypes.c_double), ("polish", ctypes.c_int), ("tol_qp", ctypes.c_double)]


class Params12(ctypes.Structure):
    """Mirror of srb12_params (the oracle's orc12_params has the same layout)."""
    _fields_ = _p12_fields

    @property
    def nv(self) -> int:
        return 24 * self.N + 1


class Batch12(ctypes.Structure):
    """Mirror of srb12_batch (struct_size filled in)."""
    _fields_ = [("struct_size", ctypes.c_int), ("x0", _dp), ("xref", _dp), ("foot", _dp), ("contact", _ip),
                ("obstacles", _dp), ("nbr_state", _dp), ("n_obs", ctypes.c_int), ("n_all", ctypes.c_int),
                ("agent_offset", ctypes.c_int), ("x_qp", _dp), ("x", _dp), ("obj", _dp), ("status", _ip),
                ("iters", _ip), ("sel", _ip), ("obstacles_version", ctypes.c_int)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(Batch12), *args, **kw)


_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        L.srb12_params_default.argtypes = [ctypes.POINTER(Params12), ctypes.c_int]
        L.srb12_lds_bytes.argtypes = [ctypes.POINTER(Params12)]
        L.srb12_ctx_create.argtypes = [ctypes.POINTER(Params12), ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_void_p)]
        L.srb12_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.srb12_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Batch12)]
        L.srb12_solve_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Batch12), ctypes.c_void_p]
        L.srb12_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        L.srb12_ctx_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _bound = True
    return L


def default_params(N: int = 10, **overrides) -> Params12:
    p = Params12()
    _lib().srb12_params_default(ctypes.byref(p), N)
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def lds_bytes(p: Params12) -> int:
    return _lib().srb12_lds_bytes(ctypes.byref(p))


def n_selected(p: Params12, n_obs: int, n_all: int):
    """(Ko, Kn) rows selected per agent for tables of these sizes (clamped as the C ABI does)."""
    Ko = min(p.K_obs, max(n_obs, 0)) if p.use_nlp else 0
    Kn = min(p.K_nbr, max(n_all - 1, 0)) if p.use_nlp else 0
    return Ko, Kn


class Solver12:
    """One HIP context solving SRB-12 batches of up to `max_agents` agents."""

    def __init__(self, params: Params12, max_agents: int, device: int = 0):
        self.params = params
        self.max_agents = int(max_agents)
        self.device = int(device)
        h = ctypes.c_void_p()
        _check(_lib().srb12_ctx_create(ctypes.byref(params), self.max_agents, self.device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib().srb12_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, x0, xref, foot, contact, obstacles=None, nbr_state=None, agent_offset: int = 0):
        """Host numpy: x0 [A,12], xref [A,N,12], foot [A,N,4,3], contact [A,N,4] int.  Returns
        dict x_qp, x [A, 24N+1], obj, status [A,2], iters [A,2], sel [A, Ko+Kn]."""
        p = self.params
        x0 = np.ascontiguousarray(x0, np.float64); A = x0.shape[0]
        xref = np.ascontiguousarray(xref, np.float64); foot = np.ascontiguousarray(foot, np.float64)
        contact = np.ascontiguousarray(contact, np.int32)
        ob = np.ascontiguousarray(obstacles if obstacles is not None else np.zeros((0, 2)), np.float64)
        nb = np.ascontiguousarray(nbr_state, np.float64) if nbr_state is not None else None
        Ko, Kn = n_selected(p, ob.shape[0], nb.shape[0] if nb is not None else 0)
        out = dict(x_qp=np.zeros((A, p.nv)), x=np.zeros((A, p.nv)), obj=np.zeros(A),
                   status=np.zeros((A, 2), np.int32), iters=np.zeros((A, 2), np.int32),
                   sel=np.full((A, Ko + Kn), -2, np.int32))
        b = Batch12(_p(x0), _p(xref), _p(foot), _p(contact), _p(ob) if ob.shape[0] else None,
                    _p(nb) if nb is not None else None, ob.shape[0], nb.shape[0] if nb is not None else 0,
                    int(agent_offset), _p(out["x_qp"]), _p(out["x"]), _p(out["obj"]), _p(out["status"]),
                    _p(out["iters"]), _p(out["sel"]) if out["sel"].size else None, 0)
        _check(_lib().srb12_solve_batch(self._h, A, ctypes.byref(b)))
        return out

    def solve_device(self, x0, xref, foot, contact, obstacles, nbr_state, out, agent_offset: int = 0, stream=None,
                     obstacles_version: int = 0):
        """torch tensors on this device (float64 / int32), contiguous; out holds x_qp (or None), x, obj,
        status, iters and optionally sel [A, Ko+Kn].  Asynchronous on `stream` (default: torch's current)."""
        def dptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _dp)

        def iptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _ip)
        A = x0.shape[0]
        import torch
        Ko, Kn = n_selected(self.params, 0 if obstacles is None else obstacles.shape[0],
                            0 if nbr_state is None else nbr_state.shape[0])
        sel = out.get("sel")
        # the kernel writes rows of stride Ko + Kn (clamped to the tables, 0 without the NLP stage):
        # anything else would be overrun or read misaligned (BatchSolver.solve_device, same check)
        if sel is not None and (sel.dtype != torch.int32 or tuple(sel.shape) != (A, Ko + Kn) or not sel.is_contiguous()):
            raise ValueError(f"out['sel'] must be a contiguous int32 tensor of shape ({A}, {Ko + Kn}) "
                             f"(n_selected(params, n_obs, n_all)), got {tuple(sel.shape)} {sel.dtype}")
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        b = Batch12(dptr(x0), dptr(xref), dptr(foot), iptr(contact), dptr(obstacles), dptr(nbr_state),
                    0 if obstacles is None else obstacles.shape[0], 0 if nbr_state is None else nbr_state.shape[0],
                    int(agent_offset), dptr(out.get("x_qp")), dptr(out["x"]), dptr(out["obj"]), iptr(out["status"]),
                    iptr(out["iters"]), iptr(out.get("sel")), int(obstacles_version))
        _check(_lib().srb12_solve_batch_device(self._h, A, ctypes.byref(b), ctypes.c_void_p(stream)))

    def last_kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(_lib().srb12_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def set_timing(self, on: bool):
        """HIP events around the kernels (srb12_ctx_set_timing; default on): last_kernel_ms needs them."""
        _check(_lib().srb12_ctx_set_timing(self._h, 1 if on else 0))


def split(p: Params12, x):
    """x [..., 24N+1] -> X [..., N, 12], U [..., N, 4, 3], s [...]"""
    N = p.N
    return (x[..., :12 * N].reshape(x.shape[:-1] + (N, 12)), x[..., 12 * N:24 * N].reshape(x.shape[:-1] + (N, 4, 3)),
            x[..., 24 * N])
