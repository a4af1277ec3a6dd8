"""Batched low-level CLF-QP controller (LowLevelCtrl::calcTorque, /root/reference/src/
LowLevelCtrl.cpp:18-113) over the srb_ll_* C ABI (include/srbnmpc.h).

    LowLevelCtrl(params, max_agents, device)
        .calc_torque(batch)                 host numpy arrays (ll_workload.make_batch layout)
        .calc_torque_device(dev, out)       torch CUDA tensors, asynchronous
        .last_kernel_ms()

No CPU fallback: without libsrbnmpc.so or a GPU the constructor raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _check, _dp, _ip, _f64, lib

IN_KEYS = ("q", "dq", "Dinv", "B", "Hv", "Jc", "dJc", "Js", "Jtoe", "Jhip", "toePos", "hipPos",
           "H0", "dH0", "y", "dy", "hd", "dhd", "fDes")
IN_SIZE = dict(q=18, dq=18, Dinv=324, B=216, Hv=18, Jc=216, dJc=12, Js=216, Jtoe=216, Jhip=216, toePos=12, hipPos=12,
               H0=324, dH0=18, y=18, dy=18, hd=18, dhd=18, fDes=12)
OUT_SIZE = dict(tau=18, QP_force=12, ddq=18, dq=18, q=18, V=1, dV=1, x=32)


class LLParams(ctypes.Structure):
    """Mirror of srb_ll_params (Settings::LL_params, global_loco_structs.hpp:96-111)."""
    _fields_ = [("mu", ctypes.c_double), ("kp", ctypes.c_double), ("kd", ctypes.c_double), ("useCLF", ctypes.c_int),
                ("tauPen", ctypes.c_double), ("dfPen", ctypes.c_double), ("auxPen", ctypes.c_double),
                ("clfPen", ctypes.c_double), ("auxMax", ctypes.c_double), ("clfEps", ctypes.c_double),
                ("maxit", ctypes.c_int), ("tol", ctypes.c_double)]


class LLIO(ctypes.Structure):
    """Mirror of srb_ll_io."""
    _fields_ = [("struct_size", ctypes.c_int), ("ind", _ip)] + [(k, _dp) for k in (
        "q", "dq", "Dinv", "B", "H", "Jc", "dJc", "Js", "Jtoe", "Jhip", "toePos", "hipPos",
        "H0", "dH0", "y", "dy", "hd", "dhd", "fDes",
        "tau", "QP_force", "ddq", "dq_out", "q_out", "V", "dV", "x")] + [("status", _ip), ("iters", _ip)]

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(LLIO), *args, **kw)


_bound = False


def _bind():
    global _bound
    L = lib()
    if not _bound:
        L.srb_ll_params_default.argtypes = [ctypes.POINTER(LLParams)]
        L.srb_ll_ctx_create.argtypes = [ctypes.POINTER(LLParams), ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_void_p)]
        L.srb_ll_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.srb_ll_calc_torque.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(LLIO)]
        L.srb_ll_calc_torque_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(LLIO), ctypes.c_void_p]
        L.srb_ll_sync.argtypes = [ctypes.c_void_p]
        L.srb_ll_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
        _bound = True
    return L


def default_params(**overrides) -> LLParams:
    p = LLParams()
    _bind().srb_ll_params_default(ctypes.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def _io_from(ptrs: dict) -> LLIO:
    io = LLIO()
    io.ind = ptrs["ind"]
    for k in IN_KEYS:
        setattr(io, "H" if k == "Hv" else k, ptrs[k])
    for k, f in (("tau", "tau"), ("QP_force", "QP_force"), ("ddq", "ddq"), ("dq", "dq_out"), ("q", "q_out"),
                 ("V", "V"), ("dV", "dV"), ("x", "x")):
        setattr(io, f, ptrs.get("out_" + k))
    io.status = ptrs["out_status"]
    io.iters = ptrs["out_iters"]
    return io


class LowLevelCtrl:
    """Batched LowLevelCtrl: one HIP context for batches of up to max_agents agents."""

    def __init__(self, params: LLParams | None = None, max_agents: int = 1, device: int = 0):
        self.params = params if params is not None else default_params()
        self.max_agents = int(max_agents)
        self.device = int(device)
        h = ctypes.c_void_p()
        _check(_bind().srb_ll_ctx_create(ctypes.byref(self.params), self.max_agents, int(device), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().srb_ll_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def calc_torque(self, batch: dict) -> dict:
        """Host arrays (ll_workload.make_batch layout) in; dict of tau, QP_force, ddq, dq, q, V,
        dV, x, status, iters out (the oracle's ll_calc_torque keys)."""
        A = int(np.asarray(batch["ind"]).shape[0])
        keep = {"ind": np.ascontiguousarray(batch["ind"], dtype=np.int32).reshape(A, 4)}
        for k in IN_KEYS:
            keep[k] = _f64(batch[k]).reshape(A, IN_SIZE[k])
        out = {k: np.zeros((A, s)) for k, s in OUT_SIZE.items()}
        out["tau"][:] = _f64(batch["tau"]).reshape(A, 18)
        out["status"] = np.zeros(A, np.int32)
        out["iters"] = np.zeros(A, np.int32)
        ptrs = {"ind": keep["ind"].ctypes.data_as(_ip)}
        for k in IN_KEYS:
            ptrs[k] = keep[k].ctypes.data_as(_dp)
        for k in OUT_SIZE:
            ptrs["out_" + k] = out[k].ctypes.data_as(_dp)
        ptrs["out_status"] = out["status"].ctypes.data_as(_ip)
        ptrs["out_iters"] = out["iters"].ctypes.data_as(_ip)
        io = _io_from(ptrs)
        _check(lib().srb_ll_calc_torque(self._h, A, ctypes.byref(io)))
        out["V"] = out["V"][:, 0]
        out["dV"] = out["dV"][:, 0]
        return out

    def calc_torque_device(self, dev: dict, out: dict, stream=None):
        """torch CUDA tensors: dev holds ind (int32 [A,4]) and the IN_KEYS arrays (float64,
        contiguous, [A, IN_SIZE]); out holds tau (in/out), QP_force, ddq, dq, q, V, dV, x
        (float64) and status, iters (int32).  Asynchronous on `stream` (a raw hipStream_t
        handle), by default torch's current stream on this device (ordered after the torch
        work that filled the inputs)."""
        def dptr(t):
            return None if t is None else ctypes.cast(ctypes.c_void_p(t.data_ptr()), _dp)

        def iptr(t):
            return ctypes.cast(ctypes.c_void_p(t.data_ptr()), _ip)
        A = dev["ind"].shape[0]
        ptrs = {"ind": iptr(dev["ind"])}
        for k in IN_KEYS:
            ptrs[k] = dptr(dev[k])
        for k in OUT_SIZE:
            ptrs["out_" + k] = dptr(out.get(k))
        ptrs["out_status"] = iptr(out["status"])
        ptrs["out_iters"] = iptr(out["iters"])
        io = _io_from(ptrs)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(self.device).cuda_stream
        s = ctypes.c_void_p(stream)
        _check(lib().srb_ll_calc_torque_device(self._h, A, ctypes.byref(io), s))

    def sync(self):
        _check(lib().srb_ll_sync(self._h))

    def last_kernel_ms(self) -> float:
        t = ctypes.c_float()
        _check(lib().srb_ll_last_kernel_ms(self._h, ctypes.byref(t)))
        return t.value
