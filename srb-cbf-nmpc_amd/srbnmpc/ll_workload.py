"""Synthetic inputs for the low-level CLF-QP controller (LowLevelCtrl::calcTorque,
/root/reference/src/LowLevelCtrl.cpp:18-113), deterministic per seed.

The reference gets these from the full-body model (RobotModel / VirtualConstraints, out of
scope here), so each agent gets an A1-sized stand-in with the same structure:
  * D: 18x18 SPD mass matrix -- base mass 12.5 kg, base inertia diag(0.07, 0.26, 0.24),
    3x3 leg blocks around diag(0.06, 0.05, 0.01), small base-leg coupling; Dinv = D^-1;
  * B = [0; I12] (joint torques act on the 12 leg coordinates, global_loco_structs.hpp:39);
  * Jtoe rows 3i..3i+2 of leg i (FR, FL, RR, RL): [I3 | -[r_i]x | leg block at cols 6+3i],
    Jhip the same at the hip offsets with no leg block, so Jtoe - Jhip has the leg block;
  * contact flags: trot pairs {FR,RL} / {FL,RR} alternating per agent, every `stand_every`-th
    agent in stand (all four legs), as the reference's gait domains switch (MPC_dist.cpp:906-916);
    Jc = stance rows of Jtoe, Js = swing rows;
  * outputs H0 = [I6 0; Js] (body pose + swing toes), small tracking errors y, dy;
  * fDes: m g / c on the stance legs plus U[-2, 2] N per axis;
  * consistency: a reference input (F*, tau*) -- F* = fDes + U[-3, 3] N, |tau*| <= sat / 2 --
    with joint accelerations ddq* = Dinv (Jc' F* + B tau* - H) defines dJc = -Jc ddq* (the
    contact equality Jc Dinv (Jc' F + B tau) = Jc Dinv H - dJc of :147-149 holds at it) and
    dH0 = -kp y - kd dy - H0 ddq* - aux* with aux* ~ N(0, 0.5^2) (the output equality holds
    with a small auxiliary input), i.e. the IO linearisation is achievable inside the torque
    limits, the regime the controller runs in on the robot.
Matrices are column-major with the leading dimensions of srb_ll_io (include/srbnmpc.h);
arrays are returned as C-contiguous numpy arrays whose memory order already is that layout
(e.g. Dinv[a] is stored transposed: Dinv[a].T is the matrix).
"""
from __future__ import annotations

import numpy as np

NQ, NU = 18, 12
MASS = 12.5
G = 9.81
TOE = np.array([[0.18, -0.13, -0.26], [0.18, 0.13, -0.26], [-0.18, -0.13, -0.26], [-0.18, 0.13, -0.26]])
HIP = np.array([[0.18, -0.05, 0.0], [0.18, 0.05, 0.0], [-0.18, -0.05, 0.0], [-0.18, 0.05, 0.0]])
TROT = ([1, 0, 0, 1], [0, 1, 1, 0])


def _skew(r):
    return np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])


def contact_flags(n_agents: int, stand_every: int = 4) -> np.ndarray:
    ind = np.zeros((n_agents, 4), np.int32)
    for a in range(n_agents):
        ind[a] = [1, 1, 1, 1] if (stand_every and a % stand_every == stand_every - 1) else TROT[a & 1]
    return ind


def make_batch(n_agents: int, seed: int = 0, stand_every: int = 4, ind=None, kp: float = 700.0, kd: float = 40.0) -> dict:
    rng = np.random.default_rng(seed)
    A = n_agents
    ind = contact_flags(A, stand_every) if ind is None else np.asarray(ind, np.int32).reshape(A, 4)
    out = {k: np.zeros((A,) + s) for k, s in dict(
        q=(NQ,), dq=(NQ,), Dinv=(NQ, NQ), B=(NU, NQ), Hv=(NQ,), Jc=(NQ, NU), dJc=(NU,), Js=(NQ, NU),
        Jtoe=(NQ, NU), Jhip=(NQ, NU), toePos=(4, 3), hipPos=(4, 3), H0=(NQ, NQ), dH0=(NQ,), y=(NQ,), dy=(NQ,),
        hd=(NQ,), dhd=(NQ,), fDes=(NU,), tau=(NQ,)).items()}
    out["ind"] = ind
    sat = np.tile([22.0, 50.0, 50.0], 4)
    for a in range(A):
        # mass matrix
        D = np.zeros((NQ, NQ))
        D[:3, :3] = MASS * np.eye(3)
        D[3:6, 3:6] = np.diag([0.07, 0.26, 0.24]) + 0.005 * rng.standard_normal((3, 3))
        for i in range(4):
            blk = np.diag([0.06, 0.05, 0.01]) + 0.004 * rng.standard_normal((3, 3))
            D[6 + 3 * i:9 + 3 * i, 6 + 3 * i:9 + 3 * i] = blk
            cpl = 0.02 * rng.standard_normal((6, 3))
            D[:6, 6 + 3 * i:9 + 3 * i] = cpl
        D = 0.5 * (D + D.T)
        w = np.linalg.eigvalsh(D)
        if w[0] < 5e-3:
            D += (5e-3 - w[0]) * np.eye(NQ)
        Dinv = np.linalg.inv(D)
        Dinv = 0.5 * (Dinv + Dinv.T)
        Bm = np.zeros((NQ, NU)); Bm[6:, :] = np.eye(NU)
        base = np.array([0.5 * rng.uniform(0, 9), rng.uniform(-2, 2), 0.26])
        Jtoe = np.zeros((NU, NQ)); Jhip = np.zeros((NU, NQ))
        toe = np.zeros((4, 3)); hip = np.zeros((4, 3))
        for i in range(4):
            r = TOE[i] + 0.01 * rng.standard_normal(3)
            rh = HIP[i]
            Jtoe[3 * i:3 * i + 3, :3] = np.eye(3); Jtoe[3 * i:3 * i + 3, 3:6] = -_skew(r)
            Jhip[3 * i:3 * i + 3, :3] = np.eye(3); Jhip[3 * i:3 * i + 3, 3:6] = -_skew(rh)
            leg = np.array([[0.0, -0.21, -0.11], [0.21, 0.0, 0.0], [0.02, 0.09, 0.11]]) + 0.01 * rng.standard_normal((3, 3))
            Jtoe[3 * i:3 * i + 3, 6 + 3 * i:9 + 3 * i] = leg
            toe[i] = base + r; hip[i] = base + rh
        st = [i for i in range(4) if ind[a, i] == 1]
        sw = [i for i in range(4) if ind[a, i] == 0]
        c = len(st)
        rows_c = np.concatenate([np.arange(3 * i, 3 * i + 3) for i in st]) if st else np.zeros(0, int)
        rows_s = np.concatenate([np.arange(3 * i, 3 * i + 3) for i in sw]) if sw else np.zeros(0, int)
        Jc = Jtoe[rows_c]; Js = Jtoe[rows_s]
        outDim = 6 + 3 * (4 - c)
        H0 = np.zeros((outDim, NQ)); H0[:6, :6] = np.eye(6); H0[6:] = Js
        Hv = np.zeros(NQ); Hv[2] = MASS * G; Hv += 0.5 * rng.standard_normal(NQ)
        fDes = np.zeros(NU)
        for i in st:
            fDes[3 * i:3 * i + 3] = [rng.uniform(-2, 2), rng.uniform(-2, 2), MASS * G / c + rng.uniform(-2, 2)]
        Fst = np.concatenate([fDes[3 * i:3 * i + 3] + rng.uniform(-3, 3, 3) for i in st]) if st else np.zeros(0)
        tau_s = 0.5 * sat * rng.uniform(-1, 1, NU)
        ddq_s = Dinv @ ((Jc.T @ Fst if c else 0.0) + Bm @ tau_s - Hv)
        dJc = -Jc @ ddq_s if c else np.zeros(0)
        q = 0.1 * rng.standard_normal(NQ); dq = 0.2 * rng.standard_normal(NQ)
        y = 0.01 * rng.standard_normal(outDim); dy = 0.05 * rng.standard_normal(outDim)
        aux_s = 0.5 * rng.standard_normal(outDim)
        dH0 = -kp * y - kd * dy - H0 @ ddq_s - aux_s
        hd = np.zeros(NQ); dhd = np.zeros(NQ)
        for k, i in enumerate(sw):
            hd[6 + 3 * k:9 + 3 * k] = toe[i] + 0.02 * rng.standard_normal(3)
            dhd[6 + 3 * k:9 + 3 * k] = 0.1 * rng.standard_normal(3)
        # column-major storage with fixed leading dimensions
        def cm(M, ld, cols):
            buf = np.zeros((cols, ld))
            buf[:M.shape[1], :M.shape[0]] = M.T
            return buf
        out["q"][a] = q; out["dq"][a] = dq
        out["Dinv"][a] = Dinv.T; out["B"][a] = Bm.T; out["Hv"][a] = Hv
        out["Jc"][a] = cm(Jc, NU, NQ); out["dJc"][a, :3 * c] = dJc
        out["Js"][a] = cm(Js, NU, NQ); out["Jtoe"][a] = Jtoe.T; out["Jhip"][a] = Jhip.T
        out["toePos"][a] = toe; out["hipPos"][a] = hip
        out["H0"][a] = cm(H0, NQ, NQ); out["dH0"][a, :outDim] = dH0
        out["y"][a, :outDim] = y; out["dy"][a, :outDim] = dy
        out["hd"][a] = hd; out["dhd"][a] = dhd; out["fDes"][a] = fDes
    return out
