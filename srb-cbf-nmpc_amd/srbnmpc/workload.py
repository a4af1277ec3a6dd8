"""Synthetic agent batches, deterministic per seed.

Distributions follow the reference's simulation setup where it has one:
  * start positions U[0,9] x U[-2,2]                     (src/A1_Sim.cpp:944-945)
  * obstacles U[0,9] x U[-2,2] + U[-0.6,0.6], clamped to [1,9] x [-3,3], 20 of them
                                                        (src/A1_Sim.cpp:946-980, NUMBER_OF_OBS)
  * reference: straight line to GOAL (10, 0) at 0.27 m/s (the speed of the logged
    instance, print_file.out), x, xdot, y, ydot per grid (copPlanner layout, MPC_dist.cpp:780)
  * footholds: default stance offsets (MPC_dist.cpp:1206-1209) around the CoM; trot pairs
    {FR,RL} / {FL,RR} alternating every gait domain of NDOMAIN = 4 grids (:906-916), so
    C = 2; C = 4 keeps all legs down (the reference's stand / first-domain case).
Deviation (documented in DESIGN.md): initial velocities are drawn toward the goal,
speed U[0, 0.3] plus U[-0.05, 0.05] per axis, instead of U[-0.3, 0.3] per axis -- with one
trot diagonal per domain the CoM-CoP rows (|p_k - u_{k+1}| <= mu h / sqrt 2) make a sideways
0.3 m/s start infeasible over a 0.43 s horizon, and the reference's QP has no slack on them.
Arenas scale with the batch so that agent density stays that of the reference's 4-agent
runs in a 9 m x 4 m field.
"""
from __future__ import annotations

import numpy as np

STANCE = np.array([[0.2188, 0.2188, -0.1472, -0.1472],     # x of FR, FL, RR, RL
                   [-0.1320, 0.1320, -0.1320, 0.1320]])    # y
TROT_PAIRS = ([0, 3], [1, 2])
GOAL = np.array([10.0, 0.0])
VREF = 0.27
TS = 43 * 0.001


def arena_scale(n_agents: int) -> float:
    return max(1.0, float(np.sqrt(n_agents / 4.0)))


def make_obstacles(rng, n_obs: int = 20, scale: float = 1.0):
    ox = rng.uniform(0, 9.0 * scale, n_obs)
    oy = rng.uniform(-2.0 * scale, 2.0 * scale, n_obs)
    ux = rng.uniform(-0.6, 0.6, n_obs)
    uy = rng.uniform(-0.6, 0.6, n_obs)
    rx = np.clip(ox + ux, 1.0, 9.0 * scale)
    ry = np.clip(oy + uy, -3.0 * scale, 3.0 * scale)
    return np.stack([rx, ry], 1)


def make_batch(n_agents: int, N: int = 10, C: int = 2, seed: int = 0, n_obs: int | None = None,
               velocity: str = "goal"):
    """Returns dict(x0 [A,4], ref [A,4N], foot [A,N,2,C], obstacles [n_obs,2],
    nbr_state [A,4] (x, y, xdot, ydot of every agent, the get_lastState layout)).
    velocity "goal" (default): initial velocities drawn toward the goal (the documented deviation);
    "free": U[-0.3, 0.3] per axis, uncorrelated with the goal and the trot support, which leaves
    some instances' CoM-CoP rows infeasible -- the hard workload of tests/test_gpu_parity.py
    (statuses other than OPTIMAL must agree with the oracle's too)."""
    rng = np.random.default_rng(seed)
    A = int(n_agents)
    sc = arena_scale(A)
    if n_obs is None:
        n_obs = int(round(20 * sc * sc))
    p0 = np.stack([rng.uniform(0, 9.0 * sc, A), rng.uniform(-2.0 * sc, 2.0 * sc, A)], 1)
    goal = GOAL * np.array([sc, 1.0]) + np.array([0.0, 0.0])
    d = goal - p0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    v0 = d * rng.uniform(0, 0.3, (A, 1)) + rng.uniform(-0.05, 0.05, (A, 2))
    if velocity == "free":
        v0 = rng.uniform(-0.3, 0.3, (A, 2))
    x0 = np.stack([p0[:, 0], v0[:, 0], p0[:, 1], v0[:, 1]], 1)
    k = np.arange(N)
    ref = np.zeros((A, N, 4))
    ref[:, :, 0] = p0[:, None, 0] + d[:, None, 0] * VREF * TS * (k + 1)
    ref[:, :, 1] = d[:, None, 0] * VREF
    ref[:, :, 2] = p0[:, None, 1] + d[:, None, 1] * VREF * TS * (k + 1)
    ref[:, :, 3] = d[:, None, 1] * VREF
    foot = np.zeros((A, N, 2, C))
    phase = rng.integers(0, 4, A)
    for a in range(A):
        for kk in range(N):
            dom = (kk + phase[a]) // 4
            k_start = max(4 * dom - phase[a], 0)
            centre = p0[a] + d[a] * VREF * TS * k_start
            legs = TROT_PAIRS[dom % 2] if C == 2 else [0, 1, 2, 3]
            foot[a, kk] = STANCE[:, legs] + centre[:, None]
    obstacles = make_obstacles(rng, n_obs, sc)
    nbr_state = np.stack([x0[:, 0], x0[:, 2], x0[:, 1], x0[:, 3]], 1)
    return dict(x0=x0, ref=ref.reshape(A, 4 * N), foot=foot, obstacles=obstacles, nbr_state=nbr_state)


HCOM12 = 0.3      # SRB-12 mode: nominal CoM height of the synthetic batches


def make_batch12(n_agents: int, N: int = 10, gait: str = "trot", seed: int = 0, n_obs: int | None = None):
    """SRB-12 extension mode: the LIP batch's arena, starts, goal, obstacles
    and trot schedule, lifted to the 12-state single rigid body.  Returns dict(x0 [A,12],
    xref [A,N,12] (states x_1..x_N), foot [A,N,4,3] (world foot positions per grid),
    contact [A,N,4] int32, obstacles [n_obs,2], nbr_state [A,4] (x, y, xdot, ydot))."""
    rng = np.random.default_rng(seed)
    A = int(n_agents)
    sc = arena_scale(A)
    if n_obs is None:
        n_obs = int(round(20 * sc * sc))
    p0 = np.stack([rng.uniform(0, 9.0 * sc, A), rng.uniform(-2.0 * sc, 2.0 * sc, A)], 1)
    goal = GOAL * np.array([sc, 1.0])
    d = goal - p0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    head = np.arctan2(d[:, 1], d[:, 0])
    v0 = d * rng.uniform(0, 0.3, (A, 1)) + rng.uniform(-0.05, 0.05, (A, 2))
    x0 = np.zeros((A, 12))
    x0[:, 0:2] = p0
    x0[:, 2] = HCOM12 + rng.uniform(-0.01, 0.01, A)
    x0[:, 3:5] = rng.uniform(-0.02, 0.02, (A, 2))
    x0[:, 5] = head + rng.uniform(-0.1, 0.1, A)
    x0[:, 6:8] = v0
    x0[:, 9:12] = rng.uniform(-0.05, 0.05, (A, 3))
    k = np.arange(1, N + 1)
    xref = np.zeros((A, N, 12))
    xref[:, :, 0] = p0[:, None, 0] + d[:, None, 0] * VREF * TS * k
    xref[:, :, 1] = p0[:, None, 1] + d[:, None, 1] * VREF * TS * k
    xref[:, :, 2] = HCOM12
    xref[:, :, 5] = head[:, None]
    xref[:, :, 6] = d[:, None, 0] * VREF
    xref[:, :, 7] = d[:, None, 1] * VREF
    foot = np.zeros((A, N, 4, 3))
    contact = np.zeros((A, N, 4), np.int32)
    phase = rng.integers(0, 4, A)
    c, s = np.cos(head), np.sin(head)
    for a in range(A):
        Rm = np.array([[c[a], -s[a]], [s[a], c[a]]])
        off = (Rm @ STANCE).T                                   # (4, 2) stance offsets along the heading
        for kk in range(N):
            dom = (kk + phase[a]) // 4
            k_start = max(4 * dom - phase[a], 0)
            centre = p0[a] + d[a] * VREF * TS * k_start
            foot[a, kk, :, :2] = centre[None, :] + off
            legs = TROT_PAIRS[dom % 2] if gait == "trot" else [0, 1, 2, 3]
            contact[a, kk, legs] = 1
    obstacles = make_obstacles(rng, n_obs, sc)
    nbr_state = np.stack([x0[:, 0], x0[:, 1], x0[:, 6], x0[:, 7]], 1)
    return dict(x0=x0, xref=xref, foot=foot, contact=contact, obstacles=obstacles, nbr_state=nbr_state)
