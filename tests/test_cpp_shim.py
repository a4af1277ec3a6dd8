"""The C++ MPC_dist shim (include/srbnmpc_mpc_dist.hpp) compiles against the C ABI, links
libsrbnmpc.so, and -- on a GPU -- reproduces the reference's logged instance (KAT-2)."""
import os
import subprocess

import numpy as np
import pytest
from conftest import ROOT

DRIVER_SRC = os.path.join(ROOT, "tests", "cpp", "mpc_dist_driver.cpp")
LIBDIR = os.path.join(ROOT, "srb-cbf-nmpc_amd", "srbnmpc")


def build_driver(tmp_path):
    exe = str(tmp_path / "mpc_dist_driver")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), DRIVER_SRC,
                    "-L", LIBDIR, "-lsrbnmpc", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def write_input(path, kat2):
    obst = np.asarray(kat2["obstacle"])
    vals = list(kat2["x0"]) + list(np.asarray(kat2["ref"]).ravel()) + [2] + list(obst) + [50.0, 50.0]
    with open(path, "w") as f:
        f.write("\n".join(repr(float(v)) if i != 20 else "2" for i, v in enumerate(vals)))


def test_shim_compiles_and_fails_cleanly_without_gpu(tmp_path, kat2):
    torch = pytest.importorskip("torch")
    exe = build_driver(tmp_path)
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_shim_on_reference_instance")
    inp = tmp_path / "in.txt"
    write_input(inp, kat2)
    r = subprocess.run([exe, str(inp), "1"], capture_output=True, text=True)
    assert r.returncode == 3 and "srb_ctx_create" in r.stderr, r.stderr


@pytest.mark.gpu
def test_shim_on_reference_instance(tmp_path, kat2):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = build_driver(tmp_path)
    inp = tmp_path / "in.txt"
    write_input(inp, kat2)
    r = subprocess.run([exe, str(inp), "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    v = r.stdout.split()
    assert v[:2] == ["0", "0"]
    nums = np.array([float(t) for t in v[2:]])
    X, xq, alpha = nums[:16], nums[16:16 + 41], nums[16 + 41:16 + 61].reshape(4, 5)   # nv = 8 N + 1 = 41
    np.testing.assert_allclose(X, np.asarray(kat2["x_nlp"])[:16], atol=1e-6)
    np.testing.assert_allclose(xq[:24], kat2["logged_qp_x"], atol=2e-9)
    import oracle
    np.testing.assert_allclose(alpha, oracle.fit_bezier([0, 0, 0, 0], X.reshape(4, 4)), atol=1e-9)


@pytest.mark.gpu
def test_shim_hl_planner_matches_oracle(tmp_path):
    """generateReferenceTrajectory through the C++ shim == the CPU restatement, bit for bit."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = build_driver(tmp_path)
    loop = 4000
    r = subprocess.run([exe, "hl", str(loop)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    nums = np.array([float(t) for t in r.stdout.split()])
    T = loop // 40
    Pr = nums[:8 * T].reshape(T, 8).T
    Prd = nums[8 * T:].reshape(T, 8).T
    import oracle
    R, Rd = oracle.hl_plan([0.0, 0.0, 0.0, -0.9, -1, 0, -1, -0.9], [[3.0, 0.2], [5.0, -0.6], [7.0, 0.4]], loop=loop)
    np.testing.assert_array_equal(Pr, R)
    np.testing.assert_array_equal(Prd, Rd)


@pytest.mark.gpu
def test_shim_horizon_10_trot_vs_oracle(tmp_path):
    """BASELINE configs[0] (one agent, horizon 10, trot) through the C++ MPC_dist shim constructed with
    horizon 10 (the reference hard-codes NDOMAIN = 4, MPC_dist.cpp:92, :104): status, predicted
    states, QP point and alpha_COM against the oracle on the same window, footholds and obstacles."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle
    from srbnmpc.mpc_dist import INIT_FOOTPRINT
    exe = build_driver(tmp_path)
    N, C = 10, 2
    x0 = np.array([0.02, 0.1, -0.01, 0.02])
    k = np.arange(N)
    ref = np.stack([0.27 * 0.043 * (k + 1), np.full(N, 0.27), np.zeros(N), np.zeros(N)], 1).ravel()
    obst = np.array([[0.9, 0.35], [2.0, -1.0], [50.0, 50.0]])
    vals = list(x0) + list(ref) + [len(obst)] + list(obst.ravel())
    inp = tmp_path / "in10.txt"
    with open(inp, "w") as f:
        f.write("\n".join(str(len(obst)) if i == 4 + 4 * N else repr(float(v)) for i, v in enumerate(vals)))
    r = subprocess.run([exe, str(inp), "1", str(N), "trot"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    v = r.stdout.split()
    nv = (6 + C) * N + 1
    nums = np.array([float(t) for t in v[2:]])
    X, xq, alpha = nums[:4 * N], nums[4 * N:4 * N + nv], nums[4 * N + nv:4 * N + nv + 20].reshape(4, 5)
    F = INIT_FOOTPRINT[[0, 3]].T                     # FR, RL stance around Pstart = 0 (gaitDomain 0)
    foot = np.repeat(F[None], N, 0)
    o = oracle.solve_batch(oracle.params(N, C, K_obs=1, use_nlp=1, tol_qp=0.0), x0[None], ref[None], foot[None], obst)
    assert [int(v[0]), int(v[1])] == o["status"][0].tolist() == [0, 0]
    np.testing.assert_allclose(X, o["x"][0, :4 * N], atol=1e-4, rtol=0)
    np.testing.assert_allclose(xq[:6 * N], o["x_qp"][0, :6 * N], atol=1e-6, rtol=0)
    np.testing.assert_allclose(alpha, oracle.fit_bezier([0.0, 0.0, 0.0, 0.0], X[:16].reshape(4, 4)), atol=1e-9)
