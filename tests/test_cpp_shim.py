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
    X, xq, alpha = nums[:16], nums[16:40], nums[40:60].reshape(4, 5)
    np.testing.assert_allclose(X, np.asarray(kat2["x_nlp"])[:16], atol=1e-6)
    np.testing.assert_allclose(xq, kat2["logged_qp_x"], atol=2e-9)
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
