"""CPU tests of the product library's C ABI and host logic (no GPU compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest
from conftest import ROOT

import oracle
import srbnmpc
from srbnmpc import workload


def _declared_functions():
    txt = open(os.path.join(ROOT, "include", "srbnmpc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(srb(?:12)?_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    names = _declared_functions()
    assert len(names) >= 12
    lib = ctypes.CDLL(srbnmpc.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n


def test_library_contains_gfx950_code_object():
    data = open(srbnmpc.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    import re
    hdr = open(os.path.join(ROOT, "srb-cbf-nmpc_amd", "csrc", "srb_kernel_params.h")).read()
    # the product list (the #else branch; SRB_DEV_INSTANCES builds only a few for register reports)
    inst = re.findall(r"X\((\d+), (\d+), (\d+), (\d+), (\d+), (\d+)\)",
                      hdr.split("#define SRB_KERNEL_INSTANCES(X) \\")[1].split("#define SRB_KI_PART0")[0])
    assert len(inst) >= 4 and any(i[2] == "4" for i in inst)
    assert any(i[3] != "0" for i in inst) and sum(i[3] == "0" for i in inst) >= 4   # compiled shapes + run-time ones
    for i in inst:                            # every register-bound instance is in the code object
        assert ("srb_nmpc_kernel_" + "_".join(i)).encode() in data


def test_param_defaults_are_the_reference_constants():
    p = srbnmpc.default_params(4, 4)
    o = oracle.params(4, 4)
    for k, _ in srbnmpc.Params._fields_:
        assert getattr(p, k) == getattr(o, k), k
    assert (p.N, p.C, p.K_obs, p.K_nbr) == (4, 4, 1, 0)             # MPC_dist.cpp:92,132,371-396
    assert (p.Qw, p.Pw, p.Rw, p.Sw) == (300.0, 2000.0, 0.1, 3000.0)  # MPC_dist.cpp:172-175
    assert p.eps_obs == float(np.float32(1.9)) and p.vsat == float(np.float32(0.35))   # float constants
    assert p.tol == 1e-6 and p.qp_maxit == 25                         # GlobalOptions.h:23-25
    assert p.nv == 41


@pytest.mark.parametrize("N,C,K", [(4, 4, 1), (10, 2, 3), (10, 2, 11), (20, 2, 11), (10, 4, 3)])
def test_lds_fits_and_sizes(N, C, K):
    p = srbnmpc.default_params(N, C, K_obs=min(K, 3), K_nbr=max(K - 3, 0))
    b = srbnmpc.lds_bytes(p)
    assert 0 < b <= 160 * 1024
    assert b % 8 == 0


def test_fit_bezier_host_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(5):
        buf = rng.normal(size=4); X = rng.normal(size=(4, 4))
        np.testing.assert_allclose(srbnmpc.fit_bezier(buf, X), oracle.fit_bezier(buf, X), atol=1e-12)


def test_ctx_create_rejects_bad_params():
    lib = srbnmpc.lib()
    p = srbnmpc.default_params(40, 4)          # nz = 121 > 64 lanes
    h = ctypes.c_void_p()
    rc = lib.srb_ctx_create(ctypes.byref(p), 8, 0, ctypes.byref(h))
    assert rc != 0
    assert b"exceeds" in lib.srb_last_error()


def test_no_silent_cpu_fallback_without_gpu():
    """Without a GPU the solver must fail loudly, never compute on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        srbnmpc.BatchSolver(srbnmpc.default_params(4, 4), 4)


def test_workload_shapes_and_determinism():
    a = workload.make_batch(16, 10, 2, seed=1)
    b = workload.make_batch(16, 10, 2, seed=1)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    assert a["x0"].shape == (16, 4) and a["ref"].shape == (16, 40) and a["foot"].shape == (16, 10, 2, 2)
    assert a["nbr_state"].shape == (16, 4)
    # footholds: each grid holds one trot diagonal of the default stance
    F = a["foot"][0, 0]
    assert np.isclose(F[0, 0] - F[0, 1], 0.2188 + 0.1472) or np.isclose(F[0, 0] - F[0, 1], -(0.2188 + 0.1472))


def test_mpcdist_host_planners():
    """copPlanner_eventbase / footholdsPlanner (MPC_dist.cpp:702-782, 1204-1266) on the host."""
    m = srbnmpc.MPCDist()
    m.setAgentID(1)
    m.setPstart(np.array([0.0, 0.0, 2.0, -1.0, 0, 0, 0, 0]))
    T = 40
    Pr = np.arange(8 * T, dtype=float).reshape(8, T)
    m.setReferenceTrajectory(Pr, -Pr)
    m.gaitDomain_ = 2
    ref = m.copPlanner_eventbase(4)
    np.testing.assert_array_equal(ref.reshape(4, 4)[:, 0], Pr[2, 8:12])    # x of grids
    np.testing.assert_array_equal(ref.reshape(4, 4)[:, 1], -Pr[2, 8:12])   # xdot
    np.testing.assert_array_equal(ref.reshape(4, 4)[:, 2], Pr[3, 8:12])    # y
    m.gaitDomain_ = 0
    m.contactInd = np.array([1, 0, 0, 1])
    F = m.footholdsPlanner()
    np.testing.assert_allclose(F, [[2.0 + 0.2188, 2.0 - 0.1472], [-1.0 - 0.1320, -1.0 + 0.1320]])
    m.contactInd = np.array([0, 1, 1, 0])
    F = m.footholdsPlanner()
    np.testing.assert_allclose(F, [[2.0 + 0.2188, 2.0 - 0.1472], [-1.0 + 0.1320, -1.0 - 0.1320]])
    np.testing.assert_array_equal(m.get_lastState(), np.zeros(4))


def test_split_layout():
    p = srbnmpc.default_params(10, 2)
    x = np.arange(p.nv, dtype=float)
    X, U, L, s = srbnmpc.split(p, x)
    assert X.shape == (10, 4) and U.shape == (10, 2) and L.shape == (10, 2) and s == p.nv - 1
    assert X[1, 0] == 4 and U[0, 0] == 40 and L[0, 0] == 60


def test_ll_params_defaults_and_validation():
    """srb_ll_params_default = Settings::LL_params defaults (Parameters.cpp:62-75) and the
    oracle's; out-of-range parameters are rejected before any device is touched."""
    from srbnmpc import lowlevel
    p = lowlevel.default_params()
    o = oracle.ll_params()
    for k in ("mu", "kp", "kd", "useCLF", "tauPen", "dfPen", "auxPen", "clfPen", "auxMax", "clfEps", "maxit", "tol"):
        assert getattr(p, k) == getattr(o, k), k
    assert (p.kp, p.kd, p.auxPen, p.clfPen, p.clfEps) == (700.0, 40.0, 1e6, 1e8, 0.8)
    lib = lowlevel._bind()
    h = ctypes.c_void_p()
    for bad in (dict(kp=-1.0), dict(clfEps=0.0), dict(tol=0.0), dict(maxit=-1), dict(auxPen=0.0)):
        q = lowlevel.default_params(**bad)
        assert lib.srb_ll_ctx_create(ctypes.byref(q), 8, 0, ctypes.byref(h)) == -1, bad
        assert b"out of range" in lib.srb_last_error()
    assert lib.srb_ll_ctx_create(ctypes.byref(p), 0, 0, ctypes.byref(h)) == -1


def test_ll_no_silent_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        srbnmpc.LowLevelCtrl(max_agents=4)


def test_abi_version_and_struct_size_checks():
    """Versioned C ABI (include/srbnmpc.h SRB_ABI_VERSION): every I/O struct starts with
    struct_size; a caller built against another layout (an older header without the field, or a
    shorter / longer struct) is rejected with SRB_ERR_ARG before any buffer or device is used."""
    from srbnmpc import lowlevel
    lib = srbnmpc.lib()
    hdr = open(os.path.join(ROOT, "include", "srbnmpc.h")).read()
    assert lib.srb_abi_version() == int(re.search(r"#define SRB_ABI_VERSION (\d+)", hdr).group(1)) == srbnmpc.ABI_VERSION
    for cls, fn in ((srbnmpc.Batch, "srb_solve_batch"), (srbnmpc.Batch, "srb_solve_qp"),
                    (srbnmpc.Batch, "srb_solve_batch_device"), (srbnmpc.Prep, "srb_prepare_batch_device"),
                    (lowlevel.LLIO, "srb_ll_calc_torque"), (lowlevel.LLIO, "srb_ll_calc_torque_device")):
        b = cls()
        assert b.struct_size == ctypes.sizeof(cls)
        f = getattr(lib if not fn.startswith("srb_ll") else lowlevel._bind(), fn)
        args = lambda s: (None, 1, ctypes.byref(s)) + ((None,) if fn.endswith("device") else ())
        f.argtypes = None
        for bad in (0, ctypes.sizeof(cls) - 8, ctypes.sizeof(cls) + 8, 0x5a5a5a5a):
            b.struct_size = bad
            assert f(*args(b)) == -1, (fn, bad)
            assert b"struct_size" in lib.srb_last_error(), fn
        b.struct_size = ctypes.sizeof(cls)
        assert f(*args(b)) == -1 and b"null argument" in lib.srb_last_error()   # passes the layout check
    # the mirrors match the C layout: struct_size first, then the pointers 8-byte aligned
    assert srbnmpc.Batch.x0.offset == 8 and srbnmpc.Prep.Pr.offset == 8 and lowlevel.LLIO.ind.offset == 8


def test_no_environment_variable_changes_the_numerics():
    """every numeric knob is a context setting (srb_ctx_set_waves,
    srb_ctx_set_option: polish on/off, its rho and waves, the selection-grid thresholds); the
    product library reads no environment variable at all, so a stray variable on a robot cannot
    change a solution.  Checked on the built library's dynamic symbols and strings."""
    path = srbnmpc.LIB_PATH
    if os.path.basename(path) != "libsrbnmpc.so":
        pytest.skip("a diagnostic build is selected (--srbnmpc-lib)")
    blob = open(path, "rb").read()
    for name in (b"SRB_POLISH_RHO", b"SRB_NMPC_NW", b"SRB_POLISH_NW", b"SRB_GRID_MIN_ROWS", b"SRB_HL_STEP"):
        assert name not in blob, name
    import subprocess
    syms = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", syms), [l for l in syms.splitlines() if "getenv" in l]
    # the option entry points validate without a context or GPU
    lib = srbnmpc.lib()
    assert lib.srb_ctx_set_option(None, srbnmpc.OPTIONS["polish"], 0.0) == -1
    v = ctypes.c_double()
    assert lib.srb_ctx_get_option(None, srbnmpc.OPTIONS["polish_rho"], ctypes.byref(v)) == -1
    hdr = open(os.path.join(ROOT, "include", "srbnmpc.h")).read()
    for k, code in srbnmpc.OPTIONS.items():
        assert re.search(rf"#define SRB_OPT_{k.upper()} {code}\b", hdr), k


def test_stray_environment_variable_does_not_change_the_library():
    """the product package loads libsrbnmpc.so whatever the environment holds; a
    diagnostic build is chosen only by an explicit srbnmpc.use_library() call (bench.py --lib,
    pytest --srbnmpc-lib), which accepts nothing but a libsrbnmpc[_<tag>].so in the package."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [sys.argv[1]]; import os, srbnmpc; "
            "print(os.path.basename(srbnmpc.LIB_PATH))")
    env = dict(os.environ, SRBNMPC_LIB="libsrbnmpc_nowpe.so", SRB_LIB="x.so")
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "srb-cbf-nmpc_amd")
    out = subprocess.run([sys.executable, "-c", code, pkg], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "libsrbnmpc.so"
    for bad in ("/tmp/libsrbnmpc_x.so", "../libsrbnmpc.so", "libother.so", "libsrbnmpc_x.txt"):
        with pytest.raises(ValueError):
            srbnmpc.use_library(bad)
