import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_addoption(parser):
    parser.addoption("--srbnmpc-lib", default=None,
                     help="diagnostics: run the tests against the variant build libsrbnmpc_<tag>.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    name = config.getoption("--srbnmpc-lib")
    if name:
        import srbnmpc
        srbnmpc.use_library(name)


def _ensure_built():
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    if not os.path.exists(os.path.join(ROOT, "srb-cbf-nmpc_amd", "srbnmpc", "libsrbnmpc.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "srb-cbf-nmpc_amd")], check=True)


_ensure_built()


QP_WARM = 4   # srbnmpc.QP_WARM: a QP stage followed by the NLP that stopped at the warm-start tolerance


def ok_elem(st):
    """Per stage: converged -- OPTIMAL, or for the QP stage (column 0) QP_WARM."""
    st = np.asarray(st)
    o = st == 0
    o[:, 0] |= st[:, 0] == QP_WARM
    return o


def converged(st):
    """Rows whose stages all converged (QP OPTIMAL or QP_WARM, NLP OPTIMAL)."""
    return ok_elem(st).all(1)


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        d = json.load(f)
    return d


@pytest.fixture(scope="session")
def kat2():
    d = load_golden("kat2.json")
    return {k: (np.asarray(v) if isinstance(v, list) else v) for k, v in d.items()}
