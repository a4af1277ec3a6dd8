"""The driver's round-end smoke check (__graft_entry__.smoke) run inside the GPU suite, so a change that
breaks it shows up with the other GPU tests (round 5: the QP warm-start tolerance broke its logged-QP
comparison until the check set the option the MPC_dist shims set)."""
import pytest


@pytest.mark.gpu
def test_graft_entry_smoke():
    import __graft_entry__
    __graft_entry__.smoke()
