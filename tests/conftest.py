import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine():
    """One engine on cuda:0 for the whole GPU session (4096+ key slots)."""
    from nebula_amd import Engine

    e = Engine(0, max_keys=8192)
    yield e
    e.close()


@pytest.fixture(autouse=True)
def _no_leaked_keys(request):
    """A test that leaves keys installed on the shared engine would shrink the key table for every
    later test (C3/C5 need 4096 slots): destroy what it left and report it."""
    yield
    if "engine" not in request.fixturenames:
        return
    e = request.getfixturevalue("engine")
    left = list(e.live.values())
    for cs in left:
        cs.destroy()
    if left:
        import warnings

        warnings.warn(f"{request.node.nodeid} left {len(left)} keys installed (destroyed)")


@pytest.fixture
def knobs():
    """knobs(name, value): set a process-wide engine knob (neb_set_knob) for this test; every knob
    it set is restored afterwards."""
    from nebula_amd import _lib as L

    saved = {}

    def set_(k, v):
        if k not in saved:
            saved[k] = L.lib().neb_get_knob(k)
        L.check(L.lib().neb_set_knob(k, int(v)), "neb_set_knob")

    yield set_
    for k, v in saved.items():
        L.lib().neb_set_knob(k, v)
