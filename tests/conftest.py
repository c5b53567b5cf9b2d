import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


@pytest.fixture(scope="session")
def engine():
    from shadow_amd.routing import Engine
    eng = Engine(0)
    yield eng
    eng.close()


@pytest.fixture
def knob(engine):
    """knob(name, value): set a tuning / testing knob of the session engine (shd_set_knob) for
    this test; every knob it touched is put back afterwards."""
    saved = {}

    def set_(name, value, eng=None):
        e = eng or engine
        key = (id(e), name)
        if key not in saved:
            saved[key] = (e, name, e.get_knob(name))
        e.set_knob(name, value)

    yield set_
    for e, name, v in saved.values():
        if e.ctx:
            e.set_knob(name, v)
