import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FACE_CFG = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
PED_CFG = os.path.join(ROOT, "surfcascade_amd", "models", "ped64x128_synth.cfg")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def face_cascade(oracle):
    with open(FACE_CFG) as f:
        return oracle.cascade_from_cfg(f.read())


@pytest.fixture(scope="session")
def ped_cascade(oracle):
    with open(PED_CFG) as f:
        return oracle.cascade_from_cfg(f.read(), tmpl_w=64, tmpl_h=128)
