import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def load_golden(name):
    with np.load(GOLDEN / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def spec_state(fx):
    spec = {k[5:]: fx[k].tolist() for k in fx if k.startswith("spec/")}
    state = {k[6:]: fx[k] for k in fx if k.startswith("state/")}
    return spec, state


@pytest.fixture
def golden():
    return load_golden
