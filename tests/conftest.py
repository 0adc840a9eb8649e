import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "panda-lang-manip_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "task_layer.npz")))


@pytest.fixture(scope="session")
def render_golden():
    import numpy as np

    return dict(np.load(os.path.join(ROOT, "tests", "golden", "render.npz")))
