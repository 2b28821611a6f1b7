import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF_DIR = "/root/reference/RayMarch Renderer"
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and librmr.so")
    config.addinivalue_line("markers", "slow: long-running")


def has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def renderer():
    from raymarchrenderer_amd import Renderer
    r = Renderer(0, 64, 64)
    yield r
    r.close()
