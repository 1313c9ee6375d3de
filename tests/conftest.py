import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


@pytest.fixture(scope="session")
def gpu_ctx():
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def golden_index():
    import json
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        return json.load(f)


def golden_image(name: str) -> bytes:
    with open(os.path.join(GOLDEN, f"edge_{name}.bin"), "rb") as f:
        return f.read()
