import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


try:  # `--hypothesis-profile=diag`: no shrinking, the first failing example is reported as it failed
    from hypothesis import Phase
    from hypothesis import settings as _hsettings
    _hsettings.register_profile("diag", phases=[Phase.explicit, Phase.reuse, Phase.generate])
    from hypothesis import Verbosity
    _hsettings.register_profile("verbose", verbosity=Verbosity.verbose, print_blob=True)
except ImportError:
    pass


def trace(*a):
    """Progress lines for GPU diagnosis runs (REVEL_TEST_TRACE=1)."""
    if os.environ.get("REVEL_TEST_TRACE"):
        print("[trace]", *a, file=sys.stderr, flush=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "experiment: kernel arms of tools/experiments (GPU, `-m experiment` only)")


def pytest_collection_modifyitems(config, items):
    """The experiment arms run only when the marker expression names them:
    `-m gpu` certifies librevel_wal.so alone, and `-m "not gpu"` (CPU) must
    not try to load libexperiments.so."""
    if "experiment" in (config.option.markexpr or ""):
        return
    skip = pytest.mark.skip(reason="experiment arm: run with -m experiment on a GPU box")
    for it in items:
        if it.get_closest_marker("experiment"):
            it.add_marker(skip)


def _traced(cls, names):
    """REVEL_TEST_TRACE=1: a trace line before every listed GpuContext call."""
    for name in names:
        f = getattr(cls, name)

        def wrap(f=f, name=name):
            def g(self, *a, **k):
                trace(name, *[getattr(x, "nbytes", x) if not isinstance(x, (list, bytes)) else len(x) for x in a][:4],
                      {kk: v for kk, v in k.items() if isinstance(v, int)})
                return f(self, *a, **k)
            return g
        setattr(cls, name, wrap())


if os.environ.get("REVEL_LIB"):  # another build of librevel_wal.so (A/B and diagnosis runs)
    from revel_amd import _lib as _revel_lib
    _revel_lib.LIB_PATH = os.path.abspath(os.environ["REVEL_LIB"])


@pytest.fixture(scope="session")
def gpu_ctx():
    from revel_amd import gpu
    if os.environ.get("REVEL_TEST_TRACE"):
        _traced(gpu.GpuContext, ["upload", "verify_image", "append_records", "replay_memory", "reassemble",
                                 "replay_file", "replay_batches"])
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
