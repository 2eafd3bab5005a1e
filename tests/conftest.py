import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librmx.so on the GPU)")


def pytest_collection_modifyitems(config, items):
    if os.path.exists("/dev/kfd"):
        return
    skip = pytest.mark.skip(reason="no AMD GPU in this container (/dev/kfd missing)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _env_tuning():
    """RMX_TEST_TUNING="k=v,k=v": run the suite with kernel knobs set (A/B of a kernel variant under
    the same parity tests); applied before every test, after any test-local knob reset."""
    spec = os.environ.get("RMX_TEST_TUNING", "")
    if spec:
        import rmx
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            rmx.set_tuning(k, int(v))
    yield
