import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "modify-sift-gpu_amd", "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _have_gpu():
    try:
        import sgpu
        return sgpu.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx():
    import sgpu
    if not _have_gpu():
        pytest.fail("GPU test requested but no gfx950 device / libsiftgpu.so is usable")
    ctx = sgpu.SiftContext(0)
    yield ctx
    ctx.close()
