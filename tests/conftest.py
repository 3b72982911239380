import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

# the library honours its test hooks (H264MI_CHECK_INJECT*,
# H264MI_DEBUG_FLAG_PICTURE) only in a process that also sets H264MI_TEST=1
# (host/capture.c h264mi_test_hooks); tests/test_knobs.py checks the gate
os.environ.setdefault("H264MI_TEST", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Native libraries are built in-tree; build them if missing."""
    need = [os.path.join(ROOT, "broadway_amd", "lib", "libh264mi.so"),
            os.path.join(ROOT, "broadway_amd", "lib", "libh264gen.so"),
            os.path.join(ROOT, "oracle", "_build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__
        __graft_entry__.build()
    yield
