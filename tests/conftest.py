import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def gpu_ctx():
    """One product context for the whole GPU session (one process on the card)."""
    from scanner_colmap_amd import Context
    ctx = Context(0)
    yield ctx
    ctx.close()
