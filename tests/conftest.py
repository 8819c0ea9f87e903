import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through libart.so's C ABI")


@pytest.fixture(scope="session")
def ctx():
    """One art_ctx for the whole GPU session (device 0)."""
    import art
    c = art.Context(1)
    yield c
    c.close()
