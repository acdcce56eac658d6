import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librt_hip.so)")


@pytest.fixture(scope="session")
def renderer():
    from bevy_raytrace_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()
