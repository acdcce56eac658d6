import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--rt-lib", default=None,
                     help="run the in-process tests against another build of the C-ABI "
                          "(e.g. bevy_raytrace_amd/librt_hip_checked.so, the bounds-checked build)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librt_hip.so)")
    lib = config.getoption("--rt-lib")
    if lib:
        from bevy_raytrace_amd import abi
        abi.LIB_PATH = os.path.abspath(lib)


@pytest.fixture(scope="session")
def _session_renderer():
    from bevy_raytrace_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


@pytest.fixture
def renderer(_session_renderer):
    """The session's context, with every A/B knob (rt_debug_tune) at its
    product default on entry and on exit."""
    _session_renderer.tune(None)
    yield _session_renderer
    _session_renderer.tune(None)
