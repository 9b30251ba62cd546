import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fractal-ray-marching_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _make(path):
    subprocess.check_call(["make", "-s", "-C", path])


@pytest.fixture(scope="session")
def frm_lib():
    """libfrm.so, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    so = os.path.join(PKG, "lib", "libfrm.so")
    if not os.path.exists(so):
        _make(PKG)
    import frm
    return frm.load()


@pytest.fixture(scope="session")
def oracle():
    from oracle import frm_oracle
    frm_oracle.load()
    return frm_oracle


@pytest.fixture(scope="session")
def host_replay():
    import ctypes
    path = os.path.join(ROOT, "tests", "native")
    _make(path)
    return ctypes.CDLL(os.path.join(path, "build", "libhost_replay.so"))


@pytest.fixture(scope="session")
def gpu_renderer_factory(frm_lib):
    import frm
    if frm.device_count() < 1:
        pytest.fail("no GPU visible to libfrm (gpu tests must run on the MI355X box)")

    def make(max_steps=0, flags=0, device=0):
        return frm.Renderer(device=device, max_steps=max_steps, flags=flags)

    return make
