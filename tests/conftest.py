"""Shared test setup.  `-m gpu` tests need a gfx950 device and call the HIP
path through the C ABI; everything else runs on the CPU (the oracle is the
checker, never the product)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "fft-convolution_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; calls the HIP path through the C ABI")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.lib()
    return oracle


def _reset_torch_stream():
    if "torch" in sys.modules:
        torch = sys.modules["torch"]
        if torch.cuda.is_available():
            torch.cuda.set_stream(torch.cuda.default_stream())


@pytest.fixture(autouse=True)
def _torch_default_stream(request):
    """Every gpu test starts and ends on torch's default stream: a test that
    leaves another current stream (torch.cuda.set_stream) would make a later
    test's torch copies and stream-0 library calls run on different streams."""
    gpu = request.node.get_closest_marker("gpu") is not None
    if gpu:
        _reset_torch_stream()
    yield
    if gpu:
        _reset_torch_stream()


@pytest.fixture(scope="session")
def amd():
    import fftconv_amd

    if fftconv_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X (there is no CPU fallback)")
    return fftconv_amd
