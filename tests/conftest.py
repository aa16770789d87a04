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


@pytest.fixture(scope="session")
def amd():
    import fftconv_amd

    if fftconv_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X (there is no CPU fallback)")
    return fftconv_amd
