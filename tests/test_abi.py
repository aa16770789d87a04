"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/fftconv.h declares (and the Python mirror binds exactly those),
its pure host functions agree with the oracle, and without a device it fails
loudly instead of falling back to the CPU."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fftconv.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fftconv_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_trait_surface():
    syms = declared_symbols()
    for kind in ("uniform", "twostage", "crossfade"):
        for op in ("init", "update", "reset", "process", "clone", "destroy"):
            assert f"fftconv_{kind}_{op}" in syms, (kind, op)


def test_library_exports_every_declared_symbol():
    import fftconv_amd

    lib = ctypes.CDLL(fftconv_amd.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(fftconv_amd.SIGNATURES) == declared_symbols()


def test_pure_host_functions_match_oracle(oracle_mod):
    import fftconv_amd

    for n in (0, 1, 2, 512, 1023):
        assert fftconv_amd.complex_size(n) == oracle_mod.complex_size(n)
    rng = np.random.default_rng(0)
    cases = [(64, 262144), (64, 12000), (1, 1), (0, 7), (7, 3)] + [
        (int(h), int(L)) for h, L in zip(rng.integers(1, 4096, 200), rng.integers(1, 2_000_000, 200))]
    for h, L in cases:
        assert fftconv_amd.compute_tail_block_size(h, L) == oracle_mod.compute_tail_block_size(h, L), (h, L)


def test_no_cpu_fallback_without_device():
    import fftconv_amd

    if fftconv_amd.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(fftconv_amd.DeviceError):
        fftconv_amd.FFTConvolver.init(np.ones(8, np.float32), 4, 8)
    with pytest.raises(fftconv_amd.DeviceError):
        fftconv_amd.TwoStageFFTConvolver.init(np.ones(8, np.float32), 4, 8)
    with pytest.raises(fftconv_amd.DeviceError):
        fftconv_amd.CrossfadeConvolver.init(np.ones(8, np.float32), 4, 8)


def test_kernel_variant_knob_range():
    """fftconv_set_kernel_variant (include/fftconv.h): -1 (automatic) and
    0..4095 are accepted (bits 0-11), anything else is FFTCONV_E_INVALID; a
    host-only setter, no device needed."""
    import fftconv_amd

    try:
        for v in (0, 64, 128, 255, 511, 1024, 2047, 4095):
            fftconv_amd.set_kernel_variant(v)
            assert fftconv_amd.get_kernel_variant() == v
        for bad in (4096, -2, -255):
            with pytest.raises(fftconv_amd.ConvolutionPanic):
                fftconv_amd.set_kernel_variant(bad)
            assert fftconv_amd.get_kernel_variant() == 4095
    finally:
        fftconv_amd.set_kernel_variant(-1)
    assert fftconv_amd.get_kernel_variant() == -1
