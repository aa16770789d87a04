"""The oracle's restatement of realfft (Fft::forward / Fft::inverse,
src/fft_convolver.rs:36-49) pinned against an independent f64 DFT (numpy):
the crates themselves are absent, so this and the reference's
delta-IR passthrough tests are what pin the transform convention --
forward unnormalised, inverse divided by n, DC / Nyquist imaginary parts 0."""
import numpy as np
import pytest


@pytest.mark.parametrize("n", [2, 4, 8, 16, 128, 512, 1024, 8192, 16384])
def test_rfft_matches_f64_dft(oracle_mod, n):
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    X = oracle_mod.rfft_forward(x)
    R = np.fft.rfft(x.astype(np.float64))
    assert X.shape == (n // 2 + 1,)
    assert X[0].imag == 0 and X[-1].imag == 0
    assert np.max(np.abs(X - R)) <= 1e-6 * np.max(np.abs(R))
    y, bad = oracle_mod.rfft_inverse(X, n)
    assert not bad
    assert np.max(np.abs(y - x)) <= 2e-6


def test_rfft_inverse_flags_input_values(oracle_mod):
    n = 64
    X = oracle_mod.rfft_forward(np.ones(n, np.float32))
    assert X[0].real == n and np.all(np.abs(X[1:]) < 1e-5)
    y, bad = oracle_mod.rfft_inverse(X, n)
    assert not bad and np.allclose(y, 1.0, atol=1e-6)
    Xb = X.copy()
    Xb[-1] += 1j  # non-zero Nyquist imaginary part: realfft's FftError::InputValues
    y2, bad2 = oracle_mod.rfft_inverse(Xb, n)
    # computed with that part taken as 0, and not divided by n: Fft::inverse
    # returns the error through `?` (src/fft_convolver.rs:42) before :44-46
    assert bad2 and np.array_equal(y2, y * n)
