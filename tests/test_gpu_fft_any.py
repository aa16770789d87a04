"""The public Fft at lengths that are not powers of two (src/fft_convolver.rs
:29-49: Fft::init takes any usize and realfft plans it -- RealToComplexOdd /
Even over rustfft's mixed-radix, Rader and Bluestein plans).  On the device
every such n runs Bluestein's chirp-z transform over power-of-two FFTs
(large.hip bs_*; the four-step passes when P = 2^ceil(log2(2n-1)) > 8192).
The oracle restates realfft for powers of two only, so these are checked
against an f64 DFT (numpy) -- bit-level parity with rustfft's plans for these
lengths is unpinned (crates absent).  Tolerance: max|gpu - f64| <= 5e-6 of the
row's peak bin (forward) and of the signal's peak (inverse)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NS = [1, 3, 5, 6, 7, 12, 100, 257, 1000, 1001, 4097, 6000, 44100, 96000]


@pytest.mark.parametrize("n", NS)
def test_fft_any_length_vs_f64(amd, n):
    rng = np.random.default_rng(n)
    rows = 3
    x = rng.uniform(-1, 1, (rows, n)).astype(np.float32)
    f = amd.Fft(n)
    X = f.forward(x)
    assert X.shape == (rows, n // 2 + 1)
    assert np.all(X[:, 0].imag == 0)
    if n % 2 == 0:
        assert np.all(X[:, -1].imag == 0)
    for r in range(rows):
        d = np.fft.rfft(x[r].astype(np.float64))
        peak = np.max(np.abs(d))
        assert np.max(np.abs(X[r] - d)) <= 5e-6 * peak, f"forward n={n}: {np.max(np.abs(X[r] - d)) / peak:.2e}"
    y, bad = f.inverse(X)
    assert not bad.any()
    for r in range(rows):
        yd = np.fft.irfft(X[r].astype(np.complex128), n=n)
        assert np.max(np.abs(y[r] - yd)) <= 5e-6 * np.max(np.abs(yd)), f"inverse n={n}"
    assert np.max(np.abs(y - x)) <= 1e-5


@pytest.mark.parametrize("n", [6, 7, 1000])
def test_fft_any_length_input_values_flag(amd, n):
    """FftError::InputValues for a non-zero DC (any n) or Nyquist (even n)
    imaginary part: flagged, the transform taken with those parts as 0, the
    row not divided by n (Fft::inverse returns through `?` at :42)."""
    rng = np.random.default_rng(50 + n)
    f = amd.Fft(n)
    X = f.forward(rng.uniform(-1, 1, (2, n)).astype(np.float32))
    X[0, 0] += 0.5j
    y, bad = f.inverse(X)
    assert bad[0] and not bad[1]
    Xc = X[0].astype(np.complex128)
    Xc[0] = Xc[0].real
    exp = np.fft.irfft(Xc, n=n) * n  # unnormalised
    assert np.max(np.abs(y[0] - exp)) <= 5e-6 * np.max(np.abs(exp))
    if n % 2 == 0:
        X2 = X[1:].copy()
        X2[0, -1] -= 1j
        _, bad2 = f.inverse(X2)
        assert bad2[0]
