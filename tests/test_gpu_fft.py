"""The public Fft (src/fft_convolver.rs:7-50) on the device, and the rocFFT
cross-check harness: the convolver's transforms against
the oracle's realfft restatement, an f64 DFT, and rocFFT (torch.fft on a
ROCm device goes through hipFFT -> rocFFT) -- and the IR spectra the
convolver holds against the same transforms, bit for bit."""
import numpy as np
import pytest

from common import ir

pytestmark = pytest.mark.gpu

NS = [2, 4, 16, 128, 256, 512, 1024, 2048, 8192, 16384]


@pytest.mark.parametrize("n", NS)
def test_fft_forward_inverse_vs_oracle_and_f64(amd, oracle_mod, n):
    rng = np.random.default_rng(700 + n)
    rows = 5
    x = rng.uniform(-1, 1, (rows, n)).astype(np.float32)
    f = amd.Fft(n)
    X = f.forward(x)
    assert X.shape == (rows, n // 2 + 1)
    assert np.all(X[:, 0].imag == 0) and np.all(X[:, -1].imag == 0)
    for r in range(rows):
        o = oracle_mod.rfft_forward(x[r])
        d = np.fft.rfft(x[r].astype(np.float64))
        peak = np.max(np.abs(d))
        assert np.max(np.abs(X[r] - o)) <= 1e-6 * peak, "vs the oracle (realfft restatement)"
        assert np.max(np.abs(X[r] - d)) <= 1e-6 * peak, "vs the f64 DFT"
    y, bad = f.inverse(X)
    assert not bad.any()
    assert np.max(np.abs(y - x)) <= 2e-6
    for r in range(rows):
        yo, bo = oracle_mod.rfft_inverse(X[r], n)
        assert not bo
        assert np.max(np.abs(y[r] - yo)) <= 1e-6


@pytest.mark.parametrize("n", [64, 512, 1024, 8192])
def test_rocfft_cross_check(amd, n):
    """R2C and C2R against rocFFT on the same device (torch.fft -> hipFFT ->
    rocFFT): forward unnormalised and inverse / n agree to f32 rounding."""
    import torch

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(800 + n)
    rows = 64
    x = rng.uniform(-1, 1, (rows, n)).astype(np.float32)
    xd = torch.from_numpy(x).to(dev)
    out = torch.empty((rows, n + 2), device=dev)
    s = torch.cuda.Stream(dev)
    f = amd.Fft(n)
    f.forward_device(xd.data_ptr(), n, out.data_ptr(), n + 2, rows, s.cuda_stream)
    s.synchronize()
    ours = torch.view_as_complex(out.view(rows, n // 2 + 1, 2))
    roc = torch.fft.rfft(xd, dim=-1)
    peak = float(roc.abs().max())
    err = float((ours - roc).abs().max())
    assert err <= 2e-6 * peak, f"forward vs rocFFT: {err / peak:.2e}"
    back = torch.empty((rows, n), device=dev)
    st = torch.zeros(rows, dtype=torch.int32, device=dev)
    f.inverse_device(out.data_ptr(), n + 2, back.data_ptr(), n, rows, st.data_ptr(), s.cuda_stream)
    s.synchronize()
    rocb = torch.fft.irfft(roc, n=n, dim=-1)
    assert int(st.sum()) == 0
    assert float((back - rocb).abs().max()) <= 2e-6
    assert float((back - xd).abs().max()) <= 2e-6


def test_fft_inverse_input_values_flag(amd, oracle_mod):
    """A non-zero DC / Nyquist imaginary part: realfft's FftError::InputValues,
    the transform of the row with those parts as 0, and NOT divided by n --
    Fft::inverse returns through `?` (src/fft_convolver.rs:42) before its
    normalisation loop (:44-46)."""
    n = 256
    rng = np.random.default_rng(900)
    X = amd.Fft(n).forward(rng.uniform(-1, 1, (3, n)).astype(np.float32))
    X[1, 0] += 0.5j   # DC imaginary part
    X[2, -1] -= 2j    # Nyquist imaginary part
    y, bad = amd.Fft(n).inverse(X)
    assert bad.tolist() == [False, True, True]
    clean = X.copy()
    clean[:, 0] = clean[:, 0].real
    clean[:, -1] = clean[:, -1].real
    ref = np.fft.irfft(clean.astype(np.complex128), n=n, axis=-1)
    for r in range(3):
        yo, bo = oracle_mod.rfft_inverse(X[r], n)
        assert bo == bad[r]
        assert np.max(np.abs(y[r] - yo)) <= 1e-6 * (n if bad[r] else 1)
        want = ref[r] * (n if bad[r] else 1)  # (unnormalised where flagged)
        assert np.max(np.abs(y[r] - want)) <= 2e-6 * (n if bad[r] else 1)


@pytest.mark.parametrize("B,L", [(64, 1000), (256, 40 * 256 + 9), (512, 3000), (1024, 4100)])
def test_ir_spectra_are_the_fft_of_the_segments(amd, B, L):
    """segments_ir[i] (src/fft_convolver.rs:126-142: copy_and_pad + Fft::forward
    of IR segment i) held by the convolver == Fft.forward of the zero-padded
    segment, bit for bit, and == rocFFT to f32 rounding."""
    import torch

    rng = np.random.default_rng(B + L)
    C = 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    S = conv.seg_count
    f = amd.Fft(2 * B)
    for c in (0, C - 1):
        segs = np.zeros((S, 2 * B), np.float32)
        for i in range(S):
            part = hs[c, i * B:(i + 1) * B]
            segs[i, :part.size] = part
        ref = f.forward(segs)
        roc = torch.fft.rfft(torch.from_numpy(segs).to("cuda:0"), dim=-1).cpu().numpy()
        for i in range(S):
            got = conv.ir_spectrum(c, i)
            assert np.array_equal(got, ref[i]), (c, i)
            assert np.max(np.abs(got - roc[i])) <= 2e-6 * max(np.max(np.abs(roc[i])), 1e-30)
