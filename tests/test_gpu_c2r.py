"""realfft's C2R error condition, exactly (src/fft_convolver.rs:264-267).

realfft rejects a non-zero imaginary part in the DC or Nyquist bin.  In the
reference that imaginary part is a sum of re * 0 + 0 * re products
(complex_multiply_accumulate over real DC / Nyquist bins), so it is NaN
exactly when some operand row's DC / Nyquist value is not finite -- and 0
when every operand is finite, even if the sum overflows to inf.  Then the
reference runs the C2R on inf without an error and outputs non-finite
samples; the device must do the same (not zero-fill), and advance its state.
Checked on every step kernel: the pipelined step (B 64), the lookahead step
(B 256, S >= 40), the generic chunk loop (B 2048, ragged calls), the long-block
path (B 16384), and the crossfade pair launch."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


def _compare(g, r, what):
    assert np.array_equal(np.isfinite(g), np.isfinite(r)), f"{what}: non-finite masks differ"
    assert np.array_equal(np.isnan(g), np.isnan(r)), f"{what}: NaN masks differ"
    m = np.isfinite(r)
    if m.any():
        assert_close(g[m], r[m], what=what)


@pytest.mark.parametrize("B,L,chunks", [(64, 1000, [64]), (256, 48 * 256, [256]), (2048, 5000, [2048, 700, 1348]),
                                        (16384, 2 * 16384, [16384])])
def test_finite_overflow_is_not_a_c2r_error(amd, oracle_mod, B, L, chunks):
    rng = np.random.default_rng(B)
    h = ir(rng, L)
    hbig = np.full(L, 1e18, np.float32)  # finite response whose DC products overflow f32
    conv = amd.FFTConvolver.init(h, B, L)
    ref = oracle_mod.FFTConvolver.init(h, B, L)
    ncalls = 3 * (L // B + 2)
    seq = [chunks[i % len(chunks)] for i in range(ncalls)]
    overflowed = False
    for i, k in enumerate(seq):
        if i == 4:
            conv.update(hbig)
            ref.update(hbig)
        if i == ncalls // 2:
            conv.update(h)
            ref.update(h)
        x = white(rng, k)
        if i in (5, 6):
            x[:] = 1e18  # finite, but X_dc * H_dc > FLT_MAX
        g, r = conv.process(x), ref.process(x)
        _compare(g, r, f"B {B} call {i}")
        assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill), f"call {i}"
        overflowed |= not np.isfinite(r).all()
    assert overflowed  # the case under test happened: no error, non-finite output


def test_finite_overflow_crossfade_pair(amd, oracle_mod):
    """The crossfade pair launch (B 512, S * B > 16384): both convolvers'
    error checks, and the non-finite mix."""
    rng = np.random.default_rng(5)
    B, L = 512, 40 * 512
    h = ir(rng, L)
    conv = amd.CrossfadeConvolver.init(h, B, L)
    ref = oracle_mod.CrossfadeConvolver.init(h, B, L)
    for i in range(12):
        x = white(rng, B)
        if i == 3:
            x[:] = 1e18
            hb = np.full(L, 1e18, np.float32)
            conv.update(hb)
            ref.update(hb)
        _compare(conv.process(x), ref.process(x), f"block {i}")
