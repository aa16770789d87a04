"""The long-block path (fft-convolution_amd/csrc/large.hip): block sizes past
the fused kernel's LDS, B = 2^14 .. 2^22, which the reference takes like any
other (src/fft_convolver.rs:115-117) and which its two-stage tail reaches for
long responses (compute_tail_block_size, :520-526: head 512 / IR 200,000 ->
T = 16,384; head 1024 / IR 1,000,000 -> T = 32,768).  Every case against the
oracle (the reference's state machines restated in C) and, for the uniform
convolver, the f64 direct convolution.  Tolerance: max|gpu - ref| <= 1e-5 *
max|ref| (REL_TOL); the public Fft at 2e-6 of the row's peak."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


def run_chunks(conv, x, chunks):
    ys, p = [], 0
    for k in chunks:
        ys.append(conv.process(x[..., p:p + k]))
        p += k
    return np.concatenate(ys, axis=-1)


@pytest.mark.parametrize("n", [32768, 65536, 1 << 20])
def test_fft_large_vs_oracle_f64_rocfft(amd, oracle_mod, n):
    """Fft::forward / inverse (src/fft_convolver.rs:36-49) at N = 2^15, 2^16
    and 2^20: four-step on the device, against the oracle's realfft
    restatement, an f64 DFT and rocFFT."""
    import torch

    rng = np.random.default_rng(n % 9973)
    rows = 3
    x = rng.uniform(-1, 1, (rows, n)).astype(np.float32)
    f = amd.Fft(n)
    X = f.forward(x)
    assert X.shape == (rows, n // 2 + 1)
    assert np.all(X[:, 0].imag == 0) and np.all(X[:, -1].imag == 0)
    roc = torch.fft.rfft(torch.from_numpy(x).to("cuda:0"), dim=-1).cpu().numpy()
    for r in range(rows):
        d = np.fft.rfft(x[r].astype(np.float64))
        peak = np.max(np.abs(d))
        o = oracle_mod.rfft_forward(x[r])
        assert np.max(np.abs(X[r] - o)) <= 2e-6 * peak, "vs the oracle"
        assert np.max(np.abs(X[r] - d)) <= 2e-6 * peak, "vs the f64 DFT"
        assert np.max(np.abs(X[r] - roc[r])) <= 2e-6 * peak, "vs rocFFT"
    y, bad = f.inverse(X)
    assert not bad.any()
    assert np.max(np.abs(y - x)) <= 4e-6
    yo, bo = oracle_mod.rfft_inverse(X[0], n)
    assert not bo
    assert np.max(np.abs(y[0] - yo)) <= 2e-6
    # FftError::InputValues: flagged, computed with the imaginary part as 0, not scaled (:42-46)
    X2 = X[:1].copy()
    X2[0, 0] += 0.25j
    y2, bad2 = f.inverse(X2)
    yo2, bo2 = oracle_mod.rfft_inverse(X2[0], n)
    assert bad2[0] and bo2
    assert np.max(np.abs(y2[0] - yo2)) <= 2e-6 * np.max(np.abs(yo2))


UNIFORM_LARGE = [
    # (block, ir_len, chunk pattern)
    (16384, 3 * 16384 + 100, [16384]),
    (16384, 2 * 16384 + 7, [5000, 16384, 30000, 11]),    # ragged chunks, multi-block calls
    (20000, 40000, [32768, 1000]),                        # block 20000 -> 32768
    (32768, 4 * 32768, [32768, 65536]),
    (1 << 17, 300000, [1 << 17]),
]


@pytest.mark.parametrize("block,L,pattern", UNIFORM_LARGE)
def test_uniform_large_vs_oracle(amd, oracle_mod, block, L, pattern):
    """FFTConvolver init / process (:105-172, :215-295) past the ring's wrap,
    two channels with distinct responses, the device state (current, active,
    fill) equal to the oracle's after every call."""
    rng = np.random.default_rng(block + L)
    C = 2
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, block, L, channels=C)
    refs = [oracle_mod.FFTConvolver.init(hs[c], block, L) for c in range(C)]
    B, S = refs[0].block_size, refs[0].seg_count
    assert conv.block_size == B and conv.seg_count == S
    chunks, tot = [], 0
    while tot < (S + 2) * B or len(chunks) < 4:
        for k in pattern:
            chunks.append(k)
            tot += k
    x = np.stack([white(rng, tot) for _ in range(C)])
    p = 0
    for k in chunks:
        got = conv.process(x[:, p:p + k])
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c, p:p + k]), what=f"B={B} ch {c} @{p}")
            assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)
        p += k
    if B <= 32768:
        conv2 = amd.FFTConvolver.init(hs, block, L, channels=C)
        y = run_chunks(conv2, x, chunks)
        for c in range(C):
            assert_close(y[c], oracle_mod.direct_convolution(x[c], hs[c]), what=f"B={B} ch {c} vs f64")


def test_uniform_large_update_reset_clone(amd, oracle_mod):
    """update (:174-213: a shorter response zeroes the rows past it, then a
    full one), update_channel, a mid-block update, reset (:296-306) and clone,
    at B = 16384."""
    rng = np.random.default_rng(1616)
    C, B, L = 3, 16384, 5 * 16384
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
    plan = [B, B, 7000, B, 9384, B, B, B, 3 * B, B]
    twin = None
    rtwins = None
    for j, k in enumerate(plan):
        if j == 2:
            hn = np.stack([ir(rng, 2 * B - 5) for _ in range(C)])
            conv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        if j == 4:  # mid-block (fill 7000): pre_multiplied and the overlap are zeroed
            h1 = ir(rng, L)
            conv.update_channel(1, h1)
            refs[1].update(h1)
        if j == 6:
            twin = conv.clone()
            rtwins = [r.clone() for r in refs]
        if j == 8:
            conv.reset()
            for r in refs:
                r.reset()
        x = np.stack([white(rng, k) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"call {j} ch {c}")
            assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)
        if twin is not None and j >= 6:
            if j > 6:
                gt = twin.process(x)
                for c in range(C):
                    assert_close(gt[c], rtwins[c].process(x[c]), what=f"clone call {j} ch {c}")


def test_uniform_large_ir_spectrum_is_fft(amd):
    """The H rows the long-block handle holds (transposed bin order inside,
    natural order through the ABI) are Fft::forward of each zero-padded
    segment (:131-142), bit for bit: the same passes run both."""
    rng = np.random.default_rng(4242)
    B, L = 16384, 2 * 16384 + 999
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, B, L)
    f = amd.Fft(2 * B)
    for s in range(conv.seg_count):
        seg = np.zeros(2 * B, np.float32)
        part = h[s * B:(s + 1) * B]
        seg[:part.size] = part
        assert np.array_equal(conv.ir_spectrum(0, s), f.forward(seg[None])[0]), f"segment {s}"


def test_uniform_large_nonfinite(amd, oracle_mod):
    """A NaN block: realfft's C2R fails, the reference zero-fills the call's
    output and leaves fill / current (:264-267); the NaN spectrum stays in the
    FDL and fails the next S - 1 blocks the same way."""
    rng = np.random.default_rng(77)
    B, L = 16384, 2 * 16384
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, B, L)
    ref = oracle_mod.FFTConvolver.init(h, B, L)
    for i in range(8):
        x = white(rng, B if i != 5 else 6000)
        if i == 2:
            x[100] = np.nan
        g, r = conv.process(x), ref.process(x)
        assert np.array_equal(np.isnan(g), np.isnan(r))
        m = ~np.isnan(r)
        assert_close(g[m], r[m], what=f"call {i}")
        assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill)


def test_uniform_large_empty_response_and_nan_batch(amd, oracle_mod):
    """One-block calls (pass C ends the call, no lg_call_end): a channel whose
    response is updated to nothing has no active segment and outputs zeros
    (:216-219) while its neighbours convolve, a NaN block in one channel
    zero-fills that call (:264-267), then a full response again -- every
    channel as the oracle, state words included."""
    rng = np.random.default_rng(78)
    C, B, L = 3, 16384, 3 * 16384
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
    for i in range(10):
        if i == 2:
            conv.update_channel(1, np.zeros(0, np.float32))
            refs[1].update(np.zeros(0, np.float32))
        if i == 7:
            h1 = ir(rng, L)
            conv.update_channel(1, h1)
            refs[1].update(h1)
        x = np.stack([white(rng, B) for _ in range(C)])
        if i == 4:
            x[2, 50] = np.nan
        got = conv.process(x)
        for c in range(C):
            r = refs[c].process(x[c])
            assert np.array_equal(np.isnan(got[c]), np.isnan(r)), (i, c)
            m = ~np.isnan(r)
            assert_close(got[c][m], r[m], what=f"call {i} ch {c}")
            assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)
        if 2 <= i < 7:
            assert not got[1].any()


@pytest.mark.parametrize("head,L", [(512, 200000), (1024, 1000000)])
def test_twostage_long_tail_vs_oracle(amd, oracle_mod, head, L):
    """TwoStageFFTConvolver (:323-512) whose tail block exceeds 8192:
    (512, 200,000) -> T = 16,384 and (1024, 1,000,000) -> T = 32,768; two
    channels, head-sized calls past both tail swaps (2 T / head + 6 calls)."""
    rng = np.random.default_rng(head + L)
    C = 2
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
    T = conv.tail_block_size
    assert T == amd.compute_tail_block_size(head, L) and T > 8192
    calls = 2 * T // head + 6
    x = np.stack([white(rng, calls * head) for _ in range(C)])
    refs = [oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
    assert refs[0].tail_block_size == T
    got = np.concatenate([conv.process(x[:, k * head:(k + 1) * head]) for k in range(calls)], axis=1)
    for c in range(C):
        exp = np.concatenate([refs[c].process(x[c, k * head:(k + 1) * head]) for k in range(calls)])
        assert float(np.max(np.abs(exp[2 * T:]))) > 0  # the tail's delay-2T output is live
        assert_close(got[c], exp, what=f"head {head} L {L} ch {c}")


def test_twostage_large_head(amd, oracle_mod):
    """A head block past 8192 (head 16384, T = 16384 by the formula's
    max(b, head)): the head, tail0 and tail all on the long-block path, with
    ragged calls through the reference's sub-chunk loop (:427-494)."""
    rng = np.random.default_rng(5150)
    head, L = 16384, 5 * 16384
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    assert conv.tail_block_size == ref.tail_block_size
    for k in [16384, 16384, 5000, 11384, 16384, 16384, 100, 16284, 16384, 16384]:
        x = white(rng, k)
        assert_close(conv.process(x), ref.process(x), what=f"call of {k}")


def test_crossfade_large_block(amd, oracle_mod):
    """CrossfadeConvolver<FFTConvolver> (src/crossfade_convolver.rs:19-105) at
    B = 16384: two updates (a fade through the pending path), the
    stand-alone mix walking mix_value into a device table (calls > 1024
    samples)."""
    rng = np.random.default_rng(9090)
    B, L = 16384, 3 * 16384
    h = ir(rng, L)
    conv = amd.CrossfadeConvolver.init(h, B, L)
    ref = oracle_mod.CrossfadeConvolver.init(h, B, L)
    for i in range(10):
        if i in (2, 4):
            hn = ir(rng, L - 1000 * i)
            conv.update(hn)
            ref.update(hn)
        x = white(rng, B)
        assert_close(conv.process(x), ref.process(x), what=f"block {i}")
        assert conv.is_crossfading() == ref.is_crossfading()
