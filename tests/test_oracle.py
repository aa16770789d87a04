"""Pins the oracle (oracle/fftconv_oracle.c) before it is trusted as the GPU
checker: the reference's own known-answer and self-consistency tests
(src/tests.rs, src/fft_convolver.rs:309-321/542-554,
src/crossfade_convolver.rs:107-124/281-316) run against it, plus the
independent f64 direct convolution that UPOLS must equal.
CPU only."""
import numpy as np
import pytest

from common import DELTA_ABS_TOL, assert_close, generate_sinusoid, ir, white


def blocks(conv, x, bs):
    return np.concatenate([conv.process(x[i:i + bs]) for i in range(0, x.size, bs)])


# ---- src/fft_convolver.rs inline tests ------------------------------------
def test_fft_convolver_passthrough(oracle_mod):
    r = np.zeros(1024, np.float32)
    r[0] = 1.0
    out = oracle_mod.FFTConvolver.init(r, 1024, 1024).process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


def test_fft_twostage_convolver_passthrough(oracle_mod):
    r = np.zeros(1024, np.float32)
    r[0] = 1.0
    out = oracle_mod.TwoStageFFTConvolver.init(r, 1024, 1024).process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


def test_crossfade_convolver_passthrough(oracle_mod):
    r = np.zeros(1024, np.float32)
    r[0] = 1.0
    conv = oracle_mod.CrossfadeConvolver.new(oracle_mod.FFTConvolver.init(r, 1024, 1024), 1024, 1024, 1024)
    out = conv.process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


def test_crossfader(oracle_mod):
    """src/crossfade_convolver.rs:281-316, exact comparisons."""
    hold, fading, a, b = 4, 4, 1.0, 10.0
    xf = oracle_mod.Crossfader.new(fading, hold)
    start = {0: b, 1: a}
    end = {0: a, 1: b}
    for target in (1, 0):
        xf.fade_into(target)
        for i in range(hold + fading):
            v = xf.mix(a, b)
            if i < hold:
                assert xf.state == (True, target)
                assert v == start[target]
            elif i < hold + fading - 1:
                assert xf.state == (True, target)
                assert v != start[target] and v != end[target]
            else:
                assert v == end[target]
                assert xf.state == (False, target)


# ---- src/tests.rs ----------------------------------------------------------
def test_fft_convolver_update_is_reset(oracle_mod):
    bs = 512
    ra = generate_sinusoid(bs, 1000.0, gain=1.0)
    rb = generate_sinusoid(bs, 2000.0, gain=0.7)
    ca = oracle_mod.FFTConvolver.init(ra, bs, bs)
    cb = oracle_mod.FFTConvolver.init(rb, bs, bs)
    cu = oracle_mod.FFTConvolver.init(ra, bs, bs)
    x = generate_sinusoid(16 * bs, 1300.0)
    for i in range(16):
        blk = x[i * bs:(i + 1) * bs]
        if i == 8:
            cu.update(rb)
        ou = cu.process(blk)
        ref = ca.process(blk) if i < 8 else cb.process(blk)
        assert np.max(np.abs(ref - ou)) < 1e-6


def test_crossfade_convolver(oracle_mod):
    bs = 512
    ra = generate_sinusoid(bs, 1000.0, gain=1.0)
    rb = generate_sinusoid(bs, 2000.0, gain=0.7)
    ca = oracle_mod.FFTConvolver.init(ra, bs, bs)
    cb = oracle_mod.FFTConvolver.init(rb, bs, bs)
    xf = oracle_mod.CrossfadeConvolver.new(ca.clone(), bs, bs, bs)
    x = generate_sinusoid(16 * bs, 1300.0)
    for i in range(16):
        blk = x[i * bs:(i + 1) * bs]
        if i == 8:
            xf.update(rb)
        oc = xf.process(blk)
        oa = ca.process(blk)
        ob = cb.process(blk) if i >= 8 else None
        if i <= 8:
            assert np.max(np.abs(oa - oc)) < 1e-6
        elif i == 9:
            j = bs // 2 - 1
            assert abs(oc[j] - (oa[j] * 0.5 + ob[j] * 0.5)) < 1e-6
        else:
            assert np.max(np.abs(ob - oc)) < 1e-6


def test_block_size_equal(oracle_mod):
    bs = 128
    r = generate_sinusoid(bs, 1000.0, gain=0.1)
    ca = oracle_mod.FFTConvolver.init(r, bs // 2, r.size)
    cb = oracle_mod.FFTConvolver.init(r, bs, r.size)
    x = generate_sinusoid(1000 * bs, 1300.0, gain=0.1)
    for i in range(1000):
        blk = x[i * bs:(i + 1) * bs]
        assert np.max(np.abs(ca.process(blk) - cb.process(blk))) < 1e-5


def test_twostage_equal(oracle_mod):
    bs = 64
    r = generate_sinusoid(12000, 1000.0, gain=0.1)
    ca = oracle_mod.FFTConvolver.init(r, bs // 2, r.size)
    cb = oracle_mod.TwoStageFFTConvolver.init(r, bs, r.size)
    x = generate_sinusoid(1000 * bs, 1300.0, gain=0.1)
    for i in range(1000):
        blk = x[i * bs:(i + 1) * bs]
        assert np.max(np.abs(ca.process(blk) - cb.process(blk))) < 1e-5


@pytest.mark.parametrize("cls", ["FFTConvolver", "TwoStageFFTConvolver"])
def test_reset(oracle_mod, cls):
    bs, n = 64, 1000
    r = generate_sinusoid(12000, 1000.0, gain=0.1)
    conv = getattr(oracle_mod, cls).init(r, bs, r.size)
    x = generate_sinusoid(n * bs, 1300.0, gain=0.1)
    a = blocks(conv, x, bs)
    conv.reset()
    b = blocks(conv, x, bs)
    assert np.max(np.abs(a - b)) < 1e-5


# ---- independent ground truth ---------------------------------------------
@pytest.mark.parametrize("B,L", [(1, 5), (2, 9), (4, 33), (64, 12000), (256, 4096), (256, 48000), (512, 1000),
                                 (1024, 3000), (4096, 20000)])
def test_uniform_equals_f64_convolution(oracle_mod, B, L):
    rng = np.random.default_rng(B * 31 + L)
    h = ir(rng, L)
    conv = oracle_mod.FFTConvolver.init(h, B, L)
    n = max((conv.seg_count + 4) * conv.block_size, 64)
    x = white(rng, n)
    chunks = rng.integers(1, 2 * conv.block_size + 2, 64)
    out, p = [], 0
    for k in np.resize(chunks, 10_000):
        if p >= n:
            break
        out.append(conv.process(x[p:p + int(k)]))
        p += int(k)
    assert_close(np.concatenate(out)[:n], oracle_mod.direct_convolution(x, h)[:n], what=f"B={B} L={L}")


@pytest.mark.parametrize("head,L", [(64, 12000), (32, 5000), (32, 3000), (128, 200), (64, 100000)])
def test_twostage_equals_f64_convolution(oracle_mod, head, L):
    rng = np.random.default_rng(head + L)
    h = ir(rng, L)
    conv = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = conv.tail_block_size
    n = 3 * T + 5 * head
    x = white(rng, n)
    out, p = [], 0
    while p < n:
        k = min(head, n - p)
        out.append(conv.process(x[p:p + k]))
        p += k
    assert_close(np.concatenate(out), oracle_mod.direct_convolution(x, h), what=f"two-stage {head}/{L}")


def test_twostage_non_power_of_two_head_panics(oracle_mod):
    """head 48 does not divide T = 512: tail_input[fill..fill+48] runs past T
    on the 11th block and the reference panics (src/fft_convolver.rs:459-460)."""
    conv = oracle_mod.TwoStageFFTConvolver.init(np.ones(5000, np.float32), 48, 5000)
    assert conv.tail_block_size == 512
    for _ in range(10):
        conv.process(np.ones(48, np.float32))
    with pytest.raises(oracle_mod.OraclePanic):
        conv.process(np.ones(48, np.float32))


def test_update_keeps_history_semantics(oracle_mod):
    """after update the first block misses the previous overlap
    tail; from the next block on the output equals conv(x, h_new)."""
    rng = np.random.default_rng(3)
    B, L = 64, 640
    h0, h1 = ir(rng, L), ir(rng, L)
    conv = oracle_mod.FFTConvolver.init(h0, B, L)
    x = white(rng, 40 * B)
    for i in range(20):
        conv.process(x[i * B:(i + 1) * B])
    conv.update(h1)
    ys = [conv.process(x[i * B:(i + 1) * B]) for i in range(20, 40)]
    full = oracle_mod.direct_convolution(x, h1)
    assert_close(np.concatenate(ys[1:]), full[21 * B:40 * B])
    assert np.max(np.abs(ys[0] - full[20 * B:21 * B])) > 1e-3


def test_tail_block_size_known_values(oracle_mod):
    # (64, 262144) -> 4096, (64, 12000) -> 1024
    assert oracle_mod.compute_tail_block_size(64, 262144) == 4096
    assert oracle_mod.compute_tail_block_size(64, 12000) == 1024
    assert oracle_mod.compute_tail_block_size(1024, 1024) == 1024


def test_panics(oracle_mod):
    with pytest.raises(oracle_mod.OraclePanic):
        oracle_mod.FFTConvolver.init(np.ones(10), 4, 5)
    conv = oracle_mod.FFTConvolver.init(np.ones(10), 4, 10)
    with pytest.raises(oracle_mod.OraclePanic):
        conv.update(np.ones(11))
    ts = oracle_mod.TwoStageFFTConvolver.init(np.ones(100), 32, 100)
    with pytest.raises(oracle_mod.OraclePanic):
        ts.process(np.ones(33))
