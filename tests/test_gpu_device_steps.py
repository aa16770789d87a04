"""`process_device_steps` over the generic / pipelined step (a uniform batch
without lookahead) and over a two-stage's aligned calls equals the same calls
made one by one, bitwise, and the oracle (src/fft_convolver.rs:215-295,
:412-495) -- through a non-finite block in one channel, and for the two-stage
from a start off a period boundary.  A two-stage's aligned calls inside a
tail period run as ONE launch (upols_run_kernel, head 64..512), and so do
the uniform batch's calls (64 <= B <= 512, no lookahead); every other call
shape one launch per call."""
import numpy as np
import pytest
import torch

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


def _device_steps(conv, x, n, K):
    C = x.shape[0]
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(np.ascontiguousarray(x.reshape(C, K, n).transpose(1, 0, 2))).to(dev)  # [K][C][n]
    yd = torch.empty_like(xd)
    s = torch.cuda.Stream(dev)
    conv.process_device_steps(xd.data_ptr(), n, C * n, yd.data_ptr(), n, C * n, n, K, s.cuda_stream)
    s.synchronize()
    return yd.cpu().numpy().transpose(1, 0, 2).reshape(C, K * n)


@pytest.mark.parametrize("B,L", [(64, 4096), (128, 3000), (512, 6000)])
def test_uniform_device_steps(amd, oracle_mod, B, L):
    rng = np.random.default_rng(800 + B)
    C, K = 5, 90
    hs = np.stack([ir(rng, L) for _ in range(C)])
    x = np.stack([white(rng, K * B) for _ in range(C)])
    x[3, 40 * B + 7] = np.nan  # a failed C2R mid-run
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert conv.lookahead_parts() == 0
    y = _device_steps(conv, x, B, K)
    one = amd.FFTConvolver.init(hs, B, L, channels=C)
    yh = np.concatenate([one.process(x[:, k * B:(k + 1) * B]) for k in range(K)], axis=1)
    assert np.array_equal(y, yh, equal_nan=True)
    for c in (0, 3):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        r = np.concatenate([ref.process(x[c, k * B:(k + 1) * B]) for k in range(K)])
        assert np.array_equal(np.isnan(y[c]), np.isnan(r))
        m = ~np.isnan(r)
        assert_close(y[c][m], r[m], what=f"channel {c}")
    for c in range(C):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        for k in range(K):
            ref.process(x[c, k * B:(k + 1) * B])
        assert conv.channel_state(c) == (ref.current, ref.active_seg_count, ref.fill)


@pytest.mark.parametrize("head,L", [(64, 20000), (32, 12000), (128, 40000), (256, 70000), (512, 200000)])
def test_twostage_device_steps(amd, oracle_mod, head, L):
    rng = np.random.default_rng(810 + head)
    C = 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
    T = conv.tail_block_size
    K = 3 * T // head + 5
    x = np.stack([white(rng, K * head) for _ in range(C)])
    x[1, (T // head + 3) * head + 5] = np.nan
    # a partial call first: the runs start off a period boundary
    first = np.stack([white(rng, head) for _ in range(C)])
    conv.process(first)
    y = _device_steps(conv, x, head, K)
    one = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
    one.process(first)
    yh = np.concatenate([one.process(x[:, k * head:(k + 1) * head]) for k in range(K)], axis=1)
    assert np.array_equal(y, yh, equal_nan=True)
    for c in range(C):
        ref = oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L)
        ref.process(first[c])
        r = np.concatenate([ref.process(x[c, k * head:(k + 1) * head]) for k in range(K)])
        assert np.array_equal(np.isnan(y[c]), np.isnan(r)), c
        m = ~np.isnan(r)
        assert_close(y[c][m], r[m], what=f"channel {c}")


NORUN = 2048  # VARIANT_NORUN: process_device_steps launches once per call


@pytest.mark.parametrize("head,L", [(64, 20000), (128, 40000)])
def test_twostage_run_after_nan_partial_call(amd, oracle_mod, head, L):
    """a C2R error on a partial call freezes the head's fill
    (src/fft_convolver.rs:264-267) while tail_input_fill advances, so the
    head's buffer is out of step with tail0's blocks: the run's calls of that
    channel cannot write tail0's pending spectra, flag the channel, and the
    flush recomputes them.  Two half calls (a NaN in channel 1's first) then
    aligned process_device_steps over more than two tail periods: bitwise
    equal to one launch per call (VARIANT_NORUN), and the oracle."""
    rng = np.random.default_rng(830 + head)
    C = 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    half = [np.stack([white(rng, head // 2) for _ in range(C)]) for _ in range(2)]
    half[0][1, 5] = np.nan
    outs = []
    for v in (-1, NORUN):
        amd.set_kernel_variant(v)
        try:
            conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
            T = conv.tail_block_size
            K = 2 * T // head + 7
            x = np.stack([white(np.random.default_rng(831 + head), K * head) for _ in range(C)])
            pre = np.concatenate([conv.process(h) for h in half], axis=1)
            outs.append(np.concatenate([pre, _device_steps(conv, x, head, K)], axis=1))
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[0], outs[1], equal_nan=True)
    for c in range(C):
        ref = oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L)
        r = np.concatenate([ref.process(h[c]) for h in half] +
                           [ref.process(x[c, k * head:(k + 1) * head]) for k in range(K)])
        assert np.array_equal(np.isnan(outs[0][c]), np.isnan(r)), c
        m = ~np.isnan(r)
        assert_close(outs[0][c][m], r[m], what=f"channel {c}")


@pytest.mark.parametrize("head,L", [(64, 40000), (64, 100000), (128, 300000)])
def test_twostage_narrow_tail_bitwise(amd, monkeypatch, head, L):
    """The T-block tail's step on 256-thread workgroups (ProcArgs::narrow,
    upols_narrow_kernel; T = 2048 / 4096 / 8192) is bit-identical to the
    512-thread kernel: aligned process_device_steps over three tail periods,
    FFTCONV_TAIL_NARROW=2 (every period) against 0, with a NaN block."""
    rng = np.random.default_rng(840 + head + L)
    C = 4
    hs = np.stack([ir(rng, L) for _ in range(C)])
    outs = []
    for nar in ("2", "0"):
        monkeypatch.setenv("FFTCONV_TAIL_NARROW", nar)
        conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
        monkeypatch.delenv("FFTCONV_TAIL_NARROW")
        T = conv.tail_block_size
        K = 3 * T // head + 3
        x = np.stack([white(np.random.default_rng(841), K * head) for _ in range(C)])
        x[2, (T // head + 1) * head + 3] = np.nan
        outs.append(_device_steps(conv, x, head, K))
    assert np.isfinite(outs[0][0]).all()
    assert np.array_equal(outs[0], outs[1], equal_nan=True)
