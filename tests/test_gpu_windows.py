"""Far-row windows of the generic step (1024 <= B <= 8192, >= 24 segments;
csrc/kernels.hip gw_anchor_kernel) and of the long-block path
(2^14 <= B <= 2^22, csrc/large.hip lg_rows: the same windows, transposed bin
order).

FFTConvolver::process (src/fft_convolver.rs:215-295) with the FDL sum of a
one-block call split as rows 1..P-1 (summed by the step) plus rows P..act-1
(summed by an anchor every P calls for the channel's next P blocks).  Checked
against the oracle (tolerance REL_TOL, as every parity test) and for the
property the design rests on: the split is canonical, so the bits do not
depend on whether a step read a window (VARIANT_NOGW), the channel's anchor
class, its shard, a clone, or the call pattern around it."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu

NOGW = 1024


def _refs(oracle_mod, hs, B, L):
    return [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(hs.shape[0])]


@pytest.mark.parametrize("B,S", [(1024, 30), (2048, 26), (4096, 40), (8192, 25), (16384, 25)])
def test_windows_vs_oracle(amd, oracle_mod, B, S):
    """Entry, the ring wrapping, partial and multi-block calls, a batch update
    that shrinks act (ring index mod act), a channel update, a reset."""
    rng = np.random.default_rng(700 + B)
    C, L = 11, S * B - 5
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert conv.far_windows() == 8
    refs = _refs(oracle_mod, hs, B, L)
    chunks = [B] * (S + 12) + [B // 3, B - B // 3] + [B] * 11 + [2 * B] + [B] * 13 + [B // 2] + [B] * 9
    for j, k in enumerate(chunks):
        if j == S + 4:
            hn = np.stack([ir(rng, L - 3 * B) for _ in range(C)])
            conv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        if j == S + 30:
            hn = ir(rng, L)
            conv.update_channel(9, hn)
            refs[9].update(hn)
        x = np.stack([white(rng, k) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"B={B} chunk {j} ch {c}")
    for c in range(C):
        assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)
    conv.reset()
    for c in range(C):
        refs[c].reset()
    for j in range(12):
        x = np.stack([white(rng, B) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"after reset, block {j}")


@pytest.mark.parametrize("B", [1024, 16384])
def test_windows_equal_full_sum(amd, B):
    """Steps served from windows give the same bits as steps that sum their
    far rows themselves (VARIANT_NOGW), through a partial call and re-entry."""
    rng = np.random.default_rng(710)
    C, L = 13, 33 * B + 7
    hs = np.stack([ir(rng, L) for _ in range(C)])
    ks = [B] * 40 + [300, B - 300] + [B] * 25 + [3 * B] + [B] * 10
    xs = [np.stack([white(rng, k) for _ in range(C)]) for k in ks]
    outs = {}
    for v in (-1, NOGW):
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(hs, B, L, channels=C)
            outs[v] = np.concatenate([conv.process(x) for x in xs], axis=1)
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[-1], outs[NOGW])


def test_windows_class_independent(amd):
    """11 identical channels in 8 anchor classes: bit-identical outputs."""
    rng = np.random.default_rng(720)
    C, B, L = 11, 2048, 30 * 2048
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(np.tile(h, (C, 1)), B, L, channels=C)
    for j in range(50):
        y = conv.process(np.tile(white(rng, B), (C, 1)))
        for c in range(1, C):
            assert np.array_equal(y[c], y[0]), (j, c)


@pytest.mark.parametrize("B", [1024, 16384])
def test_windows_shards_and_clone(amd, B):
    """A 12-channel batch split 5 + 7 (every channel changes class and index)
    stays bit-identical; a clone taken mid-window continues bit-identically."""
    rng = np.random.default_rng(730)
    C, L = 12, 28 * B
    hs = np.stack([ir(rng, L) for _ in range(C)])
    one = amd.FFTConvolver.init(hs, B, L, channels=C)
    a = amd.FFTConvolver.init(hs[:5], B, L, channels=5)
    b = amd.FFTConvolver.init(hs[5:], B, L, channels=7)
    for j in range(45):
        x = np.stack([white(rng, B) for _ in range(C)])
        assert np.array_equal(one.process(x), np.concatenate([a.process(x[:5]), b.process(x[5:])])), j
    twin = one.clone()
    for j in range(20):
        x = np.stack([white(rng, B) for _ in range(C)])
        assert np.array_equal(one.process(x), twin.process(x)), j


@pytest.mark.parametrize("B", [1024, 16384])
def test_windows_nan_block(amd, oracle_mod, B):
    """A non-finite block in one channel while its neighbours read windows:
    zero output, block kept in the input buffer, then recovery (the channel
    re-anchors) -- as the oracle."""
    rng = np.random.default_rng(740)
    C, L = 9, 30 * B
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = _refs(oracle_mod, hs, B, L)
    for j in range(60):
        x = np.stack([white(rng, B) for _ in range(C)])
        if j in (35, 36):
            x[6, 17] = np.nan
        got = conv.process(x)
        for c in range(C):
            r = refs[c].process(x[c])
            assert np.array_equal(np.isnan(got[c]), np.isnan(r)), (j, c)
            m = ~np.isnan(r)
            assert_close(got[c][m], r[m], what=f"block {j} ch {c}")
            assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)


@pytest.mark.parametrize("head,L,T", [(32, 34000, 1024), (64, 70000, 2048), (512, 450000, 16384)])
def test_windows_twostage_tail(amd, oracle_mod, head, L, T):
    """The two-stage tail (T = 1024 with 32 segments, T = 2048 with 33, and
    the long-block path's T = 16384 with 26) runs on windows: the output is
    the oracle's over 10 tail periods."""
    rng = np.random.default_rng(750 + head)
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    assert conv.tail_block_size == T and ref.tail_block_size == T
    for j in range(10 * T // head):
        x = white(rng, head)
        assert_close(conv.process(x), ref.process(x), what=f"call {j}")


def test_windows_device_steps(amd, oracle_mod):
    """process_device_steps over one-block calls with windows equals host
    calls bitwise and the oracle on sampled channels."""
    import torch

    rng = np.random.default_rng(760)
    C, B, L, K = 9, 1024, 30 * 1024, 40
    hs = np.stack([ir(rng, L) for _ in range(C)])
    x = np.stack([white(rng, K * B) for _ in range(C)])
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(np.ascontiguousarray(x.reshape(C, K, B).transpose(1, 0, 2))).to(dev)  # [K][C][B]
    yd = torch.empty_like(xd)
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert conv.far_windows() == 8
    s = torch.cuda.Stream(dev)
    conv.process_device_steps(xd.data_ptr(), B, C * B, yd.data_ptr(), B, C * B, B, K, s.cuda_stream)
    s.synchronize()
    y = yd.cpu().numpy().transpose(1, 0, 2).reshape(C, K * B)
    host = amd.FFTConvolver.init(hs, B, L, channels=C)
    yh = np.concatenate([host.process(x[:, k * B:(k + 1) * B]) for k in range(K)], axis=1)
    assert np.array_equal(y, yh)
    for c in (0, 8):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        assert_close(y[c], np.concatenate([ref.process(x[c, k * B:(k + 1) * B]) for k in range(K)]),
                     what=f"channel {c}")


@pytest.mark.parametrize("B,C", [(32768, 3), (131072, 2)])
def test_windows_long_blocks(amd, oracle_mod, B, C):
    """Far-row windows past B = 16384 (gw_anchor_kernel<15..17>, lg_rows):
    the oracle over S + 10 one-block calls with a partial call in the middle,
    and bit-identical to summing every far row (VARIANT_NOGW)."""
    rng = np.random.default_rng(790 + B)
    S = 25
    L = S * B - 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    ks = [B] * (S + 2) + [B // 5, B - B // 5] + [B] * 9
    xs = [np.stack([white(rng, k) for _ in range(C)]) for k in ks]
    outs = {}
    for v in (-1, NOGW):
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(hs, B, L, channels=C)
            assert conv.far_windows() == 8
            outs[v] = [conv.process(x) for x in xs]
        finally:
            amd.set_kernel_variant(-1)
    for a, b in zip(outs[-1], outs[NOGW]):
        assert np.array_equal(a, b)
    refs = _refs(oracle_mod, hs, B, L)
    for j, (x, got) in enumerate(zip(xs, outs[-1])):
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"B={B} call {j} ch {c}")
