"""The lookahead step (fft-convolution_amd/csrc/la.hpp) on the device.

FFTConvolver::process (src/fft_convolver.rs:215-295) for a full block with
the FDL sum re-associated in time: the step sums rows 1..4, anchors sum rows
5..16 four blocks ahead, rows 17..64 sixteen blocks ahead and rows >= 65
sixty-four blocks ahead (S >= 40; the third anchor level exists when S > 65).  Checked against the oracle (tolerance REL_TOL, as every
parity test), and for the property the design rests on -- the summation
order is canonical, so the bits do not depend on a channel's stagger phase,
its index, the shard it sits in, or whether a step was served from a window
or summed all its rows itself (VARIANT_LAFULL)."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu

NOLA, LAFULL, NOFMIX = 16, 32, 64


def _refs(oracle_mod, hs, B, L):
    return [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(hs.shape[0])]


@pytest.mark.parametrize("B", [128, 256, 512])
def test_lookahead_vs_oracle(amd, oracle_mod, B):
    """Entry, > 3 windows per channel (the FDL ring wraps), a batch update,
    partial and multi-block calls in between, a channel update and reset."""
    rng = np.random.default_rng(300 + B)
    C, L = 6, 40 * B + 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert conv.lookahead_parts() > 0
    refs = _refs(oracle_mod, hs, B, L)
    S = refs[0].seg_count
    chunks = [B] * (2 * S) + [B // 3, B - B // 3] + [B] * 20 + [2 * B] + [B] * 20 + [B // 2] + [B] * 12
    for j, k in enumerate(chunks):
        if j == S + 5:
            hn = np.stack([ir(rng, L - 7 * B) for _ in range(C)])  # act shrinks, ring indexing mod act
            conv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        if j == 2 * S + 30:
            hn = ir(rng, L)
            conv.update_channel(4, hn)
            refs[4].update(hn)
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


def test_lookahead_phase_independent(amd):
    """13 identical channels sit at 13 different stagger phases (and anchor at
    different launches): every channel's output is bit-identical, through a
    partial call and a re-entry."""
    rng = np.random.default_rng(310)
    C, B, L = 13, 256, 50 * 256
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(np.tile(h, (C, 1)), B, L, channels=C)
    assert conv.lookahead_parts() > 0
    for j in range(150):
        k = 100 if j == 70 else (B - 100 if j == 71 else B)
        x = np.tile(white(rng, k), (C, 1))
        y = conv.process(x)
        for c in range(1, C):
            assert np.array_equal(y[c], y[0]), (j, c)


def test_lookahead_window_equals_full_sum(amd):
    """Steps served from anchor windows give the same bits as steps that sum
    every FDL row themselves (VARIANT_LAFULL), and the variant without the
    lookahead step agrees within f32 rounding."""
    rng = np.random.default_rng(320)
    C, B, L = 5, 256, 60 * 256 + 11
    hs = np.stack([ir(rng, L) for _ in range(C)])
    xs = [np.stack([white(rng, B) for _ in range(C)]) for _ in range(140)]
    outs = {}
    for v in (-1, LAFULL, NOLA):
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(hs, B, L, channels=C)
            outs[v] = np.concatenate([conv.process(x) for x in xs], axis=1)
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[-1], outs[LAFULL])
    assert_close(outs[-1], outs[NOLA], what="lookahead vs generic path")


def test_lookahead_shards_bitwise(amd):
    """A 24-channel batch split 7 + 17: every channel changes its stagger phase
    and its index, and the outputs stay bit-identical."""
    rng = np.random.default_rng(330)
    C, B, L = 24, 256, 40 * 256
    hs = np.stack([ir(rng, L) for _ in range(C)])
    one = amd.FFTConvolver.init(hs, B, L, channels=C)
    a = amd.FFTConvolver.init(hs[:7], B, L, channels=7)
    b = amd.FFTConvolver.init(hs[7:], B, L, channels=17)
    assert one.lookahead_parts() > 0
    for j in range(90):
        x = np.stack([white(rng, B) for _ in range(C)])
        y = one.process(x)
        assert np.array_equal(y, np.concatenate([a.process(x[:7]), b.process(x[7:])])), j


def test_lookahead_nan_block(amd, oracle_mod):
    """A non-finite block in one channel while its neighbours run from windows:
    zero output, block kept in the input buffer, then recovery -- as the
    oracle."""
    rng = np.random.default_rng(340)
    C, B, L = 4, 256, 40 * 256
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = _refs(oracle_mod, hs, B, L)
    for j in range(70):
        x = np.stack([white(rng, B) for _ in range(C)])
        if j in (45, 46):
            x[2, 17] = np.nan
        got = conv.process(x)
        for c in range(C):
            r = refs[c].process(x[c])
            assert np.array_equal(np.isnan(got[c]), np.isnan(r)), (j, c)
            m = ~np.isnan(r)
            assert_close(got[c][m], r[m], what=f"block {j} ch {c}")
            assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)


def test_lookahead_clone_mid_window(amd):
    """A clone taken mid-window continues bit-identically (windows copied)."""
    rng = np.random.default_rng(350)
    C, B, L = 9, 256, 45 * 256
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    for _ in range(43):
        conv.process(np.stack([white(rng, B) for _ in range(C)]))
    twin = conv.clone()
    for j in range(30):
        x = np.stack([white(rng, B) for _ in range(C)])
        assert np.array_equal(conv.process(x), twin.process(x)), j


def test_lookahead_device_steps(amd, oracle_mod):
    """process_device_steps over the lookahead path equals host calls and the
    oracle (a few sampled channels)."""
    import torch

    rng = np.random.default_rng(360)
    C, B, L, K = 64, 256, 48 * 256, 120
    hs = np.stack([ir(rng, L) for _ in range(C)])
    x = np.stack([white(rng, K * B) for _ in range(C)])
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(np.ascontiguousarray(x.reshape(C, K, B).transpose(1, 0, 2))).to(dev)  # [K][C][B]
    yd = torch.empty_like(xd)
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    s = torch.cuda.Stream(dev)
    conv.process_device_steps(xd.data_ptr(), B, C * B, yd.data_ptr(), B, C * B, B, K, s.cuda_stream)
    s.synchronize()
    y = yd.cpu().numpy().transpose(1, 0, 2).reshape(C, K * B)
    host = amd.FFTConvolver.init(hs, B, L, channels=C)
    yh = np.concatenate([host.process(x[:, k * B:(k + 1) * B]) for k in range(K)], axis=1)
    assert np.array_equal(y, yh)
    for c in (0, 13, 63):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        assert_close(y[c], np.concatenate([ref.process(x[c, k * B:(k + 1) * B]) for k in range(K)]),
                     what=f"channel {c}")


@pytest.mark.parametrize("C,B", [(8, 256), (64, 256), (64, 512)])
def test_lookahead_windows_never_read_unwritten(amd, monkeypatch, C, B):
    """FFTCONV_LA_POISON fills the window buffer with NaN at init: no step may
    read a window row before an anchor (or the init / reset rebuild) wrote it,
    so the output stays finite and bit-identical to an unpoisoned handle --
    through a reset, over more than a level-3 period."""
    import torch

    rng = np.random.default_rng(370 + C + B)
    L, K = 188 * B, 200
    hs = np.stack([ir(rng, L) for _ in range(C)])
    xd = torch.from_numpy(np.stack([white(rng, C * B).reshape(C, B) for _ in range(K)])).to("cuda:0")
    outs = []
    for poison in ("1", "0"):
        monkeypatch.setenv("FFTCONV_LA_POISON", poison)
        conv = amd.FFTConvolver.init(hs, B, L, channels=C)
        monkeypatch.delenv("FFTCONV_LA_POISON")
        assert conv.lookahead_parts() > 0
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        for _ in range(2):  # (the second pass after a reset)
            yd = torch.empty_like(xd)
            conv.process_device_steps(xd.data_ptr(), B, C * B, yd.data_ptr(), B, C * B, B, K, s.cuda_stream)
            s.synchronize()
            outs.append(yd.cpu().numpy())
            conv.reset()
    assert np.isfinite(outs[0]).all() and np.isfinite(outs[1]).all()
    for y in outs[1:]:
        assert np.array_equal(y, outs[0])


def test_device_stream_zero_is_the_null_stream(amd, oracle_mod):
    """stream 0 is HIP's null stream -- torch's default stream (fftconv.h
    "Streams"): process_device_steps(..., 0) issued from the default stream,
    then .cpu() on that stream with no synchronize() in between, sees every
    call's output; it equals the same calls on an explicit stream and the
    oracle.  (Until round 5, 0 selected the handle's own non-blocking stream,
    and this read raced the last launches: the cfg4 test's failure.)"""
    import torch

    rng = np.random.default_rng(380)
    C, B, L, K = 16, 256, 48 * 256, 96
    hs = np.stack([ir(rng, L) for _ in range(C)])
    x = np.stack([white(rng, C * B).reshape(C, B) for _ in range(K)])  # [K][C][B]
    xd = torch.from_numpy(x).to("cuda:0")
    assert torch.cuda.current_stream().cuda_stream == 0
    a, b = amd.FFTConvolver.init(hs, B, L, channels=C), amd.FFTConvolver.init(hs, B, L, channels=C)
    ya = torch.full_like(xd, float("nan"))  # (queued on the default stream before the calls)
    a.process_device_steps(xd.data_ptr(), B, C * B, ya.data_ptr(), B, C * B, B, K, 0)
    got = ya.cpu().numpy()  # the default stream, no synchronisation with the handle
    yb = torch.empty_like(xd)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    b.process_device_steps(xd.data_ptr(), B, C * B, yb.data_ptr(), B, C * B, B, K, s.cuda_stream)
    s.synchronize()
    assert np.isfinite(got).all()
    assert np.array_equal(got, yb.cpu().numpy())
    # a second batch of calls on the null stream after a host update (the
    # handle's own stream) is ordered behind it
    a.update(hs[::-1].copy())
    ya2 = torch.full_like(xd, float("nan"))
    a.process_device_steps(xd.data_ptr(), B, C * B, ya2.data_ptr(), B, C * B, B, K, 0)
    got2 = ya2.cpu().numpy()
    assert np.isfinite(got2).all()
    for c in (0, 7, 15):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        yr = np.concatenate([ref.process(x[k, c]) for k in range(K)])
        assert_close(got[:, c].reshape(-1), yr, what=f"channel {c}")
        ref.update(hs[::-1][c].copy())
        yr2 = np.concatenate([ref.process(x[k, c]) for k in range(K)])
        assert_close(got2[:, c].reshape(-1), yr2, what=f"channel {c} after update")


@pytest.mark.parametrize("B,L", [(256, 40 * 256 + 5), (512, 44 * 512)])
def test_lookahead_crossfade_vs_oracle(amd, oracle_mod, B, L):
    """CrossfadeConvolver<FFTConvolver> (src/crossfade_convolver.rs:45-105)
    with both inner convolvers on the lookahead step: immediate and pending
    IR swaps (the trait init fades over the response length), against the
    oracle every block, and against the full-sum kernels within f32 rounding."""
    rng = np.random.default_rng(370 + B)
    C = 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    blocks = 70
    ups = {5: L, 17: L - 3 * B, 30: L, 52: L - B // 2}
    xs = [np.stack([white(rng, B) for _ in range(C)]) for _ in range(blocks)]
    news = {i: np.stack([ir(rng, n) for _ in range(C)]) for i, n in ups.items()}
    refs = [oracle_mod.CrossfadeConvolver.init(hs[c], B, L) for c in range(C)]
    outs = {}
    for v in (-1, NOLA):
        amd.set_kernel_variant(v)
        try:
            conv = amd.CrossfadeConvolver.init(hs, B, L, channels=C)
            ys = []
            for i in range(blocks):
                if i in news:
                    conv.update(news[i])
                ys.append(conv.process(xs[i]))
            outs[v] = np.concatenate(ys, axis=1)
        finally:
            amd.set_kernel_variant(-1)
    exp = []
    for i in range(blocks):
        if i in news:
            for c in range(C):
                refs[c].update(news[i][c])
        exp.append(np.stack([refs[c].process(xs[i][c]) for c in range(C)]))
    exp = np.concatenate(exp, axis=1)
    for c in range(C):
        assert_close(outs[-1][c], exp[c], what=f"lookahead ch {c}")
        assert_close(outs[NOLA][c], exp[c], what=f"full-sum ch {c}")


@pytest.mark.parametrize("B,L", [(128, 45 * 128 - 7), (256, 40 * 256 + 5), (512, 44 * 512)])
def test_lookahead_crossfade_fused_mix(amd, oracle_mod, B, L):
    """The crossfade mix (src/crossfade_convolver.rs:75-77, Crossfader::mix
    :242-278) fused into B's lookahead launch -- A's launch walks mix_value into
    a table, B's epilogue mixes -- is bit-identical to the stand-alone mix
    kernel (VARIANT_NOFMIX): through fades, holds, pending swaps, a short
    output (out_len < B: stand-alone mix), and a NaN block (C2R error, then the
    buffered channel's generic step inside the fused launch)."""
    rng = np.random.default_rng(410 + B)
    C = 4
    hs = np.stack([ir(rng, L) for _ in range(C)])
    blocks = 64
    ups = {3: L, 9: L - B, 20: L, 41: L - 2 * B}
    xs = [np.stack([white(rng, B) for _ in range(C)]) for _ in range(blocks)]
    for j in (44, 45):
        xs[j][2, 17] = np.nan
    news = {i: np.stack([ir(rng, n) for _ in range(C)]) for i, n in ups.items()}
    olen = {i: (B if i % 11 != 7 else B // 2) for i in range(blocks)}
    outs = {}
    for v in (-1, NOFMIX):
        amd.set_kernel_variant(v)
        try:
            conv = amd.CrossfadeConvolver.init(hs, B, L, channels=C)
            ys = []
            for i in range(blocks):
                if i in news:
                    conv.update(news[i])
                ys.append(conv.process(xs[i], olen[i]))
            outs[v] = np.concatenate(ys, axis=1)
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[-1], outs[NOFMIX], equal_nan=True)
    refs = [oracle_mod.CrossfadeConvolver.init(hs[c], B, L) for c in range(C)]
    exp = []
    for i in range(blocks):
        if i in news:
            for c in range(C):
                refs[c].update(news[i][c])
        exp.append(np.stack([refs[c].process(xs[i][c], olen[i]) for c in range(C)]))
    exp = np.concatenate(exp, axis=1)
    for c in range(C):
        m = ~np.isnan(exp[c])
        assert np.array_equal(np.isnan(outs[-1][c]), ~m), c
        assert_close(outs[-1][c][m], exp[c][m], what=f"fused ch {c}")


@pytest.mark.parametrize("B", [128, 256, 512])
def test_lookahead_three_levels_vs_oracle(amd, oracle_mod, B):
    """An FDL long enough for the third anchor level (rows >= 65, one anchor
    every 64 blocks): > 3 level-3 windows per channel, a partial call (the
    windows drop and re-enter), an update that shrinks the active segments
    below the third level's first row and one that restores them, against
    the oracle every block."""
    rng = np.random.default_rng(500 + B)
    C, L = 5, 150 * B - 9
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert conv.lookahead_parts() > 0
    refs = _refs(oracle_mod, hs, B, L)
    chunks = [B] * 230 + [B // 4, B - B // 4] + [B] * 80 + [B] * 70 + [B] * 80
    ups = {312: L - 100 * B, 382: L}  # 50 active segments, then all 150 again
    for j, k in enumerate(chunks):
        if j in ups:
            hn = np.stack([ir(rng, ups[j]) for _ in range(C)])
            conv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        x = np.stack([white(rng, k) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"B={B} chunk {j} ch {c}")
    for c in range(C):
        assert conv.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill)


def test_lookahead_three_levels_phase_and_full_sum(amd):
    """70 identical channels cover all 64 level-3 stagger phases: every
    channel's output is bit-identical to channel 0's, and to a batch whose
    steps sum every row themselves (VARIANT_LAFULL), through a partial call,
    a re-entry and an update."""
    rng = np.random.default_rng(520)
    C, B, L = 70, 256, 140 * 256
    h = ir(rng, L)
    hn = ir(rng, L - 300)
    xs = [white(rng, B) for _ in range(260)]
    outs = {}
    for v in (-1, LAFULL):
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(np.tile(h, (C, 1)), B, L, channels=C)
            ys = []
            for j, x in enumerate(xs):
                if j == 200:
                    conv.update(np.tile(hn, (C, 1)))
                if j == 150:
                    ys.append(conv.process(np.tile(x[:100], (C, 1))))
                    ys.append(conv.process(np.tile(x[100:], (C, 1))))
                else:
                    ys.append(conv.process(np.tile(x, (C, 1))))
            outs[v] = np.concatenate(ys, axis=1)
        finally:
            amd.set_kernel_variant(-1)
    for c in range(1, C):
        assert np.array_equal(outs[-1][c], outs[-1][0]), c
    assert np.array_equal(outs[-1], outs[LAFULL])


@pytest.mark.parametrize("B", [128, 256])
def test_lookahead_multi_block_calls(amd, oracle_mod, B):
    """Calls of m whole blocks (src/fft_convolver.rs:222-294 loops over any
    output.len(); src/tests.rs:119-146 feeds 2B-sample calls to a B-block
    convolver) stay on the lookahead path: bit-identical to m one-block
    calls, within tolerance of the oracle -- including a multi-block call
    that starts with buffered samples (the whole call by the chunk loop),
    and a non-finite sample in the middle block of a 3-block call (the
    reference zero-fills the whole call's output and stops, :239-240)."""
    rng = np.random.default_rng(600 + B)
    C, L = 6, 150 * B + 17
    hs = np.stack([ir(rng, L) for _ in range(C)])
    multi = amd.FFTConvolver.init(hs, B, L, channels=C)
    single = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = _refs(oracle_mod, hs, B, L)
    calls = [B] * 40 + [2 * B] * 30 + [4 * B] * 20 + [3 * B] * 10 + [B // 2] + [2 * B, B // 2] + [B] * 5 + [3 * B] * 4
    nan_call = len(calls) - 2
    filled = 0  # samples into the current block before the call
    for j, n in enumerate(calls):
        x = np.stack([white(rng, n) for _ in range(C)])
        if j == nan_call:
            x[3, B + 7] = np.nan
        got = multi.process(x)
        if n % B == 0 and filled == 0 and j < nan_call:
            one = np.concatenate([single.process(x[:, k * B:(k + 1) * B]) for k in range(n // B)], axis=1)
            assert np.array_equal(got, one), (j, n)
        else:
            # (buffered samples: the reference's chunks of one call differ
            # from those of m calls, so only the oracle comparison applies)
            single.process(x)
        filled = (filled + n) % B
        for c in range(C):
            r = refs[c].process(x[c])
            assert np.array_equal(np.isnan(got[c]), np.isnan(r)), (j, c)
            m = ~np.isnan(r)
            assert_close(got[c][m], r[m], what=f"B={B} call {j} (n={n}) ch {c}")
        for c in range(C):
            assert multi.channel_state(c) == (refs[c].current, refs[c].active_seg_count, refs[c].fill), (j, c)


@pytest.mark.parametrize("B,C", [(256, 64), (512, 24)])
def test_lookahead_post_step_state_word(amd, oracle_mod, monkeypatch, B, C):
    """The anchors never read a state word the same launch writes
    (la.hpp la_anchor_state): they read the launch-start copies
    (ProcJob::sview) that the previous launch's steps filled or the host
    refreshed after any other writer.  FFTCONV_LA_PROBE makes the race
    happen -- every step fences its word out to memory, every anchor waits,
    reads the LIVE word past its L2 and counts the ones this launch's step has
    already rewritten -- while the anchors still use the copy.  The probed
    batch must be bit-identical to an unprobed one through entry, > 2 level-3
    periods, a partial call and its re-entry, a batch update and a NaN block,
    and within tolerance of the oracle."""
    rng = np.random.default_rng(900 + B)
    L = 67 * B + 5  # S = 68 > 65: all three anchor levels
    hs = np.stack([ir(rng, L) for _ in range(C)])
    monkeypatch.setenv("FFTCONV_LA_PROBE", "1")
    probed = amd.FFTConvolver.init(hs, B, L, channels=C)
    monkeypatch.delenv("FFTCONV_LA_PROBE")
    plain = amd.FFTConvolver.init(hs, B, L, channels=C)
    assert probed.lookahead_parts() > 0 and probed.lookahead_probe() == 0
    assert plain.lookahead_probe() == -1
    refs = _refs(oracle_mod, hs, B, L)
    chunks = [B] * 150 + [B // 2, B // 2] + [B] * 20
    for j, k in enumerate(chunks):
        if j == 90:
            hn = np.stack([ir(rng, L) for _ in range(C)])
            for cv in (probed, plain):
                cv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        x = np.stack([white(rng, k) for _ in range(C)])
        if j == 120:
            x[3, 17] = np.nan  # a failed C2R: the channel leaves the lookahead path
        yp, yq = probed.process(x), plain.process(x)
        assert np.array_equal(yp, yq, equal_nan=True), f"block {j}: probed != plain"
        for c in (0, C - 1):
            assert_close(yp[c], refs[c].process(x[c]), what=f"block {j} ch {c}")
        for c in range(1, C - 1):
            refs[c].process(x[c])
    n = probed.lookahead_probe()
    print(f"\nB={B} C={C}: {n} anchors found the live word rewritten over {len(chunks)} calls")
    # every launch opens C/4 + C/16 + C/64 anchors: the race the copy removes
    # must have been there many times (a same-XCD or written-back step word)
    assert n >= len(chunks), f"only {n} rewritten live words"
