"""GPU parity: the HIP path (through the C ABI) against the oracle and the f64
ground truth, plus the reference's own tests (src/tests.rs, inline #[test]s)
re-run on the device.  Tolerance: max|gpu - ref| <= 1e-5 * max|ref|
(REL_TOL), 1e-6 absolute for the delta-IR known answers (as the reference)."""
import numpy as np
import pytest

from common import DELTA_ABS_TOL, REL_TOL, assert_close, generate_sinusoid, ir, white

pytestmark = pytest.mark.gpu


def run_chunks(conv, x, chunks):
    ys, p = [], 0
    for k in chunks:
        ys.append(conv.process(x[..., p:p + k]))
        p += k
    return np.concatenate(ys, axis=-1)


# ---------------------------------------------------------------------------
# the reference's inline tests, on the device
# ---------------------------------------------------------------------------
def test_fft_convolver_passthrough(amd):
    """src/fft_convolver.rs:309-335."""
    response = np.zeros(1024, np.float32)
    response[0] = 1.0
    conv = amd.FFTConvolver.init(response, 1024, response.size)
    out = conv.process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


def test_fft_twostage_convolver_passthrough(amd):
    """src/fft_convolver.rs:528-554."""
    response = np.zeros(1024, np.float32)
    response[0] = 1.0
    conv = amd.TwoStageFFTConvolver.init(response, 1024, response.size)
    out = conv.process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


def test_crossfade_convolver_passthrough(amd):
    """src/crossfade_convolver.rs:107-124."""
    response = np.zeros(1024, np.float32)
    response[0] = 1.0
    conv = amd.CrossfadeConvolver.new(amd.FFTConvolver.init(response, 1024, response.size), 1024, 1024, 1024)
    out = conv.process(np.ones(1024, np.float32))
    assert np.max(np.abs(out - 1.0)) < DELTA_ABS_TOL


# ---------------------------------------------------------------------------
# src/tests.rs, on the device
# ---------------------------------------------------------------------------
def test_fft_convolver_update_is_reset(amd):
    """src/tests.rs:18-59."""
    bs = 512
    ra = generate_sinusoid(bs, 1000.0, gain=1.0)
    rb = generate_sinusoid(bs, 2000.0, gain=0.7)
    ca = amd.FFTConvolver.init(ra, bs, ra.size)
    cb = amd.FFTConvolver.init(rb, bs, rb.size)
    cu = amd.FFTConvolver.init(ra, bs, ra.size)
    x = generate_sinusoid(16 * bs, 1300.0)
    for i in range(16):
        blk = x[i * bs:(i + 1) * bs]
        if i == 8:
            cu.update(rb)
        ou = cu.process(blk)
        ref = ca.process(blk) if i < 8 else cb.process(blk)
        assert np.max(np.abs(ref - ou)) < 1e-6, i


def test_crossfade_convolver(amd):
    """src/tests.rs:61-117."""
    bs = 512
    ra = generate_sinusoid(bs, 1000.0, gain=1.0)
    rb = generate_sinusoid(bs, 2000.0, gain=0.7)
    ca = amd.FFTConvolver.init(ra, bs, ra.size)
    cb = amd.FFTConvolver.init(rb, bs, rb.size)
    xf = amd.CrossfadeConvolver.new(ca.clone(), bs, bs, bs)
    x = generate_sinusoid(16 * bs, 1300.0)
    for i in range(16):
        blk = x[i * bs:(i + 1) * bs]
        if i == 8:
            xf.update(rb)
        oc = xf.process(blk)
        oa = ca.process(blk)
        if i >= 8:
            ob = cb.process(blk)
        if i <= 8:
            assert np.max(np.abs(oa - oc)) < 1e-6, i
        elif i == 9:
            j = bs // 2 - 1
            assert abs(oc[j] - (oa[j] * 0.5 + ob[j] * 0.5)) < 1e-6
        else:
            assert np.max(np.abs(ob - oc)) < 1e-6, i


def test_block_size_equal(amd):
    """src/tests.rs:119-146 (multi-block-per-call path)."""
    bs = 128
    response = generate_sinusoid(bs, 1000.0, gain=0.1)
    ca = amd.FFTConvolver.init(response, bs // 2, response.size)
    cb = amd.FFTConvolver.init(response, bs, response.size)
    x = generate_sinusoid(1000 * bs, 1300.0, gain=0.1)
    for i in range(1000):
        blk = x[i * bs:(i + 1) * bs]
        assert np.max(np.abs(ca.process(blk) - cb.process(blk))) < 1e-5, i


def test_twostage_equal(amd):
    """src/tests.rs:148-175."""
    bs = 64
    response = generate_sinusoid(12000, 1000.0, gain=0.1)
    ca = amd.FFTConvolver.init(response, bs // 2, response.size)
    cb = amd.TwoStageFFTConvolver.init(response, bs, response.size)
    assert cb.tail_block_size == 1024
    x = generate_sinusoid(1000 * bs, 1300.0, gain=0.1)
    for i in range(1000):
        blk = x[i * bs:(i + 1) * bs]
        assert np.max(np.abs(ca.process(blk) - cb.process(blk))) < 1e-5, i


@pytest.mark.parametrize("kind", ["uniform", "twostage"])
def test_reset(amd, kind):
    """src/tests.rs:177-257."""
    bs, n = 64, 1000
    response = generate_sinusoid(12000, 1000.0, gain=0.1)
    cls = amd.FFTConvolver if kind == "uniform" else amd.TwoStageFFTConvolver
    conv = cls.init(response, bs, response.size)
    x = generate_sinusoid(n * bs, 1300.0, gain=0.1)
    a = np.concatenate([conv.process(x[i * bs:(i + 1) * bs]) for i in range(n)])
    conv.reset()
    b = np.concatenate([conv.process(x[i * bs:(i + 1) * bs]) for i in range(n)])
    assert np.max(np.abs(a - b)) < 1e-5


# ---------------------------------------------------------------------------
# parity with the oracle restatement (same inputs)
# ---------------------------------------------------------------------------
UNIFORM_CASES = [
    # (block, ir_len, chunk pattern)  -- pattern repeats to cover > S blocks
    (256, 4096, [256]),                 # cfg1 geometry
    (64, 12000, [64]),
    (1, 7, [1, 3, 2]),                  # B = 1 (N = 2)
    (2, 9, [1, 2, 5]),
    (4, 33, [4, 3, 9]),
    (8, 100, [8]),
    (32, 500, [32, 7, 100]),
    (100, 1000, [128, 17, 300]),        # block 100 -> 128
    (512, 1000, [100, 300, 1000, 17, 512]),
    (1024, 5000, [1024, 2048, 5]),
    (2048, 9000, [2048]),
    (4096, 20000, [4096, 1000]),
    (8192, 20000, [8192]),
]


@pytest.mark.parametrize("block,L,pattern", UNIFORM_CASES)
def test_uniform_vs_oracle(amd, oracle_mod, block, L, pattern):
    rng = np.random.default_rng(block * 7 + L)
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, block, L)
    ref = oracle_mod.FFTConvolver.init(h, block, L)
    S = ref.seg_count
    chunks, tot = [], 0
    while tot < (S + 3) * ref.block_size or len(chunks) < 8:
        for k in pattern:
            chunks.append(k)
            tot += k
    x = white(rng, tot)
    got = run_chunks(conv, x, chunks)
    exp = run_chunks(ref, x, chunks)
    assert_close(got, exp, what=f"B={block} L={L}")
    assert_close(got, oracle_mod.direct_convolution(x, h), what="vs f64")
    assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6])
def test_uniform_kernel_variants(amd, oracle_mod, variant):
    """Every fused-kernel variant (zig-zag scan / nontemporal loads) against the
    oracle, with partial chunks, multi-block calls and an update in between."""
    rng = np.random.default_rng(40 + variant)
    C, B, L = 3, 256, 5000
    hs = np.stack([ir(rng, L) for _ in range(C)])
    amd.set_kernel_variant(variant)
    try:
        conv = amd.FFTConvolver.init(hs, B, L, channels=C)
        refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
        chunks = [B] * 25 + [100, 156, 3 * B, 7] + [B] * 5
        for j, k in enumerate(chunks):
            if j == 27:
                hn = np.stack([ir(rng, 3000) for _ in range(C)])
                conv.update(hn)
                for c in range(C):
                    refs[c].update(hn[c])
            x = np.stack([white(rng, k) for _ in range(C)])
            got = conv.process(x)
            for c in range(C):
                assert_close(got[c], refs[c].process(x[c]), what=f"variant {variant} chunk {j} ch {c}")
    finally:
        amd.set_kernel_variant(-1)


@pytest.mark.parametrize("block,lag", [(2, -1), (8, 0), (32, 5), (64, -1), (128, 0), (128, 1000), (256, -1),
                                       (256, 3), (512, -1), (512, 0)])
def test_pipelined_step(amd, oracle_mod, block, lag):
    """The pipelined full-block step (next block's pre_multiplied streamed
    under the transform chain, FLAG_PRE) against the oracle: entry after a
    full-block call, partial chunks in between (generic path, stored pre
    reused), an update() (stored pre invalidated), reset(), and a response
    shorter than three segments; the stream split is swept through `lag`."""
    rng = np.random.default_rng(60 + block)
    C, B = 3, block
    L = 37 * B + 5
    hs = np.stack([ir(rng, L) for _ in range(C)])
    amd.set_pipeline_lag(lag)
    try:
        conv = amd.FFTConvolver.init(hs, B, L, channels=C)
        refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
        chunks = [B] * 45 + [max(1, B // 3), B - max(1, B // 3)] + [B] * 6 + [B // 2 or 1] + [B] * 4 \
            + [2 * B, B, B] + [B] * 3
        for j, k in enumerate(chunks):
            if j == 50:
                hn = np.stack([ir(rng, 2 * B + 1) for _ in range(C)])  # act 3
                conv.update(hn)
                for c in range(C):
                    refs[c].update(hn[c])
            if j == 58:
                hn = np.stack([ir(rng, B) for _ in range(C)])  # act 1
                conv.update(hn)
                for c in range(C):
                    refs[c].update(hn[c])
            x = np.stack([white(rng, k) for _ in range(C)])
            got = conv.process(x)
            for c in range(C):
                assert_close(got[c], refs[c].process(x[c]), what=f"B={B} lag={lag} chunk {j} ch {c}")
        assert conv.channel_state() == (refs[0].current, refs[0].active_seg_count, refs[0].fill)
        conv.reset()
        for c in range(C):
            refs[c].reset()
        for j in range(5):
            x = np.stack([white(rng, B) for _ in range(C)])
            got = conv.process(x)
            for c in range(C):
                assert_close(got[c], refs[c].process(x[c]), what=f"after reset, block {j}")
    finally:
        amd.set_pipeline_lag(-1)


def test_pipelined_nan_block(amd, oracle_mod):
    """A non-finite block on the pipelined path: zero output, the block kept in
    the input buffer, state unchanged -- as the generic path and the oracle."""
    rng = np.random.default_rng(70)
    B, L = 256, 20 * 256
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, B, L)
    ref = oracle_mod.FFTConvolver.init(h, B, L)
    for j in range(12):
        x = white(rng, B)
        if j == 6:
            x[17] = np.nan
        g, r = conv.process(x), ref.process(x)
        assert np.array_equal(np.isnan(g), np.isnan(r))
        m = ~np.isnan(r)
        assert_close(g[m], r[m], what=f"block {j}")
        assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill)


def test_load_policy_is_bit_identical(amd):
    """Plain and nontemporal loads (the automatic choice) give the same bits."""
    rng = np.random.default_rng(50)
    C, B, L = 4, 256, 4000
    hs = np.stack([ir(rng, L) for _ in range(C)])
    outs = []
    for v in (0, 2):
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(hs, B, L, channels=C)
            r = np.random.default_rng(51)
            outs.append(np.concatenate([conv.process(np.stack([white(r, B) for _ in range(C)]))
                                        for _ in range(30)], axis=1))
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[0], outs[1])


def test_channel_shards_bitwise_equal_on_device(amd):
    """Two channel shards reproduce the one-batch run bit for bit (the
    multi-GPU path has no data-path exchange)."""
    from fftconv_amd import shard

    C, B, L, NB = 64, 256, 6000, 40
    full = range(C)
    irs = shard.synth_irs(full, L)
    dry = shard.synth_dry(full, NB, B)
    one = amd.FFTConvolver.init(irs, B, L, channels=C)
    parts = [shard.split_channels(C, 2, r) for r in range(2)]
    halves = [amd.FFTConvolver.init(irs[p.start:p.stop], B, L, channels=len(p)) for p in parts]
    for b in range(NB):
        y = one.process(dry[b])
        ys = [h.process(dry[b][p.start:p.stop]) for h, p in zip(halves, parts)]
        assert np.array_equal(y, np.concatenate(ys)), b


def test_uniform_batch_distinct_channels(amd, oracle_mod):
    rng = np.random.default_rng(5)
    C, B, L = 8, 256, 3000
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    x = np.stack([white(rng, 40 * B) for _ in range(C)])
    chunks = [B] * 30 + [100, 156, 3 * B, 256, 5 * B]
    got = run_chunks(conv, x, chunks)
    for c in range(C):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        assert_close(got[c], run_chunks(ref, x[c], chunks), what=f"channel {c}")


def test_uniform_update_sequence(amd, oracle_mod):
    """update() keeps the FDL/current/fill and zeroes overlap+pre (:174-213),
    including a mid-block update and a shrinking active_seg_count."""
    rng = np.random.default_rng(11)
    B, L = 64, 1000
    h0 = ir(rng, L)
    conv = amd.FFTConvolver.init(h0, B, L)
    ref = oracle_mod.FFTConvolver.init(h0, B, L)
    script = [("p", 64)] * 20 + [("u", 1000), ("p", 64), ("p", 30), ("u", 130), ("p", 50), ("p", 64)] \
        + [("p", 64)] * 5 + [("u", 0), ("p", 64), ("u", 700)] + [("p", 64)] * 25 + [("p", 7), ("u", 64), ("p", 200)]
    for op, n in script:
        if op == "p":
            x = white(rng, n)
            assert_close(conv.process(x), ref.process(x), what=f"{op}{n}")
        else:
            hn = ir(rng, n)
            conv.update(hn)
            ref.update(hn)
        assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill)


@pytest.mark.parametrize("kind", ["uniform", "crossfade"])
def test_update_device_matches_host_update(amd, kind):
    """update_device (HBM-resident responses, stream-ordered) == update (host)."""
    import torch

    rng = np.random.default_rng(60)
    C, B, L = 4, 128, 1200
    hs = np.stack([ir(rng, L) for _ in range(C)])
    cls = amd.FFTConvolver if kind == "uniform" else amd.CrossfadeConvolver
    a = cls.init(hs, B, L, channels=C)
    b = cls.init(hs, B, L, channels=C)
    s = torch.cuda.Stream()
    for step in range(30):
        if step in (5, 9, 17):
            hn = np.stack([ir(rng, 900) for _ in range(C)])
            a.update(hn)
            d = torch.from_numpy(hn).cuda()
            torch.cuda.synchronize()
            b.update_device(d.data_ptr(), 900, 900, s.cuda_stream)
            b.synchronize()
            s.synchronize()
        x = np.stack([white(rng, B) for _ in range(C)])
        assert np.array_equal(a.process(x), b.process(x)), step


@pytest.mark.parametrize("kind", ["uniform", "twostage", "crossfade"])
def test_process_device_steps_equals_calls(amd, kind):
    """process_device_steps(K) is bit-identical to K process_device calls."""
    import torch

    rng = np.random.default_rng(70)
    C, B, L, K = 3, 64, 3000, 40
    hs = np.stack([ir(rng, L) for _ in range(C)])
    cls = {"uniform": amd.FFTConvolver, "twostage": amd.TwoStageFFTConvolver,
           "crossfade": amd.CrossfadeConvolver}[kind]
    a, b = cls.init(hs, B, L, channels=C), cls.init(hs, B, L, channels=C)
    x = torch.from_numpy(np.stack([np.stack([white(rng, B) for _ in range(C)]) for _ in range(K)])).cuda()
    ya, yb = torch.zeros_like(x), torch.zeros_like(x)
    s = torch.cuda.Stream()
    for k in range(K):
        a.process_device(x[k].data_ptr(), B, ya[k].data_ptr(), B, B, s.cuda_stream)
    b.process_device_steps(x.data_ptr(), B, C * B, yb.data_ptr(), B, C * B, B, K, s.cuda_stream)
    s.synchronize()
    assert torch.equal(ya, yb)


def test_uniform_update_channel(amd, oracle_mod):
    rng = np.random.default_rng(12)
    C, B, L = 4, 128, 900
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
    for step in range(30):
        if step == 10:
            hn = ir(rng, 300)
            conv.update_channel(2, hn)
            refs[2].update(hn)
        x = np.stack([white(rng, B) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"step {step} ch {c}")


def test_uniform_clone(amd, oracle_mod):
    rng = np.random.default_rng(13)
    B, L = 256, 2000
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, B, L)
    ref = oracle_mod.FFTConvolver.init(h, B, L)
    for _ in range(5):
        x = white(rng, 300)
        conv.process(x)
        ref.process(x)
    twin = conv.clone()
    rtwin = ref.clone()
    for _ in range(12):
        x = white(rng, B)
        a, b = conv.process(x), twin.process(x)
        assert np.array_equal(a, b)
        assert_close(a, ref.process(x))
        rtwin.process(x)


def test_uniform_nonfinite_zero_fills(amd, oracle_mod):
    """A NaN makes realfft's C2R fail; the reference zero-fills the output and
    leaves fill/current where they were (src/fft_convolver.rs:264-267)."""
    rng = np.random.default_rng(14)
    B, L = 64, 500
    h = ir(rng, L)
    conv = amd.FFTConvolver.init(h, B, L)
    ref = oracle_mod.FFTConvolver.init(h, B, L)
    seq = []
    for i in range(20):
        x = white(rng, B if i % 3 else 40)
        if i in (6, 13):
            x[5] = np.nan
        seq.append(x)
    for x in seq:
        g, r = conv.process(x), ref.process(x)
        assert np.array_equal(np.isnan(g), np.isnan(r))
        m = ~np.isnan(r)
        assert_close(g[m], r[m])
        assert conv.channel_state() == (ref.current, ref.active_seg_count, ref.fill)


def test_uniform_edge_geometries(amd, oracle_mod):
    # empty IR / zero max length: Default-like convolver outputs zeros
    conv = amd.FFTConvolver.init(np.zeros(0, np.float32), 64, 0)
    assert np.all(conv.process(np.ones(100, np.float32)) == 0)
    conv.update(np.zeros(0, np.float32))  # ir_len == 0: early return
    # update with an empty response: active_seg_count = 0 -> zeros
    h = ir(np.random.default_rng(1), 300)
    conv = amd.FFTConvolver.init(h, 64, 300)
    conv.process(np.ones(64, np.float32))
    conv.update(np.zeros(0, np.float32))
    assert np.all(conv.process(np.ones(64, np.float32)) == 0)
    # zero-length process
    assert conv.process(np.ones(0, np.float32)).size == 0


def test_uniform_panics(amd):
    with pytest.raises(amd.ConvolutionPanic):
        amd.FFTConvolver.init(np.ones(10, np.float32), 4, 5)
    conv = amd.FFTConvolver.init(np.ones(10, np.float32), 4, 10)
    with pytest.raises(amd.ConvolutionPanic):
        conv.update(np.ones(11, np.float32))
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(4, np.float32), out_len=8)
    # block sizes up to 2^22 run (the long-block path, test_gpu_large.py);
    # past that the build returns FFTCONV_E_UNSUPPORTED
    with pytest.raises(amd.DeviceError):
        amd.FFTConvolver.init(np.ones(10, np.float32), (1 << 22) + 1, 10)


@pytest.mark.parametrize("head,L,calls", [(64, 12000, [64]), (32, 5000, [32, 13, 19]), (32, 3000, [1, 31, 32, 16]),
                                          (128, 200, [128]), (64, 262144, [64])])
def test_twostage_vs_oracle(amd, oracle_mod, head, L, calls):
    rng = np.random.default_rng(head + L)
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    assert conv.tail_block_size == ref.tail_block_size
    T = ref.tail_block_size
    n_calls = max(3 * T // max(min(calls), 1), 40)
    if L >= 200000:
        n_calls = 2 * T // head + 5  # past both tail swaps
    chunks = [calls[i % len(calls)] for i in range(n_calls)]
    x = white(rng, sum(chunks))
    got = run_chunks(conv, x, chunks)
    exp = run_chunks(ref, x, chunks)
    assert_close(got, exp, what=f"two-stage {head}/{L}")
    assert_close(got, oracle_mod.direct_convolution(x, h), what="vs f64")


def test_twostage_non_power_of_two_head_panics(amd):
    conv = amd.TwoStageFFTConvolver.init(np.ones(5000, np.float32), 48, 5000)
    assert conv.tail_block_size == 512
    for _ in range(10):
        conv.process(np.ones(48, np.float32))
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(48, np.float32))


def test_twostage_panics(amd):
    conv = amd.TwoStageFFTConvolver.init(np.ones(100, np.float32), 32, 100)
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(33, np.float32))
    with pytest.raises(amd.NotImplementedInReference):
        conv.update(np.ones(10, np.float32))


def test_twostage_clone(amd):
    rng = np.random.default_rng(21)
    h = ir(rng, 5000)
    conv = amd.TwoStageFFTConvolver.init(h, 32, 5000)
    for _ in range(50):
        conv.process(white(rng, 32))
    twin = conv.clone()
    for _ in range(80):
        x = white(rng, 32)
        assert np.array_equal(conv.process(x), twin.process(x))


@pytest.mark.parametrize("B,L,every,xfade", [(512, 2000, 5, None), (64, 700, 3, None), (128, 1000, 7, 300),
                                             (256, 256, 2, None)])
def test_crossfade_vs_oracle(amd, oracle_mod, B, L, every, xfade):
    """update every `every` blocks: exercises fade, hold, and the pending path
    (the trait init fades over response.len() samples, src/crossfade_convolver.rs:46-49)."""
    rng = np.random.default_rng(B + L + every)
    h = ir(rng, L)
    if xfade is None:
        conv = amd.CrossfadeConvolver.init(h, B, L)
        ref = oracle_mod.CrossfadeConvolver.init(h, B, L)
    else:
        conv = amd.CrossfadeConvolver.new(amd.FFTConvolver.init(h, B, L), L, B, xfade)
        ref = oracle_mod.CrossfadeConvolver.new(oracle_mod.FFTConvolver.init(h, B, L), L, B, xfade)
    for i in range(40):
        if i % every == every - 1:
            hn = ir(rng, int(rng.integers(1, L + 1)))
            conv.update(hn)
            ref.update(hn)
        x = white(rng, B)
        out_len = B if i % 4 else B // 2
        assert_close(conv.process(x, out_len), ref.process(x, out_len), what=f"block {i}")
        assert conv.is_crossfading() == ref.is_crossfading()


def _crossfade_pair_run(amd, oracle_mod, seed, lens, nan_at=None):
    """Drive a paired (automatic) and an unpaired (variant bits 3+2) crossfade
    batch through the same calls; returns both outputs and the oracle's."""
    rng = np.random.default_rng(seed)
    C, B, L = 3, 64, 20000  # S*B = 20032 bins: the pair launch applies
    hs = np.stack([ir(rng, L) for _ in range(C)])
    convs = [amd.CrossfadeConvolver.init(hs, B, L, channels=C) for _ in range(2)]
    refs = [oracle_mod.CrossfadeConvolver.init(hs[c], B, L) for c in range(C)]
    outs = [[], [], []]
    try:
        for i in range(36):
            if i % 6 == 2:
                hn = np.stack([ir(rng, lens[(i // 6) % len(lens)]) for _ in range(C)])
                if nan_at is not None and i // 6 == nan_at:
                    hn[1, 7] = np.nan
                for cv in convs:
                    cv.update(hn)
                for c in range(C):
                    refs[c].update(hn[c])
            x = np.stack([white(rng, B) for _ in range(C)])
            for k, cv in enumerate(convs):
                amd.set_kernel_variant(-1 if k == 0 else 12)  # 12: no pair, no pipelined step
                outs[k].append(cv.process(x))
            amd.set_kernel_variant(-1)
            outs[2].append(np.stack([refs[c].process(x[c]) for c in range(C)]))
    finally:
        amd.set_kernel_variant(-1)
    return [np.concatenate(o, axis=1) for o in outs]


@pytest.mark.parametrize("lens", [[20000, 19990, 19950], [20000, 12000, 20000]])
def test_crossfade_pair_launch(amd, oracle_mod, lens):
    """The crossfade pair launch (A and B of a channel in one workgroup, one
    read of the shared FDL) is bit-identical to the two-job launch and matches
    the oracle -- including after a response of another segment count makes
    the rings diverge (pairing then stops for good)."""
    paired, unpaired, ref = _crossfade_pair_run(amd, oracle_mod, 90 + len(set(lens)), lens)
    assert np.array_equal(paired, unpaired)
    for c in range(paired.shape[0]):
        assert_close(paired[c], ref[c], what=f"ch {c}")


def test_crossfade_pair_divergence_by_c2r_error(amd, oracle_mod):
    """A response with a NaN makes one convolver's C2R fail on one channel
    only: its ring stops while its partner's advances; the pair kernel must
    notice, drop FLAG_XSYNC and fall back for that channel."""
    paired, unpaired, ref = _crossfade_pair_run(amd, oracle_mod, 99, [20000], nan_at=1)
    assert np.array_equal(paired, unpaired, equal_nan=True)
    for c in range(paired.shape[0]):
        m = ~np.isnan(ref[c])
        assert np.array_equal(np.isnan(paired[c]), ~m)
        assert_close(paired[c][m], ref[c][m], what=f"ch {c}")


def test_crossfade_batch(amd, oracle_mod):
    rng = np.random.default_rng(31)
    C, B, L = 3, 128, 600
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.CrossfadeConvolver.init(hs, B, L, channels=C)
    refs = [oracle_mod.CrossfadeConvolver.init(hs[c], B, L) for c in range(C)]
    for i in range(25):
        if i in (4, 9, 15):
            hn = np.stack([ir(rng, 400) for _ in range(C)])
            conv.update(hn)
            for c in range(C):
                refs[c].update(hn[c])
        x = np.stack([white(rng, B) for _ in range(C)])
        got = conv.process(x)
        for c in range(C):
            assert_close(got[c], refs[c].process(x[c]), what=f"block {i} ch {c}")


def test_crossfade_panics(amd):
    conv = amd.CrossfadeConvolver.init(np.ones(100, np.float32), 32, 100)
    with pytest.raises(amd.NotImplementedInReference):
        conv.reset()
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(16, np.float32))          # input shorter than max_buffer_size
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(64, np.float32), out_len=33)


# ---------------------------------------------------------------------------
# the north-star geometry (cfg2) at full size
# ---------------------------------------------------------------------------
def test_cfg2_full_size_sampled_channels(amd, oracle_mod):
    """1024 channels x IR 48000, block 256, device-resident path.  Sampled
    channels against the oracle over > S blocks (the FDL ring wraps), and
    linearity of the whole batch."""
    import torch

    C, B, L, steps = 1024, 256, 48000, 200
    rng = np.random.default_rng(2024)
    hs = (rng.uniform(-1, 1, (C, L)) / np.sqrt(L)).astype(np.float32)
    x = rng.uniform(-1, 1, (C, steps * B)).astype(np.float32)
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(x).to(dev)
    yd = torch.empty_like(xd)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    stream = st.cuda_stream
    assert stream != 0
    for s in range(steps):
        conv.process_device(xd.data_ptr() + 4 * s * B, steps * B, yd.data_ptr() + 4 * s * B, steps * B, B, stream)
    torch.cuda.synchronize()
    y = yd.cpu().numpy()
    for c in (0, 1, 511, 1023):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        exp = np.concatenate([ref.process(x[c, s * B:(s + 1) * B]) for s in range(steps)])
        assert_close(y[c], exp, what=f"channel {c}")
    # linearity on every channel: conv(2x) == 2 conv(x) exactly in binary f32 scaling
    conv2 = amd.FFTConvolver.init(hs, B, L, channels=C)
    y2d = torch.empty_like(xd)
    x2d = xd * 2.0
    st.wait_stream(torch.cuda.current_stream(dev))  # (x2d is made on the default stream)
    for s in range(steps):
        conv2.process_device(x2d.data_ptr() + 4 * s * B, steps * B, y2d.data_ptr() + 4 * s * B, steps * B, B, stream)
    torch.cuda.synchronize()
    assert torch.equal(y2d, 2.0 * yd)


@pytest.mark.parametrize("B,L", [(64, 5000), (256, 40 * 256 + 5), (512, 44 * 512 - 3), (1024, 9 * 1024 + 17)])
def test_ir_transform_wave_kernel_bitwise(amd, oracle_mod, B, L):
    """FFTConvolver::init / update (src/fft_convolver.rs:131-142, :190-212): the
    IR segment transforms one per wave (default, 64 <= B <= 1024) give the same
    spectra bits as one per workgroup (variant bit 7), through init, an update
    to a shorter response (zeroed rows) and back; and match the oracle."""
    rng = np.random.default_rng(700 + B)
    C = 3
    hs = np.stack([ir(rng, L) for _ in range(C)])
    news = {4: np.stack([ir(rng, L // 3) for _ in range(C)]), 9: np.stack([ir(rng, L) for _ in range(C)])}
    xs = [np.stack([white(rng, B) for _ in range(C)]) for _ in range(14)]
    outs = []
    for v in (16, 16 | 128):  # same step kernels (16: full-sum step); 128: IR transforms per workgroup
        amd.set_kernel_variant(v)
        try:
            conv = amd.FFTConvolver.init(hs, B, L, channels=C)
            ys = []
            for i, x in enumerate(xs):
                if i in news:
                    conv.update(news[i])
                ys.append(conv.process(x))
            outs.append(np.concatenate(ys, axis=1))
        finally:
            amd.set_kernel_variant(-1)
    assert np.array_equal(outs[0], outs[1])
    for c in range(C):
        ref = oracle_mod.FFTConvolver.init(hs[c], B, L)
        exp = []
        for i, x in enumerate(xs):
            if i in news:
                ref.update(news[i][c])
            exp.append(ref.process(x[c]))
        assert_close(outs[0][c], np.concatenate(exp), what=f"ch {c}")
