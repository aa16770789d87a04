"""Two-stage tail0 deferred to the end of its period (csrc/kernels.hip
tail0_*_kernel; TwoStageFFTConvolver::process, src/fft_convolver.rs:464-475:
tail_output0 is first read after the period's swap, so the period's head
blocks are convolved by tail_convolver0 in one pass).  Checked against the
oracle through the cases that break the deferral: an unaligned call in the
middle of a period (flush, then the reference's sub-chunk loop), clone and
reset with blocks pending, and a non-finite block (realfft's C2R error) in a
pending set, which replays tail0 block by block from the untouched state.
Tolerance: REL_TOL (tests/common.py)."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


def _run(conv, ref, rng, chunks, nan_at=(), channels=1):
    """process the chunks on both; compare the whole output stream per
    channel (NaN positions exactly, the rest within REL_TOL of its maximum)."""
    refs = [ref] if channels == 1 else ref
    got, exp = [], []
    for j, k in enumerate(chunks):
        x = np.stack([white(rng, k) for _ in range(channels)])
        for (jj, c, s) in nan_at:
            if jj == j:
                x[c, s] = np.nan
        g = conv.process(x[0] if channels == 1 else x)
        got.append(g.reshape(channels, k))
        exp.append(np.stack([refs[c].process(x[c]) for c in range(channels)]))
    got, exp = np.concatenate(got, axis=1), np.concatenate(exp, axis=1)
    for c in range(channels):
        assert np.array_equal(np.isnan(got[c]), np.isnan(exp[c])), f"channel {c}"
        m = ~np.isnan(exp[c])
        assert_close(got[c][m], exp[c][m], what=f"channel {c}")


@pytest.mark.parametrize("head,L", [(64, 12000), (128, 20000), (256, 30000), (512, 40000)])
def test_deferred_periods_vs_oracle(amd, oracle_mod, head, L):
    """aligned calls only: every tail0 block deferred, several periods."""
    rng = np.random.default_rng(head + L)
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = ref.tail_block_size
    _run(conv, ref, rng, [head] * (3 * T // head + 7))


def test_deferred_flush_on_unaligned_call(amd, oracle_mod):
    rng = np.random.default_rng(6)
    head, L = 64, 12000
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = ref.tail_block_size
    per = T // head
    chunks = [head] * (per + 5) + [13, 51] + [head] * (per - 3) + [7, 57, 64, 1, 63] + [head] * (2 * per)
    _run(conv, ref, rng, chunks)


def test_deferred_clone_and_reset_mid_period(amd, oracle_mod):
    rng = np.random.default_rng(7)
    head, L = 64, 12000
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = ref.tail_block_size
    _run(conv, ref, rng, [head] * (T // head + 9))  # 9 blocks pending
    twin = conv.clone()
    for _ in range(2 * T // head):
        x = white(rng, head)
        a, b = conv.process(x), twin.process(x)
        assert np.array_equal(a, b)
        assert_close(a, ref.process(x), what="after clone")
    _run(conv, ref, rng, [head] * 5)
    conv.reset()
    ref.reset()
    _run(conv, ref, rng, [head] * (2 * T // head + 3))


def test_deferred_nan_block_replays(amd, oracle_mod):
    """a NaN sample in a pending block: tail0's C2R fails on that block, the
    flush replays the period block by block (zero output for the failing
    block, state frozen at it, as the reference)."""
    rng = np.random.default_rng(8)
    head, L = 64, 12000
    h = ir(rng, L)
    conv = amd.TwoStageFFTConvolver.init(h, head, L)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = ref.tail_block_size
    per = T // head
    _run(conv, ref, rng, [head] * (4 * per + 2), nan_at=[(per + 5, 0, 11), (2 * per + per - 1, 0, 3)])


def test_deferred_batch_one_channel_replays(amd, oracle_mod):
    """distinct channels; a non-finite block on one channel replays only that
    channel's pending blocks."""
    rng = np.random.default_rng(9)
    head, L, C = 64, 10000, 4
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
    ref = [oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
    T = ref[0].tail_block_size
    per = T // head
    _run(conv, ref, rng, [head] * (3 * per + 4), nan_at=[(per + 3, 2, 40)], channels=C)


T0BLOCK = 256  # VARIANT_T0BLOCK (include/fftconv.h): per-block tail0, read at create


def test_per_block_tail0_path(amd, oracle_mod):
    """Variant bit 8 (VARIANT_T0BLOCK, read when the convolver is created):
    the per-block tail0 launch of round 1 still matches the oracle."""
    rng = np.random.default_rng(10)
    head, L = 64, 12000
    h = ir(rng, L)
    amd.set_kernel_variant(T0BLOCK)
    try:
        conv = amd.TwoStageFFTConvolver.init(h, head, L)
    finally:
        amd.set_kernel_variant(-1)
    ref = oracle_mod.TwoStageFFTConvolver.init(h, head, L)
    T = ref.tail_block_size
    chunks = [head] * (T // head + 5) + [13, 51] + [head] * (2 * T // head)
    got = np.concatenate([conv.process(white(np.random.default_rng(k), n)) for k, n in enumerate(chunks)])
    exp = np.concatenate([ref.process(white(np.random.default_rng(k), n)) for k, n in enumerate(chunks)])
    assert_close(got, exp, what="per-block tail0")


T0FUSED = 512  # VARIANT_T0FUSED: the five-kernel flush instead of the fused one (read per launch)


@pytest.mark.parametrize("steps", [False, True])
def test_fused_flush_bitwise_equals_split(amd, oracle_mod, steps):
    """The fused end-of-period flush (tail0_fused_kernel, head block 64: the
    default; four blocks' transforms per wave) and the five-kernel one
    (VARIANT_T0FUSED) run the same arithmetic in the same order:
    bit-identical outputs, through a NaN block's replay on one channel, and
    both against the oracle -- with per-call launches (the flush transforms
    every pending block) and with process_device_steps (the head's run wrote
    the pending spectra; the flush transforms none)."""
    import torch

    head, L, C = 64, 12000, 3
    hs = np.stack([ir(np.random.default_rng(20 + c), L) for c in range(C)])
    outs = []
    for v in (-1, T0FUSED):
        amd.set_kernel_variant(v)
        try:
            conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
            T = conv.tail_block_size
            per = T // head
            rng = np.random.default_rng(21)
            xs = []
            for j in range(3 * per + 5):
                x = np.stack([white(rng, head) for _ in range(C)])
                if j == per + 4:
                    x[1, 9] = np.nan
                xs.append(x)
            if steps:
                xd = torch.from_numpy(np.stack(xs)).to("cuda:0")  # [K][C][head]
                yd = torch.empty_like(xd)
                conv.process_device_steps(xd.data_ptr(), head, C * head, yd.data_ptr(), head, C * head, head,
                                          len(xs), 0)
                outs.append(np.concatenate(list(yd.cpu().numpy()), axis=1))
            else:
                outs.append(np.concatenate([conv.process(x) for x in xs], axis=1))
        finally:
            amd.set_kernel_variant(-1)
    if not np.array_equal(outs[0], outs[1], equal_nan=True):  # (diagnostics: which one left the oracle)
        rng = np.random.default_rng(21)
        refs = [oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
        for j in range(3 * per + 5):
            x = np.stack([white(rng, head) for _ in range(C)])
            if j == per + 4:
                x[1, 9] = np.nan
            for c in range(C):
                e = refs[c].process(x[c])
                a0, a1 = outs[0][c, j * head:(j + 1) * head], outs[1][c, j * head:(j + 1) * head]
                if not np.array_equal(a0, a1, equal_nan=True):
                    print(f"call {j} ch {c}: fused err {np.nanmax(np.abs(a0 - e)):.3g}, "
                          f"five err {np.nanmax(np.abs(a1 - e)):.3g}")
    assert np.array_equal(outs[0], outs[1], equal_nan=True)
    rng = np.random.default_rng(21)
    refs = [oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
    exp = [[] for _ in range(C)]
    for j in range(3 * per + 5):
        x = np.stack([white(rng, head) for _ in range(C)])
        if j == per + 4:
            x[1, 9] = np.nan
        for c in range(C):
            exp[c].append(refs[c].process(x[c]))
    for c in range(C):
        e = np.concatenate(exp[c])
        assert np.array_equal(np.isnan(outs[0][c]), np.isnan(e))
        m = ~np.isnan(e)
        assert_close(outs[0][c][m], e[m], what=f"channel {c}")
