"""CrossfadeConvolver<TwoStageFFTConvolver> on the device.

The reference's CrossfadeConvolver is generic over `Convolution`
(src/crossfade_convolver.rs:11,45-49).  Over a TwoStageFFTConvolver it inits
and processes; every update() reaches TwoStageFFTConvolver::update, todo!()
(src/fft_convolver.rs:408-410), inside the swap (:94-105) before fade_into, so
the crossfader stays Reached(A).  The expected outputs are the reference's
process (:66-78) composed here from the oracle's TwoStageFFTConvolver (A and
B) and its Crossfader<RaisedCosineMixer> (:192-279), sample by sample.
Tolerance as tests/test_gpu_parity.py (REL_TOL); against the device's own
TwoStageFFTConvolver the output is bit-identical (same kernels, same state)."""
import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


class ComposedCrossfade:
    """CrossfadeConvolver<TwoStageFFTConvolver>::process (:66-78) over the
    oracle's pieces: convolver_a / convolver_b (:27-31, B = the convolver,
    A = its clone) and the crossfader (crossfade_samples, hold = min(mbs, mrl))."""

    def __init__(self, oracle_mod, conv, max_response_length, max_buffer_size, crossfade_samples):
        self.a, self.b = conv.clone(), conv
        self.xf = oracle_mod.Crossfader.new(crossfade_samples, min(max_buffer_size, max_response_length))
        self.m = max_buffer_size

    def process(self, x, out_len):
        assert x.size == self.m
        ba = self.a.process(x)
        bb = self.b.process(x)
        return np.array([self.xf.mix(float(ba[i]), float(bb[i])) for i in range(out_len)], np.float32)


@pytest.mark.parametrize("head,L,C", [(64, 12000, 2), (32, 3000, 3), (128, 200, 1)])
def test_crossfade_twostage_vs_composed_oracle(amd, oracle_mod, head, L, C):
    rng = np.random.default_rng(head * 7 + L)
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.CrossfadeConvolver.init(hs if C > 1 else hs[0], head, L, channels=C, inner=amd.TwoStageFFTConvolver)
    twin = amd.TwoStageFFTConvolver.init(hs if C > 1 else hs[0], head, L, channels=C)
    refs = [ComposedCrossfade(oracle_mod, oracle_mod.TwoStageFFTConvolver.init(hs[c], head, L), L, head, L)
            for c in range(C)]
    T = twin.tail_block_size
    n_calls = max(2 * T // head + 5, 40)  # past both tail swaps
    for i in range(n_calls):
        x = np.stack([white(rng, head) for _ in range(C)])
        out_len = head if i % 5 else head // 2
        got = conv.process(x if C > 1 else x[0], out_len).reshape(C, out_len)
        full = twin.process(x if C > 1 else x[0]).reshape(C, head)
        assert np.array_equal(got, full[:, :out_len]), i
        if i % 7 == 0 or i == n_calls - 1:
            for c in range(C):
                assert_close(got[c], refs[c].process(x[c], out_len), what=f"call {i} ch {c}")
        else:
            for c in range(C):
                refs[c].process(x[c], out_len)
        assert not conv.is_crossfading()


def test_crossfade_twostage_update_is_todo(amd, oracle_mod):
    """update() panics (todo!) before anything changes: later outputs are the
    ones of a convolver that never saw the update; update_device likewise."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    h = ir(rng, 5000)
    conv = amd.CrossfadeConvolver.init(h, 32, 5000, inner=amd.TwoStageFFTConvolver)
    twin = amd.TwoStageFFTConvolver.init(h, 32, 5000)
    for i in range(60):
        if i in (10, 30):
            with pytest.raises(amd.NotImplementedInReference):
                conv.update(ir(rng, 4000))
        if i == 45:
            d = torch.from_numpy(ir(rng, 3000)).to("cuda")
            with pytest.raises(amd.NotImplementedInReference):
                conv.update_device(d.data_ptr(), d.numel())
        x = white(rng, 32)
        assert np.array_equal(conv.process(x), twin.process(x)), i
    with pytest.raises(amd.NotImplementedInReference):
        conv.reset()


def test_crossfade_twostage_new_clone_and_panics(amd):
    rng = np.random.default_rng(6)
    h = ir(rng, 3000)
    inner = amd.TwoStageFFTConvolver.init(h, 64, 3000)
    for _ in range(7):
        inner.process(white(rng, 64))
    # new(): the convolver is cloned with its history; crossfade_samples and
    # max_response_length only shape the (never started) fade
    conv = amd.CrossfadeConvolver.new(inner, 3000, 64, 1000)
    assert conv.inner is amd.TwoStageFFTConvolver
    for _ in range(20):
        x = white(rng, 64)
        assert np.array_equal(conv.process(x), inner.process(x))
    twin = conv.clone()
    for _ in range(30):
        x = white(rng, 64)
        assert np.array_equal(conv.process(x), twin.process(x))
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(32, np.float32))               # input shorter than max_buffer_size
    with pytest.raises(amd.ConvolutionPanic):
        conv.process(np.ones(64, np.float32), out_len=65)   # output longer than buffer_a
    # max_buffer_size above the head block: TwoStage's assert (:414)
    big = amd.CrossfadeConvolver.new(inner, 3000, 128, 1000)
    with pytest.raises(amd.ConvolutionPanic):
        big.process(np.ones(128, np.float32))
    # input longer than max_buffer_size (but within the head): buffer_a index
    small = amd.CrossfadeConvolver.new(inner, 3000, 32, 1000)
    with pytest.raises(amd.ConvolutionPanic):
        small.process(np.ones(64, np.float32))
    y = small.process(np.ones(32, np.float32))
    assert y.shape == (32,)
