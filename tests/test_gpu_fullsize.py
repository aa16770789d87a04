"""BASELINE.json configs 3 and 5 at full size on the device (cfg2 is in
test_gpu_parity.py::test_cfg2_full_size_sampled_channels).  Sampled channels
against the oracle every call, and exact linearity of the whole batch
(conv(2x) == 2 conv(x): scaling by a power of two commutes with every f32
rounding of the path)."""
import numpy as np
import pytest

from common import assert_close

pytestmark = pytest.mark.gpu


def _dev_steps(torch, x, n):
    """[C][steps*n] host -> [steps][C][n] device."""
    C = x.shape[0]
    steps = x.shape[1] // n
    return torch.from_numpy(np.ascontiguousarray(x.reshape(C, steps, n).transpose(1, 0, 2))).to("cuda:0")


def test_cfg3_twostage_full_size(amd, oracle_mod):
    """cfg3: TwoStageFFTConvolver head 64 / tail 4096 (compute_tail_block_size,
    src/fft_convolver.rs:520-526), IR 262144, 256 channels, 64-sample calls
    (src/fft_convolver.rs:412-495) for 12 tail periods (12 T/64 + 16 calls):
    the T = 4096 tail convolver (:479-486) then runs 11 blocks, so its
    far-row windows (one anchor class in 8 per tail step, gw_anchor_kernel)
    are read by every class past entry, at cfg3 geometry with the tail on its
    CU-masked side stream beside the head and the deferred tail0 flush.
    Channels 0..7 (all 8 anchor classes), 127 and 255 against
    oracle.TwoStageFFTConvolver on every call."""
    import torch

    C, H, L = 256, 64, 262144
    rng = np.random.default_rng(3003)
    hs = (rng.uniform(-1, 1, (C, L)) / np.sqrt(L)).astype(np.float32)
    conv = amd.TwoStageFFTConvolver.init(hs, H, L, channels=C)
    T = conv.tail_block_size
    assert T == 4096
    calls = 12 * T // H + 16
    x = rng.uniform(-1, 1, (C, calls * H)).astype(np.float32)
    xd = _dev_steps(torch, x, H)
    ys = {}
    for scale in (1.0, 2.0):
        cv = conv if scale == 1.0 else amd.TwoStageFFTConvolver.init(hs, H, L, channels=C)
        xin = xd * scale
        yd = torch.empty_like(xd)
        s = torch.cuda.Stream()
        for k in range(calls):
            cv.process_device(xin[k].data_ptr(), H, yd[k].data_ptr(), H, H, s.cuda_stream)
        s.synchronize()
        ys[scale] = yd
    assert torch.equal(ys[2.0], 2.0 * ys[1.0])
    # process_device_steps: the calls inside each tail period as one launch
    # (upols_run_kernel), bit-identical to one launch per call
    cv = amd.TwoStageFFTConvolver.init(hs, H, L, channels=C)
    yr = torch.empty_like(xd)
    s = torch.cuda.Stream()
    cv.process_device_steps(xd.data_ptr(), H, C * H, yr.data_ptr(), H, C * H, H, calls, s.cuda_stream)
    s.synchronize()
    assert torch.equal(yr, ys[1.0])
    del cv, yr
    y = ys[1.0].cpu().numpy()  # [calls][C][H]
    for c in (*range(8), 127, 255):
        ref = oracle_mod.TwoStageFFTConvolver.init(hs[c], H, L)
        assert ref.tail_block_size == T
        exp = np.concatenate([ref.process(x[c, k * H:(k + 1) * H]) for k in range(calls)])
        got = y[:, c, :].reshape(-1)
        assert float(np.max(np.abs(exp[2 * T:]))) > 0  # the tail convolver's delay-2T output is live
        assert_close(got, exp, what=f"cfg3 channel {c}")
        for p in range(2, calls * H // T):  # every tail period past entry, on its own
            assert_close(got[p * T:(p + 1) * T], exp[p * T:(p + 1) * T], what=f"cfg3 channel {c} period {p}")


def test_cfg5_crossfade_full_size(amd, oracle_mod):
    """cfg5: CrossfadeConvolver<FFTConvolver> by the trait init
    (src/crossfade_convolver.rs:45-49: fade over 96000 samples, hold 512),
    512 channels, block 512, IR 96000, update() every 128 blocks for 4 swaps:
    the fade (96512 samples = 188.5 blocks) outlives the cadence, so every
    other update takes the pending path (:51-64, :66-70).  Channels 0, 255,
    511 against oracle.CrossfadeConvolver every block, and is_crossfading()
    (:85-92) on every block."""
    import torch

    C, B, L = 512, 512, 96000
    every, nup = 128, 4
    blocks = every * nup + 40
    rng = np.random.default_rng(5005)
    h0 = (rng.uniform(-1, 1, (C, L)) / np.sqrt(L)).astype(np.float32)
    news = {every * (k + 1): (rng.uniform(-1, 1, (C, L)) / np.sqrt(L)).astype(np.float32) for k in range(nup)}
    x = rng.uniform(-1, 1, (C, blocks * B)).astype(np.float32)
    xd = _dev_steps(torch, x, B)
    sampled = (0, 255, 511)
    refs = [oracle_mod.CrossfadeConvolver.init(h0[c], B, L) for c in sampled]
    ys, fading = {}, {}
    for scale in (1.0, 2.0):
        cv = amd.CrossfadeConvolver.init(h0, B, L, channels=C)
        xin = xd * scale
        yd = torch.empty_like(xd)
        s = torch.cuda.Stream()
        fl = []
        for k in range(blocks):
            if k in news:
                cv.update(news[k])
            cv.process_device(xin[k].data_ptr(), B, yd[k].data_ptr(), B, B, s.cuda_stream)
            fl.append(cv.is_crossfading())
        s.synchronize()
        ys[scale], fading[scale] = yd, fl
    assert torch.equal(ys[2.0], 2.0 * ys[1.0])
    y = ys[1.0].cpu().numpy()
    exp_fl = []
    exp = np.empty((len(sampled), blocks * B), np.float32)
    pend = 0
    for k in range(blocks):
        if k in news:
            pend += refs[0].is_crossfading()
            for i, c in enumerate(sampled):
                refs[i].update(news[k][c])
        for i, c in enumerate(sampled):
            exp[i, k * B:(k + 1) * B] = refs[i].process(x[c, k * B:(k + 1) * B])
        exp_fl.append(refs[0].is_crossfading())
    assert pend >= 2, "the 128-block cadence must hit the pending path"
    assert fading[1.0] == exp_fl
    for i, c in enumerate(sampled):
        assert_close(y[:, c, :].reshape(-1), exp[i], what=f"cfg5 channel {c}")
