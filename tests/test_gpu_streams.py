"""Stream-scoped synchronisation of the C ABI (§8(f)3; src/lib.rs:8 asks
update() to be real-time safe).  A handle waits only for its own work: a host
update() or process() must return while an unrelated stream of the same GPU is
still busy, and work submitted on different caller streams is still ordered
like the reference's sequential calls."""
import time

import numpy as np
import pytest

from common import assert_close, ir, white

pytestmark = pytest.mark.gpu


def _busy_stream(torch, dev, seconds_hint=0.4):
    """An unrelated stream kept busy with fp32 GEMMs for a while (calibrated)."""
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(4):
        a = torch.mm(a, b) * 1e-3
    torch.cuda.synchronize(dev)
    per = max((time.perf_counter() - t0) / 4, 1e-5)
    n = int(min(20000, max(50, seconds_hint / per)))
    other = torch.cuda.Stream(dev)
    with torch.cuda.stream(other):
        for _ in range(n):
            a = torch.mm(a, b) * 1e-3
    return other, n * per


@pytest.mark.parametrize("kind", ["uniform", "crossfade"])
def test_update_returns_while_unrelated_stream_busy(amd, oracle_mod, kind):
    import torch

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(501)
    C, B, L = 3, 256, 41 * 256
    hs = np.stack([ir(rng, L) for _ in range(C)])
    cls = amd.FFTConvolver if kind == "uniform" else amd.CrossfadeConvolver
    ocls = oracle_mod.FFTConvolver if kind == "uniform" else oracle_mod.CrossfadeConvolver
    conv = cls.init(hs, B, L, channels=C)
    refs = [ocls.init(hs[c], B, L) for c in range(C)]
    xs = [np.stack([white(rng, B) for _ in range(C)]) for _ in range(60)]
    hn = np.stack([ir(rng, L - 3 * B) for _ in range(C)])
    got, exp = [], []
    for j, x in enumerate(xs):
        if j == 30:
            other, est = _busy_stream(torch, dev)
            t0 = time.perf_counter()
            conv.update(hn)
            got.append(conv.process(x))  # host process: waits for the handle's own stream only
            dt = time.perf_counter() - t0
            still_busy = not other.query()
            other.synchronize()
            assert still_busy, f"the unrelated stream ({est:.2f} s of GEMMs) finished before update+process returned"
            assert dt < est, (dt, est)
            for c in range(C):
                refs[c].update(hn[c])
        else:
            got.append(conv.process(x))
        exp.append(np.stack([refs[c].process(x[c]) for c in range(C)]))
    for c in range(C):
        assert_close(np.concatenate([g[c] for g in got]), np.concatenate([e[c] for e in exp]), what=f"{kind} ch {c}")


def test_calls_on_different_caller_streams_stay_ordered(amd, oracle_mod):
    """process_device on stream s1, a host update(), process_device on s2,
    update_device on s1, host process(): each call sees the state the previous
    one left, exactly as sequential calls -- checked against the oracle."""
    import torch

    dev = torch.device("cuda:0")
    rng = np.random.default_rng(502)
    C, B, L, K = 4, 256, 44 * 256, 12
    hs = np.stack([ir(rng, L) for _ in range(C)])
    conv = amd.FFTConvolver.init(hs, B, L, channels=C)
    refs = [oracle_mod.FFTConvolver.init(hs[c], B, L) for c in range(C)]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    x = np.stack([white(rng, 4 * K * B) for _ in range(C)])  # [C][4K*B]
    xd = torch.from_numpy(np.ascontiguousarray(x.reshape(C, 4 * K, B).transpose(1, 0, 2))).to(dev)  # [4K][C][B]
    yd = torch.zeros_like(xd)
    h1 = np.stack([ir(rng, L) for _ in range(C)])
    h2 = np.stack([ir(rng, L - B) for _ in range(C)])
    h2d = torch.from_numpy(h2).to(dev)
    torch.cuda.synchronize(dev)
    conv.process_device_steps(xd[0].data_ptr(), B, C * B, yd[0].data_ptr(), B, C * B, B, K, s1.cuda_stream)
    conv.update(h1)
    conv.process_device_steps(xd[K].data_ptr(), B, C * B, yd[K].data_ptr(), B, C * B, B, K, s2.cuda_stream)
    conv.update_device(h2d.data_ptr(), L - B, L - B, s1.cuda_stream)
    conv.process_device_steps(xd[2 * K].data_ptr(), B, C * B, yd[2 * K].data_ptr(), B, C * B, B, K, s1.cuda_stream)
    tail = conv.process(np.ascontiguousarray(x[:, 3 * K * B:]))  # host call: K blocks in one call
    torch.cuda.synchronize(dev)
    y = np.concatenate([yd[:3 * K].cpu().numpy().transpose(1, 0, 2).reshape(C, 3 * K * B), tail], axis=1)
    for c in range(C):
        r = refs[c]
        e = [r.process(x[c, :K * B])]
        r.update(h1[c])
        e.append(r.process(x[c, K * B:2 * K * B]))
        r.update(h2[c])
        e.append(r.process(x[c, 2 * K * B:3 * K * B]))
        e.append(r.process(x[c, 3 * K * B:]))
        assert_close(y[c], np.concatenate(e), what=f"channel {c}")


@pytest.mark.parametrize("kind", ["uniform", "crossfade"])
def test_update_through_a_capped_stage(amd, kind):
    """fftconv_set_host_stage_limit (the pinned reservation may be
    capped or refused): a stage of 3 response rows streams an 8-channel update
    in chunks -- the outputs are bit-identical to an uncapped handle's, through
    immediate and (crossfade) pending swaps."""
    rng = np.random.default_rng(503)
    C, B, L, NB = 8, 128, 45 * 128, 48
    irs = [np.stack([ir(rng, L) for _ in range(C)]) for _ in range(4)]
    x = white(rng, C * NB * B).reshape(C, NB * B)
    outs = []
    for cap in (0, 3 * L * 4):
        amd.set_host_stage_limit(cap)
        try:
            if kind == "uniform":
                conv = amd.FFTConvolver.init(irs[0], B, L, channels=C)
            else:
                conv = amd.CrossfadeConvolver.init(irs[0], B, L, channels=C)
        finally:
            amd.set_host_stage_limit(0)
        assert amd.get_host_stage_limit() == 0
        y = []
        for j in range(NB):
            if j in (5, 9, 30):  # (crossfade: the 9 lands while the fade from 5 runs -> pending)
                conv.update(irs[1 + [5, 9, 30].index(j)])
            y.append(conv.process(x[:, j * B:(j + 1) * B]))
        outs.append(np.concatenate(y, axis=1))
    assert np.array_equal(outs[0], outs[1])
