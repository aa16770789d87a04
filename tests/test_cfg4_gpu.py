"""BASELINE.json configs[3] at its own size on the one-GPU box: 8192 channels,
block 256, IR 48,000, sharded 8 x 1024 over 8 rank processes.

The pool has one GPU per box, so the 8 ranks all run on device 0 over gloo
(tests/cfg4_worker.py); what is checked is the sharded path itself:
  * every channel of every rank's shard is bit-identical to one 8192-channel
    process (channel shards have no data-path exchange, and the lookahead
    step's summation order does not depend on the channel index or shard);
  * sampled channels (each shard edge on both sides of three rank
    boundaries) match oracle.FFTConvolver (src/fft_convolver.rs:215-295)
    within the stated f32 tolerance;
for per-channel dry input and for one shared dry source broadcast by rank 0.
NB = 208 one-block calls > S = 188, so all three anchor levels of the
lookahead step turn over (the level-3 period is 64 blocks)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from common import assert_close
from fftconv_amd import shard

HERE = os.path.dirname(os.path.abspath(__file__))
WORLD, C, B, L, NB = 8, 1024, 256, 48000, 208


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_cfg4_eight_ranks_full_size(amd, oracle_mod, tmp_path):
    import torch

    out = str(tmp_path / "y")
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "cfg4_worker.py"), out,
                                       str(C), str(B), str(L), str(NB)], env=env))
    try:
        rcs = [p.wait(timeout=420) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * WORLD

    total = WORLD * C
    full = range(total)
    irs = shard.synth_irs(full, L)
    dev = torch.device("cuda:0")
    sampled = sorted({0, 1, C - 1, C, 4 * C - 1, 4 * C, total - C - 1, total - C, total - 1})
    for mode in ("per-channel", "shared"):
        conv = amd.FFTConvolver.init(irs, B, L, channels=total, device=0)
        assert conv.lookahead_parts() > 0
        if mode == "per-channel":
            dry = shard.synth_dry(full, NB, B)  # [NB][total][B]
            d_in, in_stride = torch.from_numpy(dry).to(dev), B
        else:
            dry = np.broadcast_to(shard.synth_shared_dry(NB, B)[:, None, :], (NB, total, B))
            d_in, in_stride = torch.from_numpy(shard.synth_shared_dry(NB, B)).to(dev), 0
        yd = torch.empty(NB, total, B, device=dev)
        # an explicit stream here (the ranks use stream 0, the null stream)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        conv.process_device_steps(d_in.data_ptr(), in_stride, in_stride * total if in_stride else B, yd.data_ptr(), B,
                                  total * B, B, NB, s.cuda_stream)
        s.synchronize()
        ref = yd.cpu().numpy()
        del conv, d_in, yd
        for r in range(WORLD):
            got = np.load(f"{out}.{mode}.{r}.npy", mmap_mode="r")
            lo = r * C
            assert got.shape == (NB, C, B)
            same = np.array_equal(np.asarray(got), ref[:, lo:lo + C, :])
            assert same, f"{mode}: rank {r}'s shard differs from the 8192-channel process"
        for c in sampled:
            o = oracle_mod.FFTConvolver.init(irs[c], B, L)
            exp = np.concatenate([o.process(np.ascontiguousarray(dry[b, c])) for b in range(NB)])
            assert_close(ref[:, c, :].reshape(-1), exp, what=f"cfg4 {mode} channel {c}")
        del ref, dry
