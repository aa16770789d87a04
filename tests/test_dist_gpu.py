"""The N>1 path on the HIP library: two rank processes (gloo, both on device
0 -- the one-GPU box's rehearsal of channel sharding) must reproduce one
process's batch bit for bit, since channel shards have no data-path exchange
(SURVEY.md §8e).  Runs the lookahead step (S >= 40) for long enough that far
windows turn over."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from fftconv_amd import shard

HERE = os.path.dirname(os.path.abspath(__file__))
# L 17,000 at B 256: S = 67 > 65, so the third anchor level (rows >= 65) is
# live and its 64-step windows turn over within NB blocks
C, B, L, NB = 5, 256, 17000, 80


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
@pytest.mark.parametrize("mode,WORLD", [("per-channel", 2), ("shared", 2), ("per-channel", 8), ("shared-nccl", 1)])
def test_ranks_bitwise_equal_one_process(amd, tmp_path, mode, WORLD):
    """WORLD 8: the cfg4 shape (8 ranks, contiguous channel shards) rehearsed
    with 8 rank processes on device 0.  shared-nccl: one rank on RCCL (the
    "nccl" backend; the one-GPU pool cannot host two RCCL ranks on one
    device) -- init_process_group("nccl") and the dry-block broadcast on a
    device tensor executed, its output fed to the channels with input stride 0
    and compared bitwise with the single process."""
    out = str(tmp_path / "y.npy")
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), out, mode,
                                       str(C), str(B), str(L), str(NB)], env=env))
    rcs = [p.wait(timeout=110) for p in procs]
    assert rcs == [0] * WORLD
    got = np.load(out)  # [NB][WORLD*C][B]
    if mode == "shared-nccl":
        with open(out + ".backend") as f:
            assert f.read() == "nccl"
    full = range(0, WORLD * C)
    conv = amd.FFTConvolver.init(shard.synth_irs(full, L), B, L, channels=WORLD * C, device=0)
    assert conv.lookahead_parts() > 0
    if mode.startswith("shared"):
        dry = np.broadcast_to(shard.synth_shared_dry(NB, B)[:, None, :], (NB, WORLD * C, B))
    else:
        dry = shard.synth_dry(full, NB, B)
    ref = np.stack([conv.process(np.ascontiguousarray(dry[b])) for b in range(NB)])
    assert np.array_equal(got, ref)
