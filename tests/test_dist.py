"""Multi-process channel sharding on CPU (gloo, world_size 2).

The path shards by channel with no data-path exchange, so a sharded run must
reproduce the single-process run bit for bit; the only collective is the
optional dry-block broadcast.  The oracle stands in for the GPU compute here
(it is the checker); tests/test_dist_gpu.py runs the same two-rank gloo job on
the HIP library (-m gpu) and checks it bitwise against one process."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fftconv_amd import shard

WORLD, C, B, L, NB = 2, 3, 64, 500, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _convolve(channels, dry, irs):
    import oracle

    outs = []
    for k in range(len(channels)):
        conv = oracle.FFTConvolver.init(irs[k], B, L)
        x = dry[:, k, :] if dry.ndim == 3 else dry
        outs.append(np.concatenate([conv.process(x[b]) for b in range(NB)]))
    return np.stack(outs)


def _worker(rank, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    mine = shard.channel_range(rank, WORLD, C)
    irs = shard.synth_irs(mine, L)
    if mode == "per-channel":
        dry = shard.synth_dry(mine, NB, B)
    else:
        t = torch.from_numpy(shard.synth_shared_dry(NB, B)) if rank == 0 else torch.zeros(NB, B)
        shard.broadcast_dry(dist, t, src=0)
        dry = t.numpy()
    y = torch.from_numpy(_convolve(mine, dry, irs))
    gathered = [torch.zeros_like(y) for _ in range(WORLD)] if rank == 0 else None
    dist.gather(y, gathered, dst=0)
    if rank == 0:
        q.put(torch.cat(gathered).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["per-channel", "shared"])
def test_sharded_equals_single_process(mode):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, mode, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = range(0, WORLD * C)
    irs = shard.synth_irs(full, L)
    dry = shard.synth_dry(full, NB, B) if mode == "per-channel" else shard.synth_shared_dry(NB, B)
    ref = _convolve(full, dry, irs)
    assert np.array_equal(out, ref)


def test_channel_ranges_partition():
    seen = []
    for r in range(4):
        seen.extend(shard.channel_range(r, 4, 1024))
    assert seen == list(range(4096))
    for total in (1, 7, 8192):
        parts = [shard.split_channels(total, 8, r) for r in range(8)]
        assert sum(len(p) for p in parts) == total
        assert [c for p in parts for c in p] == list(range(total))


def test_seeds_are_global():
    a = shard.synth_irs(range(4, 6), 100)
    b = shard.synth_irs(range(0, 8), 100)
    assert np.array_equal(a, b[4:6])
    x = shard.synth_dry(range(4, 6), 3, 16)
    y = shard.synth_dry(range(0, 8), 3, 16)
    assert np.array_equal(x, y[:, 4:6])
