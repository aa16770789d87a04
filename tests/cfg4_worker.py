"""One rank of tests/test_cfg4_gpu.py: BASELINE.json configs[3] (8192 channels,
block 256, IR 48,000, 8 ranks x 1024 channels) rehearsed on the one-GPU box.

Launched as a child process with RANK / WORLD_SIZE / MASTER_* set.  Every rank
drives the HIP library on device 0 over gloo (the pool has one GPU per box),
owns the contiguous channel shard shard.channel_range(rank, world, C) and runs
NB one-block process() calls (src/fft_convolver.rs:215-295) twice, on fresh
handles:
  * per-channel dry input (seeded by global channel id);
  * one shared dry source, rank 0's blocks broadcast to every rank (the path's
    one collective, shard.broadcast_dry) and read with input stride 0.
Each rank saves its own shard's outputs, [NB][C][B] float32, to
<out>.<mode>.<rank>.npy; the parent compares them bitwise with one
8192-channel process.  Progress lines go to stderr so a slow box is visible.
"""
import gc
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import fftconv_amd as F  # noqa: E402
from fftconv_amd import shard  # noqa: E402


def run(conv, d_in, in_stride, in_step, C, B, NB):
    dev = torch.device("cuda:0")
    yd = torch.empty(NB, C, B, device=dev)
    # stream 0 = HIP's null stream, torch's default stream (fftconv.h
    # "Streams"): the read below is ordered after every launch with no explicit
    # synchronisation -- the pattern that raced while 0 meant the handle's own
    # stream (round 5)
    conv.process_device_steps(d_in.data_ptr(), in_stride, in_step, yd.data_ptr(), B, C * B, B, NB, 0)
    return yd.cpu().numpy()


def main():
    out, C, B, L, NB = sys.argv[1], *map(int, sys.argv[2:6])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    t0 = time.time()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if os.environ.get("FFTCONV_TEST_VARIANT"):  # (diagnostics: scripts/cfg4_diag.py)
        F.set_kernel_variant(int(os.environ["FFTCONV_TEST_VARIANT"]))
    mine = shard.channel_range(rank, world, C)
    dev = torch.device("cuda:0")
    irs = shard.synth_irs(mine, L)

    conv = F.FFTConvolver.init(irs, B, L, channels=C, device=0)
    assert conv.lookahead_parts() > 0, "cfg4 shards must run the lookahead step"
    dry = torch.from_numpy(shard.synth_dry(mine, NB, B)).to(dev)  # [NB][C][B]
    np.save(f"{out}.per-channel.{rank}.npy", run(conv, dry, B, C * B, C, B, NB))
    del conv, dry
    gc.collect()
    print(f"rank {rank}: per-channel done {time.time() - t0:.1f}s", file=sys.stderr, flush=True)

    t = torch.from_numpy(shard.synth_shared_dry(NB, B)) if rank == 0 else torch.zeros(NB, B)
    shard.broadcast_dry(dist, t, src=0)
    conv = F.FFTConvolver.init(irs, B, L, channels=C, device=0)
    np.save(f"{out}.shared.{rank}.npy", run(conv, t.to(dev), 0, B, C, B, NB))
    del conv
    print(f"rank {rank}: shared done {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
