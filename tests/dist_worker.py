"""One rank of the 2-process sharded run in tests/test_dist_gpu.py (launched
as a child process with RANK / WORLD_SIZE / MASTER_* set).  Every rank drives
the HIP library on device 0 (--same-device rehearsal of the N-GPU path) over
gloo; rank 0 gathers the shards and saves them for the parent to compare."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import fftconv_amd as F  # noqa: E402
from fftconv_amd import shard  # noqa: E402


def main():
    out_path, mode, C, B, L, NB = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:7])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mine = shard.channel_range(rank, world, C)
    if mode == "shared-nccl":
        # RCCL (the "nccl" backend on ROCm): the dry blocks broadcast as a
        # device tensor, then read by every channel with input stride 0
        dev = torch.device("cuda:0")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        conv = F.FFTConvolver.init(shard.synth_irs(mine, L), B, L, channels=C, device=0)
        t = (torch.from_numpy(shard.synth_shared_dry(NB, B)).to(dev) if rank == 0
             else torch.zeros(NB, B, device=dev))
        shard.broadcast_dry(dist, t, src=0)
        yd = torch.empty(NB, C, B, device=dev)
        # an explicit stream, ordered after the default stream's work: stream 0 would
        # select the handle's own stream (fftconv.h), which the default stream does not wait for
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        for b in range(NB):
            conv.process_device(t[b].data_ptr(), 0, yd[b].data_ptr(), B, B, s.cuda_stream)
        s.synchronize()
        got = [torch.zeros_like(yd) for _ in range(world)] if rank == 0 else None
        dist.gather(yd, got, dst=0)
        if rank == 0:
            np.save(out_path, torch.cat(got, dim=1).cpu().numpy())
            with open(out_path + ".backend", "w") as f:
                f.write(dist.get_backend())
        dist.barrier()
        dist.destroy_process_group()
        return
    dist.init_process_group("gloo", rank=rank, world_size=world)
    conv = F.FFTConvolver.init(shard.synth_irs(mine, L), B, L, channels=C, device=0)
    if mode == "shared":
        t = torch.from_numpy(shard.synth_shared_dry(NB, B)) if rank == 0 else torch.zeros(NB, B)
        shard.broadcast_dry(dist, t, src=0)  # the path's one collective
        dry = np.broadcast_to(t.numpy()[:, None, :], (NB, C, B))
    else:
        dry = shard.synth_dry(mine, NB, B)
    y = np.stack([conv.process(np.ascontiguousarray(dry[b])) for b in range(NB)])  # [NB][C][B]
    yt = torch.from_numpy(np.ascontiguousarray(y))
    got = [torch.zeros_like(yt) for _ in range(world)] if rank == 0 else None
    dist.gather(yt, got, dst=0)
    if rank == 0:
        np.save(out_path, torch.cat(got, dim=1).numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
