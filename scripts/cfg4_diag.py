#!/usr/bin/env python3
"""Diagnostics for tests/test_cfg4_gpu.py: the same 8-rank run (tests/
cfg4_worker.py) and 8192-channel reference process, but on a mismatch it
reports where (mode, rank, block, channel), by how much, and which side the
oracle agrees with.  usage: cfg4_diag.py OUTDIR [--nb NB]"""
import argparse
import os
import socket
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fftconv_amd as F  # noqa: E402
from fftconv_amd import shard  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the checker)

p = argparse.ArgumentParser()
p.add_argument("out")
p.add_argument("--nb", type=int, default=208)
a = p.parse_args()
WORLD, C, B, L, NB = 8, 1024, 256, 48000, a.nb
os.makedirs(a.out, exist_ok=True)
out = os.path.join(a.out, "y")
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
procs = []
for r in range(WORLD):
    env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "cfg4_worker.py"), out, str(C), str(B),
                                   str(L), str(NB)], env=env))
rcs = [pp.wait(timeout=420) for pp in procs]
print("rank exit codes", rcs, flush=True)
total = WORLD * C
full = range(total)
irs = shard.synth_irs(full, L)
dev = torch.device("cuda:0")
bad = 0
for mode in ("per-channel", "shared"):
    for rep in range(2):
        conv = F.FFTConvolver.init(irs, B, L, channels=total, device=0)
        if mode == "per-channel":
            dry = shard.synth_dry(full, NB, B)
            d_in, in_stride = torch.from_numpy(dry).to(dev), B
        else:
            dry = np.broadcast_to(shard.synth_shared_dry(NB, B)[:, None, :], (NB, total, B))
            d_in, in_stride = torch.from_numpy(shard.synth_shared_dry(NB, B)).to(dev), 0
        yd = torch.empty(NB, total, B, device=dev)
        # an explicit stream, ordered after the default stream's work: stream 0 would
        # select the handle's own stream (fftconv.h), which the default stream does not wait for
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        conv.process_device_steps(d_in.data_ptr(), in_stride, in_stride * total if in_stride else B, yd.data_ptr(), B,
                                  total * B, B, NB, st.cuda_stream)
        st.synchronize()
        ref = yd.cpu().numpy()
        del conv, d_in, yd
        if rep == 0:
            ref0 = ref
            continue
        print(f"{mode}: the 8192-channel process repeated bit-identically: {np.array_equal(ref, ref0)}", flush=True)
    for r in range(WORLD):
        got = np.asarray(np.load(f"{out}.{mode}.{r}.npy"))
        lo = r * C
        for name, mine in (("rank", got), ("rep0", ref0[:, lo:lo + C, :])):
            d = mine != ref[:, lo:lo + C, :]
            if not d.any():
                continue
            bad += 1
            blocks, chans = np.nonzero(d.any(axis=2))
            print(f"{mode} rank {r} ({name} vs 8192-ch rep1): {int(d.sum())} samples differ, blocks "
                  f"{sorted(set(blocks.tolist()))[:20]}, {len(set(chans.tolist()))} channels (first {sorted(set(chans.tolist()))[:10]})",
                  flush=True)
            for c in sorted(set(chans.tolist()))[:3]:
                gc_ = lo + c
                o = oracle.FFTConvolver.init(irs[gc_], B, L)
                exp = np.concatenate([o.process(np.ascontiguousarray(dry[b, gc_])) for b in range(NB)]).reshape(NB, B)
                for nm, y in ((name, mine[:, c, :]), ("8192-ch", ref[:, lo + c, :])):
                    err = np.abs(y - exp).max(axis=1)
                    print(f"   channel {gc_} {nm}: max |y - oracle| per block, worst {err.max():.3e} at block "
                          f"{int(err.argmax())}; scale {np.abs(exp).max():.3e}", flush=True)
                b0 = int(blocks[chans == c].min())
                print(f"   channel {gc_} first differing block {b0}: max diff {np.abs(mine[b0, c] - ref[b0, lo + c]).max():.3e}",
                      flush=True)
print("mismatching (mode, rank, side) sets:", bad)
sys.exit(1 if bad else 0)
