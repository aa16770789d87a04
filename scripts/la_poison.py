#!/usr/bin/env python3
"""Lookahead windows filled with NaN at init (FFTCONV_LA_POISON=1): which
blocks / channels read a window row no anchor wrote.  usage: la_poison.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import fftconv_amd as F  # noqa: E402
from fftconv_amd import shard  # noqa: E402

assert os.environ.get("FFTCONV_LA_POISON") == "1"
dev = torch.device("cuda:0")
for C, B, L, NB in [(1024, 256, 48000, 208), (64, 256, 48000, 208), (256, 128, 20000, 300), (512, 512, 96000, 250)]:
    irs = shard.synth_irs(range(C), L)
    for mode in ("per-channel", "shared"):
        conv = F.FFTConvolver.init(irs, B, L, channels=C, device=0)
        if mode == "per-channel":
            d_in, st = torch.from_numpy(shard.synth_dry(range(C), NB, B)).to(dev), B
        else:
            d_in, st = torch.from_numpy(shard.synth_shared_dry(NB, B)).to(dev), 0
        yd = torch.empty(NB, C, B, device=dev)
        # an explicit stream, ordered after the default stream's work: stream 0 would
        # select the handle's own stream (fftconv.h), which the default stream does not wait for
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        conv.process_device_steps(d_in.data_ptr(), st, st * C if st else B, yd.data_ptr(), B, C * B, B, NB, s.cuda_stream)
        s.synchronize()
        y = yd.cpu().numpy()
        bad = ~np.isfinite(y).all(axis=2)  # [NB][C]
        nb, nc = np.nonzero(bad)
        print(f"C={C} B={B} L={L} {mode}: lookahead parts {conv.lookahead_parts()}, non-finite (block, channel) "
              f"pairs {int(bad.sum())}; blocks {sorted(set(nb.tolist()))[:12]}; channels {sorted(set(nc.tolist()))[:12]}",
              flush=True)
        # reset: the windows hold real values now; compare with a fresh handle
        conv.reset()
        yd2 = torch.empty(NB, C, B, device=dev)
        conv.process_device_steps(d_in.data_ptr(), st, st * C if st else B, yd2.data_ptr(), B, C * B, B, NB, s.cuda_stream)
        s.synchronize()
        print(f"   after reset: equal to the first pass {np.array_equal(yd2.cpu().numpy(), y)}", flush=True)
        del conv, d_in, yd, yd2
