#!/usr/bin/env python3
"""Lookahead path: fresh handles, reset, and VARIANT_LAFULL against each other
and the oracle, per geometry.  usage: la_determinism.py [C B L NB]..."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fftconv_amd as F  # noqa: E402
from fftconv_amd import shard  # noqa: E402
import oracle  # noqa: E402  (the checker)

dev = torch.device("cuda:0")
geos = [tuple(map(int, g.split(","))) for g in sys.argv[1:]] or [(64, 256, 48000, 208)]
for C, B, L, NB in geos:
    irs = shard.synth_irs(range(C), L)
    dry = shard.synth_dry(range(C), NB, B)
    d_in = torch.from_numpy(dry).to(dev)
    # an explicit stream, ordered after the default stream's work: stream 0 would
    # select the handle's own stream (fftconv.h), which the default stream does not wait for
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))

    def run(conv):
        yd = torch.empty(NB, C, B, device=dev)
        conv.process_device_steps(d_in.data_ptr(), B, C * B, yd.data_ptr(), B, C * B, B, NB, s.cuda_stream)
        s.synchronize()
        return yd.cpu().numpy()

    c1 = F.FFTConvolver.init(irs, B, L, channels=C, device=0)
    y1 = run(c1)
    y2 = run(F.FFTConvolver.init(irs, B, L, channels=C, device=0))
    c1.reset()
    y3 = run(c1)
    c1.reset()
    y3b = run(c1)
    F.set_kernel_variant(32 | 2)
    y4 = run(F.FFTConvolver.init(irs, B, L, channels=C, device=0))
    F.set_kernel_variant(-1)
    ref = {}
    for c in (0, C // 2, C - 1):
        o = oracle.FFTConvolver.init(irs[c], B, L)
        ref[c] = np.stack([o.process(np.ascontiguousarray(dry[b, c])) for b in range(NB)])

    def rep(name, y):
        d = y != y1
        blocks = sorted(set(np.nonzero(d.any(axis=(1, 2)))[0].tolist()))
        chans = sorted(set(np.nonzero(d.any(axis=(0, 2)))[0].tolist()))
        errs = {c: float(np.abs(y[:, c] - r).max()) for c, r in ref.items()}
        worst = {c: int(np.abs(y[:, c] - r).max(axis=1).argmax()) for c, r in ref.items()}
        print(f"  {name}: equal to fresh#1 {not d.any()}; differing blocks {blocks[:16]} ({len(blocks)}), channels "
              f"{chans[:10]} ({len(chans)}); max |y - oracle| {errs} at blocks {worst}", flush=True)

    print(f"C={C} B={B} L={L} NB={NB} lookahead parts {c1.lookahead_parts()}", flush=True)
    rep("fresh#1", y1)
    rep("fresh#2", y2)
    rep("reset#1", y3)
    rep("reset#2", y3b)
    rep("LAFULL", y4)
    del c1
