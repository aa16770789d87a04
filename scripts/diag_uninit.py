#!/usr/bin/env python3
"""Diagnostic: the two-stage run path (process_device_steps, head 64, IR
12000) repeated in one process on fresh handles -- later handles get device
memory earlier handles freed, so a read of memory the path never wrote shows
up as a wrong output.  Per repetition and stream mode: the first call that
leaves the oracle, per channel."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fftconv_amd as amd  # noqa: E402
import oracle  # noqa: E402
from common import ir, white  # noqa: E402

head, L, C = 64, 12000, 3
hs = np.stack([ir(np.random.default_rng(20 + c), L) for c in range(C)])
refs = None
for rep in range(4):
    for mode in ("null", "explicit"):
        for nan in (False, True):
            conv = amd.TwoStageFFTConvolver.init(hs, head, L, channels=C)
            T = conv.tail_block_size
            per = T // head
            rng = np.random.default_rng(21)
            xs = []
            for j in range(3 * per + 5):
                x = np.stack([white(rng, head) for _ in range(C)])
                if nan and j == per + 4:
                    x[1, 9] = np.nan
                xs.append(x)
            xd = torch.from_numpy(np.stack(xs)).to("cuda:0")
            yd = torch.empty_like(xd)
            if mode == "null":
                conv.process_device_steps(xd.data_ptr(), head, C * head, yd.data_ptr(), head, C * head, head,
                                          len(xs), 0)
                y = yd.cpu().numpy()
            else:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                conv.process_device_steps(xd.data_ptr(), head, C * head, yd.data_ptr(), head, C * head, head,
                                          len(xs), s.cuda_stream)
                s.synchronize()
                y = yd.cpu().numpy()
            r = [oracle.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
            bad = []
            for j, x in enumerate(xs):
                for c in range(C):
                    e = r[c].process(x[c])
                    if np.nanmax(np.abs(y[j, c] - e)) > 1e-4:
                        bad.append((j, c))
            print(f"rep {rep} {mode:8s} nan={nan}: {len(bad)} bad (call, ch): {bad[:6]}", flush=True)
            del conv, xd, yd
