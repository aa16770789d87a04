#!/usr/bin/env python3
"""Diagnostic: the fused vs five-kernel tail0 flush (VARIANT_T0FUSED) over
aligned process_device_steps (head 64, IR 12000, T 2048): first differing
call per channel, and each against the oracle, with and without a NaN."""
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
for nan in (False, True):
    for steps in ("null", True, False):
        outs = []
        for v in (-1, 512):
            amd.set_kernel_variant(v)
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
            if steps:
                xd = torch.from_numpy(np.stack(xs)).to("cuda:0")
                yd = torch.empty_like(xd)
                if steps == "null":  # stream 0: HIP's null stream, torch's default
                    conv.process_device_steps(xd.data_ptr(), head, C * head, yd.data_ptr(), head, C * head, head,
                                              len(xs), 0)
                else:
                    s = torch.cuda.Stream()
                    s.wait_stream(torch.cuda.current_stream())
                    conv.process_device_steps(xd.data_ptr(), head, C * head, yd.data_ptr(), head, C * head, head,
                                              len(xs), s.cuda_stream)
                    s.synchronize()
                outs.append(yd.cpu().numpy())  # [K][C][head]
            else:
                outs.append(np.stack([conv.process(x) for x in xs]))
            amd.set_kernel_variant(-1)
            del conv
        refs = [oracle.TwoStageFFTConvolver.init(hs[c], head, L) for c in range(C)]
        exp = np.stack([np.stack([refs[c].process(x[c]) for c in range(C)]) for x in xs])
        print(f"nan={nan} steps={steps} T={T} per={per}")
        for c in range(C):
            d = [k for k in range(len(xs)) if not np.array_equal(outs[0][k, c], outs[1][k, c], equal_nan=True)]
            e0 = [k for k in range(len(xs)) if np.nanmax(np.abs(outs[0][k, c] - exp[k, c])) > 1e-4]
            e1 = [k for k in range(len(xs)) if np.nanmax(np.abs(outs[1][k, c] - exp[k, c])) > 1e-4]
            print(f"  ch {c}: fused vs five first diff {d[:3]} ({len(d)}); fused vs oracle bad {e0[:3]} ({len(e0)}); "
                  f"five vs oracle bad {e1[:3]} ({len(e1)})")
