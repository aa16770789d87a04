#!/usr/bin/env python3
"""Interleaved A/B of fused-kernel variants in ONE process (cfg2 geometry).
usage: ab_variants.py [variants=0,1,2,3] [rounds=5] [steps=200] [channels=1024] [block=256] [ir=48000]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import bench
import fftconv_amd as F

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
C = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
B = int(sys.argv[5]) if len(sys.argv) > 5 else 256
L = int(sys.argv[6]) if len(sys.argv) > 6 else 48000
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
conv = F.FFTConvolver.init(bench.make_irs(0, C, L), B, L, channels=C)
ring = 16
xin = torch.empty((ring, C, B), device=dev).uniform_(-1, 1)
yout = torch.empty((ring, C, B), device=dev)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
h = s.cuda_stream
bpl = bench.algorithmic_bytes_per_channel_block(B, L) * C
res = {v: [] for v in variants}
k = 0
for r in range(rounds):
    for v in variants:
        F.set_kernel_variant(v)
        for _ in range(20):
            conv.process_device(xin[k % ring].data_ptr(), B, yout[k % ring].data_ptr(), B, B, h); k += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            conv.process_device(xin[k % ring].data_ptr(), B, yout[k % ring].data_ptr(), B, B, h); k += 1
        e1.record(s)
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) * 1000 / steps)
for v in variants:
    us = statistics.median(res[v])
    print(f"variant {v}: median {us:.2f} us/step  min {min(res[v]):.2f}  -> {C*B/us:.1f} MS/s, "
          f"{bpl/us/1e3:.1f} GB/s algorithmic ({bpl/us/1e3/8000:.3f} of 8 TB/s)")
