#!/usr/bin/env python3
"""Per-call timeline of cfg3 (TwoStageFFTConvolver, head 64 / tail 4096, IR
262144, 256 channels): HIP events between consecutive head calls on the
caller's stream over a few tail periods, so the period-end work (tail0 flush,
the wait for the previous tail) shows up as the calls it delays.
usage: cfg3_steps.py [LIB] [--periods P] [--ir L]"""
import argparse
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import torch

from fftconv_amd import shard

p = argparse.ArgumentParser()
p.add_argument("lib", nargs="?", default=os.path.join(ROOT, "fft-convolution_amd", "libfftconv_amd.so"))
p.add_argument("--periods", type=int, default=4)
p.add_argument("--channels", type=int, default=256)
p.add_argument("--ir", type=int, default=262144)
a = p.parse_args()
Cn, B, L, T = a.channels, 64, a.ir, 4096
steps = T // B
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
lib = C.CDLL(os.path.abspath(a.lib), mode=os.RTLD_LOCAL)
lib.fftconv_twostage_init_batch.restype = C.c_void_p
lib.fftconv_twostage_init_batch.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                            C.c_size_t]
lib.fftconv_twostage_process_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                C.c_size_t, C.c_void_p]
irs = shard.synth_irs(range(Cn), L)
h = lib.fftconv_twostage_init_batch(0, Cn, irs.ctypes.data, L, L, B, L)
assert h
del irs
x = torch.from_numpy(shard.synth_dry(range(Cn), steps, B)).cuda()
y = torch.empty((steps, Cn, B), device="cuda")


def call(k):
    r = lib.fftconv_twostage_process_device(h, x[k].data_ptr(), B, y[k].data_ptr(), B, B, s.cuda_stream)
    assert r == 0, r


for k in range(2 * steps):  # warm: two periods
    call(k % steps)
n = a.periods * steps
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
ev[0].record(s)
for k in range(n):
    call(k % steps)
    ev[k + 1].record(s)
torch.cuda.synchronize()
dt = [ev[k].elapsed_time(ev[k + 1]) * 1000 for k in range(n)]
per_pos = [[dt[q * steps + j] for q in range(a.periods)] for j in range(steps)]
tot = sum(dt)
print(f"{n} calls, {tot / n:.3f} us/call average ({Cn * B * n / tot:.1f} MS/s)")
print("median us by call position in the period (the last call ends the period: flush, tail launch, tail wait):")
print(" ".join(f"{j}:{statistics.median(v):.2f}" for j, v in enumerate(per_pos)))
mid = statistics.median([statistics.median(v) for v in per_pos[1:-1]])
print(f"typical call {mid:.3f} us; first {statistics.median(per_pos[0]):.2f}, last {statistics.median(per_pos[-1]):.2f}")
