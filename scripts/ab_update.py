#!/usr/bin/env python3
"""Same-process, interleaved A/B of several builds of libfftconv_amd.so on the
cfg2 update (update_device: IR transform + window rebuild), each followed by a
few steps; reports the update's HIP-event time per build and checks that every
build's outputs (steps after each update) are bit-identical.
usage: ab_update.py LIB1 LIB2 ... [--rounds R] [--updates U]"""
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
p.add_argument("libs", nargs="+")
p.add_argument("--rounds", type=int, default=7)
p.add_argument("--updates", type=int, default=10)
p.add_argument("--channels", type=int, default=1024)
p.add_argument("--block", type=int, default=256)
p.add_argument("--ir", type=int, default=48000)
a = p.parse_args()
Cn, B, L = a.channels, a.block, a.ir
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
irs = shard.synth_irs(range(Cn), L)
irs2 = torch.from_numpy(shard.synth_irs(range(Cn, 2 * Cn), L)).cuda()
irs1 = torch.from_numpy(irs).cuda()
x = torch.from_numpy(shard.synth_dry(range(Cn), 4, B)).cuda()
handles, loaded = [], {}
for path in a.libs:
    if path not in loaded:
        loaded[path] = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    lib = loaded[path]
    lib.fftconv_uniform_init_batch.restype = C.c_void_p
    lib.fftconv_uniform_init_batch.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]
    lib.fftconv_uniform_update_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
    lib.fftconv_uniform_process_device_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                                         C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]
    h = lib.fftconv_uniform_init_batch(0, Cn, irs.ctypes.data, L, L, B, L)
    assert h, path
    handles.append((lib, h, torch.empty((4, Cn, B), device="cuda")))
res = [[] for _ in handles]
outs = [[] for _ in handles]
for r in range(a.rounds):
    for idx, (lib, h, y) in enumerate(handles):
        ts = []
        for u in range(a.updates):
            src = irs2 if u % 2 == 0 else irs1
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert lib.fftconv_uniform_update_device(h, src.data_ptr(), L, L, s.cuda_stream) == 0
            e1.record(s)
            assert lib.fftconv_uniform_process_device_steps(h, x.data_ptr(), B, Cn * B, y.data_ptr(), B, Cn * B, B,
                                                            4, s.cuda_stream) == 0
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        res[idx].append(statistics.median(ts))
        if r == 0:
            outs[idx] = y.clone()
for path, rr in zip(a.libs, res):
    print(f"{path}: update median {statistics.median(rr):.1f} us (min {min(rr):.1f})")
print("outputs bit-identical across builds:", all(torch.equal(outs[0], o) for o in outs[1:]))
for lib, h, _ in handles:
    lib.fftconv_uniform_destroy.argtypes = [C.c_void_p]
    lib.fftconv_uniform_destroy(h)
