#!/usr/bin/env python3
"""Same-process, interleaved A/B of several builds of libfftconv_amd.so on the
cfg2 workload (methodology rule: never rank builds across processes/boxes).
Each LIB may carry knobs applied before its timed runs: PATH,variant=6,lag=12.
usage: ab_libs.py LIB1 LIB2 ... [--rounds R] [--steps K] [--channels C] [--block B] [--ir L]"""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import numpy as np
import torch

from fftconv_amd import shard

p = argparse.ArgumentParser()
p.add_argument("libs", nargs="+")
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--steps", type=int, default=200)
p.add_argument("--channels", type=int, default=1024)
p.add_argument("--block", type=int, default=256)
p.add_argument("--ir", type=int, default=48000)
a = p.parse_args()
Cn, B, L = a.channels, a.block, a.ir
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
irs = shard.synth_irs(range(Cn), L)
x = torch.from_numpy(shard.synth_dry(range(Cn), 16, B)).cuda()
handles = []
loaded = {}
knobs = []
for spec in a.libs:
    path, *kv = spec.split(",")
    knobs.append(dict(x.split("=") for x in kv))
    if path not in loaded:
        loaded[path] = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    lib = loaded[path]
    lib.fftconv_uniform_init_batch.restype = C.c_void_p
    lib.fftconv_uniform_init_batch.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]
    lib.fftconv_uniform_process_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
    lib.fftconv_uniform_process_device_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                                         C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]
    envs = {k: v for k, v in knobs[-1].items() if k.startswith("FFTCONV_")}  # read at handle creation
    os.environ.update(envs)
    h = lib.fftconv_uniform_init_batch(0, Cn, irs.ctypes.data, L, L, B, L)
    for k in envs:
        os.environ.pop(k)
    assert h, path
    handles.append((lib, h, torch.empty((16, Cn, B), device="cuda")))
res = [[] for _ in handles]
host = [[] for _ in handles]
k = 0
for r in range(a.rounds):
    for idx, (lib, h, y) in enumerate(handles):
        kn = knobs[idx]
        if hasattr(lib, "fftconv_set_pipeline_lag"):
            lib.fftconv_set_pipeline_lag(int(kn.get("lag", -1)))
        lib.fftconv_set_kernel_variant(int(kn.get("variant", -1)))
        def run(n):
            # n steps as runs of the 16-block ring through process_device_steps
            # (the bench's submission: no Python call per step)
            nonlocal_k = run.k
            while n > 0:
                j = nonlocal_k % 16
                m = min(n, 16 - j)
                lib.fftconv_uniform_process_device_steps(h, x[j].data_ptr(), B, Cn * B, y[j].data_ptr(), B, Cn * B, B,
                                                         m, s.cuda_stream)
                nonlocal_k += m
                n -= m
            run.k = nonlocal_k
        run.k = k
        run(20)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        t0 = time.perf_counter()
        run(a.steps)
        host[idx].append((time.perf_counter() - t0) * 1e6 / a.steps)
        e1.record(s)
        k = run.k
        torch.cuda.synchronize()
        res[idx].append(e0.elapsed_time(e1) * 1000 / a.steps)
eq = [torch.equal(handles[0][2], hh[2]) for hh in handles[1:]]
same = all(eq)
if len(eq) > 1:
    print("bit-identical to the first handle, per handle:", eq)
for path, r, hr in zip(a.libs, res, host):
    us = statistics.median(r)
    print(f"{path}: median {us:.2f} us/step (min {min(r):.2f}) -> {Cn * B / us:.1f} MS/s; "
          f"host enqueue {statistics.median(hr):.2f} us/step")
print("outputs bit-identical across builds:", same)
for lib, h, _ in handles:  # (destroyed before exit: launch timelines are written at destroy)
    lib.fftconv_uniform_destroy.argtypes = [C.c_void_p]
    lib.fftconv_uniform_destroy(h)
