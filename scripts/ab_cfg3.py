#!/usr/bin/env python3
"""Same-process, interleaved A/B of several builds of libfftconv_amd.so on the
cfg3 workload (TwoStageFFTConvolver, head 64 / tail 4096, IR 262144, 256
channels; one process_device_steps call per tail period of 64 head calls).
Each LIB may carry knobs applied before its timed runs: PATH,variant=1024,lag=8,percall=1
(percall: one process_device_steps call per head call), and
environment knobs read when its handle is created: PATH,FFTCONV_TAIL_LATE=1.
usage: ab_cfg3.py LIB1 LIB2 ... [--rounds R] [--periods P]"""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import torch

from fftconv_amd import shard

p = argparse.ArgumentParser()
p.add_argument("libs", nargs="+")
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--periods", type=int, default=8)
p.add_argument("--channels", type=int, default=256)
p.add_argument("--head", type=int, default=64)
p.add_argument("--ir", type=int, default=262144)
a = p.parse_args()
Cn, B, L = a.channels, a.head, a.ir
T = 4096
steps = T // B  # head calls per tail period
torch.cuda.set_device(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
irs = shard.synth_irs(range(Cn), L)
x = torch.from_numpy(shard.synth_dry(range(Cn), steps, B)).cuda()  # [steps][C][B]
handles = []
loaded = {}
knobs = []
for spec in a.libs:
    path, *kv = spec.split(",")
    knobs.append(dict(k.split("=") for k in kv))
    if path not in loaded:
        loaded[path] = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    lib = loaded[path]
    lib.fftconv_twostage_init_batch.restype = C.c_void_p
    lib.fftconv_twostage_init_batch.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                                C.c_size_t]
    lib.fftconv_twostage_process_device_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                                          C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]
    for k, v in knobs[-1].items():  # (env knobs, read at creation: FFTCONV_TAIL_LATE=1 ...)
        if k.startswith("FFTCONV_"):
            os.environ[k] = v
    h = lib.fftconv_twostage_init_batch(0, Cn, irs.ctypes.data, L, L, B, L)
    for k in knobs[-1]:
        if k.startswith("FFTCONV_"):
            del os.environ[k]
    assert h, path
    handles.append((lib, h, torch.empty((steps, Cn, B), device="cuda"), int(knobs[-1].get("variant", -1)),
                    int(knobs[-1].get("lag", -1)), knobs[-1].get("percall", "0") == "1"))
del irs


def period(lib, h, y, percall=False):
    if percall:  # (one process_device_steps call per head call: the per-call submission)
        for k in range(steps):
            r = lib.fftconv_twostage_process_device_steps(h, x[k].data_ptr(), B, Cn * B, y[k].data_ptr(), B, Cn * B,
                                                           B, 1, s.cuda_stream)
            assert r == 0, r
        return
    r = lib.fftconv_twostage_process_device_steps(h, x.data_ptr(), B, Cn * B, y.data_ptr(), B, Cn * B, B, steps,
                                                   s.cuda_stream)
    assert r == 0, r


res = [[] for _ in handles]
host = [[] for _ in handles]
for r in range(a.rounds):
    for idx, (lib, h, y, var, lag, pc) in enumerate(handles):
        lib.fftconv_set_kernel_variant(var)
        if hasattr(lib, "fftconv_set_pipeline_lag"):
            lib.fftconv_set_pipeline_lag(lag)
        period(lib, h, y, pc)  # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        t0 = time.perf_counter()
        for _ in range(a.periods):
            period(lib, h, y, pc)
        t1 = time.perf_counter()
        e1.record(s)
        torch.cuda.synchronize()
        res[idx].append(e0.elapsed_time(e1) * 1000 / (a.periods * steps))
        host[idx].append((t1 - t0) * 1e6 / (a.periods * steps))
same = all(torch.equal(handles[0][2], hh[2]) for hh in handles[1:])
for path, r, hr in zip(a.libs, res, host):
    us = statistics.median(r)
    print(f"{path}: median {us:.3f} us/step (min {min(r):.3f}) -> {Cn * B / us:.1f} MS/s; "
          f"host enqueue {statistics.median(hr):.3f} us/step")
print("outputs bit-identical across builds:", same)
for lib, h, *_ in handles:  # (destroyed before exit: no live handle at library teardown)
    lib.fftconv_twostage_destroy.argtypes = [C.c_void_p]
    lib.fftconv_twostage_destroy(h)
