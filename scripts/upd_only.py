#!/usr/bin/env python3
"""cfg2 update_device only (IR transform + window rebuild), N times: a small
driver for rocprofv3 --pmc passes on the update's kernels."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fft-convolution_amd"))
import torch

from fftconv_amd import shard

Cn, B, L, N = 1024, 256, 48000, int(sys.argv[1]) if len(sys.argv) > 1 else 6
lib = C.CDLL(os.path.join(ROOT, "fft-convolution_amd", "libfftconv_amd.so"))
lib.fftconv_uniform_init_batch.restype = C.c_void_p
lib.fftconv_uniform_init_batch.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]
lib.fftconv_uniform_update_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
lib.fftconv_uniform_destroy.argtypes = [C.c_void_p]
irs = shard.synth_irs(range(Cn), L)
h = lib.fftconv_uniform_init_batch(0, Cn, irs.ctypes.data, L, L, B, L)
assert h
d = torch.from_numpy(shard.synth_irs(range(Cn, 2 * Cn), L)).cuda()
torch.cuda.synchronize()
for _ in range(N):
    assert lib.fftconv_uniform_update_device(h, d.data_ptr(), L, L, None) == 0
torch.cuda.synchronize()
lib.fftconv_uniform_destroy(h)
print("ok")
