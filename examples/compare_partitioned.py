#!/usr/bin/env python3
"""examples/compare_partitioned.rs on the GPU path: a 64-sample-block uniform
FFTConvolver and a TwoStageFFTConvolver over the same 128000-tap sinusoid
response, 1000 blocks of a 1300 Hz sinusoid fed one block per process() call
(reference: examples/compare_partitioned.rs:9-68, util/mod.rs:7-40).  Prints
both timings and the max |a - b| and writes output_a.wav / output_b.wav
(16-bit PCM, the same f32 -> i16 truncation as util::save_wav)."""
import argparse
import math
import os
import sys
import time
import wave

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fft-convolution_amd"))
import fftconv_amd as F  # noqa: E402

SAMPLE_RATE = 44100


def generate_sinusoid(num_samples: int, freq: float, sample_rate: int, gain: float) -> np.ndarray:
    """util::generate_sinusoid (examples/util/mod.rs:7-19): f64 phase, cast to f32."""
    t = np.arange(num_samples, dtype=np.float64) / float(sample_rate)
    return (gain * np.sin(2.0 * math.pi * freq * t)).astype(np.float32)


def save_wav(filename: str, samples: np.ndarray, sample_rate: int):
    """util::save_wav (examples/util/mod.rs:21-40): mono, 16-bit, `as i16`
    (truncation toward zero, saturating)."""
    scaled = np.clip(np.trunc(samples.astype(np.float32) * np.float32(32767.0)), -32768, 32767).astype("<i2")
    with wave.open(filename, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(scaled.tobytes())
    print(f"Saved: {filename}")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block-size", type=int, default=64)
    p.add_argument("--blocks", type=int, default=1000)
    p.add_argument("--response-len", type=int, default=128_000)
    p.add_argument("--out-dir", default=".")
    p.add_argument("--no-wav", action="store_true")
    a = p.parse_args()
    block_size, n_blocks = a.block_size, a.blocks

    response = generate_sinusoid(a.response_len, 1000.0, SAMPLE_RATE, 0.1)
    convolver_a = F.FFTConvolver.init(response, block_size, len(response))
    convolver_b = F.TwoStageFFTConvolver.init(response, block_size, len(response))
    inp = generate_sinusoid(n_blocks * block_size, 1300.0, SAMPLE_RATE, 0.1)
    output_a = np.zeros(block_size * n_blocks, np.float32)
    output_b = np.zeros(block_size * n_blocks, np.float32)

    t = time.perf_counter()
    for i in range(n_blocks):
        s, e = i * block_size, (i + 1) * block_size
        output_a[s:e] = convolver_a.process(inp[s:e])
    print(f"Uniform took = {(time.perf_counter() - t) * 1000:.2f} ms")

    t = time.perf_counter()
    for i in range(n_blocks):
        s, e = i * block_size, (i + 1) * block_size
        output_b[s:e] = convolver_b.process(inp[s:e])
    print(f"Partitioned took = {(time.perf_counter() - t) * 1000:.2f} ms")

    max_abs_diff = float(np.max(np.abs(output_a - output_b)))
    print(f"max_abs_diff = {max_abs_diff!r}")
    if not a.no_wav:
        save_wav(os.path.join(a.out_dir, "output_a.wav"), output_a, SAMPLE_RATE)
        save_wav(os.path.join(a.out_dir, "output_b.wav"), output_b, SAMPLE_RATE)
    return max_abs_diff


if __name__ == "__main__":
    main()
