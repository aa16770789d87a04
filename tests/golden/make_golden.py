#!/usr/bin/env python3
"""Generates tests/golden/*.npz from the oracle (oracle/fftconv_oracle.c, the
CPU restatement of the reference) on seeded inputs.  The reference itself
cannot run here (Rust crate; no cargo/rustc and no realfft/rustfft sources in
this image), so these vectors are oracle outputs pinned by the reference's own
known-answer tests (tests/test_oracle.py); uniform cases also carry the
independent f64 direct convolution.  Re-run:  python tests/golden/make_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from replay import flatten, replay  # noqa: E402


def white(rng, n, s=1.0):
    return (rng.uniform(-1, 1, n) * s).astype(np.float32)


def irv(rng, n):
    return white(rng, n, 1.0 / np.sqrt(max(n, 1)))


def scenarios():
    rng = np.random.default_rng(20261015)
    out = {}
    # cfg1 geometry (BASELINE configs[0]): B=256, IR=4096, full-block calls
    h = irv(rng, 4096)
    out["uniform_cfg1"] = ("uniform", dict(block=256, max_len=4096), h,
                           [("process", white(rng, 256)) for _ in range(40)])
    # ragged chunking incl. 1-sample and multi-block calls
    h = irv(rng, 1000)
    ops = [("process", white(rng, k)) for k in [64, 1, 5, 58, 200, 64, 3, 61, 640, 17, 64, 64, 111, 13]]
    out["uniform_ragged"] = ("uniform", dict(block=64, max_len=1000), h, ops)
    # updates: full, shorter (active shrinks), mid-block, empty
    h = irv(rng, 900)
    ops = [("process", white(rng, 128)) for _ in range(10)]
    ops += [("update", irv(rng, 900)), ("process", white(rng, 128)), ("process", white(rng, 50)),
            ("update", irv(rng, 130)), ("process", white(rng, 78)), ("process", white(rng, 128)),
            ("update", irv(rng, 0)), ("process", white(rng, 128)), ("update", irv(rng, 600))]
    ops += [("process", white(rng, 128)) for _ in range(10)]
    out["uniform_update"] = ("uniform", dict(block=128, max_len=900), h, ops)
    # block 1 (N = 2) and a non-power-of-two block (100 -> 128)
    h = irv(rng, 7)
    out["uniform_b1"] = ("uniform", dict(block=1, max_len=7), h, [("process", white(rng, k)) for k in [1, 3, 2, 9]])
    h = irv(rng, 700)
    out["uniform_b100"] = ("uniform", dict(block=100, max_len=700), h,
                           [("process", white(rng, k)) for k in [100, 128, 28, 300, 256]])
    # two-stage, head 64 / IR 12000 (T = 1024) past both tail swaps
    h = irv(rng, 12000)
    out["twostage_64_12000"] = ("twostage", dict(block=64, max_len=12000), h,
                                [("process", white(rng, 64)) for _ in range(40)] +
                                [("process", white(rng, k)) for k in [10, 54, 64, 1, 63]] +
                                [("process", white(rng, 64)) for _ in range(20)])
    # crossfade (trait init: crossfade over response.len()), pending path
    h = irv(rng, 2000)
    ops = []
    for i in range(30):
        if i % 5 == 4:
            ops.append(("update", irv(rng, int(rng.integers(1, 2001)))))
        ops.append(("process", white(rng, 512), 512 if i % 3 else 256))
    out["crossfade_512_2000"] = ("crossfade", dict(block=512, max_len=2000), h, ops)
    # the reference's delta-IR known answer (src/fft_convolver.rs:309-321)
    d = np.zeros(1024, np.float32)
    d[0] = 1.0
    out["uniform_delta_1024"] = ("uniform", dict(block=1024, max_len=1024), d,
                                 [("process", np.ones(1024, np.float32))])
    return out


def make(kind, geo, h):
    cls = {"uniform": oracle.FFTConvolver, "twostage": oracle.TwoStageFFTConvolver,
           "crossfade": oracle.CrossfadeConvolver}[kind]
    return cls.init(h, geo["block"], geo["max_len"])


def main():
    for name, (kind, geo, h, ops) in scenarios().items():
        k, n, o, data = flatten(ops)
        exp = replay(make(kind, geo, h), k, n, o, data)
        extra = {}
        if kind == "uniform" and not np.any(k == 1):
            x = data
            extra["f64"] = oracle.direct_convolution(x, h).astype(np.float64)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), convolver=np.array(kind), block=geo["block"],
                            max_len=geo["max_len"], ir=h, kind=k, n=n, out_len=o, data=data, expected=exp, **extra)
        print(f"{name}: {kind} ops={len(k)} samples_out={exp.size}")


if __name__ == "__main__":
    main()
