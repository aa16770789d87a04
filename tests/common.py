"""Input generators and tolerance helpers shared by the tests."""
import numpy as np

SAMPLE_RATE = 44100.0

# Stated f32 tolerance: max|got - ref| <= REL_TOL * max|ref|,
# and 1e-6 absolute for the reference's delta-IR known-answer tests.
REL_TOL = 1e-5
DELTA_ABS_TOL = 1e-6


def generate_sinusoid(length, frequency, sample_rate=SAMPLE_RATE, gain=1.0):
    """src/tests.rs:9-16, f32 arithmetic in the reference's evaluation order."""
    i = np.arange(length, dtype=np.float32)
    two_pi = np.float32(2.0) * np.float32(np.pi)
    arg = (two_pi * np.float32(frequency)) * i / np.float32(sample_rate)
    return (np.float32(gain) * np.sin(arg)).astype(np.float32)


def white(rng, n, scale=1.0):
    return (rng.uniform(-1.0, 1.0, n) * scale).astype(np.float32)


def ir(rng, n):
    """White-noise IR U[-1,1) / sqrt(L)."""
    return white(rng, n, 1.0 / np.sqrt(max(n, 1)))


def max_rel_err(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    peak = float(np.max(np.abs(ref))) if ref.size else 0.0
    err = float(np.max(np.abs(got - ref))) if ref.size else 0.0
    return err / peak if peak > 0 else err


def assert_close(got, ref, rel=REL_TOL, what=""):
    e = max_rel_err(got, ref)
    assert e <= rel, f"{what}: max|got-ref|/max|ref| = {e:.3e} > {rel:.1e}"
