"""The reference's example (examples/compare_partitioned.rs) on the GPU path:
the Python mirror and the native C-ABI host both run; the uniform and the
two-stage outputs agree with each other and with the oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

from common import assert_close
from conftest import ROOT

EX = os.path.join(ROOT, "examples")


@pytest.mark.gpu
def test_compare_partitioned_python(amd, oracle_mod, tmp_path):
    sys.path.insert(0, EX)
    try:
        import compare_partitioned as ex
    finally:
        sys.path.remove(EX)
    B, n = 64, 300
    resp = ex.generate_sinusoid(128_000, 1000.0, ex.SAMPLE_RATE, 0.1)
    inp = ex.generate_sinusoid(n * B, 1300.0, ex.SAMPLE_RATE, 0.1)
    a = amd.FFTConvolver.init(resp, B, len(resp))
    b = amd.TwoStageFFTConvolver.init(resp, B, len(resp))
    ref = oracle_mod.FFTConvolver.init(resp, B, len(resp))
    ya = np.concatenate([a.process(inp[i * B:(i + 1) * B]) for i in range(n)])
    yb = np.concatenate([b.process(inp[i * B:(i + 1) * B]) for i in range(n)])
    yr = np.concatenate([ref.process(inp[i * B:(i + 1) * B]) for i in range(n)])
    assert_close(ya, yr, what="uniform vs oracle")
    assert_close(yb, yr, what="two-stage vs oracle")
    ex.save_wav(str(tmp_path / "a.wav"), ya, ex.SAMPLE_RATE)
    assert (tmp_path / "a.wav").stat().st_size == 44 + 2 * n * B


@pytest.mark.gpu
def test_compare_partitioned_native():
    exe = os.path.join(EX, "compare_partitioned")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", EX], check=True)
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = dict(l.split(" = ", 1) for l in r.stdout.splitlines() if " = " in l)
    assert float(lines["max_abs_diff"]) < 1e-5, r.stdout


def test_save_wav_matches_hound_truncation(tmp_path):
    """util::save_wav: `(sample * i16::MAX as f32) as i16` truncates toward
    zero and saturates (examples/util/mod.rs:33-36)."""
    sys.path.insert(0, EX)
    try:
        import compare_partitioned as ex
    finally:
        sys.path.remove(EX)
    import wave

    x = np.array([0.0, 0.5, -0.5, 1.0, -1.0, 2.0, -2.0, 1e-5, -0.99999], np.float32)
    ex.save_wav(str(tmp_path / "t.wav"), x, 44100)
    with wave.open(str(tmp_path / "t.wav"), "rb") as w:
        assert (w.getnchannels(), w.getsampwidth(), w.getframerate()) == (1, 2, 44100)
        got = np.frombuffer(w.readframes(w.getnframes()), "<i2")
    assert got.tolist() == [0, 16383, -16383, 32767, -32767, 32767, -32768, 0, -32766]
