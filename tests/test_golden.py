"""Committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py
from the oracle): the oracle must keep reproducing them (CPU), and the HIP
path must match them within the stated f32 tolerance (GPU).  Fixtures are
data only; they never read /root/reference at run time."""
import glob
import os

import numpy as np
import pytest

from common import REL_TOL, assert_close
from replay import replay

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "*.npz")))
IDS = [os.path.basename(p)[:-4] for p in GOLDEN]


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make(mod, f):
    kind = str(f["convolver"])
    cls = {"uniform": mod.FFTConvolver, "twostage": mod.TwoStageFFTConvolver,
           "crossfade": mod.CrossfadeConvolver}[kind]
    return cls.init(f["ir"], int(f["block"]), int(f["max_len"]))


def test_fixtures_present():
    assert len(GOLDEN) >= 8


@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_oracle_reproduces_golden(oracle_mod, path):
    f = load(path)
    got = replay(make(oracle_mod, f), f["kind"], f["n"], f["out_len"], f["data"])
    assert_close(got, f["expected"], rel=1e-6, what="oracle vs fixture")
    if "f64" in f:
        assert_close(got, f["f64"], what="oracle vs f64 direct convolution")
    if os.path.basename(path).startswith("uniform_delta"):
        assert np.max(np.abs(got - 1.0)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_hip_matches_golden(amd, path):
    f = load(path)
    got = replay(make(amd, f), f["kind"], f["n"], f["out_len"], f["data"])
    assert_close(got, f["expected"], rel=REL_TOL, what="HIP vs fixture")
    if "f64" in f:
        assert_close(got, f["f64"], rel=REL_TOL, what="HIP vs f64 direct convolution")
