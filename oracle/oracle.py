"""ctypes view of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The classes mirror the reference's `Convolution` trait (src/lib.rs:5-14) over
the C restatement in fftconv_oracle.c.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product path never
does.  A reference panic surfaces here as OraclePanic.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of the same restatement (make asan: liboracle_asan.so)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")

_f32p = C.POINTER(C.c_float)
_sz = C.c_size_t


class OraclePanic(RuntimeError):
    """Raised where the reference would panic (assert!/panic!/todo!)."""


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        sig = {
            "ou_init": (vp, [_f32p, _sz, _sz, _sz]),
            "ou_default": (vp, []),
            "ou_update": (C.c_int, [vp, _f32p, _sz]),
            "ou_process": (None, [vp, _f32p, _f32p, _sz]),
            "ou_reset": (None, [vp]),
            "ou_clone": (vp, [vp]),
            "ou_free": (None, [vp]),
            "ou_block_size": (_sz, [vp]),
            "ou_seg_count": (_sz, [vp]),
            "ou_active_seg_count": (_sz, [vp]),
            "ou_current": (_sz, [vp]),
            "ou_fill": (_sz, [vp]),
            "oracle_compute_tail_block_size": (_sz, [_sz, _sz]),
            "oracle_complex_size": (_sz, [_sz]),
            "ots_init": (vp, [_f32p, _sz, _sz, _sz]),
            "ots_process": (C.c_int, [vp, _f32p, _f32p, _sz]),
            "ots_reset": (None, [vp]),
            "ots_clone": (vp, [vp]),
            "ots_free": (None, [vp]),
            "ots_tail_block_size": (_sz, [vp]),
            "ocf_init": (vp, [_f32p, _sz, _sz, _sz]),
            "ocf_new": (vp, [vp, _sz, _sz, _sz]),
            "ocf_update": (C.c_int, [vp, _f32p, _sz]),
            "ocf_process": (C.c_int, [vp, _f32p, _sz, _f32p, _sz]),
            "ocf_is_crossfading": (C.c_int, [vp]),
            "ocf_response_pending": (C.c_int, [vp]),
            "ocf_free": (None, [vp]),
            "oracle_xfader_new": (vp, [_sz, _sz]),
            "oracle_xfader_free": (None, [vp]),
            "oracle_xfader_fade_into": (None, [vp, C.c_int]),
            "oracle_xfader_mix": (C.c_float, [vp, C.c_float, C.c_float]),
            "oracle_xfader_state": (C.c_int, [vp]),
            "oracle_bench_uniform": (C.c_double, [_sz, _sz, _sz, _sz, _sz, _sz, C.c_uint64]),
            "oracle_bench": (C.c_double, [C.c_int, _sz, _sz, _sz, _sz, _sz, _sz, C.c_uint64, _sz]),
            "oracle_rfft_forward": (C.c_int, [_sz, _f32p, _f32p]),
            "oracle_rfft_inverse": (C.c_int, [_sz, _f32p, _f32p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def compute_tail_block_size(head_len: int, response_len: int) -> int:
    """src/fft_convolver.rs:520-540."""
    return int(lib().oracle_compute_tail_block_size(head_len, response_len))


def complex_size(n: int) -> int:
    """src/fft_convolver.rs:52-68."""
    return int(lib().oracle_complex_size(n))


class _Handle:
    _free = ""

    def __init__(self, h):
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            getattr(_lib, self._free)(h)
            self._h = None


class FFTConvolver(_Handle):
    """src/fft_convolver.rs:86-321."""

    _free = "ou_free"

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int):
        r = _f32(response)
        h = lib().ou_init(_ptr(r), r.size, max_block_size, max_response_length)
        if not h:
            raise OraclePanic("max_response_length must be at least the length of the initial impulse response")
        return cls(h)

    @classmethod
    def default(cls):
        return cls(lib().ou_default())

    def update(self, response):
        r = _f32(response)
        if lib().ou_update(self._h, _ptr(r), r.size):
            raise OraclePanic("New impulse response is longer than initialized length")

    def reset(self):
        lib().ou_reset(self._h)

    def process(self, inp, out_len: int | None = None) -> np.ndarray:
        x = _f32(inp)
        n = x.size if out_len is None else out_len
        if x.size < n:
            raise OraclePanic("input slice shorter than output")
        y = np.zeros(n, np.float32)
        lib().ou_process(self._h, _ptr(x), _ptr(y), n)
        return y

    def clone(self):
        return FFTConvolver(lib().ou_clone(self._h))

    @property
    def block_size(self):
        return int(lib().ou_block_size(self._h))

    @property
    def seg_count(self):
        return int(lib().ou_seg_count(self._h))

    @property
    def active_seg_count(self):
        return int(lib().ou_active_seg_count(self._h))

    @property
    def current(self):
        return int(lib().ou_current(self._h))

    @property
    def fill(self):
        return int(lib().ou_fill(self._h))


class TwoStageFFTConvolver(_Handle):
    """src/fft_convolver.rs:323-526."""

    _free = "ots_free"

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int):
        r = _f32(response)
        h = lib().ots_init(_ptr(r), r.size, max_block_size, max_response_length)
        if not h:
            raise OraclePanic("max_response_length must be at least the length of the initial impulse response")
        return cls(h)

    def update(self, response):
        raise OraclePanic("not yet implemented")  # todo!() at src/fft_convolver.rs:408-410

    def reset(self):
        lib().ots_reset(self._h)

    def process(self, inp) -> np.ndarray:
        x = _f32(inp)
        y = np.zeros(x.size, np.float32)
        if lib().ots_process(self._h, _ptr(x), _ptr(y), x.size):
            raise OraclePanic("assertion failed: input.len() <= self.head_block_size")
        return y

    def clone(self):
        return TwoStageFFTConvolver(lib().ots_clone(self._h))

    @property
    def tail_block_size(self):
        return int(lib().ots_tail_block_size(self._h))


class CrossfadeConvolver(_Handle):
    """CrossfadeConvolver<FFTConvolver>, src/crossfade_convolver.rs:3-105."""

    _free = "ocf_free"

    def __init__(self, h, max_buffer_size: int):
        super().__init__(h)
        self.max_buffer_size = max_buffer_size

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int):
        r = _f32(response)
        h = lib().ocf_init(_ptr(r), r.size, max_block_size, max_response_length)
        if not h:
            raise OraclePanic("max_response_length must be at least the length of the initial impulse response")
        return cls(h, max_block_size)

    @classmethod
    def new(cls, convolver: FFTConvolver, max_response_length: int, max_buffer_size: int, crossfade_samples: int):
        inner = lib().ou_clone(convolver._h)
        h = lib().ocf_new(inner, max_response_length, max_buffer_size, crossfade_samples)
        return cls(h, max_buffer_size)

    def update(self, response):
        r = _f32(response)
        if lib().ocf_update(self._h, _ptr(r), r.size):
            raise OraclePanic("crossfade update: response too long")

    def reset(self):
        raise OraclePanic("not yet implemented")  # todo!() at src/crossfade_convolver.rs:80-82

    def process(self, inp, out_len: int | None = None) -> np.ndarray:
        x = _f32(inp)
        n = x.size if out_len is None else out_len
        y = np.zeros(n, np.float32)
        if lib().ocf_process(self._h, _ptr(x), x.size, _ptr(y), n):
            raise OraclePanic("crossfade process: slice out of bounds")
        return y

    def is_crossfading(self) -> bool:
        return bool(lib().ocf_is_crossfading(self._h))

    @property
    def response_pending(self) -> bool:
        return bool(lib().ocf_response_pending(self._h))


class Crossfader(_Handle):
    """Crossfader<RaisedCosineMixer>, src/crossfade_convolver.rs:192-279."""

    _free = "oracle_xfader_free"
    A, B = 0, 1

    @classmethod
    def new(cls, fading_samples: int, hold_samples: int):
        return cls(lib().oracle_xfader_new(fading_samples, hold_samples))

    def fade_into(self, target: int):
        lib().oracle_xfader_fade_into(self._h, target)

    def mix(self, a: float, b: float) -> float:
        return float(lib().oracle_xfader_mix(self._h, a, b))

    @property
    def state(self):
        """(approaching: bool, target: 0=A/1=B)."""
        s = int(lib().oracle_xfader_state(self._h))
        return (s // 2 == 1, s % 2)


def bench_uniform(channels, block, ir_len, nblocks, warm, threads, seed=1234) -> float:
    return float(lib().oracle_bench_uniform(channels, block, ir_len, nblocks, warm, threads, seed))


def rfft_forward(x) -> np.ndarray:
    """Fft::forward (src/fft_convolver.rs:36-39): unnormalised R2C of an even
    length row -> complex64[n/2 + 1] (the restatement of realfft's algorithm)."""
    x = _f32(x)
    out = np.zeros(x.size + 2, np.float32)
    if lib().oracle_rfft_forward(x.size, _ptr(x), _ptr(out)):
        raise ValueError("length must be even and > 0")
    return out.view(np.complex64)


def rfft_inverse(spec, n: int):
    """Fft::inverse (src/fft_convolver.rs:41-49): C2R of n/2+1 bins, / n.
    Returns (x, input_error): realfft's FftError::InputValues when DC or
    Nyquist has a non-zero imaginary part (the output is computed anyway)."""
    z = np.ascontiguousarray(np.asarray(spec, np.complex64)).view(np.float32)
    x = np.zeros(n, np.float32)
    rc = lib().oracle_rfft_inverse(n, _ptr(z), _ptr(x))
    if rc < 0:
        raise ValueError("length must be even and > 0")
    return x, bool(rc)


BENCH_KINDS = {"uniform": 0, "twostage": 1, "crossfade": 2}


def bench(kind, channels, block, ir_len, nblocks, warm, threads, seed=1234, every=0) -> float:
    """Seconds of `nblocks` process() calls of `block` samples on every one of
    `channels` instances of `kind` (twostage: block = head block; crossfade:
    update() with a fresh response every `every` blocks), split over threads."""
    return float(lib().oracle_bench(BENCH_KINDS[kind], channels, block, ir_len, nblocks, warm, threads, seed, every))


def direct_convolution(x, h) -> np.ndarray:
    """Independent f64 ground truth: causal linear convolution y[n] = sum_k h[k] x[n-k]
    truncated to len(x); what UPOLS computes with zero latency."""
    x = np.asarray(x, np.float64)
    h = np.asarray(h, np.float64)
    if h.size == 0 or x.size == 0:
        return np.zeros(x.size)
    n = x.size + h.size - 1
    nfft = 1 << (n - 1).bit_length()
    y = np.fft.irfft(np.fft.rfft(x, nfft) * np.fft.rfft(h, nfft), nfft)[: x.size]
    return y
