"""fftconv_amd -- Python mirror of the reference's `Convolution` trait over the
MI355X C ABI (include/fftconv.h, libfftconv_amd.so).

    FFTConvolver.init(response, max_block_size, max_response_length)   src/fft_convolver.rs:105
    .update(response) / .reset() / .process(input[, out_len]) / .clone()
    TwoStageFFTConvolver.init(...)                                      src/fft_convolver.rs:340
    CrossfadeConvolver.init(...) / CrossfadeConvolver.new(conv, ...)    src/crossfade_convolver.rs:19-49

Every object is a batch of `channels` independent convolvers on one GPU
(channels=1 is exactly one reference instance).  Host arrays are
[channels][samples] (1-D for a single channel).  `process_device` takes raw
device pointers (e.g. torch tensors' data_ptr()) and a HIP stream and is
asynchronous.  Stream 0 is HIP's null stream -- torch's default stream --
as everywhere in HIP: work enqueued there after a call sees its results.

A reference panic surfaces as `ConvolutionPanic`; HIP failures as
`DeviceError`.  There is no CPU fallback: importing works anywhere, but
creating a convolver needs the HIP library and a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FFTCONV_AMD_LIB: another build of the same library (A/B of kernel revisions)
LIB_PATH = os.environ.get("FFTCONV_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "libfftconv_amd.so")

FFTCONV_OK = 0
FFTCONV_E_INVALID = -1
FFTCONV_E_UNIMPLEMENTED = -2
FFTCONV_E_UNSUPPORTED = -3
FFTCONV_E_DEVICE = -4
FFTCONV_E_NOMEM = -5

# every symbol include/fftconv.h declares: name -> (restype, argtypes)
_vp, _sz, _fp, _i = C.c_void_p, C.c_size_t, C.POINTER(C.c_float), C.c_int
SIGNATURES = {
    "fftconv_abi_version": (_i, []),
    "fftconv_last_error": (C.c_char_p, []),
    "fftconv_device_count": (_i, []),
    "fftconv_complex_size": (_sz, [_sz]),
    "fftconv_compute_tail_block_size": (_sz, [_sz, _sz]),
    "fftconv_fft_forward": (_i, [_i, _sz, _sz, _vp, _sz, _vp, _sz, _vp]),
    "fftconv_fft_inverse": (_i, [_i, _sz, _sz, _vp, _sz, _vp, _sz, _vp, _vp]),
    "fftconv_fft_forward_host": (_i, [_i, _sz, _sz, _fp, _fp]),
    "fftconv_fft_inverse_host": (_i, [_i, _sz, _sz, _fp, _fp, C.POINTER(_i)]),
    "fftconv_set_kernel_variant": (_i, [_i]),
    "fftconv_get_kernel_variant": (_i, []),
    "fftconv_set_pipeline_lag": (_i, [_i]),
    "fftconv_get_pipeline_lag": (_i, []),
    "fftconv_set_host_stage_limit": (_i, [_sz]),
    "fftconv_get_host_stage_limit": (_sz, []),
    "fftconv_uniform_init": (_vp, [_fp, _sz, _sz, _sz]),
    "fftconv_uniform_init_batch": (_vp, [_i, _sz, _fp, _sz, _sz, _sz, _sz]),
    "fftconv_uniform_update": (_i, [_vp, _fp, _sz]),
    "fftconv_uniform_update_batch": (_i, [_vp, _fp, _sz, _sz]),
    "fftconv_uniform_update_channel": (_i, [_vp, _sz, _fp, _sz]),
    "fftconv_uniform_update_device": (_i, [_vp, _vp, _sz, _sz, _vp]),
    "fftconv_uniform_reset": (_i, [_vp]),
    "fftconv_uniform_process": (_i, [_vp, _fp, _sz, _fp, _sz]),
    "fftconv_uniform_process_device": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _vp]),
    "fftconv_uniform_process_device_steps": (_i, [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _sz, _sz, _vp]),
    "fftconv_uniform_clone": (_vp, [_vp]),
    "fftconv_uniform_destroy": (None, [_vp]),
    "fftconv_uniform_synchronize": (_i, [_vp]),
    "fftconv_uniform_channels": (_sz, [_vp]),
    "fftconv_uniform_lookahead_parts": (_i, [_vp]),
    "fftconv_uniform_far_windows": (_i, [_vp]),
    "fftconv_uniform_lookahead_probe": (_i, [_vp]),
    "fftconv_uniform_block_size": (_sz, [_vp]),
    "fftconv_uniform_seg_count": (_sz, [_vp]),
    "fftconv_uniform_ir_spectrum": (_i, [_vp, _sz, _sz, _fp]),
    "fftconv_uniform_channel_state": (_i, [_vp, _sz, C.POINTER(_sz)]),
    "fftconv_twostage_init": (_vp, [_fp, _sz, _sz, _sz]),
    "fftconv_twostage_init_batch": (_vp, [_i, _sz, _fp, _sz, _sz, _sz, _sz]),
    "fftconv_twostage_update": (_i, [_vp, _fp, _sz]),
    "fftconv_twostage_reset": (_i, [_vp]),
    "fftconv_twostage_process": (_i, [_vp, _fp, _fp, _sz]),
    "fftconv_twostage_process_device": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _vp]),
    "fftconv_twostage_process_device_steps": (_i, [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _sz, _sz, _vp]),
    "fftconv_twostage_clone": (_vp, [_vp]),
    "fftconv_twostage_destroy": (None, [_vp]),
    "fftconv_twostage_synchronize": (_i, [_vp]),
    "fftconv_twostage_tail_block_size": (_sz, [_vp]),
    "fftconv_crossfade_init": (_vp, [_fp, _sz, _sz, _sz]),
    "fftconv_crossfade_init_batch": (_vp, [_i, _sz, _fp, _sz, _sz, _sz, _sz]),
    "fftconv_crossfade_new": (_vp, [_vp, _sz, _sz, _sz]),
    "fftconv_crossfade_init_twostage": (_vp, [_fp, _sz, _sz, _sz]),
    "fftconv_crossfade_init_twostage_batch": (_vp, [_i, _sz, _fp, _sz, _sz, _sz, _sz]),
    "fftconv_crossfade_new_twostage": (_vp, [_vp, _sz, _sz, _sz]),
    "fftconv_crossfade_update": (_i, [_vp, _fp, _sz]),
    "fftconv_crossfade_update_batch": (_i, [_vp, _fp, _sz, _sz]),
    "fftconv_crossfade_update_device": (_i, [_vp, _vp, _sz, _sz, _vp]),
    "fftconv_crossfade_reset": (_i, [_vp]),
    "fftconv_crossfade_process": (_i, [_vp, _fp, _sz, _fp, _sz]),
    "fftconv_crossfade_process_device": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _vp]),
    "fftconv_crossfade_process_device_steps": (_i, [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _sz, _sz, _vp]),
    "fftconv_crossfade_is_crossfading": (_i, [_vp]),
    "fftconv_crossfade_clone": (_vp, [_vp]),
    "fftconv_crossfade_destroy": (None, [_vp]),
    "fftconv_crossfade_synchronize": (_i, [_vp]),
}


class ConvolutionPanic(RuntimeError):
    """Where the reference panics (assert!/panic!/slice bounds)."""


class NotImplementedInReference(ConvolutionPanic):
    """Where the reference has todo!()."""


class DeviceError(RuntimeError):
    """HIP runtime failure or no usable device."""


_lib = None


def lib():
    """Load libfftconv_amd.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DeviceError(f"{LIB_PATH} not built -- run __graft_entry__.build() or make -C fft-convolution_amd")
        # One HIP runtime per process: torch's libc10_hip loads its bundled
        # libamdhip64 by the unversioned name, while this library NEEDs
        # libamdhip64.so.7.  Loading torch first makes the dynamic linker bind
        # our NEEDED entry to torch's copy (same SONAME), so device pointers and
        # hipStream_t handles from torch are valid here; loading us first would
        # put two HIP/HSA runtimes in the process and torch would see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.fftconv_abi_version() != 1:
            raise DeviceError("ABI version mismatch")
        _lib = L
    return _lib


def last_error() -> str:
    return lib().fftconv_last_error().decode()


def _check(rc: int):
    if rc == FFTCONV_OK:
        return
    msg = last_error()
    if rc == FFTCONV_E_INVALID:
        raise ConvolutionPanic(msg)
    if rc == FFTCONV_E_UNIMPLEMENTED:
        raise NotImplementedInReference(msg)
    raise DeviceError(f"status {rc}: {msg}")


def _handle(h):
    if not h:
        msg = last_error()
        if "max_response_length" in msg or "longer" in msg:
            raise ConvolutionPanic(msg)
        raise DeviceError(msg or "handle creation failed")
    return h


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a: np.ndarray):
    return a.ctypes.data_as(_fp)


def complex_size(n: int) -> int:
    return int(lib().fftconv_complex_size(n))


def compute_tail_block_size(head_len: int, response_len: int) -> int:
    return int(lib().fftconv_compute_tail_block_size(head_len, response_len))


def set_kernel_variant(v: int):
    _check(lib().fftconv_set_kernel_variant(v))


def get_kernel_variant() -> int:
    return int(lib().fftconv_get_kernel_variant())


def set_host_stage_limit(nbytes: int):
    """Cap (bytes, 0 = none) on the pinned host staging a handle reserves at
    creation for update(); larger updates stream through it in chunks."""
    _check(lib().fftconv_set_host_stage_limit(nbytes))


def get_host_stage_limit() -> int:
    return int(lib().fftconv_get_host_stage_limit())


def set_pipeline_lag(rows: int):
    """FDL rows the pipelined step leaves to its stream waves (-1 = automatic)."""
    _check(lib().fftconv_set_pipeline_lag(rows))


def get_pipeline_lag() -> int:
    return int(lib().fftconv_get_pipeline_lag())


def device_count() -> int:
    return int(lib().fftconv_device_count())


class Fft:
    """Fft (src/fft_convolver.rs:7-50) of length n on the GPU: realfft's
    R2C / C2R (forward unnormalised, inverse / n), batched over rows.  Any n in
    1..2^21 (Bluestein for a length that is not a power of two), or a power of
    two up to 2^23."""

    def __init__(self, length: int, device: int = 0):
        self.n = int(length)
        self.device = device

    def forward(self, x) -> np.ndarray:
        """[rows][n] (or [n]) reals -> complex64 [rows][n/2 + 1]."""
        x = _f32(x)
        flat = x.ndim == 1
        x2 = x.reshape(-1, self.n)
        out = np.zeros((x2.shape[0], 2 * (self.n // 2 + 1)), np.float32)
        _check(lib().fftconv_fft_forward_host(self.device, self.n, x2.shape[0], _p(x2), _p(out)))
        out = out.view(np.complex64)
        return out[0] if flat else out

    def inverse(self, spec):
        """complex [rows][n/2 + 1] -> ([rows][n] reals / n, per-row
        FftError::InputValues flags (non-zero DC / Nyquist imaginary part))."""
        z = np.ascontiguousarray(np.asarray(spec, np.complex64))
        flat = z.ndim == 1
        z2 = z.reshape(-1, self.n // 2 + 1)
        zf = np.ascontiguousarray(z2).view(np.float32)
        out = np.zeros((z2.shape[0], self.n), np.float32)
        st = np.zeros(z2.shape[0], np.int32)
        _check(lib().fftconv_fft_inverse_host(self.device, self.n, z2.shape[0], _p(zf), _p(out),
                                              st.ctypes.data_as(C.POINTER(_i))))
        return (out[0], bool(st[0])) if flat else (out, st.astype(bool))

    def forward_device(self, d_in: int, in_stride: int, d_out: int, out_stride: int, rows: int, stream: int = 0):
        _check(lib().fftconv_fft_forward(self.device, self.n, rows, C.c_void_p(d_in), in_stride, C.c_void_p(d_out),
                                         out_stride, C.c_void_p(stream) if stream else None))

    def inverse_device(self, d_in: int, in_stride: int, d_out: int, out_stride: int, rows: int, d_status: int = 0,
                       stream: int = 0):
        _check(lib().fftconv_fft_inverse(self.device, self.n, rows, C.c_void_p(d_in), in_stride, C.c_void_p(d_out),
                                         out_stride, C.c_void_p(d_status) if d_status else None,
                                         C.c_void_p(stream) if stream else None))


def _responses(responses, channels):
    r = _f32(responses)
    if r.ndim == 1:
        return r, r.size, 0
    if r.shape[0] != channels:
        raise ValueError("responses must be [channels][len]")
    return r, r.shape[1], r.shape[1]


class _Base:
    _prefix = ""

    def __init__(self, h, channels: int):
        self._h = h
        self.channels = channels

    def _fn(self, name):
        return getattr(lib(), f"fftconv_{self._prefix}_{name}")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            getattr(_lib, f"fftconv_{self._prefix}_destroy")(h)
            self._h = None

    def _shape_in(self, x):
        x = _f32(x)
        if self.channels == 1 and x.ndim == 1:
            return x, x.size, True
        if x.ndim != 2 or x.shape[0] != self.channels:
            raise ValueError(f"input must be [{self.channels}][n]")
        return x, x.shape[1], False

    def synchronize(self):
        _check(self._fn("synchronize")(self._h))

    def process_device(self, d_in: int, in_stride: int, d_out: int, out_stride: int, n: int, stream: int = 0):
        """process() on device buffers, enqueued on `stream` (0 = HIP's null
        stream, torch's default stream; fftconv.h "Streams"): ordered after the
        handle's previous work, and work enqueued on `stream` afterwards sees
        the output."""
        _check(self._fn("process_device")(self._h, C.c_void_p(d_in), in_stride, C.c_void_p(d_out), out_stride, n,
                                          C.c_void_p(stream) if stream else None))

    def process_device_steps(self, d_in: int, in_stride: int, in_step: int, d_out: int, out_stride: int,
                             out_step: int, n: int, steps: int, stream: int = 0):
        """`steps` consecutive process_device calls (offsets in floats); stream 0 =
        HIP's null stream, as process_device."""
        _check(self._fn("process_device_steps")(self._h, C.c_void_p(d_in), in_stride, in_step, C.c_void_p(d_out),
                                                out_stride, out_step, n, steps,
                                                C.c_void_p(stream) if stream else None))

    def __copy__(self):
        return self.clone()


class FFTConvolver(_Base):
    """FFTConvolver, src/fft_convolver.rs:86-307 (a batch of `channels`)."""

    _prefix = "uniform"

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int, *, channels: int = 1, device: int = 0):
        r, n, stride = _responses(response, channels)
        h = lib().fftconv_uniform_init_batch(device, channels, _p(r), n, stride, max_block_size, max_response_length)
        return cls(_handle(h), channels)

    def update(self, response):
        r = _f32(response)
        if r.ndim == 2:
            _check(lib().fftconv_uniform_update_batch(self._h, _p(r), r.shape[1], r.shape[1]))
        else:
            _check(lib().fftconv_uniform_update(self._h, _p(r), r.size))

    def update_device(self, d_responses: int, response_len: int, stride: int = 0, stream: int = 0):
        """update() from device memory (channel c at d_responses + 4*c*stride;
        stride 0 = same response for all channels), stream-ordered."""
        _check(self._fn("update_device")(self._h, C.c_void_p(d_responses), response_len, stride,
                                         C.c_void_p(stream) if stream else None))

    def update_channel(self, channel: int, response):
        r = _f32(response)
        _check(lib().fftconv_uniform_update_channel(self._h, channel, _p(r), r.size))

    def reset(self):
        _check(lib().fftconv_uniform_reset(self._h))

    def process(self, inp, out_len: int | None = None) -> np.ndarray:
        x, n_in, flat = self._shape_in(inp)
        n = n_in if out_len is None else out_len
        y = np.zeros((self.channels, n), np.float32)
        _check(lib().fftconv_uniform_process(self._h, _p(x), n_in, _p(y), n))
        return y[0] if flat else y

    def clone(self):
        return FFTConvolver(_handle(lib().fftconv_uniform_clone(self._h)), self.channels)

    @property
    def block_size(self) -> int:
        return int(lib().fftconv_uniform_block_size(self._h))

    @property
    def seg_count(self) -> int:
        return int(lib().fftconv_uniform_seg_count(self._h))

    def lookahead_parts(self) -> int:
        """Anchor workgroups per channel of the lookahead step (0 = not used)."""
        return int(lib().fftconv_uniform_lookahead_parts(self._h))

    def far_windows(self) -> int:
        """Window rows per channel of the far-row windows (B >= 1024; 0 = not used)."""
        return int(lib().fftconv_uniform_far_windows(self._h))

    def lookahead_probe(self) -> int:
        """(tests) live state words the FFTCONV_LA_PROBE launches' anchors found
        already rewritten by their own launch's steps (the anchors compute from
        launch-start copies); -1 when the probe is off."""
        return int(lib().fftconv_uniform_lookahead_probe(self._h))

    def ir_spectrum(self, channel: int, segment: int) -> np.ndarray:
        """segments_ir[segment] of a channel: complex64[B + 1]."""
        out = np.zeros(2 * (self.block_size + 1), np.float32)
        _check(lib().fftconv_uniform_ir_spectrum(self._h, channel, segment, _p(out)))
        return out.view(np.complex64)

    def channel_state(self, channel: int = 0):
        """(current, active_seg_count, input_buffer_fill)."""
        out = (C.c_size_t * 3)()
        _check(lib().fftconv_uniform_channel_state(self._h, channel, out))
        return tuple(int(v) for v in out)


class TwoStageFFTConvolver(_Base):
    """TwoStageFFTConvolver, src/fft_convolver.rs:323-526."""

    _prefix = "twostage"

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int, *, channels: int = 1, device: int = 0):
        r, n, stride = _responses(response, channels)
        h = lib().fftconv_twostage_init_batch(device, channels, _p(r), n, stride, max_block_size, max_response_length)
        return cls(_handle(h), channels)

    def update(self, response):
        r = _f32(response)
        _check(lib().fftconv_twostage_update(self._h, _p(r), r.size))

    def reset(self):
        _check(lib().fftconv_twostage_reset(self._h))

    def process(self, inp) -> np.ndarray:
        x, n, flat = self._shape_in(inp)
        y = np.zeros((self.channels, n), np.float32)
        _check(lib().fftconv_twostage_process(self._h, _p(x), _p(y), n))
        return y[0] if flat else y

    def clone(self):
        return TwoStageFFTConvolver(_handle(lib().fftconv_twostage_clone(self._h)), self.channels)

    @property
    def tail_block_size(self) -> int:
        return int(lib().fftconv_twostage_tail_block_size(self._h))


class CrossfadeConvolver(_Base):
    """CrossfadeConvolver<T>, src/crossfade_convolver.rs:3-105, for T =
    FFTConvolver (the default) or TwoStageFFTConvolver (`inner=`, or `new`
    with a TwoStageFFTConvolver).  Over a TwoStageFFTConvolver every update()
    reaches its todo!() (src/fft_convolver.rs:408-410) and raises
    NotImplementedInReference, as the reference panics."""

    _prefix = "crossfade"

    def __init__(self, h, channels: int, max_buffer_size: int, inner: type = None):
        super().__init__(h, channels)
        self.max_buffer_size = max_buffer_size
        self.inner = inner or FFTConvolver

    @classmethod
    def init(cls, response, max_block_size: int, max_response_length: int, *, channels: int = 1, device: int = 0,
             inner: type = None):
        """Convolution::init (:46-49); `inner` is the T of CrossfadeConvolver<T>."""
        r, n, stride = _responses(response, channels)
        fn = lib().fftconv_crossfade_init_twostage_batch if inner is TwoStageFFTConvolver \
            else lib().fftconv_crossfade_init_batch
        if inner not in (None, FFTConvolver, TwoStageFFTConvolver):
            raise TypeError("inner must be FFTConvolver or TwoStageFFTConvolver")
        h = fn(device, channels, _p(r), n, stride, max_block_size, max_response_length)
        return cls(_handle(h), channels, max_block_size, inner)

    @classmethod
    def new(cls, convolver, max_response_length: int, max_buffer_size: int, crossfade_samples: int):
        """CrossfadeConvolver::new (:19-43); the convolver is cloned."""
        if isinstance(convolver, TwoStageFFTConvolver):
            fn = lib().fftconv_crossfade_new_twostage
        elif isinstance(convolver, FFTConvolver):
            fn = lib().fftconv_crossfade_new
        else:
            raise TypeError("convolver must be an FFTConvolver or a TwoStageFFTConvolver")
        h = fn(convolver._h, max_response_length, max_buffer_size, crossfade_samples)
        return cls(_handle(h), convolver.channels, max_buffer_size, type(convolver))

    def update(self, response):
        r = _f32(response)
        if r.ndim == 2:
            _check(lib().fftconv_crossfade_update_batch(self._h, _p(r), r.shape[1], r.shape[1]))
        else:
            _check(lib().fftconv_crossfade_update(self._h, _p(r), r.size))

    def update_device(self, d_responses: int, response_len: int, stride: int = 0, stream: int = 0):
        """update() from device memory (channel c at d_responses + 4*c*stride;
        stride 0 = same response for all channels), stream-ordered."""
        _check(self._fn("update_device")(self._h, C.c_void_p(d_responses), response_len, stride,
                                         C.c_void_p(stream) if stream else None))

    def reset(self):
        _check(lib().fftconv_crossfade_reset(self._h))

    def process(self, inp, out_len: int | None = None) -> np.ndarray:
        x, n_in, flat = self._shape_in(inp)
        n = n_in if out_len is None else out_len
        y = np.zeros((self.channels, n), np.float32)
        _check(lib().fftconv_crossfade_process(self._h, _p(x), n_in, _p(y), n))
        return y[0] if flat else y

    def is_crossfading(self) -> bool:
        return bool(lib().fftconv_crossfade_is_crossfading(self._h))

    def clone(self):
        return CrossfadeConvolver(_handle(lib().fftconv_crossfade_clone(self._h)), self.channels,
                                  self.max_buffer_size, self.inner)


__all__ = [
    "Fft", "FFTConvolver", "TwoStageFFTConvolver", "CrossfadeConvolver", "ConvolutionPanic",
    "NotImplementedInReference", "DeviceError", "complex_size", "compute_tail_block_size", "device_count",
    "lib", "LIB_PATH", "SIGNATURES",
]
