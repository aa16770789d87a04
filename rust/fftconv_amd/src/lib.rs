//! GPU-backed drop-ins for the reference crate's convolvers.
//!
//! `GpuFFTConvolver`, `GpuTwoStageFFTConvolver` and `GpuCrossfadeConvolver`
//! implement `fft_convolution::Convolution` (src/lib.rs:5-14) over the C ABI
//! of libfftconv_amd.so (include/fftconv.h).  Error behaviour follows the
//! reference: where it panics (`FFTCONV_E_INVALID`) or has `todo!()`
//! (`FFTCONV_E_UNIMPLEMENTED`) these panic with the library's message; a
//! failed C2R (realfft's error path, src/fft_convolver.rs:264-267) zero-fills
//! the output inside the library exactly as the reference does.
//! `GpuFFTConvolverBatch` exposes the batched, HBM-resident path
//! (`process_device`) used for throughput.

pub mod ffi;

use fft_convolution::Convolution;
use realfft::FftError;
use rustfft::num_complex::Complex;
use std::ffi::CStr;
use std::os::raw::{c_int, c_void};
use std::ptr::NonNull;

fn last_error() -> String {
    unsafe {
        let p = ffi::fftconv_last_error();
        if p.is_null() { String::new() } else { CStr::from_ptr(p).to_string_lossy().into_owned() }
    }
}

fn check(rc: c_int) {
    match rc {
        ffi::FFTCONV_OK => {}
        ffi::FFTCONV_E_UNIMPLEMENTED => panic!("not yet implemented: {}", last_error()),
        _ => panic!("{}", last_error()),
    }
}

fn handle<T>(p: *mut T) -> NonNull<T> {
    NonNull::new(p).unwrap_or_else(|| panic!("{}", last_error()))
}

macro_rules! gpu_convolver {
    ($name:ident, $raw:ident, $init:ident, $update:ident, $reset:ident, $clone:ident, $destroy:ident) => {
        pub struct $name {
            h: NonNull<ffi::$raw>,
        }
        // one caller thread at a time (`&mut self`), as the reference
        unsafe impl Send for $name {}
        impl Clone for $name {
            fn clone(&self) -> Self {
                Self { h: handle(unsafe { ffi::$clone(self.h.as_ptr()) }) }
            }
        }
        impl Drop for $name {
            fn drop(&mut self) {
                unsafe { ffi::$destroy(self.h.as_ptr()) }
            }
        }
        impl $name {
            fn init_raw(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self {
                let p = unsafe { ffi::$init(response.as_ptr(), response.len(), max_block_size, max_response_length) };
                Self { h: handle(p) }
            }
            fn update_raw(&mut self, response: &[f32]) {
                check(unsafe { ffi::$update(self.h.as_ptr(), response.as_ptr(), response.len()) })
            }
            fn reset_raw(&mut self) {
                check(unsafe { ffi::$reset(self.h.as_ptr()) })
            }
        }
    };
}

gpu_convolver!(GpuFFTConvolver, fftconv_uniform, fftconv_uniform_init, fftconv_uniform_update,
               fftconv_uniform_reset, fftconv_uniform_clone, fftconv_uniform_destroy);
gpu_convolver!(GpuTwoStageFFTConvolver, fftconv_twostage, fftconv_twostage_init, fftconv_twostage_update,
               fftconv_twostage_reset, fftconv_twostage_clone, fftconv_twostage_destroy);
gpu_convolver!(GpuCrossfadeConvolver, fftconv_crossfade, fftconv_crossfade_init, fftconv_crossfade_update,
               fftconv_crossfade_reset, fftconv_crossfade_clone, fftconv_crossfade_destroy);
gpu_convolver!(GpuCrossfadeTwoStageConvolver, fftconv_crossfade, fftconv_crossfade_init_twostage,
               fftconv_crossfade_update, fftconv_crossfade_reset, fftconv_crossfade_clone, fftconv_crossfade_destroy);

/// FFTConvolver (src/fft_convolver.rs:86-307).
impl Convolution for GpuFFTConvolver {
    fn init(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self {
        Self::init_raw(response, max_block_size, max_response_length)
    }
    fn update(&mut self, response: &[f32]) {
        self.update_raw(response)
    }
    fn reset(&mut self) {
        self.reset_raw()
    }
    fn process(&mut self, input: &[f32], output: &mut [f32]) {
        check(unsafe {
            ffi::fftconv_uniform_process(self.h.as_ptr(), input.as_ptr(), input.len(), output.as_mut_ptr(),
                                         output.len())
        })
    }
}

/// TwoStageFFTConvolver (src/fft_convolver.rs:323-512); `update` is the
/// reference's `todo!()` and panics the same way.
impl Convolution for GpuTwoStageFFTConvolver {
    fn init(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self {
        Self::init_raw(response, max_block_size, max_response_length)
    }
    fn update(&mut self, response: &[f32]) {
        self.update_raw(response)
    }
    fn reset(&mut self) {
        self.reset_raw()
    }
    fn process(&mut self, input: &[f32], output: &mut [f32]) {
        // the reference slices input[..output.len()] (panics if shorter)
        assert!(input.len() >= output.len(), "range end index {} out of range for slice of length {}",
                output.len(), input.len());
        check(unsafe {
            ffi::fftconv_twostage_process(self.h.as_ptr(), input.as_ptr(), output.as_mut_ptr(), output.len())
        })
    }
}

/// CrossfadeConvolver<FFTConvolver> (src/crossfade_convolver.rs:10-105): the
/// two inner convolvers and the raised-cosine mix run on the device.
impl Convolution for GpuCrossfadeConvolver {
    fn init(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self {
        Self::init_raw(response, max_block_size, max_response_length)
    }
    fn update(&mut self, response: &[f32]) {
        self.update_raw(response)
    }
    fn reset(&mut self) {
        self.reset_raw()
    }
    fn process(&mut self, input: &[f32], output: &mut [f32]) {
        check(unsafe {
            ffi::fftconv_crossfade_process(self.h.as_ptr(), input.as_ptr(), input.len(), output.as_mut_ptr(),
                                           output.len())
        })
    }
}

impl GpuCrossfadeConvolver {
    /// CrossfadeConvolver::new (src/crossfade_convolver.rs:20-43) around a GPU FFTConvolver.
    pub fn new(convolver: GpuFFTConvolver, max_response_length: usize, max_buffer_size: usize,
               crossfade_samples: usize) -> Self {
        let p = unsafe {
            ffi::fftconv_crossfade_new(convolver.h.as_ptr(), max_response_length, max_buffer_size,
                                       crossfade_samples)
        };
        Self { h: handle(p) }
    }
    /// src/crossfade_convolver.rs:85-92
    pub fn is_crossfading(&self) -> bool {
        unsafe { ffi::fftconv_crossfade_is_crossfading(self.h.as_ptr()) != 0 }
    }
}

/// CrossfadeConvolver<TwoStageFFTConvolver> (the reference's CrossfadeConvolver
/// is generic, src/crossfade_convolver.rs:11,45-49).  `update` reaches
/// TwoStageFFTConvolver::update's `todo!()` through the swap and panics the
/// same way; `process` needs input.len() == max_buffer_size <= the head block.
impl Convolution for GpuCrossfadeTwoStageConvolver {
    fn init(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self {
        Self::init_raw(response, max_block_size, max_response_length)
    }
    fn update(&mut self, response: &[f32]) {
        self.update_raw(response)
    }
    fn reset(&mut self) {
        self.reset_raw()
    }
    fn process(&mut self, input: &[f32], output: &mut [f32]) {
        check(unsafe {
            ffi::fftconv_crossfade_process(self.h.as_ptr(), input.as_ptr(), input.len(), output.as_mut_ptr(),
                                           output.len())
        })
    }
}

impl GpuCrossfadeTwoStageConvolver {
    /// CrossfadeConvolver::new (src/crossfade_convolver.rs:20-43) around a GPU TwoStageFFTConvolver.
    pub fn new(convolver: GpuTwoStageFFTConvolver, max_response_length: usize, max_buffer_size: usize,
               crossfade_samples: usize) -> Self {
        let p = unsafe {
            ffi::fftconv_crossfade_new_twostage(convolver.h.as_ptr(), max_response_length, max_buffer_size,
                                                crossfade_samples)
        };
        Self { h: handle(p) }
    }
    /// src/crossfade_convolver.rs:85-92
    pub fn is_crossfading(&self) -> bool {
        unsafe { ffi::fftconv_crossfade_is_crossfading(self.h.as_ptr()) != 0 }
    }
}

/// A batch of independent FFTConvolver channels on one GPU (the throughput
/// path): responses and blocks are channel-major, device pointers are HBM
/// resident, work is queued on `stream` (a hipStream_t, null = HIP's null stream).
pub struct GpuFFTConvolverBatch {
    h: NonNull<ffi::fftconv_uniform>,
}
unsafe impl Send for GpuFFTConvolverBatch {}
impl Drop for GpuFFTConvolverBatch {
    fn drop(&mut self) {
        unsafe { ffi::fftconv_uniform_destroy(self.h.as_ptr()) }
    }
}
impl GpuFFTConvolverBatch {
    pub fn init(device: i32, channels: usize, responses: &[f32], response_len: usize, max_block_size: usize,
                max_response_length: usize) -> Self {
        assert!(responses.len() >= channels * response_len);
        let p = unsafe {
            ffi::fftconv_uniform_init_batch(device, channels, responses.as_ptr(), response_len, response_len,
                                            max_block_size, max_response_length)
        };
        Self { h: handle(p) }
    }
    /// One process() call of `len` samples on every channel; `d_input` /
    /// `d_output` are device pointers with the given channel strides.
    ///
    /// # Safety
    /// The pointers must address `channels` rows of `len` floats on the batch's device.
    pub unsafe fn process_device(&mut self, d_input: *const f32, in_stride: usize, d_output: *mut f32,
                                 out_stride: usize, len: usize, stream: *mut c_void) {
        check(unsafe {
            ffi::fftconv_uniform_process_device(self.h.as_ptr(), d_input, in_stride, d_output, out_stride, len,
                                                stream)
        })
    }
    pub fn synchronize(&mut self) {
        check(unsafe { ffi::fftconv_uniform_synchronize(self.h.as_ptr()) })
    }
    pub fn channels(&self) -> usize {
        unsafe { ffi::fftconv_uniform_channels(self.h.as_ptr()) }
    }
}

/// Fft (src/fft_convolver.rs:7-50): realfft's R2C / C2R of length n on the
/// GPU.  n is any length in 1..2^21, or a power of two up to 2^23 (the library
/// returns FFTCONV_E_UNSUPPORTED, and this panics, otherwise).  A power of two
/// runs the convolver's own transforms, so its spectrum is bit-identical to
/// the row a handle holds; any other length runs Bluestein's chirp-z
/// transform (within f32 rounding of an f64 DFT, not bit-identical to a
/// convolver kernel).
#[derive(Clone, Default, Debug)]
pub struct GpuFft {
    n: usize,
    device: i32,
}
impl GpuFft {
    /// Fft::init (:30-34); the device tables are built on first use
    pub fn init(&mut self, length: usize) {
        self.n = length;
    }
    /// Fft::forward (:36-39): n reals -> n/2 + 1 bins, unnormalised
    pub fn forward(&self, input: &mut [f32], output: &mut [Complex<f32>]) -> Result<(), FftError> {
        assert!(input.len() == self.n && output.len() == self.n / 2 + 1, "Fft::forward: slice lengths");
        check(unsafe {
            ffi::fftconv_fft_forward_host(self.device, self.n, 1, input.as_ptr(), output.as_mut_ptr() as *mut f32)
        });
        Ok(())
    }
    /// Fft::inverse (:41-49): n/2 + 1 bins -> n reals / n; a non-zero DC /
    /// Nyquist imaginary part is realfft's FftError::InputValues, returned
    /// before the normalisation (the row then stays unscaled, as :42 returns)
    pub fn inverse(&self, input: &mut [Complex<f32>], output: &mut [f32]) -> Result<(), FftError> {
        assert!(output.len() == self.n && input.len() == self.n / 2 + 1, "Fft::inverse: slice lengths");
        let mut bad: c_int = 0;
        check(unsafe {
            ffi::fftconv_fft_inverse_host(self.device, self.n, 1, input.as_ptr() as *const f32, output.as_mut_ptr(),
                                          &mut bad)
        });
        if bad != 0 {
            // realfft's odd-length C2R checks the DC bin only: input[n/2] is
            // then an ordinary bin, so its flag is false
            return Err(FftError::InputValues(input[0].im != 0.0,
                                             self.n % 2 == 0 && input[self.n / 2].im != 0.0));
        }
        Ok(())
    }
}
