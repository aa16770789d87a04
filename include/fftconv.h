/*
 * fftconv.h -- C ABI of the MI355X-native partitioned FFT convolver.
 *
 * Drop-in boundary for Sin-tel/fft-convolution's `Convolution` trait
 * (src/lib.rs:5-14):
 *
 *     trait Convolution: Clone {
 *         fn init(response: &[f32], max_block_size: usize, max_response_length: usize) -> Self;
 *         fn update(&mut self, response: &[f32]);          // real-time safe
 *         fn reset(&mut self);
 *         fn process(&mut self, input: &[f32], output: &mut [f32]);
 *     }
 *
 * Every handle is a *batch* of `channels` independent convolvers that share
 * one geometry (block size, max response length) and live on one GPU.  A
 * handle created by the single-channel `*_init` entry point is a batch of 1
 * and is the exact counterpart of one reference instance.  Batched host
 * buffers are laid out channel-major: sample j of channel c at [c*len + j]
 * (or [c*stride + j] where a stride is taken).
 *
 * Errors: where the reference panics (assert!/panic!/todo!/slice bounds) the
 * call returns a negative status and leaves the instance unchanged; the
 * message is available from fftconv_last_error().  A runtime FFT error
 * (realfft's C2R rejecting a non-finite DC/Nyquist bin) zero-fills that
 * channel's output and leaves its block state where the reference leaves it
 * (src/fft_convolver.rs:264-267); it is not an error status.
 *
 * There is no CPU fallback: creating a handle without a usable gfx950 device
 * fails with FFTCONV_E_DEVICE.
 *
 * Streams: every `void *hip_stream` argument is a hipStream_t, and NULL is
 * HIP's null (legacy default) stream -- the same meaning it has in every HIP
 * API and the stream PyTorch's default stream maps to.  A call enqueued on a
 * stream is ordered after the handle's previous work wherever that ran (one
 * event wait when the stream differs from the last one used), and anything
 * enqueued on the same stream afterwards sees its results.  Host-synchronous
 * entry points use the handle's own (non-blocking) stream and wait for it;
 * *_synchronize waits for all of a handle's work.
 */
#ifndef FFTCONV_H
#define FFTCONV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFTCONV_ABI_VERSION 1

enum {
    FFTCONV_OK = 0,
    FFTCONV_E_INVALID = -1,       /* a reference panic!/assert!/slice-bounds precondition */
    FFTCONV_E_UNIMPLEMENTED = -2, /* a reference todo!() */
    FFTCONV_E_UNSUPPORTED = -3,   /* geometry outside this build (block size > 2^22) */
    FFTCONV_E_DEVICE = -4,        /* HIP runtime error / no device */
    FFTCONV_E_NOMEM = -5
};

typedef struct fftconv_uniform fftconv_uniform;     /* FFTConvolver        src/fft_convolver.rs:86-307 */
typedef struct fftconv_twostage fftconv_twostage;   /* TwoStageFFTConvolver src/fft_convolver.rs:323-512 */
typedef struct fftconv_crossfade fftconv_crossfade; /* CrossfadeConvolver<FFTConvolver | TwoStageFFTConvolver> src/crossfade_convolver.rs:10-105 */

/* ---- library ----------------------------------------------------------- */
int fftconv_abi_version(void);
const char *fftconv_last_error(void);            /* thread-local, "" if none */
int fftconv_device_count(void);                   /* visible HIP devices, 0 if none */
size_t fftconv_complex_size(size_t size);         /* src/fft_convolver.rs:52-54 */
size_t fftconv_compute_tail_block_size(size_t head_len, size_t response_len); /* :520-526 */

/* ---- Fft (src/fft_convolver.rs:7-50) ----------------------------------- */
/* The reference's public real FFT (realfft's RealToComplex / ComplexToReal of
 * length n; Fft::init takes any usize, :30-34) as batched device transforms.
 * n: any length in 1..2^21, or a power of two up to 2^23.
 *   - A power of two runs the convolver's own kernels (n > 16384: the
 *     four-step passes of the long-block path), so a spectrum here is
 *     bit-identical to the convolver's.
 *   - Any other length runs Bluestein's chirp-z transform over power-of-two
 *     FFTs of P >= 2n-1 points (its tables are cached per length, at most
 *     256 MiB of device memory, least recently used first out).  Those
 *     spectra are within f32 rounding of an f64 DFT, not bit-identical to any
 *     convolver kernel (the convolver's block sizes are powers of two).
 * A row of bins is 2*(n/2+1) floats: n+2 for even n, n+1 for odd n.
 * Forward (Fft::forward :36-39): rows of n reals -> n/2+1 bins,
 * interleaved (re, im), unnormalised, DC (and, for even n, Nyquist)
 * imaginary parts 0.
 * Inverse (Fft::inverse :41-49): n/2+1 bins -> n reals divided by n;
 * d_status[row] (optional) = 1 where realfft returns FftError::InputValues
 * (non-zero DC imaginary part, or for even n a non-zero Nyquist imaginary
 * part; the transform runs with those parts as 0).  Such a row is NOT divided
 * by n: Fft::inverse returns the error through `?` (:42) before its
 * normalisation loop (:44-46).  Strides in floats; enqueued on `hip_stream`
 * (NULL = HIP's null stream). */
int fftconv_fft_forward(int device, size_t n, size_t rows, const float *d_in, size_t in_stride, float *d_out,
                        size_t out_stride, void *hip_stream);
int fftconv_fft_inverse(int device, size_t n, size_t rows, const float *d_in, size_t in_stride, float *d_out,
                        size_t out_stride, int *d_status, void *hip_stream);
/* Host-memory forms, rows packed ([rows][n] reals, [rows][2*(n/2+1)] bin floats);
 * synchronous (temporary device buffers: not for the real-time path). */
int fftconv_fft_forward_host(int device, size_t n, size_t rows, const float *input, float *output);
int fftconv_fft_inverse_host(int device, size_t n, size_t rows, const float *input, float *output, int *status);
/* Tuning knob (process-wide): spectral-MAC scan variant of the fused kernel,
 * -1 = automatic (default: nontemporal loads when the per-step H+X stream
 * exceeds the Infinity Cache, plain loads otherwise -- the load policy never
 * changes a result bit; the pipelined full-block step when B <= 512 and a
 * channel's FDL holds <= 16384 bins, chosen per geometry, never by channel
 * count, so channel shards stay bit-identical; for a CrossfadeConvolver
 * with a longer FDL, one workgroup runs A and B on one FDL stream, which
 * never changes a result bit),
 * else bit 0 = zig-zag segment order on alternate blocks, bit 1 =
 * nontemporal H/X loads, bit 2 = no pipelined step (every call computes
 * its pre_multiplied at block start, as the reference does) -- when none
 * of bits 0-2 is set, the automatic load and step policy stays --, bit 3 = no
 * crossfade pair launch (A and B stream the shared FDL separately), bit 4 =
 * no lookahead step (see below), bit 5 = lookahead launches without anchors
 * (every full block sums all its FDL rows itself; bit-identical to the
 * lookahead path, for tests), bit 6 = crossfade on the lookahead step with
 * the stand-alone mix kernel (by default B's launch mixes in its epilogue,
 * from gains A's launch precomputed; bit-identical either way), bit 7 = IR
 * transforms (init / update) one segment per workgroup (by default one per
 * wave for 64 <= B <= 1024; bit-identical), bit 8 = two-stage tail0 runs
 * per head block (by default its blocks are convolved together at the end
 * of each tail period; read when a TwoStageFFTConvolver is created), bit 9 =
 * that end-of-period flush in one fused kernel instead of five (head block
 * 64; bit-identical), bit 10 = no far-row windows for B >= 1024 (every
 * one-block call sums its far rows itself; bit-identical), bit 11 =
 * process_device_steps launches once per call (by default, for 64 <= B <= 512,
 * a TwoStageFFTConvolver's aligned calls inside one tail period, and the
 * calls of an FFTConvolver batch on the generic / pipelined step with at most
 * two channels per CU, run as ONE launch in which each channel's workgroup
 * loops over its calls; bit-identical).
 * Lookahead (automatic for standalone FFTConvolver batches with
 * 128 <= B <= 512 and >= 40 segments, full-block calls from an empty input
 * buffer): the FDL sum of each block is re-associated in time over a near
 * level and three anchor levels with geometric periods -- the step sums
 * rows 1..4 itself, an anchor every 4 blocks sums rows 5..16 for the next 4
 * blocks, one every 16 blocks rows 17..64 for the next 16, one every 64
 * blocks rows >= 65 for the next 64 -- so a full-block call streams ~1/10
 * of the reference's bytes; its summation order does not depend on the
 * channel index, the shard or the call history (bit-identical to summing
 * every row).
 * -1 selects automatic; any other negative value is FFTCONV_E_INVALID.
 * Results agree within f32 rounding across variants. */
int fftconv_set_kernel_variant(int variant);
int fftconv_get_kernel_variant(void);
/* Tuning knob (process-wide): FDL rows the pipelined step leaves to its
 * stream waves while its first wave runs the transform chain; -1 = automatic
 * (all of them: the first wave never streams).  Does not change results beyond
 * f32 summation order. */
int fftconv_set_pipeline_lag(int rows);
int fftconv_get_pipeline_lag(void);
/* Pinned host staging of update() (process-wide, read when a handle is
 * created).  A standalone FFTConvolver batch, and a crossfade, reserve
 * channels x max_response_length floats of pinned host memory at init, so
 * update() copies the response and returns without waiting for the upload
 * (src/lib.rs:8 asks update to be real-time safe: it never allocates).  A cap
 * in bytes (0 = none, the default) -- or a reservation the host refuses, which
 * falls back to smaller ones down to one response row -- makes update() stream
 * the rows through the stage in chunks, waiting for each chunk's copy before
 * refilling it: no allocation either way, same results. */
int fftconv_set_host_stage_limit(size_t bytes);
size_t fftconv_get_host_stage_limit(void);

/* ---- FFTConvolver (uniformly partitioned, zero latency) ---------------- */
/* FFTConvolver::init, src/fft_convolver.rs:105-172.  NULL on error. */
fftconv_uniform *fftconv_uniform_init(const float *response, size_t response_len,
                                      size_t max_block_size, size_t max_response_length);
/* Batched init on `device`: channel c's response is responses[c*response_stride ..
 * + response_len] (host memory). */
fftconv_uniform *fftconv_uniform_init_batch(int device, size_t channels, const float *responses,
                                            size_t response_len, size_t response_stride,
                                            size_t max_block_size, size_t max_response_length);
/* FFTConvolver::update, src/fft_convolver.rs:174-213; every channel gets the
 * same response.  No allocation (staging is reserved at init). */
int fftconv_uniform_update(fftconv_uniform *h, const float *response, size_t response_len);
/* Per-channel responses, host memory, channel c at responses[c*stride ..]. */
int fftconv_uniform_update_batch(fftconv_uniform *h, const float *responses, size_t response_len,
                                 size_t response_stride);
/* One channel only. */
int fftconv_uniform_update_channel(fftconv_uniform *h, size_t channel, const float *response,
                                   size_t response_len);
/* update() from device-resident responses (channel c at d_responses[c*stride],
 * stride 0 = one response for every channel), enqueued on `hip_stream`
 * (NULL = HIP's null stream) without a host synchronisation or an allocation. */
int fftconv_uniform_update_device(fftconv_uniform *h, const float *d_responses, size_t response_len,
                                  size_t response_stride, void *hip_stream);
/* FFTConvolver::reset, src/fft_convolver.rs:296-306 (all channels). */
int fftconv_uniform_reset(fftconv_uniform *h);
/* FFTConvolver::process, src/fft_convolver.rs:215-295, host buffers:
 * input [channels][input_len], output [channels][output_len]; reads
 * input[0..output_len] of each channel (input_len >= output_len, else
 * FFTCONV_E_INVALID like the reference's slice panic).  Synchronous. */
int fftconv_uniform_process(fftconv_uniform *h, const float *input, size_t input_len,
                            float *output, size_t output_len);
/* Same on device-resident buffers, enqueued on `hip_stream` (NULL = HIP's
 * null stream), asynchronous: channel c reads d_input[c*in_stride ..
 * + len] and writes d_output[c*out_stride .. + len]. */
int fftconv_uniform_process_device(fftconv_uniform *h, const float *d_input, size_t in_stride,
                                   float *d_output, size_t out_stride, size_t len, void *hip_stream);
/* `steps` consecutive process() calls of `len` samples each, from one host
 * call: call k reads d_input + k*in_step (channel stride in_stride) and writes
 * d_output + k*out_step.  Identical to `steps` calls of _process_device; it
 * removes the per-call host overhead when blocks are already resident. */
int fftconv_uniform_process_device_steps(fftconv_uniform *h, const float *d_input, size_t in_stride,
                                         size_t in_step, float *d_output, size_t out_stride,
                                         size_t out_step, size_t len, size_t steps, void *hip_stream);
/* #[derive(Clone)]: a deep, device-side copy of every buffer and scalar. */
fftconv_uniform *fftconv_uniform_clone(const fftconv_uniform *h);
void fftconv_uniform_destroy(fftconv_uniform *h);
int fftconv_uniform_synchronize(fftconv_uniform *h);
size_t fftconv_uniform_channels(const fftconv_uniform *h);
/* anchor workgroups per channel of the lookahead step, 0 = not used */
int fftconv_uniform_lookahead_parts(const fftconv_uniform *h);
/* window rows per channel of the generic step's far-row windows (automatic
 * for standalone batches with B >= 1024 and >= 24 segments: an
 * anchor every P blocks sums rows >= P for a channel's next P one-block
 * calls; bit-identical to summing them every block), 0 = not used */
int fftconv_uniform_far_windows(const fftconv_uniform *h);
/* (tests) with FFTCONV_LA_PROBE=1 in the environment when the handle was
 * created, the lookahead launches make their anchors wait for the steps and
 * read the live state words, which they do not compute from (they use the
 * launch-start copies, la.hpp la_anchor_state): the number of live words
 * found already rewritten by the same launch so far; -1 when the probe is
 * off (the default) */
int fftconv_uniform_lookahead_probe(const fftconv_uniform *h);
size_t fftconv_uniform_block_size(const fftconv_uniform *h);   /* next_power_of_two(max_block_size) */
size_t fftconv_uniform_seg_count(const fftconv_uniform *h);
/* segments_ir[segment] of one channel (src/fft_convolver.rs:92): B+1 bins,
 * interleaved (re, im), into host `out` ((B+1)*2 floats) */
int fftconv_uniform_ir_spectrum(const fftconv_uniform *h, size_t channel, size_t segment, float *out);
/* copies {current, active_seg_count, input_buffer_fill} of one channel */
int fftconv_uniform_channel_state(const fftconv_uniform *h, size_t channel, size_t out3[3]);

/* ---- TwoStageFFTConvolver (head block + García-optimal tail block) ----- */
fftconv_twostage *fftconv_twostage_init(const float *response, size_t response_len,
                                        size_t max_block_size, size_t max_response_length);
fftconv_twostage *fftconv_twostage_init_batch(int device, size_t channels, const float *responses,
                                              size_t response_len, size_t response_stride,
                                              size_t max_block_size, size_t max_response_length);
/* todo!() in the reference (src/fft_convolver.rs:408-410): FFTCONV_E_UNIMPLEMENTED. */
int fftconv_twostage_update(fftconv_twostage *h, const float *response, size_t response_len);
int fftconv_twostage_reset(fftconv_twostage *h);
/* len must be <= max_block_size (assert at src/fft_convolver.rs:414); input and
 * output both [channels][len]. */
int fftconv_twostage_process(fftconv_twostage *h, const float *input, float *output, size_t len);
int fftconv_twostage_process_device(fftconv_twostage *h, const float *d_input, size_t in_stride,
                                    float *d_output, size_t out_stride, size_t len, void *hip_stream);
int fftconv_twostage_process_device_steps(fftconv_twostage *h, const float *d_input, size_t in_stride,
                                          size_t in_step, float *d_output, size_t out_stride,
                                          size_t out_step, size_t len, size_t steps, void *hip_stream);
fftconv_twostage *fftconv_twostage_clone(const fftconv_twostage *h);
void fftconv_twostage_destroy(fftconv_twostage *h);
int fftconv_twostage_synchronize(fftconv_twostage *h);
size_t fftconv_twostage_tail_block_size(const fftconv_twostage *h);

/* ---- CrossfadeConvolver<FFTConvolver> ---------------------------------- */
/* Convolution::init, src/crossfade_convolver.rs:46-49: crossfade_samples =
 * response_len, hold = min(max_block_size, response_len). */
fftconv_crossfade *fftconv_crossfade_init(const float *response, size_t response_len,
                                          size_t max_block_size, size_t max_response_length);
fftconv_crossfade *fftconv_crossfade_init_batch(int device, size_t channels, const float *responses,
                                                size_t response_len, size_t response_stride,
                                                size_t max_block_size, size_t max_response_length);
/* CrossfadeConvolver::new, src/crossfade_convolver.rs:19-43.  `convolver` is
 * cloned (the reference moves it; the caller keeps ownership of its handle). */
fftconv_crossfade *fftconv_crossfade_new(const fftconv_uniform *convolver, size_t max_response_length,
                                         size_t max_buffer_size, size_t crossfade_samples);
/* CrossfadeConvolver<TwoStageFFTConvolver> (the reference's CrossfadeConvolver
 * is generic over `Convolution`, src/crossfade_convolver.rs:11,45-49): the same
 * handle type and the same functions below.  Its update() reaches
 * TwoStageFFTConvolver::update, todo!() (src/fft_convolver.rs:408-410), before
 * anything changes: FFTCONV_E_UNIMPLEMENTED and the handle is unchanged.
 * process() needs input_len == max_buffer_size <= the inner head block size
 * (:412-414 and the head / tail slice bounds). */
fftconv_crossfade *fftconv_crossfade_init_twostage(const float *response, size_t response_len,
                                                   size_t max_block_size, size_t max_response_length);
fftconv_crossfade *fftconv_crossfade_init_twostage_batch(int device, size_t channels, const float *responses,
                                                         size_t response_len, size_t response_stride,
                                                         size_t max_block_size, size_t max_response_length);
fftconv_crossfade *fftconv_crossfade_new_twostage(const fftconv_twostage *convolver, size_t max_response_length,
                                                  size_t max_buffer_size, size_t crossfade_samples);
/* src/crossfade_convolver.rs:51-64; same response for every channel. */
int fftconv_crossfade_update(fftconv_crossfade *h, const float *response, size_t response_len);
int fftconv_crossfade_update_batch(fftconv_crossfade *h, const float *responses, size_t response_len,
                                   size_t response_stride);
/* update() from device-resident responses, stream-ordered (see uniform). */
int fftconv_crossfade_update_device(fftconv_crossfade *h, const float *d_responses, size_t response_len,
                                    size_t response_stride, void *hip_stream);
/* todo!() in the reference (src/crossfade_convolver.rs:80-82): FFTCONV_E_UNIMPLEMENTED. */
int fftconv_crossfade_reset(fftconv_crossfade *h);
/* src/crossfade_convolver.rs:66-78: input_len >= max_buffer_size and
 * output_len <= max_buffer_size (the reference's slice bounds). */
int fftconv_crossfade_process(fftconv_crossfade *h, const float *input, size_t input_len,
                              float *output, size_t output_len);
int fftconv_crossfade_process_device(fftconv_crossfade *h, const float *d_input, size_t in_stride,
                                     float *d_output, size_t out_stride, size_t output_len,
                                     void *hip_stream);
int fftconv_crossfade_process_device_steps(fftconv_crossfade *h, const float *d_input, size_t in_stride,
                                           size_t in_step, float *d_output, size_t out_stride,
                                           size_t out_step, size_t output_len, size_t steps,
                                           void *hip_stream);
int fftconv_crossfade_is_crossfading(const fftconv_crossfade *h); /* :85-92, 1/0 */
fftconv_crossfade *fftconv_crossfade_clone(const fftconv_crossfade *h);
void fftconv_crossfade_destroy(fftconv_crossfade *h);
int fftconv_crossfade_synchronize(fftconv_crossfade *h);

#ifdef __cplusplus
}
#endif

#endif /* FFTCONV_H */
