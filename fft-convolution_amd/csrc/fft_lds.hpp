// fft_lds.hpp -- workgroup-cooperative real FFT of length N = 2B on gfx950.
//
// Replaces the reference's Fft wrapper (src/fft_convolver.rs:1-50), which
// delegates to realfft/rustfft on the CPU.  The transform is the same
// algorithm realfft publishes for even lengths: pack the N real samples as
// M = N/2 complex points z[n] = x[2n] + i x[2n+1], run an M-point complex
// FFT, then separate the even/odd spectra with one post-twiddle pass.
//
// GPU layout decisions:
//  * the complex FFT is a self-sorting Stockham transform in LDS (ping-pong
//    buffers, one barrier per stage), radix-4 stages plus a final radix-2
//    stage when log2(M) is odd; stage indices are compile-time constants so
//    every address is a shift/mask;
//  * spectra are stored *packed*: B complex slots, slot 0 holds
//    (DC.re, Nyquist.re).  The DC and Nyquist bins of a real signal are real,
//    so the reference's B+1 bins carry exactly the same information and a
//    row becomes a power of two (2 KB at B = 256) -- aligned float4 streams;
//  * twiddles come from a table W_N^k = exp(-2 pi i k / N), k < N, computed
//    on the host in double precision and rounded to f32 (the accuracy
//    rustfft's compute_twiddle gives).
#pragma once
#include <hip/hip_runtime.h>

namespace fftconv {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// Complex products with explicit fused multiply-adds.  The kernels are built
// with -ffp-contract=off, so every rounding is spelled out here and every
// instantiation (load policy, block size, shard size) computes the same bits.
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(w)
__device__ __forceinline__ float2 cmulc(float2 a, float2 w) {
    return make_float2(fmaf(a.x, w.x, a.y * w.y), fmaf(a.y, w.x, -(a.x * w.y)));
}
template <bool INV>
__device__ __forceinline__ float2 twmul(float2 a, float2 w) { return INV ? cmulc(a, w) : cmul(a, w); }

// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) { return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x); }

// Wave-local LDS ordering point: one wave's LDS writes are visible to all its
// lanes' later reads (DS ops of a wave execute in order; the wait and the
// compiler barrier keep the reads behind the writes).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool WAVE>
__device__ __forceinline__ void stage_sync() {
    if constexpr (WAVE) wave_sync();
    else __syncthreads();
}

// M-point complex FFT (M = 2^LOG2M) over LDS, executed by NT threads.
// Input in buf0; returns the buffer that holds the naturally ordered result
// (buf0 or buf1).  INV = unnormalised inverse (conjugate twiddles).
// `tw` is the W_N table with N = 2M.  Every thread of the block must call it
// (WAVE: a single wave -- NT = 64, any wave of the block -- calls it,
// synchronising at wave level).
template <int LOG2M, int NT, bool INV, bool WAVE = false>
__device__ __forceinline__ float2 *lds_cfft(float2 *buf0, float2 *buf1, const float2 *__restrict__ tw) {
    constexpr int M = 1 << LOG2M;
    constexpr int N = 2 * M;
    constexpr int R4 = LOG2M / 2;
    float2 *src = buf0;
    float2 *dst = buf1;
    const int tid = WAVE ? (int)(threadIdx.x & (NT - 1)) : (int)threadIdx.x;  // WAVE: any one wave
#pragma unroll
    for (int s = 0; s < R4; ++s) {
        const int Ns = 1 << (2 * s);        // sub-transform length so far
        const int step = N / (Ns * 4);      // table stride for this stage
        for (int j = tid; j < M / 4; j += NT) {
            const int k = j & (Ns - 1);
            float2 v0 = src[j];
            float2 v1 = src[j + M / 4];
            float2 v2 = src[j + M / 2];
            float2 v3 = src[j + 3 * M / 4];
            if (s > 0) {
                v1 = twmul<INV>(v1, tw[k * step]);
                v2 = twmul<INV>(v2, tw[2 * k * step]);
                v3 = twmul<INV>(v3, tw[3 * k * step]);
            }
            const float2 a02 = cadd(v0, v2), s02 = csub(v0, v2);
            const float2 a13 = cadd(v1, v3), s13 = mul_mi<INV>(csub(v1, v3));
            const int base = (j - k) * 4 + k;
            dst[base] = cadd(a02, a13);
            dst[base + Ns] = cadd(s02, s13);
            dst[base + 2 * Ns] = csub(a02, a13);
            dst[base + 3 * Ns] = csub(s02, s13);
        }
        stage_sync<WAVE>();
        float2 *t = src; src = dst; dst = t;
    }
    if constexpr ((LOG2M & 1) != 0) {
        constexpr int Ns = M / 2;
        constexpr int step = N / (Ns * 2);  // = 2
        for (int j = tid; j < M / 2; j += NT) {
            const int k = j & (Ns - 1);
            float2 v0 = src[j];
            float2 v1 = src[j + M / 2];
            if constexpr (Ns > 1) v1 = twmul<INV>(v1, tw[k * step]);
            const int base = (j - k) * 2 + k;
            dst[base] = cadd(v0, v1);
            dst[base + Ns] = csub(v0, v1);
        }
        stage_sync<WAVE>();
        float2 *t = src; src = dst; dst = t;
    }
    return src;
}

// Post-twiddle: packed real spectrum from the complex FFT Z of the packed
// samples (realfft's RealToComplexEven post-processing).  Writes
// spec[0] = (DC, Nyquist), spec[k] = X[k] for 1 <= k < M.  Caller syncs.
template <int LOG2M, int NT>
__device__ __forceinline__ float2 real_post(const float2 *Z, int k, const float2 *__restrict__ tw) {
    constexpr int M = 1 << LOG2M;
    const float2 a = Z[k];
    if (k == 0) return make_float2(a.x + a.y, a.x - a.y);
    const float2 zb = Z[M - k];
    const float2 b = make_float2(zb.x, -zb.y);
    const float2 e = make_float2((a.x + b.x) * 0.5f, (a.y + b.y) * 0.5f);
    const float2 o = make_float2((a.y - b.y) * 0.5f, -(a.x - b.x) * 0.5f);
    return cadd(e, cmul(tw[k], o));
}

// Pre-twiddle for the C2R: from a packed spectrum to the M complex points
// whose inverse FFT interleaves the even/odd output samples.
template <int LOG2M, int NT>
__device__ __forceinline__ float2 real_pre(const float2 *X, int k, const float2 *__restrict__ tw) {
    constexpr int M = 1 << LOG2M;
    const float2 a = X[k];
    if (k == 0) return make_float2(a.x + a.y, a.x - a.y);
    const float2 xb = X[M - k];
    const float2 b = make_float2(xb.x, -xb.y);
    const float2 e = cadd(a, b);
    const float2 o = cmulc(csub(a, b), tw[k]);
    return make_float2(e.x - o.y, e.y + o.x);
}

}  // namespace fftconv
