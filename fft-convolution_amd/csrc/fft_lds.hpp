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

// Twiddle sources.  A stage reads W_N^(m k step) (m = 1..3); with the full
// W_N table (`const float2 *`) the lanes of a wave read it at stride m step,
// which piles the middle stages' reads on a few LDS banks.  TwStaged is the
// same values regathered per stage -- [post: W^k, k < M][stage 1..R4-1: three
// rows of Ns, row m-1 holding W^(m k step)][radix-2 stage: W^(2k), k < M/2]
// (2M - 4 entries, it fits the full table's 2M) -- so every stage reads
// consecutive entries.  Same f32 values, so the same bits either way.
template <int LOG2M>
struct TwStaged {
    const float2 *t;
};
template <int LOG2M>
constexpr int tws_off4(int S) { return (1 << LOG2M) + (1 << (2 * S)) - 4; }  // M + sum_{s=1}^{S-1} 3 4^s
template <int LOG2M>
constexpr int tws_off2() { return tws_off4<LOG2M>(LOG2M / 2); }
template <int LOG2M>
constexpr int tws_size() { return tws_off2<LOG2M>() + ((LOG2M & 1) ? (1 << LOG2M) / 2 : 0); }
template <int LOG2M, int S>
__device__ __forceinline__ float2 tw_r4(const float2 *__restrict__ tw, int m, int k) {
    constexpr int N = 2 << LOG2M;
    constexpr int step = N / ((1 << (2 * S)) * 4);
    return tw[m * k * step];
}
template <int LOG2M, int S>
__device__ __forceinline__ float2 tw_r4(TwStaged<LOG2M> tw, int m, int k) {
    return tw.t[tws_off4<LOG2M>(S) + (m - 1) * (1 << (2 * S)) + k];
}
template <int LOG2M>
__device__ __forceinline__ float2 tw_r2(const float2 *__restrict__ tw, int k) { return tw[2 * k]; }
template <int LOG2M>
__device__ __forceinline__ float2 tw_r2(TwStaged<LOG2M> tw, int k) { return tw.t[tws_off2<LOG2M>() + k]; }
__device__ __forceinline__ float2 tw_post(const float2 *__restrict__ tw, int k) { return tw[k]; }
template <int LOG2M>
__device__ __forceinline__ float2 tw_post(TwStaged<LOG2M> tw, int k) { return tw.t[k]; }
// Gather the staged table (tws_size entries) from the full W_N table, by NT
// threads; caller syncs.
template <int LOG2M, int NT>
__device__ __forceinline__ void tws_build(float2 *dst, const float2 *__restrict__ tw, int tid) {
    constexpr int M = 1 << LOG2M;
    constexpr int N = 2 * M;
    for (int e = tid; e < tws_size<LOG2M>(); e += NT) {
        int src;
        if (e < M) {
            src = e;
        } else if (e >= tws_off2<LOG2M>()) {
            src = 2 * (e - tws_off2<LOG2M>());
        } else {
            int S = 1;
            while (e >= tws_off4<LOG2M>(S + 1)) ++S;
            const int Ns = 1 << (2 * S), r = e - tws_off4<LOG2M>(S);
            src = (r / Ns + 1) * (r % Ns) * (N / (Ns * 4));
        }
        dst[e] = tw[src];
    }
}

// One radix-4 Stockham stage s (sub-transform length Ns = 4^s so far) of an
// M-point complex FFT over LDS, by NT threads; `tw` is the W_N table, N = 2M.
// The four outputs of butterfly j go to base + q Ns.  For Ns < 16 the 16
// lanes of a ds_write_b64 group would hit 4 bank pairs (writes at stride 4
// Ns float2); each lane therefore stores its outputs in the order
// q = (r + j/4) mod 4, r = 0..3, which spreads every store instruction over
// all 16 bank pairs.  Only the store order changes, not a value.
template <int LOG2M, int NT, bool INV, int S, class TW>
__device__ __forceinline__ void fft_stage_r4(const float2 *src, float2 *dst, TW tw, int tid) {
    constexpr int M = 1 << LOG2M;
    constexpr int Ns = 1 << (2 * S);      // sub-transform length so far
    for (int j = tid; j < M / 4; j += NT) {
        const int k = j & (Ns - 1);
        float2 v0 = src[j];
        float2 v1 = src[j + M / 4];
        float2 v2 = src[j + M / 2];
        float2 v3 = src[j + 3 * M / 4];
        if constexpr (S > 0) {
            v1 = twmul<INV>(v1, tw_r4<LOG2M, S>(tw, 1, k));
            v2 = twmul<INV>(v2, tw_r4<LOG2M, S>(tw, 2, k));
            v3 = twmul<INV>(v3, tw_r4<LOG2M, S>(tw, 3, k));
        }
        const float2 a02 = cadd(v0, v2), s02 = csub(v0, v2);
        const float2 a13 = cadd(v1, v3), s13 = mul_mi<INV>(csub(v1, v3));
        const float2 o0 = cadd(a02, a13), o1 = cadd(s02, s13), o2 = csub(a02, a13), o3 = csub(s02, s13);
        const int base = (j - k) * 4 + k;
        if constexpr (Ns < 16) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int q = (r + (j >> 2)) & 3;
                dst[base + q * Ns] = q == 0 ? o0 : (q == 1 ? o1 : (q == 2 ? o2 : o3));
            }
        } else {
            dst[base] = o0;
            dst[base + Ns] = o1;
            dst[base + 2 * Ns] = o2;
            dst[base + 3 * Ns] = o3;
        }
    }
}
// The final radix-2 stage when log2(M) is odd (Ns = M/2).
template <int LOG2M, int NT, bool INV, class TW>
__device__ __forceinline__ void fft_stage_r2(const float2 *src, float2 *dst, TW tw, int tid) {
    constexpr int M = 1 << LOG2M;
    constexpr int Ns = M / 2;
    for (int j = tid; j < M / 2; j += NT) {
        const int k = j & (Ns - 1);
        float2 v0 = src[j];
        float2 v1 = src[j + M / 2];
        if constexpr (Ns > 1) v1 = twmul<INV>(v1, tw_r2<LOG2M>(tw, k));  // (W^(2k))
        const int base = (j - k) * 2 + k;
        dst[base] = cadd(v0, v1);
        dst[base + Ns] = csub(v0, v1);
    }
}

// Stages [S0, S1) of the M-point FFT (radix-4 stages 0 .. R4-1, then the
// radix-2 stage R4 when log2(M) is odd), ping-ponging src -> dst; returns
// the buffer holding the result.
template <int LOG2M, int NT, bool INV, bool WAVE, int S0, int S1, class TW>
__device__ __forceinline__ float2 *fft_stages(float2 *src, float2 *dst, TW tw, int tid) {
    constexpr int R4 = LOG2M / 2;
    if constexpr (S0 >= S1) {
        return src;
    } else {
        if constexpr (S0 < R4) fft_stage_r4<LOG2M, NT, INV, S0>(src, dst, tw, tid);
        else fft_stage_r2<LOG2M, NT, INV>(src, dst, tw, tid);
        stage_sync<WAVE>();
        return fft_stages<LOG2M, NT, INV, WAVE, S0 + 1, S1, TW>(dst, src, tw, tid);
    }
}
template <int LOG2M>
constexpr int fft_nstages() { return LOG2M / 2 + (LOG2M & 1); }

// M-point complex FFT (M = 2^LOG2M) over LDS, executed by NT threads.
// Input in buf0; returns the buffer that holds the naturally ordered result
// (buf0 or buf1).  INV = unnormalised inverse (conjugate twiddles).
// `tw` is the W_N table with N = 2M.  Every thread of the block must call it
// (WAVE: a single wave -- NT = 64, any wave of the block -- calls it,
// synchronising at wave level).
template <int LOG2M, int NT, bool INV, bool WAVE = false, class TW = const float2 *>
__device__ __forceinline__ float2 *lds_cfft(float2 *buf0, float2 *buf1, TW tw) {
    const int tid = WAVE ? (int)(threadIdx.x & (NT - 1)) : (int)threadIdx.x;  // WAVE: any one wave
    return fft_stages<LOG2M, NT, INV, WAVE, 0, fft_nstages<LOG2M>()>(buf0, buf1, tw, tid);
}

// Post-twiddle: packed real spectrum from the complex FFT Z of the packed
// samples (realfft's RealToComplexEven post-processing).  Writes
// spec[0] = (DC, Nyquist), spec[k] = X[k] for 1 <= k < M.  Caller syncs.
template <int LOG2M, int NT, class TW = const float2 *>
__device__ __forceinline__ float2 real_post(const float2 *Z, int k, TW tw) {
    constexpr int M = 1 << LOG2M;
    const float2 a = Z[k];
    if (k == 0) return make_float2(a.x + a.y, a.x - a.y);
    const float2 zb = Z[M - k];
    const float2 b = make_float2(zb.x, -zb.y);
    const float2 e = make_float2((a.x + b.x) * 0.5f, (a.y + b.y) * 0.5f);
    const float2 o = make_float2((a.y - b.y) * 0.5f, -(a.x - b.x) * 0.5f);
    return cadd(e, cmul(tw_post(tw, k), o));
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

// ---------------------------------------------------------------------------
// Wave-level transforms of the step chain (one wave per transform, M >= 128):
// the ends of the R2C / C2R exchange data across the wavefront by __shfl
// instead of an LDS round trip.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float2 shfl2(float2 v, int src) {
    return make_float2(__shfl(v.x, src, 64), __shfl(v.y, src, 64));
}
// realfft's post-twiddle of bin k from Z[k] (a) and Z[M-k] (zb): real_post
template <class TW>
__device__ __forceinline__ float2 real_post_pair(float2 a, float2 zb, int k, TW tw) {
    if (k == 0) return make_float2(a.x + a.y, a.x - a.y);
    const float2 b = make_float2(zb.x, -zb.y);
    const float2 e = make_float2((a.x + b.x) * 0.5f, (a.y + b.y) * 0.5f);
    const float2 o = make_float2((a.y - b.y) * 0.5f, -(a.x - b.x) * 0.5f);
    return cadd(e, cmul(tw_post(tw, k), o));
}

// One wave's radix-4 stage S (or the final radix-2 stage) IN PLACE: each lane
// reads the inputs of all its butterflies into registers before any store
// (the stores depend on the loaded values, and a wave's LDS operations
// execute in order, so no lane overwrites an input another lane has yet to
// read).  Same butterflies, twiddles and store order as fft_stage_r4/_r2:
// the same bits, in half the LDS.
template <int LOG2M, int S, class TW>
__device__ __forceinline__ void wave_stage_inplace(float2 *buf, TW tw) {
    constexpr int M = 1 << LOG2M;
    constexpr int R4 = LOG2M / 2;
    const int lane = (int)(threadIdx.x & 63);
    if constexpr (S < R4) {
        constexpr int Ns = 1 << (2 * S);
        constexpr int NB = (M / 4 + 63) / 64;
        float2 v[NB][4];
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int j = lane + 64 * t;
            if (j < M / 4) {
                v[t][0] = buf[j];
                v[t][1] = buf[j + M / 4];
                v[t][2] = buf[j + M / 2];
                v[t][3] = buf[j + 3 * M / 4];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (no store moves above a load)
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int j = lane + 64 * t;
            if (j < M / 4) {
                const int k = j & (Ns - 1);
                float2 v1 = v[t][1], v2 = v[t][2], v3 = v[t][3];
                if constexpr (S > 0) {
                    v1 = twmul<false>(v1, tw_r4<LOG2M, S>(tw, 1, k));
                    v2 = twmul<false>(v2, tw_r4<LOG2M, S>(tw, 2, k));
                    v3 = twmul<false>(v3, tw_r4<LOG2M, S>(tw, 3, k));
                }
                const float2 a02 = cadd(v[t][0], v2), s02 = csub(v[t][0], v2);
                const float2 a13 = cadd(v1, v3), s13 = mul_mi<false>(csub(v1, v3));
                const float2 o0 = cadd(a02, a13), o1 = cadd(s02, s13), o2 = csub(a02, a13), o3 = csub(s02, s13);
                const int base = (j - k) * 4 + k;
                if constexpr (Ns < 16) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int qq = (r + (j >> 2)) & 3;
                        buf[base + qq * Ns] = qq == 0 ? o0 : (qq == 1 ? o1 : (qq == 2 ? o2 : o3));
                    }
                } else {
                    buf[base] = o0;
                    buf[base + Ns] = o1;
                    buf[base + 2 * Ns] = o2;
                    buf[base + 3 * Ns] = o3;
                }
            }
        }
    } else {
        constexpr int Ns = M / 2;
        constexpr int NB = (M / 2 + 63) / 64;
        float2 v[NB][2];
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int j = lane + 64 * t;
            if (j < M / 2) {
                v[t][0] = buf[j];
                v[t][1] = buf[j + M / 2];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int t = 0; t < NB; ++t) {
            const int j = lane + 64 * t;
            if (j < M / 2) {
                const int k = j & (Ns - 1);
                float2 v1 = v[t][1];
                if constexpr (Ns > 1) v1 = twmul<false>(v1, tw_r2<LOG2M>(tw, k));
                const int base = (j - k) * 2 + k;
                buf[base] = cadd(v[t][0], v1);
                buf[base + Ns] = csub(v[t][0], v1);
            }
        }
    }
}
template <int LOG2M, int S0, int S1, class TW>
__device__ __forceinline__ float2 *wave_stages_inplace(float2 *buf, TW tw) {
    if constexpr (S0 < S1) {
        wave_stage_inplace<LOG2M, S0, TW>(buf, tw);
        wave_sync();
        return wave_stages_inplace<LOG2M, S0 + 1, S1, TW>(buf, tw);
    } else {
        return buf;
    }
}

// R2C of the packed block in buf0 (one wave): every stage but the last
// through LDS, the last stage in registers -- lane L then holds Z[j + q QS]
// for its butterflies j = L + 64 i -- and the post-twiddle pairs bin k with
// bin M - k, which sits in lane (64 - L) mod 64 at butterfly NJ-1-i, output
// NQ-1-q (lane 0: its own registers): one __shfl per bin, no LDS round trip
// and no wave barrier.  Same butterflies and post-twiddle as lds_cfft +
// real_post (bit-identical).  Writes the packed spectrum to q (LDS; must not
// be the buffer the last LDS stage ended in, fft_r2c_q_is_buf1) and g (HBM).
template <int LOG2M>
constexpr bool fft_r2c_q_is_buf1() { return ((fft_nstages<LOG2M>() - 1) & 1) == 0; }
// S0 > 0: stages [0, S0) already ran (buf0 holds their output; see
// wave_stage0_padded).  q == nullptr: the spectrum goes to g only.
// INPLACE: the LDS stages run in buf0 alone (wave_stages_inplace; buf1 unused).
// GNT: the stores to g are nontemporal (streamed out instead of left dirty in L2).
template <int LOG2M, int S0 = 0, class TW = const float2 *, bool INPLACE = false, bool GNT = false>
__device__ __forceinline__ void wave_r2c_post(float2 *buf0, float2 *buf1, TW tw, float2 *q, float2 *g) {
    constexpr int M = 1 << LOG2M;
    constexpr bool R2 = (LOG2M & 1) != 0;     // last stage radix-2 (else radix-4, Ns = M/4)
    constexpr int NQ = R2 ? 2 : 4;             // outputs per butterfly
    constexpr int QS = R2 ? M / 2 : M / 4;     // index stride between them
    constexpr int NJ = QS / 64;                // butterflies per lane
    constexpr int SL = fft_nstages<LOG2M>() - 1;  // the last stage
    static_assert(NJ >= 1 && LOG2M >= 3, "wave transforms: M >= 128");
    const int lane = (int)(threadIdx.x & 63);
    const float2 *src;
    if constexpr (INPLACE) src = wave_stages_inplace<LOG2M, S0, SL, TW>(buf0, tw);
    else src = fft_stages<LOG2M, 64, false, true, S0, SL, TW>(buf0, buf1, tw, lane);
    float2 z[NJ][NQ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
        const int j = lane + 64 * i;  // (k = j: the last stage has Ns = QS; table stride 2)
        if constexpr (R2) {
            const float2 v0 = src[j];
            const float2 v1 = twmul<false>(src[j + M / 2], tw_r2<LOG2M>(tw, j));
            z[i][0] = cadd(v0, v1);
            z[i][1] = csub(v0, v1);
        } else {
            const float2 v0 = src[j];
            const float2 v1 = twmul<false>(src[j + M / 4], tw_r4<LOG2M, SL>(tw, 1, j));
            const float2 v2 = twmul<false>(src[j + M / 2], tw_r4<LOG2M, SL>(tw, 2, j));
            const float2 v3 = twmul<false>(src[j + 3 * M / 4], tw_r4<LOG2M, SL>(tw, 3, j));
            const float2 a02 = cadd(v0, v2), s02 = csub(v0, v2);
            const float2 a13 = cadd(v1, v3), s13 = mul_mi<false>(csub(v1, v3));
            z[i][0] = cadd(a02, a13);
            z[i][1] = cadd(s02, s13);
            z[i][2] = csub(a02, a13);
            z[i][3] = csub(s02, s13);
        }
    }
    const int mirror = (64 - lane) & 63;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
            const int k = lane + 64 * i + qq * QS;
            float2 b = shfl2(z[NJ - 1 - i][NQ - 1 - qq], mirror);
            if (lane == 0) b = i == 0 ? z[0][(NQ - qq) % NQ] : z[(NJ - i) % NJ][NQ - 1 - qq];
            const float2 v = real_post_pair(z[i][qq], b, k, tw);
            if (q) q[k] = v;
            if constexpr (GNT) {
                typedef float f32x2_t __attribute__((ext_vector_type(2)));
                const f32x2_t w = {v.x, v.y};
                __builtin_nontemporal_store(w, reinterpret_cast<f32x2_t *>(g + k));
            } else {
                g[k] = v;
            }
        }
    }
}

// Stage 0 of the R2C of a zero-padded block, in registers: the packed points
// z[m], m >= M/2, are the padding (copy_and_pad, src/fft_convolver.rs:56-60),
// so butterfly j reads v0 = z[j], v1 = z[j + M/4] and v2 = v3 = 0.  Lane L
// passes v0[t], v1[t] of its butterflies j = L + 64 t; the outputs go to
// dst[4j + q] in fft_stage_r4's conflict-free order.  The arithmetic is
// fft_stage_r4<S = 0>'s with the zero operands kept, so the same bits.
template <int LOG2M>
constexpr int stage0_per_lane() { return ((1 << LOG2M) / 4 + 63) / 64; }
template <int LOG2M, bool INV = false>
__device__ __forceinline__ void wave_stage0_padded(const float2 (&v0)[stage0_per_lane<LOG2M>()],
                                                   const float2 (&v1)[stage0_per_lane<LOG2M>()], float2 *dst) {
    constexpr int M = 1 << LOG2M;
    const int lane = (int)(threadIdx.x & 63);
    const float2 zero = make_float2(0.f, 0.f);
#pragma unroll
    for (int t = 0; t < stage0_per_lane<LOG2M>(); ++t) {
        const int j = lane + 64 * t;
        if (j < M / 4) {
            const float2 a02 = cadd(v0[t], zero), s02 = csub(v0[t], zero);
            const float2 a13 = cadd(v1[t], zero), s13 = mul_mi<INV>(csub(v1[t], zero));
            const float2 o0 = cadd(a02, a13), o1 = cadd(s02, s13), o2 = csub(a02, a13), o3 = csub(s02, s13);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qq = (r + (j >> 2)) & 3;
                dst[4 * j + qq] = qq == 0 ? o0 : (qq == 1 ? o1 : (qq == 2 ? o2 : o3));
            }
        }
    }
}

// C2R of the packed spectrum X (LDS, one wave): realfft's pre-twiddle fused
// with the first radix-4 stage -- lane L's four stage-0 inputs are its own
// pre-twiddled bins j + q M/4, so they never go through LDS -- then the other
// stages b0 <-> b1 (b1 may be X's buffer).  Bit-identical to real_pre +
// lds_cfft<INV>.  Returns the result (2M reals, not yet scaled by 1/N).
template <int LOG2M>
__device__ __forceinline__ const float *wave_c2r(const float2 *X, float2 *b0, float2 *b1,
                                                 const float2 *__restrict__ tw) {
    constexpr int M = 1 << LOG2M;
    const int lane = (int)(threadIdx.x & 63);
    for (int j = lane; j < M / 4; j += 64) {
        const float2 v0 = real_pre<LOG2M, 64>(X, j, tw);
        const float2 v1 = real_pre<LOG2M, 64>(X, j + M / 4, tw);
        const float2 v2 = real_pre<LOG2M, 64>(X, j + M / 2, tw);
        const float2 v3 = real_pre<LOG2M, 64>(X, j + 3 * M / 4, tw);
        const float2 a02 = cadd(v0, v2), s02 = csub(v0, v2);
        const float2 a13 = cadd(v1, v3), s13 = mul_mi<true>(csub(v1, v3));
        const float2 o0 = cadd(a02, a13), o1 = cadd(s02, s13), o2 = csub(a02, a13), o3 = csub(s02, s13);
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // (stage 0: conflict-free store order, fft_stage_r4)
            const int qq = (r + (j >> 2)) & 3;
            b0[4 * j + qq] = qq == 0 ? o0 : (qq == 1 ? o1 : (qq == 2 ? o2 : o3));
        }
    }
    wave_sync();
    return reinterpret_cast<const float *>(fft_stages<LOG2M, 64, true, true, 1, fft_nstages<LOG2M>()>(b0, b1, tw, lane));
}

}  // namespace fftconv
