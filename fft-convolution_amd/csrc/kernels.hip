// kernels.hip -- gfx950 kernels of the batched partitioned convolver.
//
// One workgroup owns one channel (one reference FFTConvolver instance) for
// the whole call, so every piece of per-channel state stays private to a CU
// and no inter-workgroup protocol is needed.
//
// HBM layout (per uniform batch: C channels, block B, S segments):
//   H   float2 [C][S][B]  packed IR segment spectra      (segments_ir)
//   X   float2 [C][S][B]  packed frequency-domain delay line (segments)
//   ovl float  [C][B]     overlap                        (overlap)
//   ib  float  [C][B]     input buffer, only touched for partial blocks
//   pre float2 [C][B]     pre_multiplied, only touched for partial blocks
//   st  int4   [C]        {current, active_seg_count, input_buffer_fill, flags}
// A packed row is B complex = 8B bytes (slot 0 = (DC, Nyquist)), so each
// channel's H and X are contiguous 8*S*B-byte streams read with 16-byte
// loads (float4 = 2 bins per lane).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "fft_lds.hpp"
#include "kernels.hpp"
#include <hip/hip_ext.h>

namespace fftconv {

// ---------------------------------------------------------------------------
// Geometry of the fused step kernel for a given block size
// ---------------------------------------------------------------------------
template <int LOG2B, int NT>
struct Geo {
    static constexpr int B = 1 << LOG2B;
    static constexpr int VEC = B >= 2 ? 2 : 1;          // complex bins per lane-slot
    static constexpr int F = B / VEC;                   // slots per row
    static constexpr int G = F >= NT ? 1 : NT / F;      // row groups (segment split)
    static constexpr int SPT = F >= NT ? F / NT : 1;    // slots per thread
    // rows in flight per thread (B 4096 on 512 threads: 2 rows measured no
    // faster than 1 -- its near-row MAC streams at the chip's rate, r5o)
    static constexpr int U = SPT == 1 ? 8 : (SPT == 2 ? 2 : 1);
    static constexpr size_t red_bytes = G > 1 ? (size_t)NT * VEC * sizeof(float2) : 0;
    // B <= 512: the prologue stages by LDS-DMA the twiddle table (2B float2),
    // H[0] (B float2), overlap, and the two tail slices (B floats each)
    static constexpr bool PREFETCH = LOG2B <= 9;
    static constexpr size_t tw_bytes = PREFETCH ? 2 * (size_t)B * sizeof(float2) : 0;
    static constexpr size_t pre_bytes = PREFETCH ? (size_t)B * sizeof(float2) + 3 * (size_t)B * sizeof(float) : 0;
    static constexpr size_t gen_bytes = ((2 * (size_t)B * sizeof(float2) + red_bytes + tw_bytes + pre_bytes + 15) / 16) * 16;
    // pipelined full-block step (pipelined_step): bufA | bufB | tw (2B) | H0 | H1 | pre | overlap | tail0 | tail1
    static constexpr bool PIPE = LOG2B >= 1 && LOG2B <= 9 && NT == 256;
    // the next block's pre is reduced and stored while the chain runs its C2R
    // (B <= 256): the reduction slots (4 waves x 64 lanes x 16 B x slots/lane)
    // after the chain's buffers; at B = 512 they reuse the front once the
    // chain is done (the process kernel's LDS stays below 40 KB there)
    static constexpr bool PIPE_EARLY = LOG2B <= 8;
    static constexpr size_t pipe_red = 4 * 64 * 16 * (size_t)(B >= 128 ? B / 128 : 1);
    static constexpr size_t pipe_bytes =
        PIPE ? (PIPE_EARLY ? 68 * (size_t)B + pipe_red : (68 * (size_t)B > pipe_red ? 68 * (size_t)B : pipe_red)) : 0;
    static constexpr size_t lds_bytes = (gen_bytes > pipe_bytes ? gen_bytes : pipe_bytes) + 16;
};

template <int VEC> struct VecT;
template <> struct VecT<2> { using type = float4; };
template <> struct VecT<1> { using type = float2; };

// Complex multiply-accumulate over one lane-slot, complex_multiply_accumulate
// (src/fft_convolver.rs:62-74) for 2 bins.  dc/ny carry the products of the
// packed real bins so that slot 0 can be resolved as (DC, Nyquist).
struct Acc2 {
    float4 a;
    float dc, ny;
    __device__ __forceinline__ void zero() { a = make_float4(0.f, 0.f, 0.f, 0.f); dc = ny = 0.f; }
    __device__ __forceinline__ void mac(float4 h, float4 x) {
        a.x = fmaf(-h.y, x.y, fmaf(h.x, x.x, a.x));
        a.y = fmaf(h.y, x.x, fmaf(h.x, x.y, a.y));
        a.z = fmaf(-h.w, x.w, fmaf(h.z, x.z, a.z));
        a.w = fmaf(h.w, x.z, fmaf(h.z, x.w, a.w));
        dc = fmaf(h.x, x.x, dc);
        ny = fmaf(h.y, x.y, ny);
    }
    __device__ __forceinline__ float4 get(int slot) const {
        return slot == 0 ? make_float4(dc, ny, a.z, a.w) : a;
    }
};
struct Acc1 {  // B == 1: the only bin pair is (DC, Nyquist)
    float2 a;
    __device__ __forceinline__ void zero() { a = make_float2(0.f, 0.f); }
    __device__ __forceinline__ void mac(float2 h, float2 x) { a.x = fmaf(h.x, x.x, a.x); a.y = fmaf(h.y, x.y, a.y); }
    __device__ __forceinline__ float2 get(int) const { return a; }
};
template <int VEC> using AccT = std::conditional_t<VEC == 2, Acc2, Acc1>;

__device__ __forceinline__ float4 vadd(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float2 vadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
// streaming accesses (nontemporal): rows used once, which must not evict the
// working set of latency-bound launches running beside them (a two-stage head)
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ntld4(const float4 *p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void ntst4(float4 *p, float4 v) {
    const f32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<f32x4 *>(p));
}

// conv = pre + x (.) h for one slot, packed-aware (slot 0 bin 0 is (DC, Nyquist)).
__device__ __forceinline__ float4 slot_mac(float4 pre, float4 x, float4 h, int slot) {
    float4 r;
    if (slot == 0) {
        r.x = fmaf(x.x, h.x, pre.x);
        r.y = fmaf(x.y, h.y, pre.y);
    } else {
        r.x = fmaf(-x.y, h.y, fmaf(x.x, h.x, pre.x));
        r.y = fmaf(x.y, h.x, fmaf(x.x, h.y, pre.y));
    }
    r.z = fmaf(-x.w, h.w, fmaf(x.z, h.z, pre.z));
    r.w = fmaf(x.w, h.z, fmaf(x.z, h.w, pre.w));
    return r;
}
__device__ __forceinline__ float2 slot_mac(float2 pre, float2 x, float2 h, int) {
    return make_float2(fmaf(x.x, h.x, pre.x), fmaf(x.y, h.y, pre.y));
}
// a state word written by a non-lookahead step: no live window, this launch's tag
__device__ __forceinline__ int la_clear(int flags, const ProcArgs &a) {
    return (flags & ~(LA_MASK | SEQ_MASK)) | (a.la_seq << SEQ_SHIFT);
}
__device__ __forceinline__ bool slot0_finite(float4 v) { return isfinite(v.x) && isfinite(v.y); }
__device__ __forceinline__ bool slot0_finite(float2 v) { return isfinite(v.x) && isfinite(v.y); }
__device__ __forceinline__ float2 slot0_of(float4 v) { return make_float2(v.x, v.y); }
__device__ __forceinline__ float2 slot0_of(float2 v) { return v; }

// realfft's C2R error (:264-267) once conv's slot 0 = pre0 + x0 (.) h0 came
// out non-finite.  The reference's DC / Nyquist imaginary parts are sums of
// re * 0 + 0 * re products (complex_multiply_accumulate on real bins): NaN
// exactly when one operand row's (DC, Nyquist) pair is not finite, and 0 when
// all are finite -- a finite overflow then runs the C2R on inf without an
// error.  pre0 was summed from rows 1..act-1 of H and of the ring, which are
// unchanged since (an update zeroes pre_multiplied), so only a non-finite pre0
// needs them scanned.  Rare path: one lane.
__device__ __attribute__((noinline)) bool c2r_rejects(const float2 *Hc, const float2 *Xc, int B, int cur, int act,
                                                      float2 pre0, float2 x0, float2 h0) {
    if (!slot0_finite(x0) || !slot0_finite(h0)) return true;
    if (slot0_finite(pre0)) return false;
    for (int i = 1; i < act; ++i) {
        const int xi = (cur + i) % act;  // index_audio (:248; current may exceed act after an update)
        if (!slot0_finite(Hc[(size_t)i * B]) || !slot0_finite(Xc[(size_t)xi * B])) return true;
    }
    return false;
}

// Buffer-resource streams (guide T8): one wave-uniform descriptor per channel
// stream, the row offset in an SGPR (soffset) when the row is wave-uniform,
// one shared per-lane voffset -- no per-load 64-bit address registers.
// aux 2 = nontemporal.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// FFTCONV_DEBUG_BOUNDS (debug builds only): DBG_CHECK (kernels.hpp) reports
// out-of-range stream rows and window/state indices with printf instead of
// touching the memory
struct RowStream {
    __amdgpu_buffer_rsrc_t r;
#ifdef FFTCONV_DEBUG_BOUNDS
    int nbytes;
#endif
    __device__ __forceinline__ RowStream(const float2 *base, size_t bytes) {
        r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2 *>(base), 0, (int)bytes, 0x00020000);
#ifdef FFTCONV_DEBUG_BOUNDS
        nbytes = (int)bytes;
#endif
    }
    // (an explicitly typed vector + memcpy: indexing the builtin's result
    // through __builtin_bit_cast made hipcc emit a single-dword load)
    template <bool NTL>
    __device__ __forceinline__ float4 ld4(int voff, int soff) const {
#ifdef FFTCONV_DEBUG_BOUNDS
        if (voff < nbytes && (soff < 0 || soff + voff + 16 > nbytes)) {
            dbg_bounds(3, voff, soff, nbytes, 0);  // (site 3: a stream row past the buffer)
            soff = 0;
        }
#endif
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, NTL ? 2 : 0);
        float4 f;
        __builtin_memcpy(&f, &v, sizeof(f));
        return f;
    }
    template <bool NTL>
    __device__ __forceinline__ float2 ld2(int voff, int soff) const {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, NTL ? 2 : 0);
        float2 f;
        __builtin_memcpy(&f, &v, sizeof(f));
        return f;
    }
    template <bool NTL>
    __device__ __forceinline__ float4 ld(int voff, int soff, float4 *) const { return ld4<NTL>(voff, soff); }
    template <bool NTL>
    __device__ __forceinline__ float2 ld(int voff, int soff, float2 *) const { return ld2<NTL>(voff, soff); }
};

// pre_multiplied = sum_{i=i0}^{i1-1} H[i] (.) X[(cur+i) % act] over this
// thread's slots (src/fft_convolver.rs:244-255; the whole sum is rows
// 1..act-1).  The rows are visited in scan order t = 0..i1-i0-1, group g
// taking t = g (mod G).  ZZ: every other block scans the rows backwards (rows
// read last by one step are read first by the next).  NTL: nontemporal loads.
template <int LOG2B, int NT, bool ZZ, bool NTL, class AccArr>
__device__ __forceinline__ void mac_rows(AccArr &acc, const float2 *Hc, const float2 *Xc, int S, int cur, int act,
                                         int i0, int i1, int flags, int f0, int g) {
    using Gm = Geo<LOG2B, NT>;
    constexpr int B = Gm::B, VEC = Gm::VEC, F = Gm::F, G = Gm::G, SPT = Gm::SPT, U = Gm::U;
    constexpr int ROWB = B * (int)sizeof(float2);  // bytes per row
    constexpr bool UNIFORM = F >= 64;              // a row group spans whole waves
    using vec_t = typename VecT<VEC>::type;
    const size_t bytes = (size_t)S * ROWB;
    const RowStream hs(Hc, bytes), xs(Xc, bytes);
    const int lane_off = f0 * VEC * (int)sizeof(float2);
#pragma unroll
    for (int s = 0; s < SPT; ++s) acc[s].zero();
    const bool rev = ZZ && (flags & FLAG_REV);
    const int di = rev ? -G : G;
    const int nr = i1 - i0;
    int t = g;
    int i = rev ? i1 - 1 - t : i0 + t;
    int xi = (cur + i) % act;  // index_audio = (current + i) % active
    for (; t + (U - 1) * G < nr; t += U * G) {
        vec_t hv[U][SPT], xv[U][SPT];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ho = i * ROWB, xo = xi * ROWB;
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                const int lo = lane_off + s * NT * VEC * (int)sizeof(float2);
                hv[u][s] = UNIFORM ? hs.ld<NTL>(lo, ho, (vec_t *)nullptr) : hs.ld<NTL>(lo + ho, 0, (vec_t *)nullptr);
                xv[u][s] = UNIFORM ? xs.ld<NTL>(lo, xo, (vec_t *)nullptr) : xs.ld<NTL>(lo + xo, 0, (vec_t *)nullptr);
            }
            i += di;
            xi += di;
            if (xi >= act) xi -= act;
            if (xi < 0) xi += act;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < SPT; ++s) acc[s].mac(hv[u][s], xv[u][s]);
    }
    for (; t < nr; t += G) {
        const int ho = i * ROWB, xo = xi * ROWB;
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
            const int lo = lane_off + s * NT * VEC * (int)sizeof(float2);
            const vec_t h = UNIFORM ? hs.ld<NTL>(lo, ho, (vec_t *)nullptr) : hs.ld<NTL>(lo + ho, 0, (vec_t *)nullptr);
            const vec_t x = UNIFORM ? xs.ld<NTL>(lo, xo, (vec_t *)nullptr) : xs.ld<NTL>(lo + xo, 0, (vec_t *)nullptr);
            acc[s].mac(h, x);
        }
        i += di;
        xi += di;
        if (xi >= act) xi -= act;
        if (xi < 0) xi += act;
    }
}

// Crossfade pair: the two convolvers' pre_multiplied from ONE read of the
// shared FDL (A and B see the same input, so while their ring states agree
// their FDL rows are equal).  Same row walk and per-accumulator order as
// mac_rows (non-zig-zag), so each sum is bit-identical to the unpaired one.
template <int LOG2B, int NT, bool NTL, class AccArr>
__device__ __forceinline__ void mac_rows_pair(AccArr &accA, AccArr &accB, const float2 *HA, const float2 *HB,
                                              const float2 *Xc, int S, int cur, int act, int f0, int g) {
    using Gm = Geo<LOG2B, NT>;
    constexpr int B = Gm::B, VEC = Gm::VEC, G = Gm::G, SPT = Gm::SPT;
    constexpr int U = SPT == 1 ? 8 : (SPT == 2 ? 4 : 2);
    constexpr int ROWB = B * (int)sizeof(float2);
    constexpr bool UNIFORM = Gm::F >= 64;
    using vec_t = typename VecT<VEC>::type;
    const size_t bytes = (size_t)S * ROWB;
    const RowStream ha(HA, bytes), hb(HB, bytes), xs(Xc, bytes);
    const int lane_off = f0 * VEC * (int)sizeof(float2);
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
        accA[s].zero();
        accB[s].zero();
    }
    int t = g;
    int i = 1 + t;
    int xi = (cur + i) % act;
    for (; t + (U - 1) * G < act - 1; t += U * G) {
        vec_t av[U][SPT], bv[U][SPT], xv[U][SPT];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ho = i * ROWB, xo = xi * ROWB;
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                const int lo = lane_off + s * NT * VEC * (int)sizeof(float2);
                av[u][s] = UNIFORM ? ha.ld<NTL>(lo, ho, (vec_t *)nullptr) : ha.ld<NTL>(lo + ho, 0, (vec_t *)nullptr);
                bv[u][s] = UNIFORM ? hb.ld<NTL>(lo, ho, (vec_t *)nullptr) : hb.ld<NTL>(lo + ho, 0, (vec_t *)nullptr);
                xv[u][s] = UNIFORM ? xs.ld<NTL>(lo, xo, (vec_t *)nullptr) : xs.ld<NTL>(lo + xo, 0, (vec_t *)nullptr);
            }
            i += G;
            xi += G;
            if (xi >= act) xi -= act;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                accA[s].mac(av[u][s], xv[u][s]);
                accB[s].mac(bv[u][s], xv[u][s]);
            }
    }
    for (; t < act - 1; t += G) {
        const int ho = i * ROWB, xo = xi * ROWB;
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
            const int lo = lane_off + s * NT * VEC * (int)sizeof(float2);
            const vec_t x = UNIFORM ? xs.ld<NTL>(lo, xo, (vec_t *)nullptr) : xs.ld<NTL>(lo + xo, 0, (vec_t *)nullptr);
            accA[s].mac(UNIFORM ? ha.ld<NTL>(lo, ho, (vec_t *)nullptr) : ha.ld<NTL>(lo + ho, 0, (vec_t *)nullptr), x);
            accB[s].mac(UNIFORM ? hb.ld<NTL>(lo, ho, (vec_t *)nullptr) : hb.ld<NTL>(lo + ho, 0, (vec_t *)nullptr), x);
        }
        i += G;
        xi += G;
        if (xi >= act) xi -= act;
    }
}

// Asynchronous global -> LDS copies (LDS-DMA, global_load_lds): lane l of a
// wave writes dst + l*W for a wave-uniform dst, no VGPR destination, drained
// by the next __syncthreads (s_waitcnt vmcnt(0) before s_barrier).
typedef __attribute__((address_space(1))) const void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;
template <int NT>
__device__ __forceinline__ void dma_f32(float *dst, const float *src, int count) {  // any alignment
    const int lane = threadIdx.x & 63;
    // NT threads copy: the caller's wave w of them starts at w (NT = 64: any single wave)
    for (int base = ((threadIdx.x >> 6) % (NT / 64)) * 64; base < count; base += NT)
        if (base + lane < count)
            __builtin_amdgcn_global_load_lds((gptr_t)(src + base + lane), (lptr_t)(dst + base), 4, 0, 0);
}
template <int NT>
__device__ __forceinline__ void dma_16b(void *dst, const void *src, int bytes) {  // 16-byte aligned, bytes % 16 == 0
    const int lane = threadIdx.x & 63;
    const char *s = static_cast<const char *>(src);
    char *d = static_cast<char *>(dst);
    for (int base = ((threadIdx.x >> 6) % (NT / 64)) * 1024; base < bytes; base += NT * 16)
        if (base + lane * 16 < bytes)
            __builtin_amdgcn_global_load_lds((gptr_t)(s + base + lane * 16), (lptr_t)(d + base), 16, 0, 0);
}

// TwoStageFFTConvolver::process sub-chunk (src/fft_convolver.rs:438-461) fused
// into the head job: output += precalculated0, then += precalculated (two
// separate adds, like the reference's two loops), and tail_input <- input.
// Generic form: a pass over the finished output.
template <int NT>
__device__ __forceinline__ void twostage_epilogue(const ProcJob &J, size_t c, float *outc, const float *inc, int n) {
    if (!J.add0 && !J.tin) return;
    __syncthreads();  // outc[] was written by other threads of this workgroup
    const float *p0 = J.add0 ? J.add0 + c * J.add_stride : nullptr;
    const float *p1 = J.add1 ? J.add1 + c * J.add_stride : nullptr;
    float *ti = J.tin ? J.tin + c * J.tin_stride : nullptr;
    for (int j = threadIdx.x; j < n; j += NT) {
        if (p0) {
            float v = outc[j];
            v += p0[j];
            if (p1) v += p1[j];
            outc[j] = v;
        }
        if (ti) ti[j] = inc[j];
    }
}

// FDL stream of the pipelined step: rows i = 2 + t of the NEXT block's
// pre_multiplied (block start `curp`) for t in [t_begin, t_end), split over
// nw waves (this is wave sw of them); a wave covers RPW rows at once when a
// row has fewer than 64 slots.  Accumulates into acc (not zeroed here).
template <int LOG2B, bool NTL, class AccArr>
__device__ __forceinline__ void mac_rows_range(AccArr &acc, const float2 *Hc, const float2 *Xc, int S, int curp,
                                               int act, int t_begin, int t_end, int nw, int sw, int rsub, int f0) {
    constexpr int B = 1 << LOG2B, F = B / 2;
    constexpr int RPW = F >= 64 ? 1 : 64 / F, SPL = F >= 64 ? F / 64 : 1;
    // (11 rows per half-wave in flight: cfg3's head stream -- 62 rows over 3
    // waves of 2 half-waves -- in one round trip instead of two: head step
    // 5.41 -> 5.05 us, cfg3 6.96 -> 6.86 us; 16 spills: 6.57 us; r4l A/B)
    constexpr int U = SPL == 1 ? 11 : (SPL == 2 ? 4 : 2);
    constexpr int ROWB = B * (int)sizeof(float2);
    constexpr bool UNIFORM = RPW == 1;  // one row per wave-iteration: row offset in an SGPR
    const int STEP = nw * RPW;
    const size_t bytes = (size_t)S * ROWB;
    const RowStream hs(Hc, bytes), xs(Xc, bytes);
    const int lane_off = f0 * 16;
    constexpr int OOB = 0x7ffffff0;  // a voffset past the stream: the load returns 0, no memory access
    int t = t_begin + sw * RPW + rsub;
    int i = 2 + t;
    int xi = (curp + i) % act;
    // batches of U rows, the last one partial: rows past t_end are loaded from
    // the out-of-range offset and not accumulated, so the last rows of a walk
    // are in flight together instead of one round trip each (cfg3 head, r3)
    for (; t < t_end; t += U * STEP) {
        float4 hv[U][SPL], xv[U][SPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = t + u * STEP < t_end;
            const int ho = in ? i * ROWB : 0, xo = in ? xi * ROWB : 0;
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                const int lo = in ? lane_off + s * 64 * 16 : OOB;
                hv[u][s] = UNIFORM ? hs.ld4<NTL>(lo, ho) : hs.ld4<NTL>(in ? lo + ho : OOB, 0);
                xv[u][s] = UNIFORM ? xs.ld4<NTL>(lo, xo) : xs.ld4<NTL>(in ? lo + xo : OOB, 0);
            }
            i += STEP;
            xi += STEP;
            if (xi >= act) xi -= act;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t + u * STEP < t_end) {
#pragma unroll
                for (int s = 0; s < SPL; ++s) acc[s].mac(hv[u][s], xv[u][s]);
            }
    }
}

// mac_rows_range over a multi-call run's LDS copies of the IR rows (hl) and
// the FDL ring (xl): the same rows in the same order per slot, so the same
// bits -- without the HBM / L2 round trip the stream waves otherwise wait on
// every call (cfg3's head: 62 rows of H and X per call, ~1.6 us)
template <int LOG2B, class AccArr>
__device__ __forceinline__ void mac_rows_lds(AccArr &acc, const float2 *hl, const float2 *xl, int curp, int act,
                                             int t_begin, int t_end, int nw, int sw, int rsub, int f0) {
    constexpr int B = 1 << LOG2B, F = B / 2;
    constexpr int RPW = F >= 64 ? 1 : 64 / F, SPL = F >= 64 ? F / 64 : 1;
    // batches of U rows, every LDS read of a batch issued before its MACs
    // (one LDS round trip per batch, not per row); rows past t_end read row 0
    // and are not accumulated
    constexpr int U = SPL == 1 ? 12 : (SPL == 2 ? 6 : 3);
    const int STEP = nw * RPW;
    const float4 *h4 = reinterpret_cast<const float4 *>(hl), *x4 = reinterpret_cast<const float4 *>(xl);
    int t = t_begin + sw * RPW + rsub;
    int i = 2 + t;
    int xi = (curp + i) % act;
    for (; t < t_end; t += U * STEP) {
        float4 hv[U][SPL], xv[U][SPL];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = t + u * STEP < t_end;
            const int ho = in ? i * F : 0, xo = in ? xi * F : 0;
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                hv[u][s] = h4[ho + f0 + s * 64];
                xv[u][s] = x4[xo + f0 + s * 64];
            }
            i += STEP;
            xi += STEP;
            if (xi >= act) xi -= act;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t + u * STEP < t_end) {
#pragma unroll
                for (int s = 0; s < SPL; ++s) acc[s].mac(hv[u][s], xv[u][s]);
            }
    }
}

// ProcArgs::sig: a tail step's workgroups arrive when their stores are done
// (each releases at agent scope, then one relaxed add; the last acquires them
// all and releases sig[1] = sig_val); a run waits for sig[1] >= sig_val
// (wrap-safe), acquires, and the workgroup's loads of the tail's output come
// after.  The wait is bounded (~100 ms, counted in sig[2]): the tail it waits
// for was enqueued a period earlier on a stream of its own, fits a CU beside
// a run workgroup, and in practice finished long before.
__device__ __forceinline__ void sig_arrive(const ProcArgs &a) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned n = gridDim.x * gridDim.y;
        const unsigned prev = __hip_atomic_fetch_add(a.sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == n - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(a.sig, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sig + 1, a.sig_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
__device__ __forceinline__ void sig_wait(const ProcArgs &a) {
    if (threadIdx.x == 0) {
        const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
        while ((int)(__hip_atomic_load(a.sig + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.sig_val) < 0) {
            __builtin_amdgcn_s_sleep(8);
            if ((unsigned)__builtin_amdgcn_s_memrealtime() - t0 > 10000000u) {  // (100 MHz: 100 ms)
                __hip_atomic_fetch_add(a.sig + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// launch timeline phase stamp k (0..3) of this wave of a process launch
// (FFTCONV_PROC_TRACE; job 0 only)
__device__ __forceinline__ void proc_stamp(const ProcArgs &a, int k) {
    if (a.la_trace && blockIdx.y == 0 && (threadIdx.x >> 6) < 4 && (threadIdx.x & 63) == 0) {
        int *p = reinterpret_cast<int *>(a.la_trace + ((size_t)a.la_trace_grid * 4 + (size_t)blockIdx.x * 4 + (threadIdx.x >> 6)));
        p[k] = (int)(unsigned)__builtin_amdgcn_s_memrealtime();
    }
}

// A multi-call launch's chain state between two calls of one channel
// (upols_run_kernel, pipelined steps at B <= 256): when the previous call ran
// the pipelined step without a C2R error (`hot`), the twiddles, H[0], H[1]
// and the next pre_multiplied are still in LDS, the next call's input block
// was prefetched into LDS stage[par] by a helper wave, and the overlap is in
// registers -- the call starts its R2C without a memory round trip.  The
// same values as the loads it replaces: bit-identical.
struct RunCarry {
    int hot;
    int par;                // stage buffer holding this call's input (hot)
    const float *next_in;   // the next call's input (null: the run's last call)
    float ov[4];            // overlap samples of the chain's lanes (B <= 256)
    int4 st;                // the state word the call stored (hot): the next call's, without a reload
    // the run's LDS copies of the IR rows and the FDL (ProcArgs::run_lds_rows;
    // null = the helpers stream the rows from memory): row r at hl / xl + r*B
    const float2 *hl;
    float2 *xl;
};

// Workgroup barrier for LDS data only: this wave's LDS operations complete,
// then s_barrier -- unlike __syncthreads, no wait for the wave's outstanding
// global stores (the pipelined step's chain has just issued its FDL row,
// tail_input and tail0 spectrum stores; nothing behind this barrier reads
// them, and the call's closing __syncthreads orders them for the next call).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------
// Pipelined full-block step (2 <= B <= 512): the common call -- one whole
// block from an empty input buffer -- when pre[] already holds
// pre_multiplied for the block at `current` (FLAG_PRE).  The work of
// FFTConvolver::process (:215-295) is re-timed, not changed:
//   wave 0   : R2C of the block -> FDL row `current`; conv = pre + X.H[0];
//              C2R, x1/N; overlap-add and overlap save -- all out of LDS,
//              staged by its own LDS-DMA, synchronised at wave level; then
//              row 1 (H[1] (.) X_new) of the NEXT block's pre_multiplied,
//              then the last w0 = max(0, (S-2-lag)/4) FDL rows of it
//   waves 1-3: stream the other FDL rows of the NEXT block's pre_multiplied
// so the latency chain hides under the FDL stream instead of following it
// (lag ~ the chain's duration in rows of stream; set by the host).
// The next block's pre is reduced in a fixed order and stored (FLAG_PRE).
// B <= 256 (PIPE_EARLY): the chain parks its share of that pre right after
// the conv (row 1 needs only the new spectrum) and the helper waves, long
// done with their rows, reduce and store it and the state word while the
// chain runs its C2R -- the reduction leaves the launch's critical path
// (cfg3 head timeline, profiles/r3: it ran after the chain, 0.5 of 5.5 us).
// ---------------------------------------------------------------------------
template <int LOG2B, int NT, bool NTL, bool RUN = false>
__device__ __forceinline__ bool pipelined_step(const ProcArgs &a, const ProcJob &J, size_t c, int cur, int act,
                                               int flags, unsigned char *smem, RunCarry *rc = nullptr) {
    using Gm = Geo<LOG2B, NT>;
    constexpr int B = Gm::B, F = B / 2;
    constexpr int RPW = F >= 64 ? 1 : 64 / F, SPL = F >= 64 ? F / 64 : 1;
    constexpr int NSW = NT / 64 - 1;
    constexpr float invN = 1.0f / (float)(2 * B);
    float2 *bufA = reinterpret_cast<float2 *>(smem);
    float2 *bufB = bufA + B;
    float2 *twl = bufB + B;
    float2 *h0l = twl + 2 * B;
    float2 *h1l = h0l + B;
    float2 *prel = h1l + B;
    float *ovl = reinterpret_cast<float *>(prel + B);
    float *p0l = ovl + B;
    float *p1l = p0l + B;
    int &s_err = *reinterpret_cast<int *>(smem + Gm::lds_bytes - 16);
    // the next block's pre: partial sums [wave][slot/64][lane]
    float4 *red = reinterpret_cast<float4 *>(Gm::PIPE_EARLY ? reinterpret_cast<unsigned char *>(p1l + B) : smem);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const size_t rows = (size_t)J.S * B;
    const float2 *Hc = J.H + c * rows;
    float2 *Xc = J.X + c * rows;
    float *ovc = J.overlap + c * B;
    float2 *prec = J.pre + c * B;
    float *outc = J.out + c * J.out_stride;
    const float *inc = J.in + c * J.in_stride;
    const int curp = cur > 0 ? cur - 1 : act - 1;  // current after this block (:287-291)
    const int rsub = F >= 64 ? 0 : lane / F;
    const int f0 = F >= 64 ? lane : lane % F;

    Acc2 acc[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) acc[s].zero();
    constexpr int CNB = (B + 63) / 64;  // the chain's samples per lane
    float ovr[CNB], p0r[CNB], p1r[CNB];
#pragma unroll
    for (int i = 0; i < CNB; ++i) ovr[i] = p0r[i] = p1r[i] = 0.f;
    float2 *Z = bufA, *Q = bufB;  // (the chain's transform buffers, across B1)
    bool err = false;
    constexpr bool RH = RUN && Gm::PIPE_EARLY && CNB <= 4;  // (run-carried state: B <= 256)
    float *stage[2] = {ovl, p0l};  // (a run's prefetched input blocks: LDS the step leaves unused)
    const bool hot = RH && rc->hot;
    // (a run: the spectra of the calls' blocks, double-buffered by stage
    // parity -- the last helper wave transforms the NEXT call's block while
    // the chain runs this call's C2R, so a hot call's chain starts at the
    // conv; then the helper's two transform buffers.  Past the step's LDS:
    // the run kernel allocates run_lds_bytes)
    float2 *nxs = reinterpret_cast<float2 *>(smem + Gm::lds_bytes);
    float2 *nfa = nxs + 2 * B, *nfb = nfa + B;
    // (a run: the state word this step stores when its block succeeds; every
    // thread holds it, so the next call starts without reloading it)
    if constexpr (RH) rc->st = make_int4(curp, act, 0, la_clear(((flags & ~FLAG_INBUF) ^ FLAG_REV) | FLAG_PRE, a));
    if (wave == 0) {
        // ---- critical chain, one wave: R2C, conv, the C2R error check ----
        if (hot) {
            // tw, H[0], H[1], pre and this block's spectrum in LDS already
        } else {
            dma_f32<64>(reinterpret_cast<float *>(bufA), inc, B);   // x[0..B) as packed z[0..B/2)
            for (int m = B / 2 + lane; m < B; m += 64) bufA[m] = make_float2(0.f, 0.f);
            dma_16b<64>(twl, a.tw, 2 * B * (int)sizeof(float2));
            dma_16b<64>(h0l, Hc, B * (int)sizeof(float2));
            if (act > 1) dma_16b<64>(h1l, Hc + B, B * (int)sizeof(float2));
            dma_16b<64>(prel, prec, B * (int)sizeof(float2));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        wave_sync();
        // the overlap and the two-stage adds are read only by the overlap-add
        // at the chain's end: plain loads issued now arrive under the
        // transforms, instead of holding the R2C behind the prologue wait
        // (cfg3 head: the adds come from the tail buffers, HBM-cold)
#pragma unroll
        for (int i = 0; i < CNB; ++i) {
            const int j = lane + 64 * i;
            if (j < B) {
                if constexpr (RH) ovr[i] = hot ? rc->ov[i] : ovc[j];
                else ovr[i] = ovc[j];
                if (J.add0) p0r[i] = J.add0[c * J.add_stride + j];
                if (J.add1) p1r[i] = J.add1[c * J.add_stride + j];
            }
        }
        proc_stamp(a, 0);
        if (J.tin) {  // two-stage: append the block to tail_input (:459-461)
            const float *xb = hot ? stage[rc->par] : reinterpret_cast<const float *>(bufA);
            float *ti = J.tin + c * J.tin_stride;
            for (int j = lane; j < B; j += 64) ti[j] = xb[j];
        }
        float2 *Xcur = Xc + (size_t)cur * B;
        float2 *t0r = J.t0x ? J.t0x + c * J.t0x_stride : nullptr;  // (a run: tail0's copy of the spectrum)
        if (hot) {
            // the spectrum the last helper wave computed during the previous
            // call (the same transform, bit for bit): to the FDL row, tail0's row
            Q = nxs + rc->par * B;
            Z = bufA;
            float2 *xlc = rc->xl ? rc->xl + (size_t)cur * B : nullptr;  // (the run's LDS ring)
            for (int m = lane; m < B; m += 64) {
                const float2 v = Q[m];
                Xcur[m] = v;
                if (t0r) t0r[m] = v;
                if (xlc) xlc[m] = v;
            }
        } else {
            wave_sync();
            Z = lds_cfft<LOG2B, 64, false, true>(bufA, bufB, twl);  // :229-241
            Q = Z == bufA ? bufB : bufA;
            float2 *xlc = nullptr;
            if constexpr (RH) xlc = rc->xl ? rc->xl + (size_t)cur * B : nullptr;
            for (int m = lane; m < B; m += 64) {
                const float2 v = real_post<LOG2B, 64>(Z, m, twl);
                Q[m] = v;
                Xcur[m] = v;
                if (t0r) t0r[m] = v;
                if (xlc) xlc[m] = v;
            }
            wave_sync();
        }
        bool bad = false;  // conv = pre + X (.) H[0] (:256-261), then the C2R error check
        for (int f = lane; f < F; f += 64) {
            const float4 cv = slot_mac(reinterpret_cast<const float4 *>(prel)[f], reinterpret_cast<const float4 *>(Q)[f],
                                       reinterpret_cast<const float4 *>(h0l)[f], f);
            reinterpret_cast<float4 *>(Z)[f] = cv;
            if (f == 0 && !slot0_finite(cv) &&
                c2r_rejects(Hc, Xc, B, cur, act, slot0_of(reinterpret_cast<const float4 *>(prel)[0]),
                            slot0_of(reinterpret_cast<const float4 *>(Q)[0]), slot0_of(reinterpret_cast<const float4 *>(h0l)[0])))
                bad = true;
        }
        // row 1 of the next block's pre_multiplied: H[1] (.) X_new (X_new is row (curp+1) % act = cur)
        if (act > 1 && rsub == 0) {
#pragma unroll
            for (int s = 0; s < SPL; ++s) {
                const int f = f0 + s * 64;
                if (f < F) acc[s].mac(reinterpret_cast<const float4 *>(h1l)[f], reinterpret_cast<const float4 *>(Q)[f]);
            }
        }
        err = __ballot(bad) != 0ull;
        if constexpr (Gm::PIPE_EARLY) {
            // the chain's share of the next block's pre (row 1, and the last
            // w0 rows with a pipeline lag) to the reduction slots; the helper
            // waves reduce and store it, and the state, during the C2R below
            const int R = act > 2 ? act - 2 : 0;
            const int w0 = R > a.lag ? (R - a.lag) / (NSW + 1) : 0;
            if (w0 > 0) {
                bool inl = false;
                if constexpr (RH) inl = rc->xl != nullptr;
                if (inl) mac_rows_lds<LOG2B>(acc, rc->hl, rc->xl, curp, act, R - w0, R, 1, 0, rsub, f0);
                else mac_rows_range<LOG2B, NTL>(acc, Hc, Xc, J.S, curp, act, R - w0, R, 1, 0, rsub, f0);
            }
#pragma unroll
            for (int s = 0; s < SPL; ++s) red[s * 64 + lane] = acc[s].get(f0 + s * 64);
            if (lane == 0) s_err = err ? 1 : 0;
        }
    } else if constexpr (Gm::PIPE_EARLY) {
        // ---- helper waves: FDL rows 2..act-1 - w0 of the next block's pre ----
        // (a run: wave 1 first prefetches the next call's block into the other stage)
        if (RH && wave == 1 && rc->next_in) dma_f32<64>(stage[rc->par ^ 1], rc->next_in + c * J.in_stride, B);
        const int R = act > 2 ? act - 2 : 0;
        const int w0 = R > a.lag ? (R - a.lag) / (NSW + 1) : 0;
        bool inl = false;
        if constexpr (RH) inl = rc->xl != nullptr;
        if (inl) mac_rows_lds<LOG2B>(acc, rc->hl, rc->xl, curp, act, 0, R - w0, NSW, wave - 1, rsub, f0);
        else mac_rows_range<LOG2B, NTL>(acc, Hc, Xc, J.S, curp, act, 0, R - w0, NSW, wave - 1, rsub, f0);
#pragma unroll
        for (int s = 0; s < SPL; ++s) red[(wave * SPL + s) * 64 + lane] = acc[s].get(f0 + s * 64);
        // (the stage DMA has landed before B1: the last wave transforms it after B1)
        if constexpr (RH) {
            if (wave == 1 && rc->next_in) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        proc_stamp(a, 2);
    }
    // B1 (B <= 256): every wave at this one barrier -- the chain's share of
    // the next block's pre and its error flag, and the helpers' shares, are
    // in the reduction slots (LDS only: the chain's global stores stay in
    // flight across it)
    if constexpr (Gm::PIPE_EARLY) lds_barrier();
    if (wave == 0) {
        // ---- the chain's C2R and overlap-add ----
        wave_sync();
        proc_stamp(a, 1);
        if (!err) {
            for (int m = lane; m < B; m += 64) Q[m] = real_pre<LOG2B, 64>(Z, m, twl);
            wave_sync();
            const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2B, 64, true, true>(Q, Z, twl));
#pragma unroll
            for (int i = 0; i < CNB; ++i) {  // overlap-add (:270-274) + two-stage adds (:439-454)
                const int j = lane + 64 * i;
                if (j >= B) continue;
                float v = y[j] * invN + ovr[i];
                if (J.add0) {
                    v += p0r[i];
                    if (J.add1) v += p1r[i];
                }
                outc[j] = v;
                ovc[j] = y[B + j] * invN;  // :283-284
                if constexpr (RH) rc->ov[i] = y[B + j] * invN;
            }
        } else {
            // output.fill(0); return (:264-267): the block stays in the input
            // buffer, fill / current unchanged, pre still describes this block
            float *ibc = J.inbuf + c * B;
#pragma unroll
            for (int i = 0; i < CNB; ++i) {
                const int j = lane + 64 * i;
                if (j >= B) continue;
                float v = 0.f;
                if (J.add0) {
                    v += p0r[i];
                    if (J.add1) v += p1r[i];
                }
                outc[j] = v;
                ibc[j] = inc[j];
            }
        }
        if (!Gm::PIPE_EARLY && lane == 0) s_err = err ? 1 : 0;
        proc_stamp(a, 2);  // (timelines: the chain's C2R and overlap-add done)
        if constexpr (Gm::PIPE_EARLY) return !err;
    }
    if constexpr (Gm::PIPE_EARLY) {
        // ---- helper waves: the next block's pre in its fixed-order
        // reduction, and the state, while the chain runs its C2R ----
        const int ht = tid - 64;
        if (s_err) {
            if (ht == 0) J.state[c] = make_int4(cur, act, 0, la_clear(flags | FLAG_INBUF, a));
            if constexpr (RH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the stage DMA)
            return false;
        }
        for (int f = ht; f < F; f += NT - 64) {
            float4 p = red[f];
            for (int w = 0; w <= NSW; ++w)
                for (int r = (w == 0 ? 1 : 0); r < RPW; ++r) p = vadd(p, red[w * SPL * 64 + f + r * F]);
            reinterpret_cast<float4 *>(prec)[f] = p;
            if constexpr (RH) reinterpret_cast<float4 *>(prel)[f] = p;  // (the chain's C2R no longer reads prel)
        }
        if constexpr (RH) {
            // the last wave (never in the reduction at B <= 256): the R2C of the
            // next call's block (:229-241), from the stage wave 1 filled, into
            // the spectrum buffer of the other parity
            if (wave == NSW && rc->next_in) {
                const float *sg = stage[rc->par ^ 1];
                float *za = reinterpret_cast<float *>(nfa);
                for (int j = lane; j < B; j += 64) za[j] = sg[j];
                for (int m = B / 2 + lane; m < B; m += 64) nfa[m] = make_float2(0.f, 0.f);
                wave_sync();
                const float2 *Zn = lds_cfft<LOG2B, 64, false, true>(nfa, nfb, twl);
                float2 *qn = nxs + (rc->par ^ 1) * B;
                for (int m = lane; m < B; m += 64) qn[m] = real_post<LOG2B, 64>(Zn, m, twl);
            }
        }
        if (ht == 0) J.state[c] = make_int4(curp, act, 0, la_clear(((flags & ~FLAG_INBUF) ^ FLAG_REV) | FLAG_PRE, a));
        if constexpr (RH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the stage DMA has landed)
        // (RunCarry::st above is this word)
        proc_stamp(a, 3);
        return true;
    }
    // ---- FDL rows 2..act-1 of the next block's pre: waves 1..NSW take
    // t in [0, R0), wave 0 (after its chain) the last w0 rows ----
    {
        const int R = act > 2 ? act - 2 : 0;
        const int w0 = R > a.lag ? (R - a.lag) / (NSW + 1) : 0;
        const int R0 = R - w0;
        if (wave == 0) mac_rows_range<LOG2B, NTL>(acc, Hc, Xc, J.S, curp, act, R0, R, 1, 0, rsub, f0);
        else mac_rows_range<LOG2B, NTL>(acc, Hc, Xc, J.S, curp, act, 0, R0, NSW, wave - 1, rsub, f0);
    }
    proc_stamp(a, 2);
    __syncthreads();
    if (s_err) {
        if (tid == 0) J.state[c] = make_int4(cur, act, 0, la_clear(flags | FLAG_INBUF, a));
        return false;
    }
    // next block's pre: every lane parks its partial sums in LDS (the whole
    // workgroup's staging is dead now), then slot f sums waves 0..NSW and
    // sub-rows in a fixed order -- deterministic for a given geometry and lag
#pragma unroll
    for (int s = 0; s < SPL; ++s) red[(wave * SPL + s) * 64 + lane] = acc[s].get(f0 + s * 64);
    __syncthreads();
    for (int f = tid; f < F; f += NT) {
        const int base = (f / 64) * 64 + f % 64;
        float4 p = red[base];
        for (int w = 0; w <= NSW; ++w)
            for (int r = (w == 0 ? 1 : 0); r < RPW; ++r) p = vadd(p, red[w * SPL * 64 + base + r * F]);
        reinterpret_cast<float4 *>(prec)[f] = p;
    }
    if (tid == 0) J.state[c] = make_int4(curp, act, 0, la_clear(((flags & ~FLAG_INBUF) ^ FLAG_REV) | FLAG_PRE, a));
    proc_stamp(a, 3);
    return false;  // (B = 512: no run-carried state)
}

// ---------------------------------------------------------------------------
// Fused UPOLS step: FFTConvolver::process (src/fft_convolver.rs:215-295) for
// one channel per workgroup, the whole chunk loop of one call on device.
//
// Latency structure: every load that does not depend on the MAC is issued in
// the prologue, so its round trip overlaps the FDL stream -- the twiddle table
// (into LDS), H[0], and for the common one-full-block call the input block,
// the overlap and the two-stage tail slices.  After the MAC the FFT / C2R /
// overlap-add tail then runs out of LDS and registers only.
// ---------------------------------------------------------------------------
// returns true when the call ran the pipelined step without a C2R error and
// left a multi-call launch's chain state in LDS (RunCarry::hot)
template <int LOG2B, int NT, bool ZZ, bool NTL, bool RUN = false>
__device__ __forceinline__ bool process_job(const ProcArgs &a, const ProcJob &J, const size_t c, const int4 st,
                                            unsigned char *smem, RunCarry *rc = nullptr) {
    using Gm = Geo<LOG2B, NT>;
    constexpr int B = Gm::B, VEC = Gm::VEC, F = Gm::F, G = Gm::G, SPT = Gm::SPT;
    constexpr float invN = 1.0f / (float)(2 * B);
    using vec_t = typename VecT<VEC>::type;

    float2 *bufA = reinterpret_cast<float2 *>(smem);
    float2 *bufB = bufA + B;
    vec_t *red = reinterpret_cast<vec_t *>(bufB + B);
    int &s_err = *reinterpret_cast<int *>(smem + Gm::lds_bytes - 16);

    const int tid = threadIdx.x;
    int cur = st.x;
    const int act = st.y;
    int fill = st.z;
    int flags = st.w;
    float *outc = J.out + c * J.out_stride;
    const float *inc = J.in + c * J.in_stride;
    const int n = J.n;

    if (act == 0) {  // :216-219 -- zero output, state untouched
        for (int j = tid; j < n; j += NT) outc[j] = 0.f;
        twostage_epilogue<NT>(J, c, outc, inc, n);
        return false;
    }

    if constexpr (Gm::PIPE) {
        if (a.pipe && fill == 0 && n == B && !(flags & FLAG_INBUF) && (flags & FLAG_PRE) && cur < act && !ZZ)
            return pipelined_step<LOG2B, NT, NTL, RUN>(a, J, c, cur, act, flags, smem, rc);
    }

    const size_t rows = (size_t)J.S * B;
    const float2 *Hc = J.H + c * rows;
    float2 *Xc = J.X + c * rows;
    float *ovc = J.overlap + c * B;
    float *ibc = J.inbuf + c * B;
    float2 *prec = J.pre + c * B;

    // slot ownership: the MAC splits rows over G groups; the owner of slot f
    // after the reduction is thread f (G > 1) or thread f % NT (G == 1).
    const int f0 = G > 1 ? tid % F : tid;
    // a row group spans whole waves when F >= 64: make g wave-uniform so the
    // row walk (i, xi, row addresses) lives in scalar registers
    const int g = G > 1 ? (F >= 64 ? __builtin_amdgcn_readfirstlane(tid / F) : tid / F) : 0;
    const bool owner = G > 1 ? tid < F : true;

    // ---- prologue: loads independent of the MAC ------------------------------
    constexpr bool PF = Gm::PREFETCH;
    float2 *twl = reinterpret_cast<float2 *>(smem + 2 * (size_t)B * sizeof(float2) + Gm::red_bytes);
    float2 *h0l = twl + 2 * B;
    float *ovl = reinterpret_cast<float *>(h0l + B);
    float *p0l = ovl + B;
    float *p1l = p0l + B;
    // the common call: exactly one full block from an empty input buffer
    const bool one_block = PF && fill == 0 && n == B && !(flags & FLAG_INBUF);
    const bool epi = J.add0 != nullptr || J.tin != nullptr;
    // far-row windows (B >= 1024): pre_multiplied is summed as
    // rows 1..sp-1 plus rows sp..act-1, in every launch of such a batch, so
    // the result does not depend on which steps read a window; a one-block
    // call of a channel whose window is live reads the far part from it
    constexpr bool GW = G == 1 && VEC == 2 && !ZZ && LOG2B >= 10;
    const int sp = GW && a.gw_p > 0 && act > a.gw_p ? a.gw_p : 0;
    const bool gwin = sp && a.gw && fill == 0 && n == B && !(flags & (FLAG_INBUF | FLAG_PRE)) && (flags & FLAG_GW);
    if constexpr (PF) {
        dma_16b<NT>(twl, a.tw, 2 * B * (int)sizeof(float2));
        if constexpr (B >= 2) dma_16b<NT>(h0l, Hc, B * (int)sizeof(float2));
        else dma_f32<NT>(reinterpret_cast<float *>(h0l), reinterpret_cast<const float *>(Hc), 2 * B);
        if (one_block) {
            // the zero-padded block, packed z[m] = (x[2m], x[2m+1]): x[0..B) lands
            // as raw floats in bufA[0..B/2), the padding half is zero
            dma_f32<NT>(reinterpret_cast<float *>(bufA), inc, B);
            if constexpr (B >= 2) {
                for (int m = B / 2 + tid; m < B; m += NT) bufA[m] = make_float2(0.f, 0.f);
            } else {
                if (tid == 0) bufA[0].y = 0.f;  // x[1] is padding when B == 1
            }
            dma_f32<NT>(ovl, ovc, B);
            if (J.add0) dma_f32<NT>(p0l, J.add0 + c * J.add_stride, B);
            if (J.add1) dma_f32<NT>(p1l, J.add1 + c * J.add_stride, B);
        }
    }
    const float2 *tw = PF ? twl : a.tw;
    const float2 *h0g = PF ? h0l : Hc;

    vec_t pacc[SPT];
    if (fill != 0 && owner) {  // a partial block carries pre_multiplied over
#pragma unroll
        for (int s = 0; s < SPT; ++s) pacc[s] = reinterpret_cast<const vec_t *>(prec)[f0 + s * NT];
    }

    int processed = 0;
    bool err = false, pre_next = false;
    bool t0w = false;  // (a run's two-stage head: this call wrote its block's spectrum to t0x)
    for (;;) {
        const bool was_empty = fill == 0;                               // :223
        const int k = min(n - processed, B - fill);                      // :224-227
        if (processed >= n) {
            // a full-block call that ended on a block boundary: one more MAC
            // pass (no transform) computes the next block's pre_multiplied so
            // the following full-block call takes pipelined_step
            if (!Gm::PIPE || ZZ || !a.pipe || n != B || !was_empty || (flags & FLAG_PRE) || cur >= act) break;
            pre_next = true;
        }

        if (was_empty && (flags & FLAG_PRE) && cur < act) {
            // pre[] already holds this block's pre_multiplied (computed at the
            // end of the previous block)
            if (owner) {
#pragma unroll
                for (int s = 0; s < SPT; ++s) pacc[s] = reinterpret_cast<const vec_t *>(prec)[f0 + s * NT];
            }
        } else if (was_empty) {                                          // :244-255
            AccT<VEC> acc[SPT];
            mac_rows<LOG2B, NT, ZZ, NTL>(acc, Hc, Xc, J.S, cur, act, 1, sp ? sp : act, flags, f0, g);
            if constexpr (GW) {
#pragma unroll
                for (int s = 0; s < SPT; ++s) pacc[s] = acc[s].get(f0 + s * NT);
                // far rows sp..act-1: this block's window row (the anchor
                // summed them, gw_anchor_kernel), else summed here; near +
                // far either way
                if (gwin) {
                    const int k = (int)(((long long)a.gw_t - 1 - (long long)c) % sp + sp) % sp;
                    DBG_CHECK(k >= 0 && k < sp, 40, k, a.gw_t, sp, (int)c);
                    const float4 *wr = reinterpret_cast<const float4 *>(a.gw + ((size_t)c * sp + k) * B);
#pragma unroll
                    for (int s = 0; s < SPT; ++s) pacc[s] = vadd(pacc[s], ntld4(wr + f0 + s * NT));
                } else if (sp) {  // (acc reused: one accumulator set live)
                    mac_rows<LOG2B, NT, ZZ, NTL>(acc, Hc, Xc, J.S, cur, act, sp, act, flags, f0, g);
#pragma unroll
                    for (int s = 0; s < SPT; ++s) pacc[s] = vadd(pacc[s], acc[s].get(f0 + s * NT));
                }
            } else if constexpr (G > 1) {
                red[g * F + f0] = acc[0].get(f0);
                __syncthreads();
                if (owner) {
                    vec_t p = red[f0];
#pragma unroll
                    for (int q = 1; q < G; ++q) p = vadd(p, red[q * F + f0]);
                    pacc[0] = p;
                }
            } else {
#pragma unroll
                for (int s = 0; s < SPT; ++s) pacc[s] = acc[s].get(f0 + s * NT);
            }
        }
        if (pre_next) {
            flags |= FLAG_PRE;
            break;
        }
        proc_stamp(a, 0);  // (timelines: pre_multiplied ready)

        // forward FFT of the zero-padded input buffer into segments[current]
        // (:229-241): x[i] = chunk sample, else the carried input buffer.
        if (one_block) {
            // the block is already in bufA (prologue DMA); two-stage: append it
            // to tail_input from LDS (:459-461)
            __syncthreads();
            if (J.tin) {
                const float *xb = reinterpret_cast<const float *>(bufA);
                float *ti = J.tin + c * J.tin_stride;
                for (int j = tid; j < B; j += NT) ti[j] = xb[j];
            }
        } else {
            for (int m = tid; m < B; m += NT) {
                float2 z = make_float2(0.f, 0.f);
                const int i0 = 2 * m, i1 = 2 * m + 1;
                if (i0 < B) {
                    z.x = (i0 >= fill && i0 < fill + k) ? inc[processed + i0 - fill]
                                                         : ((flags & FLAG_INBUF) ? ibc[i0] : 0.f);
                }
                if (i1 < B) {
                    z.y = (i1 >= fill && i1 < fill + k) ? inc[processed + i1 - fill]
                                                         : ((flags & FLAG_INBUF) ? ibc[i1] : 0.f);
                }
                bufA[m] = z;
            }
        }
        if (tid == 0) s_err = 0;
        __syncthreads();
        float2 *Z = lds_cfft<LOG2B, NT, false>(bufA, bufB, tw);
        float2 *Q = Z == bufA ? bufB : bufA;
        float2 *Xcur = Xc + (size_t)cur * B;
        // (a run's two-stage head: tail0's copy of a whole block's spectrum)
        float2 *t0r = J.t0x && fill == 0 && k == B ? J.t0x + c * J.t0x_stride : nullptr;
        t0w = t0w || t0r != nullptr;
        for (int m = tid; m < B; m += NT) {
            const float2 v = real_post<LOG2B, NT>(Z, m, tw);
            Q[m] = v;
            Xcur[m] = v;
            if (t0r) t0r[m] = v;
        }
        __syncthreads();
        proc_stamp(a, 1);  // (R2C done)

        // conv = pre_multiplied + segments[current] (.) segments_ir[0] (:256-261)
        if (owner) {
            const vec_t *q = reinterpret_cast<const vec_t *>(Q);
            vec_t *zc = reinterpret_cast<vec_t *>(Z);
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                const int f = f0 + s * NT;
                const vec_t cv = slot_mac(pacc[s], q[f], reinterpret_cast<const vec_t *>(h0g)[f], f);
                zc[f] = cv;
                // realfft's C2R rejects a non-zero DC/Nyquist imaginary part
                // (:264-267), which only a non-finite operand produces
                if (f == 0 && !slot0_finite(cv) &&
                    c2r_rejects(Hc, Xc, B, cur, act, slot0_of(pacc[s]), slot0_of(q[f]),
                                slot0_of(reinterpret_cast<const vec_t *>(h0g)[f])))
                    s_err = 1;
            }
        }
        __syncthreads();
        if (s_err) { err = true; break; }

        // inverse FFT (:264) with the 1/N of Fft::inverse (:44-46)
        for (int m = tid; m < B; m += NT) Q[m] = real_pre<LOG2B, NT>(Z, m, tw);
        __syncthreads();
        float2 *Y = lds_cfft<LOG2B, NT, true>(Q, Z, tw);
        const float *y = reinterpret_cast<const float *>(Y);
        proc_stamp(a, 2);  // (C2R done)

        // overlap-add (:270-274)
        if (one_block) {
            for (int j = tid; j < B; j += NT) {
                float v = y[j] * invN + ovl[j];
                if (J.add0) {  // two-stage sub-chunk adds (:439-454), same rounding order
                    v += p0l[j];
                    if (J.add1) v += p1l[j];
                }
                outc[j] = v;
            }
        } else {
            for (int j = tid; j < k; j += NT) outc[processed + j] = y[fill + j] * invN + ovc[fill + j];
        }
        const bool complete = fill + k == B;                              // :277-278
        if (complete) {
            if (!one_block) __syncthreads();  // every overlap read above is done
            for (int j = tid; j < B; j += NT) ovc[j] = y[B + j] * invN;  // :283-284
            if (flags & FLAG_INBUF)
                for (int j = tid; j < B; j += NT) ibc[j] = 0.f;           // :280
            flags &= ~(FLAG_INBUF | FLAG_PRE);
            flags ^= FLAG_REV;
            fill = 0;
            cur = cur > 0 ? cur - 1 : act - 1;                            // :287-291
        } else {
            for (int j = tid; j < k; j += NT) ibc[fill + j] = inc[processed + j];
            flags |= FLAG_INBUF;
            fill += k;
        }
        processed += k;
        __syncthreads();
    }

    if (err) {
        // output.fill(0); return -- state stays at the failing chunk: its
        // input is in the buffer, fill and current unchanged.
        const int k = min(n - processed, B - fill);
        for (int j = tid; j < k; j += NT) ibc[fill + j] = inc[processed + j];
        flags |= FLAG_INBUF;
        for (int j = tid; j < n; j += NT) outc[j] = 0.f;
    }
    if ((fill != 0 || err || pre_next) && owner) {
#pragma unroll
        for (int s = 0; s < SPT; ++s) reinterpret_cast<vec_t *>(prec)[f0 + s * NT] = pacc[s];
    }
    // (a live window stays live only across a step that read it and advanced)
    if (tid == 0) J.state[c] = make_int4(cur, act, fill, la_clear(flags, a) | (gwin && !err ? FLAG_GW : 0));
    // a run's call whose head buffer is out of step with tail_input wrote no
    // spectrum for tail0's pending block: the flush recomputes this channel's
    if (J.t0x && !t0w && tid == 0) J.t0m[c] = 1;
    if (epi && (!one_block || err)) twostage_epilogue<NT>(J, c, outc, inc, n);
    proc_stamp(a, 3);
    return false;
}

// ---------------------------------------------------------------------------
// Far-row windows of the generic step (B >= 1024).  After step t
// of a batch, the channels of class t mod P (c = t mod P + P j) sum, for each
// of their next P blocks k = 0..P-1 (current = cur' - k, cur' = the state
// after step t), the far rows
//   W[k] = sum_{i=P}^{act-1} H[i] (.) X[(cur' - k + i) % act]
// (src/fft_convolver.rs:244-255 restricted to i >= P): rows written by block t
// or earlier, still in the ring at block t+1+k.  One pass over the far rows
// serves all P windows -- each X row meets P IR rows from a register ring.
// Each window accumulates its rows in the step's order with the step's
// arithmetic (Acc2), so near + W is bit-identical to the step summing the
// far rows itself.  A workgroup: one channel, 256 slots (512 bins).  Channels
// whose ring is off the block path (a buffered partial block, a failed C2R)
// or too short get no window: FLAG_GW cleared.
// long blocks (B > 2^kMaxLog2Fused): windows K0 .. K0+KH-1 of one slot, the
// far rows walked P at a time, software-pipelined (the next P rows' loads
// issued before this batch's MACs); each window sums its rows in the same
// order and arithmetic as the full walk below
#ifndef FFTCONV_GW_SPLIT
#define FFTCONV_GW_SPLIT 1  // threads per slot (2: window halves per thread, 41.9 vs 30.4 us at lgu, rejected)
#endif
template <int LOG2B, int K0, int KH>
__device__ __forceinline__ void gw_walk_long(Acc2 (&w)[KH], const float4 *H4, const float4 *X4, int cur, int act) {
    constexpr int F = (1 << LOG2B) / 2, P = kGwP;
    float4 xr[P];  // X at ring offset o (from cur') in xr[o % P]
#pragma unroll
    for (int o = 1; o < P; ++o) xr[o] = ntld4(X4 + (size_t)((cur + o) % act) * F);
    xr[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    int i0 = P;
    float4 h[P], xn[P];
    if (i0 + P <= act) {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            h[j] = ntld4(H4 + (size_t)(i0 + j) * F);
            xn[j] = ntld4(X4 + (size_t)((cur + i0 + j) % act) * F);
        }
    }
    for (; i0 + P <= act; i0 += P) {
        float4 h2[P], x2[P];
        const bool more = i0 + 2 * P <= act;
        if (more) {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                h2[j] = ntld4(H4 + (size_t)(i0 + P + j) * F);
                x2[j] = ntld4(X4 + (size_t)((cur + i0 + P + j) % act) * F);
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int kk = 0; kk < KH; ++kk) {
                const int k = K0 + kk;
                w[kk].mac(h[j], j >= k ? xn[j - k] : xr[j - k + P]);
            }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            xr[j] = xn[j];
            if (more) {
                h[j] = h2[j];
                xn[j] = x2[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
        if (i0 + j < act) {
            const float4 hv = ntld4(H4 + (size_t)(i0 + j) * F);
            xr[j] = ntld4(X4 + (size_t)((cur + i0 + j) % act) * F);
#pragma unroll
            for (int kk = 0; kk < KH; ++kk) w[kk].mac(hv, xr[(j - (K0 + kk) + P) % P]);
        }
    }
}

template <int LOG2B>
__global__ __launch_bounds__(256) void gw_anchor_kernel(ProcArgs a) {
    constexpr int B = 1 << LOG2B, F = B / 2, P = kGwP;
    const ProcJob &J = a.job[0];
    const int cls = a.gw_t % P;
    const int c = cls + P * (int)blockIdx.y;
    if (c >= a.la_channels) return;
    const int4 st = J.state[c];
    const int cur = st.x, act = st.y;
    if (st.z != 0 || (st.w & (FLAG_INBUF | FLAG_PRE)) || act <= P) {
        if (blockIdx.x == 0 && threadIdx.x == 0) J.state[c].w = st.w & ~FLAG_GW;
        return;
    }
    const size_t rows = (size_t)J.S * B;
    if constexpr (LOG2B > kMaxLog2Fused) {
        // long blocks: FFTCONV_GW_SPLIT threads per slot, each summing P / SPLIT
        // of the windows (SPLIT 2 doubles the waves, one per SIMD at 1, but
        // measured slower: anchor 41.9 vs 30.4 us at lgu, r5ar)
        constexpr int SPLIT = FFTCONV_GW_SPLIT, KH = P / SPLIT, SL = 256 / SPLIT;
        static_assert(P % SPLIT == 0 && SL % 64 == 0, "window split");
        const int part = (int)threadIdx.x / SL;  // (wave-uniform)
        const int f = (int)blockIdx.x * SL + (int)threadIdx.x % SL;
        const float4 *H4 = reinterpret_cast<const float4 *>(J.H + (size_t)c * rows) + f;
        const float4 *X4 = reinterpret_cast<const float4 *>(J.X + (size_t)c * rows) + f;
        Acc2 w[KH];
#pragma unroll
        for (int k = 0; k < KH; ++k) w[k].zero();
        if constexpr (SPLIT == 1) {
            gw_walk_long<LOG2B, 0, KH>(w, H4, X4, cur, act);
        } else if constexpr (SPLIT == 2) {
            if (part == 0) gw_walk_long<LOG2B, 0, KH>(w, H4, X4, cur, act);
            else gw_walk_long<LOG2B, KH, KH>(w, H4, X4, cur, act);
        } else {
            static_assert(SPLIT <= 2, "window split");
        }
        float4 *W4 = reinterpret_cast<float4 *>(a.gw + (size_t)c * P * B) + f;
#pragma unroll
        for (int k = 0; k < KH; ++k) ntst4(W4 + (size_t)(part * KH + k) * F, w[k].get(f));
        if (blockIdx.x == 0 && threadIdx.x == 0) J.state[c].w = st.w | FLAG_GW;
        return;
    }
    const int f = (int)blockIdx.x * 256 + (int)threadIdx.x;  // float4 slot
    const float4 *H4 = reinterpret_cast<const float4 *>(J.H + (size_t)c * rows) + f;
    const float4 *X4 = reinterpret_cast<const float4 *>(J.X + (size_t)c * rows) + f;
    Acc2 w[P];
    float4 xr[P];  // X at ring offset o (from cur') in xr[o % P]
#pragma unroll
    for (int k = 0; k < P; ++k) w[k].zero();
#pragma unroll
    for (int o = 1; o < P; ++o) {
        DBG_CHECK((cur + o) % act < J.S, 41, cur, o, act, J.S);
        xr[o] = ntld4(X4 + (size_t)((cur + o) % act) * F);
    }
    // P rows in flight (B <= 8192: the two-stage tail's anchor beside the
    // head on few CUs -- the plain loop's lower register count measured
    // faster there than the pipelined walk of gw_walk_long)
    int i0 = P;
    for (; i0 + P <= act; i0 += P) {
        float4 h[P], xn[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            h[j] = ntld4(H4 + (size_t)(i0 + j) * F);
            xn[j] = ntld4(X4 + (size_t)((cur + i0 + j) % act) * F);
        }
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int k = 0; k < P; ++k) w[k].mac(h[j], j >= k ? xn[j - k] : xr[j - k + P]);
#pragma unroll
        for (int j = 0; j < P; ++j) xr[j] = xn[j];
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
        if (i0 + j < act) {
            const float4 hv = ntld4(H4 + (size_t)(i0 + j) * F);
            xr[j] = ntld4(X4 + (size_t)((cur + i0 + j) % act) * F);
#pragma unroll
            for (int k = 0; k < P; ++k) w[k].mac(hv, xr[(j - k + P) % P]);
        }
    }
    float4 *W4 = reinterpret_cast<float4 *>(a.gw + (size_t)c * P * B) + f;
#pragma unroll
    for (int k = 0; k < P; ++k) ntst4(W4 + (size_t)k * F, w[k].get(f));
    if (blockIdx.x == 0 && threadIdx.x == 0) J.state[c].w = st.w | FLAG_GW;
}

template <int LOG2B, int NT, bool ZZ, bool NTL>
__global__ __launch_bounds__(NT, NT == 512 ? 2 : 4) void upols_process_kernel(ProcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const size_t c = blockIdx.x;
    const ProcJob &J = a.job[blockIdx.y];
    unsigned t0 = 0;
    if (a.la_trace) t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
    process_job<LOG2B, NT, ZZ, NTL>(a, J, c, J.state[c], smem);
    if (a.sig_mode == 1) sig_arrive(a);
    if (a.la_trace && blockIdx.y == 0 && (threadIdx.x >> 6) < 4 && (threadIdx.x & 63) == 0) {
        // launch timeline (FFTCONV_PROC_TRACE, tuning): role 6, as upols_la_kernel's record
        const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
        const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(0xF804);   // HW_REG_HW_ID
        const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
        const int wave = (int)(threadIdx.x >> 6);
        a.la_trace[(size_t)blockIdx.x * 4 + wave] =
            make_int4(6 | (wave << 4), (int)((hw & 0xffffu) | ((xcc & 0xffu) << 24)), (int)t0, (int)t1);
    }
}

// ---------------------------------------------------------------------------
// A run of consecutive process() calls in ONE launch (process_device_steps of
// a TwoStageFFTConvolver inside one tail period): call k is job[0] with its
// input / output advanced by k steps and its two-stage slices (tail
// precalculated, tail_input) by k blocks.  Channels are independent, so each
// workgroup loops over its channel's calls with no grid-wide sync: call k+1
// reads the state, FDL row, pre_multiplied and overlap call k stored, which
// the barrier between calls makes visible to every wave of the workgroup.
// The body is process_job, the one-call kernel's, so the bits are the same.
// The kernel boundary between calls goes away (cfg3's head: ~1 us of its
// ~4.9 us per launch).  At most 2 workgroups per CU (256 VGPRs):
// the loop keeps its addresses live, and a 128-VGPR body spilled (r4p).
// ---------------------------------------------------------------------------
template <int LOG2B, int NT, bool NTL>
__global__ __launch_bounds__(NT, 2) void upols_run_kernel(ProcArgs a, RunSteps r) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const size_t c = blockIdx.x;
    ProcJob J = a.job[0];
    RunCarry rc{};
    // (issue priority over the waves of other kernels on the same SIMD: the
    // two-stage tail beside the run; 1 = the chain wave, 2 = every wave)
    if (a.prio == 2 || (a.prio == 1 && threadIdx.x < 64)) __builtin_amdgcn_s_setprio(3);
    if (a.sig_mode == 2) sig_wait(a);  // (the previous tail step's output, which the calls add)
    unsigned t0 = 0;
    using Gm = Geo<LOG2B, NT>;
    const int rl = a.run_lds_rows;  // (the IR rows and the FDL in LDS for the run: their row count)
    if (rl > 0) {
        float2 *hl = reinterpret_cast<float2 *>(smem + Gm::lds_bytes + 4 * (size_t)Gm::B * sizeof(float2));
        rc.hl = hl;
        rc.xl = hl + (size_t)rl * Gm::B;
        dma_16b<NT>(hl, J.H + c * (size_t)J.S * Gm::B, rl * Gm::B * (int)sizeof(float2));
    }
    for (int k = 0; k < r.n; ++k) {
        if (a.la_trace && k == r.n - 1) t0 = (unsigned)__builtin_amdgcn_s_memrealtime();  // (the last call's start)
        if (rl > 0 && !rc.hot) {
            // the FDL into LDS: at the run's start, and after a call that
            // did not run the pipelined step to its end (the generic step and
            // a failed C2R touch only the FDL in memory)
            dma_16b<NT>(rc.xl, J.X + c * (size_t)J.S * Gm::B, rl * Gm::B * (int)sizeof(float2));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        rc.next_in = k + 1 < r.n ? J.in + r.in_step : nullptr;
        // (a hot call's state word is the one the previous call stored; the
        // reload stays behind the branch -- a speculated load would put a
        // memory round trip at the start of every call)
        int4 st = rc.st;
        if (!rc.hot) {
            asm volatile("" ::: "memory");
            st = J.state[c];
        }
        const bool kept = process_job<LOG2B, NT, false, NTL, true>(a, J, c, st, smem, &rc);
        rc.hot = kept && rc.next_in != nullptr;  // (the next call's block is in stage[par ^ 1])
        rc.par ^= 1;
        __syncthreads();
        J.in += r.in_step;
        J.out += r.out_step;
        if (J.add0) J.add0 += J.n;
        if (J.add1) J.add1 += J.n;
        if (J.tin) J.tin += J.n;
        if (J.t0x) J.t0x += J.n;
    }
    if (a.la_trace && (threadIdx.x >> 6) < 4 && (threadIdx.x & 63) == 0) {
        // launch timeline (FFTCONV_PROC_TRACE, tuning): the run's last call,
        // role 6 as upols_process_kernel's record (the phase stamps are that call's)
        const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
        const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(0xF804);   // HW_REG_HW_ID
        const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
        const int wave = (int)(threadIdx.x >> 6);
        a.la_trace[(size_t)blockIdx.x * 4 + wave] =
            make_int4(6 | (wave << 4), (int)((hw & 0xffffu) | ((xcc & 0xffu) << 24)), (int)t0, (int)t1);
    }
}

// ---------------------------------------------------------------------------
// Crossfade mix (src/crossfade_convolver.rs:75-77 + Crossfader::mix :242-278
// + RaisedCosineMixer :160-169), all channels in lockstep.  mix_value is
// walked by the same sequential f32 additions the reference performs (once
// per workgroup into LDS, or per sample for calls longer than 1024), so the
// gains are bit-identical to a serial walk.
// ---------------------------------------------------------------------------
// Crossfader::mix for sample j of the call.  vtab (if given) holds the
// sequential mix_value walk: vtab[k] = mix_value0 + step + ... (k adds).
// RaisedCosineMixer (:160-169): gain g1 = cos^2(pi/2 * v) of A, 1 - g1 of B
__device__ __forceinline__ float mix_gain(float v) {
    const float PI_HALF = 3.14159265358979323846f * 0.5f;
    const float rad = __fmul_rn(PI_HALF, v);
    const float cs = cosf(rad);
    return __fmul_rn(cs, cs);
}
__device__ __forceinline__ float mix_apply(float va, float vb, float g1) {
    const float g2 = __fsub_rn(1.0f, g1);
    return __fadd_rn(__fmul_rn(va, g1), __fmul_rn(vb, g2));
}

__device__ __forceinline__ float mix_sample(const CrossfadeMixArgs &a, int j, float va, float vb,
                                            const float *vtab) {
    if (!a.approaching) return a.target == 0 ? va : vb;
    const long long cj = a.counter0 + j + 1;
    if (cj <= 0) return a.target == 0 ? vb : va;                   // hold the previous target
    if (a.fading >= 1 && cj >= a.fading) return a.target == 0 ? va : vb;  // reached (snap)
    const long long inc = cj - (a.counter0 > 0 ? a.counter0 : 0);
    float v;
    if (vtab) {
        v = vtab[inc];
    } else {
        v = a.mix_value0;
        for (long long q = 0; q < inc; ++q) v = __fadd_rn(v, a.step);
    }
    return mix_apply(va, vb, mix_gain(v));
}

// Crossfader::mix for sample j as a selector word: MIX_SEL_A / MIX_SEL_B take
// that convolver's sample as is (hold, snap, not fading), anything else is the
// gain g1 in [0, 1] of the blend.  mix_select(va, vb, mix_selector(...)) is
// bit-identical to mix_sample.
constexpr float MIX_SEL_A = 2.0f, MIX_SEL_B = 3.0f;
__device__ __forceinline__ float mix_selector(const CrossfadeMixArgs &a, int j, const float *vtab) {
    const float sa = a.target == 0 ? MIX_SEL_A : MIX_SEL_B, sb = a.target == 0 ? MIX_SEL_B : MIX_SEL_A;
    if (!a.approaching) return sa;
    const long long cj = a.counter0 + j + 1;
    if (cj <= 0) return sb;                            // hold the previous target
    if (a.fading >= 1 && cj >= a.fading) return sa;    // reached (snap)
    return mix_gain(vtab[cj - (a.counter0 > 0 ? a.counter0 : 0)]);
}
__device__ __forceinline__ float mix_select(float va, float vb, float sel) {
    return sel == MIX_SEL_A ? va : (sel == MIX_SEL_B ? vb : mix_apply(va, vb, sel));
}

// The mix_value walk of one call into LDS: vtab[k] = v0 + step + ... + step
// (k sequential f32 additions, n + 1 entries), one thread, bit-identical to
// the reference's per-sample `mix_value += step` (:259).  The additions are a
// dependent chain on one lane; unrolled by 8 with the stores batched after
// them, the loop is little more than that chain (the rolled loop -- an
// address, a store and the loop test per add -- took ~9 us for 512 samples in
// the cfg5 step workgroups, more than their whole transform chain, r3).
__device__ __forceinline__ void mix_walk_lane(float *vtab, float v, float step, int n) {
    vtab[0] = v;
    int k = 1;
    for (; k + 7 <= n; k += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            v = __fadd_rn(v, step);
            t[u] = v;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) vtab[k + u] = t[u];
    }
    for (; k <= n; ++k) {
        v = __fadd_rn(v, step);
        vtab[k] = v;
    }
}
__device__ __forceinline__ void mix_walk(const CrossfadeMixArgs &a, float *vtab) {
    mix_walk_lane(vtab, a.mix_value0, a.step, a.n);
}

// IR transform (init / update): H rows stored nontemporal, so the window
// rebuild behind it finds them written out instead of dirty in L2 (cfg2
// update: rebuild 277 -> 261 us, cfg2u +1.1 %, profiles/r5/r5i_*)
#ifndef FFTCONV_IR_NTST
#define FFTCONV_IR_NTST 1
#endif
#include "la.hpp"  // (after the mix helpers: B's lookahead launch can fuse the mix)

__global__ void crossfade_mix_kernel(CrossfadeMixArgs a) {
    __shared__ float vtab[1025];
    const size_t c = blockIdx.x;
    const float *A = a.buf_a + c * a.buf_stride;
    const float *Bv = a.buf_b + c * a.buf_stride;
    float *o = a.out + c * a.out_stride;
    const bool tab = a.approaching && a.n <= 1024;
    if (tab) {
        if (threadIdx.x == 0) mix_walk(a, vtab);
        __syncthreads();
    }
    const float *vt = tab ? vtab : (a.approaching ? a.vtab : nullptr);
    for (int j = threadIdx.x; j < a.n; j += blockDim.x) o[j] = mix_sample(a, j, A[j], Bv[j], vt);
}

// the mix_value walk of a call longer than crossfade_mix_kernel's LDS table
// (n > 1024) into a device table, once (one lane), before the mix reads it
__global__ void crossfade_walk_kernel(CrossfadeMixArgs a, float *vtab) {
    if (threadIdx.x == 0) mix_walk(a, vtab);
}

// ---------------------------------------------------------------------------
// Crossfade pair step: CrossfadeConvolver::process (src/crossfade_convolver.rs
// :66-78) runs convolver_a and convolver_b on the same input block.  While
// the two ring states agree (and FLAG_XSYNC says they always have), their
// FDLs are equal row for row, so one workgroup per channel does both with
// one FDL stream (H_A, H_B, X: 24 instead of 32 B per bin-row), one forward
// transform written to both FDL rows, and the two C2Rs.  Each convolver's
// arithmetic is exactly the unpaired kernel's (same sum order): pairing never
// changes a result bit.  Any other call runs the two generic jobs in turn;
// if the states disagree the channel drops FLAG_XSYNC for good.
// B in [2, 512]; LDS: bufA | bufB | bufC | redA | redB | tw | H0a | H0b | ovA | ovB
// ---------------------------------------------------------------------------
template <int LOG2B, int NT>
struct PairGeo {
    using Gm = Geo<LOG2B, NT>;
    static constexpr int B = Gm::B;
    // ... | s_err[2] (16 B) | A's output (B floats) | mix_value walk (B + 1 floats)
    static constexpr size_t pair_bytes = 3 * 8 * (size_t)B + 2 * Gm::red_bytes + 16 * (size_t)B + 16 * (size_t)B +
                                         8 * (size_t)B + 16 + 4 * (size_t)B + 4 * ((size_t)B + 4);
    static constexpr size_t lds_bytes = pair_bytes > Gm::lds_bytes ? pair_bytes : Gm::lds_bytes;
};

template <int LOG2B, int NT, bool NTL>
__device__ __forceinline__ void pair_step(const ProcArgs &a, size_t c, int cur, int act, int flags,
                                          unsigned char *smem) {
    using Gm = Geo<LOG2B, NT>;
    constexpr int B = Gm::B, VEC = Gm::VEC, F = Gm::F, G = Gm::G, SPT = Gm::SPT;
    constexpr float invN = 1.0f / (float)(2 * B);
    using vec_t = typename VecT<VEC>::type;
    static_assert(VEC == 2 && B <= 512, "pair step: 2 <= B <= 512");
    float2 *bufA = reinterpret_cast<float2 *>(smem);
    float2 *bufB = bufA + B;
    float2 *bufC = bufB + B;
    vec_t *redA = reinterpret_cast<vec_t *>(bufC + B);
    vec_t *redB = reinterpret_cast<vec_t *>(reinterpret_cast<unsigned char *>(redA) + Gm::red_bytes);
    float2 *twl = reinterpret_cast<float2 *>(reinterpret_cast<unsigned char *>(redB) + Gm::red_bytes);
    float2 *h0[2] = {twl + 2 * B, twl + 3 * B};
    float *ovl[2] = {reinterpret_cast<float *>(twl + 4 * B), reinterpret_cast<float *>(twl + 4 * B) + B};
    int *s_err = reinterpret_cast<int *>(ovl[1] + B);  // [2]
    float *ya = reinterpret_cast<float *>(s_err + 4);   // A's output, for the fused mix
    float *vtab = ya + B;                               // mix_value walk
    const bool fuse = a.fuse_mix != 0;

    const ProcJob *Js[2] = {&a.job[0], &a.job[1]};
    const int tid = threadIdx.x;
    const size_t rows = (size_t)Js[0]->S * B;
    const float2 *Hc[2] = {Js[0]->H + c * rows, Js[1]->H + c * rows};
    const float *inc = Js[0]->in + c * Js[0]->in_stride;
    const int f0 = G > 1 ? tid % F : tid;
    const int g = G > 1 ? (F >= 64 ? __builtin_amdgcn_readfirstlane(tid / F) : tid / F) : 0;
    const bool owner = G > 1 ? tid < F : true;

    // prologue (LDS-DMA): twiddles, both H[0], the packed block, both overlaps
    dma_16b<NT>(twl, a.tw, 2 * B * (int)sizeof(float2));
    dma_16b<NT>(h0[0], Hc[0], B * (int)sizeof(float2));
    dma_16b<NT>(h0[1], Hc[1], B * (int)sizeof(float2));
    dma_f32<NT>(reinterpret_cast<float *>(bufA), inc, B);
    for (int m = B / 2 + tid; m < B; m += NT) bufA[m] = make_float2(0.f, 0.f);
    dma_f32<NT>(ovl[0], Js[0]->overlap + c * B, B);
    dma_f32<NT>(ovl[1], Js[1]->overlap + c * B, B);
    // the crossfader's mix_value walk (one lane; hides under the FDL stream)
    if (fuse && a.mix.approaching && tid == 0) mix_walk(a.mix, vtab);

    // both pre_multiplied from one FDL stream (:244-255)
    vec_t pacc[2][SPT];
    {
        AccT<VEC> accA[SPT], accB[SPT];
        mac_rows_pair<LOG2B, NT, NTL>(accA, accB, Hc[0], Hc[1], Js[0]->X + c * rows, Js[0]->S, cur, act, f0, g);
        if constexpr (G > 1) {
            redA[g * F + f0] = accA[0].get(f0);
            redB[g * F + f0] = accB[0].get(f0);
            __syncthreads();
            if (owner) {
                vec_t p = redA[f0], q = redB[f0];
#pragma unroll
                for (int r = 1; r < G; ++r) {
                    p = vadd(p, redA[r * F + f0]);
                    q = vadd(q, redB[r * F + f0]);
                }
                pacc[0][0] = p;
                pacc[1][0] = q;
            }
        } else {
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                pacc[0][s] = accA[s].get(f0 + s * NT);
                pacc[1][s] = accB[s].get(f0 + s * NT);
            }
        }
    }
    if (tid < 2) s_err[tid] = 0;
    __syncthreads();

    // one R2C (:229-241), written to both FDL rows `current`
    float2 *Z = lds_cfft<LOG2B, NT, false>(bufA, bufB, twl);
    float2 *W = Z == bufA ? bufB : bufA;
    float2 *XA = Js[0]->X + c * rows + (size_t)cur * B;
    float2 *XB = Js[1]->X + c * rows + (size_t)cur * B;
    for (int m = tid; m < B; m += NT) {
        const float2 v = real_post<LOG2B, NT>(Z, m, twl);
        bufC[m] = v;
        XA[m] = v;
        XB[m] = v;
    }
    __syncthreads();

    for (int j = 0; j < 2; ++j) {
        const ProcJob &J = *Js[j];
        // conv = pre + X (.) H[0] (:256-261), then the C2R error check
        if (owner) {
#pragma unroll
            for (int s = 0; s < SPT; ++s) {
                const int f = f0 + s * NT;
                const vec_t cv = slot_mac(pacc[j][s], reinterpret_cast<const vec_t *>(bufC)[f],
                                          reinterpret_cast<const vec_t *>(h0[j])[f], f);
                reinterpret_cast<vec_t *>(Z)[f] = cv;
                if (f == 0 && !slot0_finite(cv) &&
                    c2r_rejects(J.H + c * rows, Js[0]->X + c * rows, B, cur, act, slot0_of(pacc[j][s]),
                                slot0_of(reinterpret_cast<const vec_t *>(bufC)[f]),
                                slot0_of(reinterpret_cast<const vec_t *>(h0[j])[f])))
                    s_err[j] = 1;
            }
        }
        __syncthreads();
        float *outc = J.out + c * J.out_stride;
        if (!s_err[j]) {
            for (int m = tid; m < B; m += NT) W[m] = real_pre<LOG2B, NT>(Z, m, twl);
            __syncthreads();
            const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2B, NT, true>(W, Z, twl));
            float *ovc = J.overlap + c * B;
            for (int k = tid; k < B; k += NT) {
                const float v = y[k] * invN + ovl[j][k];  // :270-274
                ovc[k] = y[B + k] * invN;                  // :283-284
                if (!fuse) {
                    outc[k] = v;
                } else if (j == 0) {
                    ya[k] = v;
                } else if (k < a.mix.n) {                  // crossfade_convolver.rs:75-77
                    a.mix.out[c * a.mix.out_stride + k] = mix_sample(a.mix, k, ya[k], v, vtab);
                }
            }
            if (tid == 0) J.state[c] = make_int4(cur > 0 ? cur - 1 : act - 1, act, 0, la_clear((flags & ~FLAG_INBUF) ^ FLAG_REV, a));
        } else {
            // output.fill(0); return (:264-267): block kept in the input buffer
            float *ibc = J.inbuf + c * B;
            for (int k = tid; k < B; k += NT) {
                if (!fuse) outc[k] = 0.f;
                else if (j == 0) ya[k] = 0.f;
                else if (k < a.mix.n) a.mix.out[c * a.mix.out_stride + k] = mix_sample(a.mix, k, ya[k], 0.f, vtab);
                ibc[k] = inc[k];
            }
            if (owner) {
#pragma unroll
                for (int s = 0; s < SPT; ++s) reinterpret_cast<vec_t *>(J.pre + c * B)[f0 + s * NT] = pacc[j][s];
            }
            if (tid == 0) J.state[c] = make_int4(cur, act, 0, la_clear(flags | FLAG_INBUF, a));
        }
        __syncthreads();  // Z / W are reused by the next convolver
    }
}

// the generic body for both jobs in turn, out of line: the rare fallback
// keeps its registers out of the pair step's allocation
template <int LOG2B, int NT, bool NTL>
__device__ __attribute__((noinline)) void pair_fallback(const ProcArgs &a, size_t c, int4 sa, int4 sb,
                                                        unsigned char *smem) {
    process_job<LOG2B, NT, false, NTL>(a, a.job[0], c, sa, smem);
    __syncthreads();
    process_job<LOG2B, NT, false, NTL>(a, a.job[1], c, sb, smem);
    if (a.fuse_mix) {  // the jobs wrote buf_a / buf_b (this workgroup's own stores)
        __threadfence_block();
        __syncthreads();
        const float *A = a.mix.buf_a + c * a.mix.buf_stride, *Bv = a.mix.buf_b + c * a.mix.buf_stride;
        for (int k = threadIdx.x; k < a.mix.n; k += NT)
            a.mix.out[c * a.mix.out_stride + k] = mix_sample(a.mix, k, A[k], Bv[k], nullptr);
    }
}

// (2 waves/SIMD suffice: C workgroups of 3 streams x 8 rows x 16 B per lane
// in flight; the rarely-taken generic fallback then needs no spills)
template <int LOG2B, int NT, bool NTL>
__global__ __launch_bounds__(NT, 2) void upols_pair_kernel(ProcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const size_t c = blockIdx.x;
    int4 sa = a.job[0].state[c], sb = a.job[1].state[c];
    constexpr int KEY = FLAG_INBUF | FLAG_REV | FLAG_PRE;
    const bool same = sa.x == sb.x && sa.y == sb.y && sa.z == sb.z && ((sa.w ^ sb.w) & KEY) == 0;
    if (same && (sa.w & sb.w & FLAG_XSYNC) && sa.y > 0 && sa.z == 0 && a.job[0].n == (1 << LOG2B) &&
        !(sa.w & (FLAG_INBUF | FLAG_PRE)) && sa.x < sa.y) {
        pair_step<LOG2B, NT, NTL>(a, c, sa.x, sa.y, sa.w, smem);
        return;
    }
    if (!same) {  // the rings have diverged (a C2R error in one of them): never pair again
        sa.w &= ~FLAG_XSYNC;
        sb.w &= ~FLAG_XSYNC;
    }
    pair_fallback<LOG2B, NT, NTL>(a, c, sa, sb, smem);
}

// ---------------------------------------------------------------------------
// IR partition: FFTConvolver::init (:131-142) / update (:190-212).
// grid (S, channels): workgroup (i, c) transforms segment i of channel
// chan0 + c; segments at or past ceil(len_active / B) are zeroed.
// ---------------------------------------------------------------------------
template <int LOG2B, int NT>
__global__ __launch_bounds__(NT) void ir_segments_kernel(IrArgs a) {
    constexpr int B = 1 << LOG2B;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *bufA = reinterpret_cast<float2 *>(smem);
    float2 *bufB = bufA + B;
    const int tid = threadIdx.x;
    const int i = blockIdx.x;
    const size_t c = a.chan0 + blockIdx.y;
    const size_t rows = (size_t)a.S * B;
    float2 *row = a.H + c * rows + (size_t)i * B;
    const long long active = (a.len_active + B - 1) / B;

    if (a.update_state && i == 0) {
        // update(): zero overlap / pre_multiplied / conv, set active (:185-190)
        for (int j = tid; j < B; j += NT) {
            a.overlap[c * B + j] = 0.f;
            a.pre[c * B + j] = make_float2(0.f, 0.f);
        }
        if (tid == 0) {
            a.state[c].y = (int)active;
            a.state[c].w &= ~(FLAG_PRE | LA_MASK | SEQ_MASK);  // the stored pre / window used the old response
        }
    }
    if (i >= active) {  // :210-212
        for (int j = tid; j < B; j += NT) row[j] = make_float2(0.f, 0.f);
        return;
    }
    const float *src = a.src + blockIdx.y * a.src_stride;
    const long long base = (long long)i * B;
    for (int m = tid; m < B; m += NT) {
        const long long i0 = base + 2 * m, i1 = base + 2 * m + 1;
        float2 z;
        z.x = (2 * m < B && i0 < a.len_data) ? src[i0] : 0.f;
        z.y = (2 * m + 1 < B && i1 < a.len_data) ? src[i1] : 0.f;
        bufA[m] = z;
    }
    __syncthreads();
    const float2 *Z = lds_cfft<LOG2B, NT, false>(bufA, bufB, a.tw);
    for (int m = tid; m < B; m += NT) row[m] = real_post<LOG2B, NT>(Z, m, a.tw);
}

// The same transforms one segment per wave (64 <= B <= 1024), each wave
// walking IR_SPW segments and loading the next segment's samples into
// registers while it transforms the current one (the transform was a
// dependent load -> FFT -> store chain per segment).  For B >= 128 (M = B
// complex points, the upper half the zero padding):
//  * stage 0 runs in registers from the loaded samples (wave_stage0_padded:
//    two of a butterfly's four inputs are padding), so neither the samples
//    nor the padding go through LDS;
//  * the middle stages read the per-stage twiddle table (TwStaged: gathered
//    once per workgroup, consecutive entries per stage -- the full table's
//    strided reads were the kernel's LDS bank conflicts);
//  * the last stage and realfft's post-twiddle run in registers with the
//    mirror bin fetched by __shfl (wave_r2c_post), straight to HBM.
// Same butterflies and twiddle values in the same order as
// ir_segments_kernel, so the same bits.
//  * B >= 128: the middle stages run in place (wave_stages_inplace), so a
//    wave needs one B-point buffer and a workgroup runs IR_NW = 8 waves --
//    twice the segment loads in flight per CU of the ping-pong layout.
// grid (ceil(S / (NW * IR_SPW)), channels); LDS: tw (2B) | NW x bufA (| bufB: B < 128)
#ifndef FFTCONV_IR_SPW
#define FFTCONV_IR_SPW 2
#endif
constexpr int IR_SPW = FFTCONV_IR_SPW;
// segments loaded ahead of the one being transformed (1: the next one only)
#ifndef FFTCONV_IR_PF
#define FFTCONV_IR_PF 1
#endif
constexpr int IR_PF = FFTCONV_IR_PF;
static_assert(IR_PF >= 1 && IR_PF <= IR_SPW, "prefetch depth");
template <int LOG2B>
constexpr int ir_nw() { return LOG2B >= 7 ? 8 : 4; }
template <int LOG2B>
constexpr size_t ir_wave_lds() { return (size_t)(2 + ir_nw<LOG2B>() * (LOG2B >= 7 ? 1 : 2)) * (1 << LOG2B) * sizeof(float2); }
template <int LOG2B>
__global__ __launch_bounds__(64 * ir_nw<LOG2B>()) void ir_segments_wave_kernel(IrArgs a) {
    constexpr int B = 1 << LOG2B;
    constexpr bool REG = LOG2B >= 7;                        // register stage 0 / __shfl last stage
    constexpr int NW = ir_nw<LOG2B>(), NT = 64 * NW;
    constexpr int NPL = REG ? stage0_per_lane<LOG2B>() : (B / 2 + 63) / 64;  // per lane: butterflies / points
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *twl = reinterpret_cast<float2 *>(smem);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float2 *bufA = twl + 2 * B + (size_t)wave * (REG ? 1 : 2) * B;
    float2 *bufB = bufA + B;
    const size_t c = a.chan0 + blockIdx.y;
    const size_t rows = (size_t)a.S * B;
    const long long active = (a.len_active + B - 1) / B;
    if constexpr (REG) tws_build<LOG2B, NT>(twl, a.tw, tid);
    else dma_16b<NT>(twl, a.tw, 2 * B * (int)sizeof(float2));
    if (a.update_state && blockIdx.x == 0) {
        // update(): zero overlap / pre_multiplied / conv, set active (:185-190)
        for (int j = tid; j < B; j += NT) {
            a.overlap[c * B + j] = 0.f;
            a.pre[c * B + j] = make_float2(0.f, 0.f);
        }
        if (tid == 0) {
            a.state[c].y = (int)active;
            a.state[c].w &= ~(FLAG_PRE | LA_MASK | SEQ_MASK);  // the stored pre / window used the old response
        }
    }
    const float *src = a.src + blockIdx.y * a.src_stride;
    // (a channel's response 8-byte aligned: a point inside the data is one
    // 8-byte load, half the load instructions of two 4-byte ones)
    const bool al8 = ((uintptr_t)src & 7) == 0;
    // copy_and_pad (:56-60) of segment i as packed points z[m] = (x[2m], x[2m+1]), m < B/2
    auto point = [&](long long base, int m) {
        const long long i0 = base + 2 * m, i1 = i0 + 1;
        if (al8 && 2 * m + 1 < B && i1 < a.len_data) return *reinterpret_cast<const float2 *>(src + i0);
        float2 z;
        z.x = (2 * m < B && i0 < a.len_data) ? src[i0] : 0.f;
        z.y = (2 * m + 1 < B && i1 < a.len_data) ? src[i1] : 0.f;
        return z;
    };
    // REG: lo[t] = z[j], hi[t] = z[j + B/4] for butterflies j = lane + 64 t < B/4;
    // else lo[u] = z[lane + 64 u]
    auto load = [&](int i, float2 (&lo)[NPL], float2 (&hi)[NPL]) {
        const long long base = (long long)i * B;
#pragma unroll
        for (int u = 0; u < NPL; ++u) {
            const int m = lane + 64 * u;
            if constexpr (REG) {
                if (m < B / 4) {
                    lo[u] = point(base, m);
                    hi[u] = point(base, m + B / 4);
                }
            } else {
                lo[u] = point(base, m);
            }
        }
    };
    const int i0 = (blockIdx.x * NW + wave) * IR_SPW;
    // a ring of IR_PF + 1 segments in registers: segment q + IR_PF is loaded
    // while segment q is transformed (the loop is unrolled, so every ring
    // index is a constant and no in-flight load is ever copied)
    constexpr int RING = IR_PF + 1;
    float2 rl[RING][NPL], rh[RING][NPL];
#pragma unroll
    for (int k = 0; k < IR_PF && k < IR_SPW; ++k)
        if (i0 + k < a.S && i0 + k < active) load(i0 + k, rl[k], rh[k]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (the twiddle table)
#pragma unroll
    for (int q = 0; q < IR_SPW; ++q) {
        const int i = i0 + q;
        if (i >= a.S) break;
        float2 *row = a.H + c * rows + (size_t)i * B;
        if (q + IR_PF < IR_SPW && i + IR_PF < a.S && i + IR_PF < active)
            load(i + IR_PF, rl[(q + IR_PF) % RING], rh[(q + IR_PF) % RING]);  // (in flight under these FFTs)
        if (i >= active) {  // :210-212
            for (int m = lane; m < B; m += 64) row[m] = make_float2(0.f, 0.f);
            continue;
        }
        float2(&cur)[NPL] = rl[q % RING];
        if constexpr (REG) {
            wave_stage0_padded<LOG2B>(cur, rh[q % RING], bufA);
            wave_sync();
            wave_r2c_post<LOG2B, 1, TwStaged<LOG2B>, true, (FFTCONV_IR_NTST != 0)>(bufA, nullptr, TwStaged<LOG2B>{twl},
                                                                                 nullptr, row);
        } else {
#pragma unroll
            for (int u = 0; u < NPL; ++u) {
                const int m = lane + 64 * u;
                if (m < B) bufA[m] = m < B / 2 ? cur[u] : make_float2(0.f, 0.f);
            }
            for (int m = B / 2 + lane; m < B; m += 64) bufA[m] = make_float2(0.f, 0.f);
            wave_sync();
            const float2 *Z = lds_cfft<LOG2B, 64, false, true>(bufA, bufB, twl);
            for (int m = lane; m < B; m += 64) row[m] = real_post<LOG2B, 64>(Z, m, twl);
        }
        wave_sync();  // (the next segment overwrites both buffers)
    }
}

// ---------------------------------------------------------------------------
// Fft::forward / Fft::inverse as a batched API (src/fft_convolver.rs:36-49):
// realfft's even-length algorithm, the same butterflies and twiddles as the
// convolver's transforms, so an IR segment's spectrum here is bit-identical
// to the row the convolver holds for it.  Forward: N reals -> M+1 bins,
// unnormalised, DC / Nyquist imaginary parts exactly 0.  Inverse: M+1 bins ->
// N reals divided by N (:44-46); a non-zero DC / Nyquist imaginary part is
// realfft's FftError::InputValues -- flagged in status, and (like the oracle's
// restatement) the transform runs with those parts taken as 0.
// ---------------------------------------------------------------------------
template <int LOG2M, int NT, bool INV>
__global__ __launch_bounds__(NT) void fft_rows_kernel(FftArgs a) {
    constexpr int M = 1 << LOG2M;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *bufA = reinterpret_cast<float2 *>(smem);
    float2 *bufB = bufA + M;
    const int tid = threadIdx.x;
    const float *in = a.in + (size_t)blockIdx.x * a.in_stride;
    float *out = a.out + (size_t)blockIdx.x * a.out_stride;
    if constexpr (!INV) {
        for (int m = tid; m < M; m += NT) bufA[m] = make_float2(in[2 * m], in[2 * m + 1]);
        __syncthreads();
        const float2 *Z = lds_cfft<LOG2M, NT, false>(bufA, bufB, a.tw);
        for (int k = tid; k < M; k += NT) {
            const float2 v = real_post<LOG2M, NT>(Z, k, a.tw);
            if (k == 0) {  // packed (DC, Nyquist)
                out[0] = v.x;
                out[1] = 0.f;
                out[2 * M] = v.y;
                out[2 * M + 1] = 0.f;
            } else {
                out[2 * k] = v.x;
                out[2 * k + 1] = v.y;
            }
        }
    } else {
        constexpr float invN = 1.0f / (float)(2 * M);
        for (int k = tid; k < M; k += NT)
            bufA[k] = k == 0 ? make_float2(in[0], in[2 * M]) : make_float2(in[2 * k], in[2 * k + 1]);
        // FftError::InputValues: realfft still writes the transform (with the
        // imaginary parts as 0), and Fft::inverse returns through `?` (:42)
        // before its normalisation loop (:44-46) -- that row is not scaled
        const bool bad = in[1] != 0.f || in[2 * M + 1] != 0.f;
        if (tid == 0 && a.status) a.status[blockIdx.x] = bad ? 1 : 0;
        __syncthreads();
        for (int m = tid; m < M; m += NT) bufB[m] = real_pre<LOG2M, NT>(bufA, m, a.tw);
        __syncthreads();
        const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2M, NT, true>(bufB, bufA, a.tw));
        const float sc = bad ? 1.0f : invN;
        for (int j = tid; j < 2 * M; j += NT) out[j] = y[j] * sc;  // (x / N: N is a power of two)
    }
}

template <int LOG2M>
static hipError_t launch_fft_t(bool inverse, const FftArgs &a, int rows, hipStream_t s) {
    constexpr int NT = LOG2M <= 6 ? 64 : 256;
    constexpr size_t lds = 2 * (size_t)(1 << LOG2M) * sizeof(float2) + 16;
    auto kern = inverse ? fft_rows_kernel<LOG2M, NT, true> : fft_rows_kernel<LOG2M, NT, false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(rows), dim3(NT), lds, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// TwoStage sub-chunk (src/fft_convolver.rs:438-461): output += precalculated0
// then += precalculated (two passes, like the reference), and append the
// input to tail_input.
// ---------------------------------------------------------------------------
__global__ void twostage_accum_kernel(TwoStageAccumArgs a) {
    const size_t c = blockIdx.x;
    float *o = a.out + c * a.out_stride + a.sb;
    const float *p0 = a.p0 + c * a.T + a.pos;
    const float *p1 = a.p1 + c * a.T + a.pos;
    const float *x = a.in + c * a.in_stride + a.sb;
    float *ti = a.tail_input + c * a.T + a.fill;
    for (int j = threadIdx.x; j < a.cnt; j += blockDim.x) {
        float v = o[j];
        v += p0[j];
        v += p1[j];
        o[j] = v;
        ti[j] = x[j];
    }
}

// FFTConvolver::reset (src/fft_convolver.rs:296-306) scalar part: current = 0,
// input_buffer_fill = 0; active_seg_count is kept.
__global__ void reset_state_kernel(int4 *state, int channels) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < channels) {
        int4 s = state[c];
        state[c] = make_int4(0, s.y, 0, 0);
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
constexpr int kNT = 256;

// threads per workgroup of the fused kernel: 256 up to B = 1024; larger
// blocks get more lanes so each owns <= 4 slots (no spills at 4 waves/SIMD)
// (B >= 2048 on 512 threads at 2 waves per SIMD: B 4096 197 VGPRs, no
// spills -- on 1024 threads the 128-VGPR cap spilled 34 (B 8192: 96).  A
// one-block step at 256 channels: B 2048 73.1 -> 70.3 us, B 4096 99.8 ->
// 92.2 us, B 8192 125.9 -> 117.5 us; bit-identical; r4e / r4f A/Bs)
constexpr int proc_nt(int log2b) { return log2b <= 10 ? 256 : 512; }

// ---------------------------------------------------------------------------
// Two-stage tail0 deferred to the end of its period (Tail0Args, kernels.hpp).
// TwoStageFFTConvolver::process runs tail_convolver0 on every head block
// (src/fft_convolver.rs:464-472), but tail_output0 is first read after the
// period's swap (:473-475).  So the period's blocks are convolved together:
// one pass over tail0's IR rows and FDL serves all of them, instead of one
// pass per block (cfg3: 64 passes of 64 rows per period).  The state
// (FDL, overlap, current) is committed exactly as the per-block calls leave
// it.
// ---------------------------------------------------------------------------
// (1) copy_and_pad + Fft::forward (:229-241) of pending block k of channel c
// -- the step's own transform -- into xs[c][k]
template <int LOG2B>
__global__ __launch_bounds__(64) void tail0_r2c_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *bufA = reinterpret_cast<float2 *>(smem), *bufB = bufA + B, *twl = bufB + B;
    const ProcJob &J = t.pa.job[0];
    const size_t c = blockIdx.x;
    // grid.y: every pending block; blocks [0, k0) have their spectra from the
    // head's run unless the run missed some of this channel's (t.miss)
    const int k = (int)blockIdx.y, lane = threadIdx.x;
    if (k < t.k0 && !t.miss[c]) return;
    dma_f32<64>(reinterpret_cast<float *>(bufA), J.in + c * J.in_stride + (size_t)k * B, B);  // packed z[0..B/2)
    for (int m = B / 2 + lane; m < B; m += 64) bufA[m] = make_float2(0.f, 0.f);              // the padding half
    dma_16b<64>(twl, t.pa.tw, 2 * B * (int)sizeof(float2));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    float2 *Z = lds_cfft<LOG2B, 64, false, true>(bufA, bufB, twl);
    float2 *xr = t.xs + ((size_t)c * t.nmax + k) * B;
    for (int m = lane; m < B; m += 64) xr[m] = real_post<LOG2B, 64>(Z, m, twl);
    if (k == 0) {  // the overlap before the period's blocks, for (3) (whose tiles overwrite it; k0 = 0)
        for (int j = lane; j < B; j += 64) t.ov0[c * B + j] = J.overlap[c * B + j];
    }
}

// (2) conv_k = sum_{i=1}^{act-1} H[i] (.) X_{k-i} + H[0] (.) X_k (:244-261,
// rows in the reference's order) for every pending block k, one slot chunk
// of FC float4 per workgroup.  X_m is pending block m (m >= 0) or, for m < 0,
// the FDL row (cur0 - m) % act of the previous period (untouched so far).
// The chunk's IR rows and every X row it meets are staged in LDS once; a
// thread owns one slot and J consecutive blocks and walks the rows with the
// X values in a register ring (one H and one X read per row for J MACs).
constexpr int T0_J = 8, T0_FC = 32;
template <int LOG2B>
__host__ __device__ constexpr size_t tail0_mac_lds(int act, int n) {
    return (size_t)(2 * act + 1 + n + T0_J) * T0_FC * 16;  // (+ zero rows: H[act], X[-1], X[nq..nq+J))
}
template <int LOG2B>
__global__ __launch_bounds__(256) void tail0_mac_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B, F = B / 2, FC = F < T0_FC ? F : T0_FC, J = T0_J, RS = J + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ProcJob &J0 = t.pa.job[0];
    const size_t c = blockIdx.x;
    const int fc0 = blockIdx.y * FC;
    const int tid = threadIdx.x, fl = tid % FC, g = tid / FC;
    const int4 st = J0.state[c];
    const int cur0 = st.x, act = st.y, n = t.n;
    if (t.k0 > 0 && blockIdx.y == 0) {
        // the overlap before the period's blocks, for (3) (tail0_r2c copies it
        // at block 0; with k0 > 0 the head's run made block 0's spectrum)
        for (int j = tid; j < B; j += 256) t.ov0[c * B + j] = J0.overlap[c * B + j];
    }
    if (act != t.act) {  // (not a geometry the LDS was sized for: the replay path runs it)
        if (tid == 0) t.err[c] = 1;
        return;
    }
    const size_t rows = (size_t)J0.S * B;
    const float4 *H = reinterpret_cast<const float4 *>(J0.H + c * rows) + fc0;
    const float4 *X = reinterpret_cast<const float4 *>(J0.X + c * rows) + fc0;
    const float4 *xs = reinterpret_cast<const float4 *>(t.xs + (size_t)c * t.nmax * B) + fc0;
    // LDS: H rows [0, act) and a zero row; then X rows q = m + act - 1 in
    // [-1, nq + J) (q = -1 and q >= nq zero), so the walk reads unguarded
    const int nq = act - 1 + n;
    float4 *Hs = reinterpret_cast<float4 *>(smem);  // [act + 1][FC]
    float4 *Xs = Hs + (size_t)(act + 2) * FC;        // Xs[q * FC], q >= -1
    for (int idx = tid; idx < FC; idx += 256) Hs[(size_t)act * FC + idx] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int idx = tid; idx < (J + 1) * FC; idx += 256) {
        const int q = idx < FC ? -1 : nq + idx / FC - 1;
        Xs[(size_t)q * FC + idx % FC] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // LDS-DMA of every row chunk (no VGPRs, all in flight): a wave copies
    // two rows per instruction, lanes 0..31 the first, 32..63 the second
    static_assert(FC == 32, "a row chunk is half a wave of 16-byte lanes");
    {
        const int wave = tid >> 6, lane = tid & 63, half = lane >> 5, f = lane & 31;
        for (int r2 = wave * 2; r2 < act; r2 += 8) {  // IR rows
            if (r2 + half < act)
                __builtin_amdgcn_global_load_lds((gptr_t)(H + (size_t)(r2 + half) * F + f),
                                                 (lptr_t)(Hs + (size_t)r2 * FC), 16, 0, 0);
        }
        for (int r2 = wave * 2; r2 < nq; r2 += 8) {  // X rows
            const int q = r2 + half;
            const float4 *src;
            if (q < act - 1) {
                int r = cur0 + act - 1 - q;
                if (r >= act) r -= act;
                src = X + (size_t)r * F;
            } else {
                src = xs + (size_t)(q - (act - 1)) * F;
            }
            if (q < nq)
                __builtin_amdgcn_global_load_lds((gptr_t)(src + f), (lptr_t)(Xs + (size_t)r2 * FC), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int kb0 = g * J;
    if (kb0 >= n) return;
    auto xq = [&](int q) { return Xs[q * FC + fl]; };  // (q in [-1, nq + J): zero rows at the ends)
    LaAcc acc[J];  // (packed FMAs, la.hpp)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j].zero();
    const bool z0 = fc0 + fl == 0;
    // load e of the walk is X at q = Q1 + J - 1 - e; row i = s + 1 of step s
    // meets, for block kb0 + j, load e = s + J - 1 - j
    const int Q1 = kb0 + act - 2;
    float4 xr[RS];
#pragma unroll
    for (int e = 0; e < J; ++e) xr[e] = xq(Q1 + J - 1 - e);
    float4 hn = Hs[(size_t)min(1, act) * FC + fl];
    const int ns = act - 1;
    for (int s0 = 0; s0 < ns; s0 += RS) {
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            const int sidx = s0 + u;
            if (sidx >= ns) break;
            const float4 h = hn;
            xr[(u + J) % RS] = xq(Q1 - 1 - sidx);
            hn = Hs[(size_t)min(sidx + 2, act) * FC + fl];  // (row act is zero)
            const LaH ho = la_ops(h, z0);
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j].mac(ho, xr[(u + J - 1 - j) % RS]);
        }
    }
    const float4 h0 = Hs[fl];
    const int f = fc0 + fl;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int k = kb0 + j;
        if (k < n) {
            const float4 cv = slot_mac(acc[j].get(), Xs[(size_t)(k + act - 1) * FC + fl], h0, f);
            reinterpret_cast<float4 *>(t.cv + ((size_t)c * t.nmax + k) * B)[f] = cv;
        }
    }
}

// (2b) the C2R of conv_k (:264, the 1/N applied by (3)), one wave per block;
// realfft's C2R error (a non-finite DC / Nyquist bin, :264-267) flags the
// channel for (4)
template <int LOG2B>
__global__ __launch_bounds__(64) void tail0_c2r_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *Z = reinterpret_cast<float2 *>(smem), *q = Z + B, *twl = q + B;
    const size_t c = blockIdx.x;
    const int k = blockIdx.y, lane = threadIdx.x;
    const float2 *cr = t.cv + ((size_t)c * t.nmax + k) * B;
    dma_16b<64>(Z, cr, B * (int)sizeof(float2));
    dma_16b<64>(twl, t.pa.tw, 2 * B * (int)sizeof(float2));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (lane == 0 && !(isfinite(Z[0].x) && isfinite(Z[0].y))) t.err[c] = 1;
    for (int m = lane; m < B; m += 64) q[m] = real_pre<LOG2B, 64>(Z, m, twl);
    wave_sync();
    const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2B, 64, true, true>(q, Z, twl));
    float *yr = t.ys + ((size_t)c * t.nmax + k) * 2 * B;
    for (int j = lane; j < 2 * B; j += 64) yr[j] = y[j];
}

// (3) overlap-add (:270-274) over a tile of pending blocks, the overlap
// save (:283-284) by the last tile, and the FDL rows (:229-241; block k at
// (cur0 - k) % act, the last act blocks stay) -- channels without a C2R error
template <int LOG2B>
__global__ __launch_bounds__(256) void tail0_commit_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B, KT = 256 / (B / 2), NT = 256;
    constexpr float invN = 1.0f / (float)(2 * B);
    const ProcJob &J = t.pa.job[0];
    const size_t c = blockIdx.x;
    if (t.err[c]) return;  // (replayed by tail0_replay_kernel)
    const int tid = threadIdx.x, n = t.n;
    const int k0 = blockIdx.y * KT, k1 = min(n, k0 + KT);
    const int4 st = J.state[c];
    const int cur0 = st.x, act = st.y;
    const float *ys = t.ys + (size_t)c * t.nmax * 2 * B;
    float *outc = J.out + c * J.out_stride;
    for (int idx = k0 * B + tid; idx < k1 * B; idx += NT) {
        const int k = idx >> LOG2B, j = idx & (B - 1);
        const float ov = k == 0 ? t.ov0[c * B + j] : ys[(size_t)(k - 1) * 2 * B + B + j] * invN;
        outc[idx] = ys[(size_t)k * 2 * B + j] * invN + ov;
    }
    if (k1 == n) {  // (the input buffer is empty after a completed block, :280)
        for (int j = tid; j < B; j += NT) J.overlap[c * B + j] = ys[(size_t)(n - 1) * 2 * B + B + j] * invN;
        if (st.w & FLAG_INBUF)
            for (int j = tid; j < B; j += NT) J.inbuf[c * B + j] = 0.f;
    }
    const size_t rows = (size_t)J.S * B;
    float2 *Xc = J.X + c * rows;
    const float2 *xs = t.xs + (size_t)c * t.nmax * B;
    const int kf = max(k0, n - act);
    for (int idx = tid; idx < (k1 - kf) * B; idx += NT) {
        const int k = kf + (idx >> LOG2B), m = idx & (B - 1);
        int r = (cur0 - k) % act;
        if (r < 0) r += act;
        Xc[(size_t)r * B + m] = xs[(size_t)k * B + m];
    }
}

// (4) per channel: the state word of a committed channel (current, the
// flags of n completed blocks) -- or, for a channel whose C2R failed on a
// pending block, tail_convolver0.process block by block (:464-472) from the
// untouched state by the generic step, so the failing block leaves exactly
// the reference's state
template <int LOG2B>
constexpr int t0_replay_nt();
template <int LOG2B>
__global__ __launch_bounds__(LOG2B == 6 ? 512 : proc_nt(LOG2B)) void tail0_replay_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B, NT = LOG2B == 6 ? 512 : proc_nt(LOG2B);  // (t0_replay_nt: the fused flush's)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ProcJob &J = t.pa.job[0];
    const size_t c = blockIdx.x;
    const int n = t.n;
    if (threadIdx.x == 0) t.miss[c] = 0;  // (every pending spectrum was recomputed or is the run's)
    if (!t.err[c]) {
        if (threadIdx.x == 0) {
            const int4 st = J.state[c];
            const int act = st.y;
            int cur = (st.x - n) % act;
            if (cur < 0) cur += act;
            const int flags = (st.w & ~(FLAG_PRE | FLAG_INBUF)) ^ ((n & 1) ? FLAG_REV : 0);
            J.state[c] = make_int4(cur, act, 0, la_clear(flags, t.pa));
        }
        return;
    }
    for (int k = 0; k < n; ++k) {
        ProcJob Jk = J;
        Jk.in = J.in + (size_t)k * B;
        Jk.out = J.out + (size_t)k * B;
        Jk.n = B;
        __syncthreads();  // the previous block's state word is stored
        const int4 st = J.state[c];
        process_job<LOG2B, NT, false, false>(t.pa, Jk, c, st, smem);
    }
    __syncthreads();
    if (threadIdx.x == 0) t.err[c] = 0;
}

// The whole flush in ONE launch at B = 64 (cfg3's head; one slot chunk per
// channel), the default there: per channel one 512-thread workgroup
//   (0) every row by LDS-DMA: tail0's IR rows, the previous period's FDL rows,
//       the pending spectra the head's run wrote (blocks [0, k0)), the
//       overlap, and the inputs of the blocks still to transform;
//   (1) the R2C of blocks [r0, n) (r0 = k0, or 0 if the run missed some of
//       this channel's spectra) into their LDS X rows;
//   (2) the MAC of tail0_mac_kernel, conv rows to LDS; realfft's C2R error
//       (a non-finite DC / Nyquist of some block's conv) decided right here;
//   (3) the FDL rows committed, then each block's C2R;
//   (4) overlap-add, overlap save and the state -- or, on a C2R error, the
//       block-by-block replay of tail0_replay_kernel from the untouched state.
// The same arithmetic in the same order as the five kernels (bit-identical:
// a block's MAC sums its rows in the same order whatever the blocks per
// thread, and both replays run the generic step on 512 threads).
// The B = 64 transforms use 16 of a wave's 64 lanes (16 radix-4 butterflies
// per stage), so each wave runs FOUR blocks' transforms at once, one per
// 16-lane group, each in its own LDS buffers: the same butterflies per lane
// group.  (r4's fused kernel ran one at a time, 16 per wave: 46 us per
// flush; 256 threads with four groups per wave: 22.4 us per cfg3 flush --
// MAC 9.4, C2R 6.0, commit 3.4 -- r6o FFTCONV_T0_TRACE.)
// LDS: [H rows + zero | X rows (q >= -1) + zero rows] (the C2R outputs reuse
// the H rows once the MAC is done, the second 16 transform buffers the X
// rows once the FDL is committed) | tw | 16 groups x 2 B-point buffers |
// conv rows (the inputs to transform before the MAC) | overlap | flag
constexpr int T0F_NT = 512, T0F_J = 4, T0F_G = 16;  // threads; blocks per MAC thread; transform groups of waves 0-3
template <int LOG2B>
constexpr int t0_replay_nt() { return LOG2B == 6 ? T0F_NT : proc_nt(LOG2B); }
template <int LOG2B>
__host__ __device__ constexpr size_t tail0_fused_lds(int act, int n) {
    constexpr size_t B = (size_t)1 << LOG2B;
    return (size_t)(2 * act + 1 + n + T0F_J) * T0_FC * 16 + 2 * B * 8 + T0F_G * 2 * B * 8 + (size_t)n * (B / 2) * 16 +
           B * 4 + 16;
}
template <int LOG2B>
__host__ __device__ constexpr bool tail0_fused_fits(int act, int n) {
    constexpr size_t B = (size_t)1 << LOG2B;
    // (the C2R's second 16 transform buffers live in the X rows: 2 x 16 x B float2)
    return LOG2B == 6 && act >= 1 && n >= 1 && n <= (T0F_NT / T0_FC) * T0F_J && n <= act + 1 &&
           (size_t)(act + n + T0F_J) * T0_FC * 16 >= T0F_G * 2 * B * 8 && tail0_fused_lds<LOG2B>(act, n) <= 160 * 1024;
}
template <int LOG2B>
__global__ __launch_bounds__(T0F_NT) void tail0_fused_kernel(Tail0Args t) {
    constexpr int B = 1 << LOG2B, F = B / 2, FC = T0_FC, J = T0F_J, RS = J + 1, NT = T0F_NT, GL = 16;
    static_assert(F == FC && B / 4 == GL, "one slot chunk per channel, 16 butterflies per stage (B = 64)");
    constexpr float invN = 1.0f / (float)(2 * B);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ProcJob &J0 = t.pa.job[0];
    const size_t c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave * 4 + (lane >> 4), gl = lane & 15;  // this lane's transform group (0..31), its lane in it
    const int4 st = J0.state[c];
    const int cur0 = st.x, act = st.y, n = t.n;
    const size_t rows = (size_t)J0.S * B;
    float4 *Hs = reinterpret_cast<float4 *>(smem);   // [act + 1][FC]
    float4 *Xs = Hs + (size_t)(t.act + 2) * FC;       // Xs[q * FC], q >= -1
    unsigned char *rest = smem + (size_t)(2 * t.act + 1 + n + J) * FC * 16;
    float2 *twl = reinterpret_cast<float2 *>(rest);
    float2 *wb = twl + 2 * B;
    // groups 0-15: their buffers after tw; groups 16-31 (the C2R only): the X rows' region
    float2 *gA = grp < T0F_G ? wb + (size_t)grp * 2 * B : reinterpret_cast<float2 *>(Xs - FC) + (size_t)(grp - T0F_G) * 2 * B;
    float2 *gB = gA + B;
    float4 *cvs = reinterpret_cast<float4 *>(wb + (size_t)T0F_G * 2 * B);  // [n][F]
    float *ins = reinterpret_cast<float *>(cvs);       // [n][B] inputs to transform, before the MAC
    float *ovs = reinterpret_cast<float *>(cvs + (size_t)n * F);
    int &s_err = *reinterpret_cast<int *>(ovs + B);
    float *ys = reinterpret_cast<float *>(smem);       // [n][2B], over the H rows after the MAC
    const bool geo = act == t.act;  // (not the geometry the LDS was sized for: replay)
    const int r0 = t.miss[c] ? 0 : min(t.k0, n);      // blocks [r0, n) are transformed here
    // (FFTCONV_T0_TRACE, tuning: phase stamps of thread 0, s_memrealtime)
    int *tst = t.pa.la_trace ? reinterpret_cast<int *>(t.pa.la_trace) + c * 8 : nullptr;
    auto stamp = [&](int k) {
        if (tst && tid == 0) tst[k] = (int)(unsigned)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);

    // ---- (0) every row by LDS-DMA (no VGPRs, all in flight) ----
    const float4 *H = reinterpret_cast<const float4 *>(J0.H + c * rows);
    const float4 *X = reinterpret_cast<const float4 *>(J0.X + c * rows);
    const float4 *xs = reinterpret_cast<const float4 *>(t.xs + (size_t)c * t.nmax * B);
    const int nq = act - 1 + n;
    constexpr int NWV = NT / 64;
    if (tid == 0) s_err = geo ? 0 : 1;
    if (geo) {
        for (int idx = tid; idx < FC; idx += NT) Hs[(size_t)act * FC + idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int idx = tid; idx < (J + 1) * FC; idx += NT) {
            const int q = idx < FC ? -1 : nq + idx / FC - 1;
            Xs[(size_t)q * FC + idx % FC] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const int half = lane >> 5, f = lane & 31;
        for (int r2 = wave * 2; r2 < act; r2 += 2 * NWV)  // IR rows, two per wave instruction
            if (r2 + half < act)
                __builtin_amdgcn_global_load_lds((gptr_t)(H + (size_t)(r2 + half) * F + f),
                                                 (lptr_t)(Hs + (size_t)r2 * FC), 16, 0, 0);
        // X rows q < act - 1 + r0: the previous period's FDL rows, then the
        // spectra of pending blocks [0, r0) (the run's)
        for (int r2 = wave * 2; r2 < act - 1 + r0; r2 += 2 * NWV) {
            const int q = r2 + half;
            const float4 *src;
            if (q < act - 1) {
                int r = cur0 + act - 1 - q;
                if (r >= act) r -= act;
                src = X + (size_t)r * F;
            } else {
                src = xs + (size_t)(q - (act - 1)) * F;
            }
            if (q < act - 1 + r0)
                __builtin_amdgcn_global_load_lds((gptr_t)(src + f), (lptr_t)(Xs + (size_t)r2 * FC), 16, 0, 0);
        }
        dma_16b<NT>(twl, t.pa.tw, 2 * B * (int)sizeof(float2));
        dma_f32<NT>(ovs, J0.overlap + c * B, B);
        for (int k = r0 + wave; k < n; k += NWV)  // (tail_input blocks: the job's input, stride T)
            dma_f32<64>(ins + (size_t)k * B, J0.in + c * J0.in_stride + (size_t)k * B, B);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(1);
    if (!geo) goto replay;
    {
        // ---- (1) R2C of blocks [r0, n) (:229-241) into their X rows, 16 at a time (waves 0-3) ----
        if (grp < T0F_G) {
            for (int k0 = r0; k0 < n; k0 += T0F_G) {
                const int k = k0 + grp;
                const bool live = k < n;
                for (int m = gl; m < B; m += GL)
                    gA[m] = live && m < B / 2 ? make_float2(ins[(size_t)k * B + 2 * m], ins[(size_t)k * B + 2 * m + 1])
                                              : make_float2(0.f, 0.f);
                wave_sync();
                float2 *Z = lds_cfft<LOG2B, GL, false, true>(gA, gB, twl);
                if (live) {
                    float2 *xr = reinterpret_cast<float2 *>(Xs + (size_t)(k + act - 1) * FC);
                    for (int m = gl; m < B; m += GL) xr[m] = real_post<LOG2B, 64>(Z, m, twl);
                }
                wave_sync();
            }
        }
        __syncthreads();
        stamp(2);
        // ---- (2) the MAC of tail0_mac_kernel (J blocks per thread), conv rows to LDS ----
        const int fl = tid % FC, g = tid / FC, kb0 = g * J;
        if (kb0 < n) {
            auto xq = [&](int q) { return Xs[q * FC + fl]; };
            LaAcc acc[J];
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j].zero();
            const bool z0 = fl == 0;
            const int Q1 = kb0 + act - 2;
            float4 xr[RS];
#pragma unroll
            for (int e = 0; e < J; ++e) xr[e] = xq(Q1 + J - 1 - e);
            float4 hn = Hs[(size_t)min(1, act) * FC + fl];
            const int ns = act - 1;
            for (int s0 = 0; s0 < ns; s0 += RS) {
#pragma unroll
                for (int u = 0; u < RS; ++u) {
                    const int sidx = s0 + u;
                    if (sidx >= ns) break;
                    const float4 h = hn;
                    xr[(u + J) % RS] = xq(Q1 - 1 - sidx);
                    hn = Hs[(size_t)min(sidx + 2, act) * FC + fl];
                    const LaH ho = la_ops(h, z0);
#pragma unroll
                    for (int j = 0; j < J; ++j) acc[j].mac(ho, xr[(u + J - 1 - j) % RS]);
                }
            }
            const float4 h0 = Hs[fl];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int k = kb0 + j;
                if (k < n) cvs[(size_t)k * F + fl] = slot_mac(acc[j].get(), Xs[(size_t)(k + act - 1) * FC + fl], h0, fl);
            }
        }
        __syncthreads();
        stamp(3);
        // realfft's C2R error (:264-267): a block's conv DC / Nyquist not finite
        if (tid < n) {
            const float2 z = reinterpret_cast<const float2 *>(cvs + (size_t)tid * F)[0];
            if (!(isfinite(z.x) && isfinite(z.y))) s_err = 1;
        }
        __syncthreads();
        if (s_err) goto replay;
        // ---- (3) the FDL rows (block k at (cur0 - k) % act, the last act blocks stay) ----
        float2 *Xc = J0.X + c * rows;
        const int kf = max(0, n - act);
        for (int idx = tid; idx < (n - kf) * B; idx += NT) {
            const int k = kf + (idx >> LOG2B), m = idx & (B - 1);
            int r = (cur0 - k) % act;
            if (r < 0) r += act;
            Xc[(size_t)r * B + m] = reinterpret_cast<const float2 *>(Xs + (size_t)(k + act - 1) * FC)[m];
        }
        __syncthreads();  // (the X rows are read: groups 16-31 take their region)
        // ... then each block's C2R, 32 at a time
        for (int k0 = 0; k0 < n; k0 += 2 * T0F_G) {
            const int k = k0 + grp;
            const bool live = k < n;
            const float2 *Zc = reinterpret_cast<const float2 *>(cvs + (size_t)min(k, n - 1) * F);
            for (int m = gl; m < B; m += GL) gA[m] = real_pre<LOG2B, 64>(Zc, m, twl);
            wave_sync();
            const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2B, GL, true, true>(gA, gB, twl));
            if (live) {
                float *yr = ys + (size_t)k * 2 * B;
                for (int j = gl; j < 2 * B; j += GL) yr[j] = y[j];
            }
            wave_sync();
        }
        __syncthreads();
        stamp(4);
        // ---- (4) overlap-add (:270-274), overlap save (:283-284), state ----
        float *outc = J0.out + c * J0.out_stride;
        for (int idx = tid; idx < n * B; idx += NT) {
            const int k = idx >> LOG2B, j = idx & (B - 1);
            const float ov = k == 0 ? ovs[j] : ys[(size_t)(k - 1) * 2 * B + B + j] * invN;
            outc[idx] = ys[(size_t)k * 2 * B + j] * invN + ov;
        }
        for (int j = tid; j < B; j += NT) J0.overlap[c * B + j] = ys[(size_t)(n - 1) * 2 * B + B + j] * invN;
        if (st.w & FLAG_INBUF)
            for (int j = tid; j < B; j += NT) J0.inbuf[c * B + j] = 0.f;
        if (tid == 0) {
            int cur = (cur0 - n) % act;
            if (cur < 0) cur += act;
            const int flags = (st.w & ~(FLAG_PRE | FLAG_INBUF)) ^ ((n & 1) ? FLAG_REV : 0);
            J0.state[c] = make_int4(cur, act, 0, la_clear(flags, t.pa));
            t.miss[c] = 0;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(5);
        return;
    }
replay:
    // tail_convolver0.process block by block from the untouched state (the
    // FDL, the overlap and the state word are not written above), on the
    // generic step of 512 threads, as tail0_replay_kernel at B = 64
    if (tid == 0) t.miss[c] = 0;
    for (int k = 0; k < n; ++k) {
        ProcJob Jk = J0;
        Jk.in = J0.in + (size_t)k * B;
        Jk.out = J0.out + (size_t)k * B;
        Jk.n = B;
        __syncthreads();  // (the LDS is the generic step's now; the previous block's state word is stored)
        const int4 sk = J0.state[c];
        process_job<LOG2B, NT, false, false>(t.pa, Jk, c, sk, smem);
    }
}

static int g_variant = VARIANT_AUTO;
// the scan bits 0-2 (zig-zag, nontemporal, no pipelined step) override the
// automatic load / step policy only when one of them is set: a variant of
// feature bits alone (bits 3-10) keeps the automatic policy
static bool scan_variant_set() { return g_variant != VARIANT_AUTO && (g_variant & 7) != 0; }
static int g_lag = -1;

// Pipelined step: FDL rows the three stream waves take alone while wave 0
// runs the transform chain.  Auto: all of them -- wave 0 never streams (cfg3
// head, S = 64, swept in-process: lag 0 1527, 16 1586, 32 1635, 48 1754,
// >= 62 1844 MS/s; the chain is the critical path, any row given to wave 0
// lengthens it).  Never a function of the channel count, so channel shards
// of any size stay bit-identical.
static int pipeline_lag(int) { return g_lag >= 0 ? g_lag : (1 << 30); }

// Automatic variant: a per-step H+X stream larger than the 256 MiB Infinity
// Cache is re-read from HBM every step whatever the load policy, and there
// nontemporal loads stream 12-14 % faster (measured, cfg2: 137 -> 121 us);
// a stream that stays cache-resident across steps is 1.5x faster with plain
// loads (S = 8: 9.5 vs 14.3 us).  Both variants perform identical arithmetic,
// so the choice never changes a result bit; zig-zag (+0.6 % on top of NT)
// changes the summation order and is therefore opt-in only, keeping channel
// shards bit-identical whatever the shard size.
//
// The pipelined full-block step pays off where a channel's FDL stream is
// short next to its transform chain (cfg3's head, S*B = 4096: 1630 -> 1860
// MS/s) and costs ~3 % on long ones (cfg2, S*B = 48128: the other resident
// workgroups' streams already cover each chain, and three stream waves issue
// fewer loads than four).  It changes the summation order, so it is chosen
// per channel geometry (never by channel count): shards stay bit-identical.
static int pick_variant(const ProcArgs &a, int channels, int log2b) {
    if (scan_variant_set()) return g_variant;
    double stream = 0.0;
    long long rows = 0;
    for (int j = 0; j < a.njobs; ++j) {
        stream += 16.0 * (double)channels * (double)a.job[j].S * (double)(1 << log2b);
        rows = std::max(rows, (long long)a.job[j].S);
    }
    const int nt = stream > 192.0 * 1024 * 1024 ? VARIANT_NT : 0;
    return nt | ((rows << log2b) > 16384 ? VARIANT_NOPIPE : 0) | (g_variant == VARIANT_AUTO ? 0 : g_variant);
}

template <int LOG2B>
static hipError_t launch_gw_anchor_t(const ProcArgs &a, int channels, hipStream_t s) {
    constexpr int F = (1 << LOG2B) / 2;
    constexpr int SL = LOG2B > kMaxLog2Fused ? 256 / FFTCONV_GW_SPLIT : 256;  // slots per workgroup
    static_assert(F % 256 == 0, "a workgroup covers 256 slots");
    const int cls = a.gw_t % kGwP;
    if (channels <= cls || a.gw == nullptr) return hipSuccess;
    ProcArgs args = a;
    args.la_channels = channels;
    const int ny = (channels - cls + kGwP - 1) / kGwP;
    hipLaunchKernelGGL(gw_anchor_kernel<LOG2B>, dim3(F / SL, ny), dim3(256), 0, s, args);
    return hipGetLastError();
}

hipError_t launch_gw_anchor(int log2b, const ProcArgs &a, int channels, hipStream_t s) {
    switch (log2b) {
        case 10: return launch_gw_anchor_t<10>(a, channels, s);
        case 11: return launch_gw_anchor_t<11>(a, channels, s);
        case 12: return launch_gw_anchor_t<12>(a, channels, s);
        case 13: return launch_gw_anchor_t<13>(a, channels, s);
        case 14: return launch_gw_anchor_t<14>(a, channels, s);
        case 15: return launch_gw_anchor_t<15>(a, channels, s);
        case 16: return launch_gw_anchor_t<16>(a, channels, s);
        case 17: return launch_gw_anchor_t<17>(a, channels, s);
        case 18: return launch_gw_anchor_t<18>(a, channels, s);
        case 19: return launch_gw_anchor_t<19>(a, channels, s);
        case 20: return launch_gw_anchor_t<20>(a, channels, s);
        case 21: return launch_gw_anchor_t<21>(a, channels, s);
        case 22: return launch_gw_anchor_t<22>(a, channels, s);
        default: return hipErrorInvalidValue;
    }
}

bool gw_supported(int log2b, int S) { return log2b >= 10 && log2b <= kMaxLog2Block && S >= 3 * kGwP; }

// The generic step on 256 threads for 2048 <= B <= 8192 (ProcArgs::narrow):
// one wave per SIMD and up to 512 VGPRs, so that the workgroup fits a CU
// beside a multi-call run's workgroup (4 waves of ~208 VGPRs) -- the
// 512-thread kernel's 2 waves per SIMD of ~200 VGPRs do not, and the cfg3
// tail then waited for the few CUs the run left free (227 us per period
// beside the run vs 44 us alone, profiles/r5/r5ai).  The MAC keeps each
// slot's row order and the transforms the same butterflies: same bits.
// (at most 256 registers: 2 waves per SIMD -- with a run workgroup's ~240 on
// the same SIMD; unbounded it took 255 VGPRs + 30 AGPRs, and beside the
// run's LDS-resident rows (237 VGPRs) it no longer fit: 200 us per tail
// step instead of 58, profiles/r6/r6h)
template <int LOG2B, bool ZZ, bool NTL>
__global__ __launch_bounds__(256, 2) void upols_narrow_kernel(ProcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const size_t c = blockIdx.x;
    const ProcJob &J = a.job[blockIdx.y];
    process_job<LOG2B, 256, ZZ, NTL>(a, J, c, J.state[c], smem);
    if (a.sig_mode == 1) sig_arrive(a);
}

template <int LOG2B>
static hipError_t launch_process_t(const ProcArgs &a, int channels, hipStream_t s) {
    if constexpr (LOG2B >= 11 && LOG2B <= kMaxLog2Fused) {
        if (a.narrow) {
            using Gn = Geo<LOG2B, 256>;
            auto kern = upols_narrow_kernel<LOG2B, false, false>;
            const int var = pick_variant(a, channels, LOG2B);
            ProcArgs args = a;
            args.pipe = 0;
            args.lag = pipeline_lag(LOG2B);
            switch (var & 3) {
                case 1: kern = upols_narrow_kernel<LOG2B, true, false>; break;
                case 2: kern = upols_narrow_kernel<LOG2B, false, true>; break;
                case 3: kern = upols_narrow_kernel<LOG2B, true, true>; break;
                default: break;
            }
            if (Gn::lds_bytes > 64 * 1024) {
                hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)Gn::lds_bytes);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(kern, dim3(channels, a.njobs), dim3(256), Gn::lds_bytes, s, args);
            return hipGetLastError();
        }
    }
    constexpr int PNT = proc_nt(LOG2B);
    using Gm = Geo<LOG2B, PNT>;
    auto kern = upols_process_kernel<LOG2B, PNT, false, false>;
    const int var = pick_variant(a, channels, LOG2B);
    ProcArgs args = a;
    args.pipe = (var & VARIANT_NOPIPE) ? 0 : 1;
    args.lag = pipeline_lag(LOG2B);
    switch (var & 3) {
        case 1: kern = upols_process_kernel<LOG2B, PNT, true, false>; break;
        case 2: kern = upols_process_kernel<LOG2B, PNT, false, true>; break;
        case 3: kern = upols_process_kernel<LOG2B, PNT, true, true>; break;
        default: break;
    }
    if (Gm::lds_bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)Gm::lds_bytes);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(channels, a.njobs), dim3(PNT), Gm::lds_bytes, s, args);
    return hipGetLastError();
}

template <int LOG2B>
static hipError_t launch_run_t(const ProcArgs &a, const RunSteps &r, int channels, hipStream_t s) {
    if constexpr (LOG2B >= 6 && LOG2B <= 9) {
        constexpr int PNT = proc_nt(LOG2B);
        using Gm = Geo<LOG2B, PNT>;
        if (a.njobs != 1 || r.n < 1) return hipErrorInvalidValue;
        const int var = pick_variant(a, channels, LOG2B);
        if (var & 1) return hipErrorInvalidValue;  // (zig-zag order: per-call launches only)
        ProcArgs args = a;
        args.pipe = (var & VARIANT_NOPIPE) ? 0 : 1;
        args.lag = pipeline_lag(LOG2B);
        auto kern = (var & VARIANT_NT) ? upols_run_kernel<LOG2B, PNT, true> : upols_run_kernel<LOG2B, PNT, false>;
        // (+ the run-carried spectra and the next block's transform buffers,
        // pipelined_step; + the IR rows and the FDL when they fit)
        const size_t lds = Gm::lds_bytes + 4 * (size_t)Gm::B * sizeof(float2) +
                           (size_t)a.run_lds_rows * 2 * Gm::B * sizeof(float2);
        if (a.run_lds_rows < 0 || lds > 160 * 1024) return hipErrorInvalidValue;
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(kern, dim3(channels), dim3(PNT), lds, s, args, r);
        return hipGetLastError();
    } else {
        return hipErrorNotSupported;
    }
}
// the row count of a run's LDS-resident IR rows + FDL (ProcArgs::run_lds_rows):
// S when a run workgroup's LDS stays within 96 KiB -- room left for a 64 KiB
// two-stage tail workgroup on the same CU (cfg3: B 64, S 64 -> 74 KiB) -- and
// only for the run-carried pipelined step (B <= 256); else 0
int run_lds_rows(int log2b, int S) {
    if (log2b < 6 || log2b > 8 || S < 2) return 0;
    if (g_variant != VARIANT_AUTO && (g_variant & VARIANT_NORUNLDS)) return 0;
    const size_t B = (size_t)1 << log2b;
    const size_t base = (log2b == 6 ? Geo<6, 256>::lds_bytes : (log2b == 7 ? Geo<7, 256>::lds_bytes : Geo<8, 256>::lds_bytes)) +
                        4 * B * sizeof(float2);
    return base + (size_t)S * 2 * B * sizeof(float2) <= 96 * 1024 ? S : 0;
}
bool run_supported(int log2b) {
    if (g_variant != VARIANT_AUTO && (g_variant & VARIANT_NORUN)) return false;
    return log2b >= 6 && log2b <= 9 && !(scan_variant_set() && (g_variant & VARIANT_ZIGZAG));
}
hipError_t launch_process_run(int log2b, const ProcArgs &a, const RunSteps &r, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    switch (log2b) {
        case 6: return launch_run_t<6>(a, r, channels, s);
        case 7: return launch_run_t<7>(a, r, channels, s);
        case 8: return launch_run_t<8>(a, r, channels, s);
        case 9: return launch_run_t<9>(a, r, channels, s);
        default: return hipErrorNotSupported;
    }
}

template <int LOG2B>
static hipError_t launch_tail0_t(const Tail0Args &a, int channels, hipStream_t s, hipEvent_t done) {
    if constexpr (LOG2B >= 6 && LOG2B <= 9) {
        constexpr int B = 1 << LOG2B, KT = 256 / (B / 2), NT = proc_nt(LOG2B);
        if (a.n <= 0 || a.n > a.nmax) return hipErrorInvalidValue;
        Tail0Args t = a;
        const int var = pick_variant(a.pa, channels, LOG2B);
        t.pa.pipe = (var & VARIANT_NOPIPE) ? 0 : 1;  // (the replay path's generic step)
        t.pa.lag = pipeline_lag(LOG2B);
        // (every check before the first launch: a failure leaves the pending
        // blocks and tail0's state untouched)
        constexpr int F = B / 2, FC = F < T0_FC ? F : T0_FC;
        const size_t lds = tail0_mac_lds<LOG2B>(a.act, a.n);
        auto mk = tail0_mac_kernel<LOG2B>;
        if (lds > 160 * 1024 || (256 / FC) * T0_J < a.n) return hipErrorInvalidValue;
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)mk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        if constexpr (LOG2B == 6) {
            // (VARIANT_T0FUSED: the five kernels instead, bit-identical)
            if (tail0_fused_fits<LOG2B>(a.act, a.n) && !(g_variant != VARIANT_AUTO && (g_variant & VARIANT_T0FUSED))) {
                const size_t fl = tail0_fused_lds<LOG2B>(a.act, a.n);
                auto fk = tail0_fused_kernel<LOG2B>;
                if (hipError_t e = hipFuncSetAttribute((const void *)fk, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)fl);
                    e != hipSuccess)
                    return e;
                if (done) {  // (the event on the kernel's own completion: no marker packet of its own)
                    hipExtLaunchKernelGGL(fk, dim3(channels), dim3(T0F_NT), fl, s, nullptr, done, 0, t);
                    return hipGetLastError();
                }
                hipLaunchKernelGGL(fk, dim3(channels), dim3(T0F_NT), fl, s, t);
                return hipGetLastError();
            }
        }
        // (blocks [0, k0) have their spectra from the head's run; the overlap
        // copy tail0_r2c makes at block 0 is then tail0_mac's)
        if (t.k0 < 0 || t.k0 > a.n) return hipErrorInvalidValue;
        // (always: with k0 == n its workgroups only test the channel's miss flag)
        hipLaunchKernelGGL(tail0_r2c_kernel<LOG2B>, dim3(channels, a.n), dim3(64), 4 * B * sizeof(float2), s, t);
        hipLaunchKernelGGL(mk, dim3(channels, F / FC), dim3(256), lds, s, t);
        hipLaunchKernelGGL(tail0_c2r_kernel<LOG2B>, dim3(channels, a.n), dim3(64), 4 * B * sizeof(float2), s, t);
        hipLaunchKernelGGL(tail0_commit_kernel<LOG2B>, dim3(channels, (a.n + KT - 1) / KT), dim3(256), 0, s, t);
        constexpr int RNT = t0_replay_nt<LOG2B>();
        static_assert(RNT == (LOG2B == 6 ? 512 : proc_nt(LOG2B)), "tail0_replay_kernel's thread count");
        constexpr size_t rep_lds = Geo<LOG2B, RNT>::lds_bytes;  // (the generic step)
        if (done) {
            hipExtLaunchKernelGGL(tail0_replay_kernel<LOG2B>, dim3(channels), dim3(RNT), (std::uint32_t)rep_lds, s,
                                  nullptr, done, 0, t);
            return hipGetLastError();
        }
        hipLaunchKernelGGL(tail0_replay_kernel<LOG2B>, dim3(channels), dim3(RNT), rep_lds, s, t);
        return hipGetLastError();
    } else {
        return hipErrorNotSupported;
    }
}
bool tail0_defer_supported(int log2b, int act, int nmax) {
    if (log2b < 6 || log2b > 9 || act < 1 || nmax < 1) return false;
    const int F = (1 << log2b) / 2, FC = F < T0_FC ? F : T0_FC;
    return nmax <= (256 / FC) * T0_J && tail0_mac_lds<6>(act, nmax) <= 160 * 1024;
}
hipError_t launch_tail0_flush(int log2b, const Tail0Args &a, int channels, hipStream_t s, hipEvent_t done) {
    if (channels <= 0) return hipSuccess;
    switch (log2b) {
        case 6: return launch_tail0_t<6>(a, channels, s, done);
        case 7: return launch_tail0_t<7>(a, channels, s, done);
        case 8: return launch_tail0_t<8>(a, channels, s, done);
        case 9: return launch_tail0_t<9>(a, channels, s, done);
        default: return hipErrorNotSupported;
    }
}

template <int LOG2B>
static hipError_t launch_ir_t(const IrArgs &a, int channels, hipStream_t s) {
    if constexpr (LOG2B >= 6 && LOG2B <= 10) {
        if (g_variant == VARIANT_AUTO || !(g_variant & VARIANT_IRBLOCK)) {
            constexpr size_t lds = ir_wave_lds<LOG2B>();
            constexpr int NW = ir_nw<LOG2B>();
            auto kern = ir_segments_wave_kernel<LOG2B>;
            if (lds > 64 * 1024) {
                hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(kern, dim3((a.S + NW * IR_SPW - 1) / (NW * IR_SPW), channels), dim3(64 * NW), lds, s, a);
            return hipGetLastError();
        }
    }
    constexpr size_t lds = 2 * (size_t)(1 << LOG2B) * sizeof(float2) + 16;
    auto kern = ir_segments_kernel<LOG2B, kNT>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(a.S, channels), dim3(kNT), lds, s, a);
    return hipGetLastError();
}

#define FFTCONV_DISPATCH(FN, LOG2B, ...)                      \
    switch (LOG2B) {                                          \
        case 0: return FN<0>(__VA_ARGS__);                    \
        case 1: return FN<1>(__VA_ARGS__);                    \
        case 2: return FN<2>(__VA_ARGS__);                    \
        case 3: return FN<3>(__VA_ARGS__);                    \
        case 4: return FN<4>(__VA_ARGS__);                    \
        case 5: return FN<5>(__VA_ARGS__);                    \
        case 6: return FN<6>(__VA_ARGS__);                    \
        case 7: return FN<7>(__VA_ARGS__);                    \
        case 8: return FN<8>(__VA_ARGS__);                    \
        case 9: return FN<9>(__VA_ARGS__);                    \
        case 10: return FN<10>(__VA_ARGS__);                  \
        case 11: return FN<11>(__VA_ARGS__);                  \
        case 12: return FN<12>(__VA_ARGS__);                  \
        case 13: return FN<13>(__VA_ARGS__);                  \
        default: return hipErrorInvalidValue;                 \
    }

hipError_t launch_process(int log2b, const ProcArgs &a, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    if (log2b > kMaxLog2Fused) return launch_process_large(log2b, a, a.lg, a.lg_chunks, channels, s);
    FFTCONV_DISPATCH(launch_process_t, log2b, a, channels, s)
}

// Lookahead geometry policy: block sizes whose row is whole waves of float4
// slots (128..512) and FDLs long enough that the anchor levels dominate.  A
// function of (B, S) only, never of the channel count.
int la_parts(int log2b, int S) {
    if (log2b < 7 || log2b > 9) return 0;
    if (g_variant != VARIANT_AUTO && (g_variant & VARIANT_NOLA)) return 0;
    if (S < 40) return 0;  // (channels whose active segments drop below D0 + 2 step generically)
    return 1;
}
LaDims la_dims(int log2b, int S, int jw) {
    LaDims d{};
    d.nlv = la_nlv(S);
    for (int lv = 1; lv <= 3; ++lv) d.per[lv - 1] = la_per(lv);
    const int nsl = log2b >= 7 ? (1 << (log2b - 1)) / 64 : 1;  // LaGeo::NSL
    d.wg[0] = log2b <= LA_MIDIN_MAXLOG ? 0 : 1;                // LaStep::MIDIN: level 1 in the step workgroups
    d.wg[1] = nsl * (LA_P2 / jw);
    d.wg[2] = d.nlv == 3 ? nsl * (LA_P3 / jw) : 0;
    d.pt = LA_PT;
    d.per_all = LA_PER;
    return d;
}

// anchor workgroups of a launch (ProcArgs::la_n): per level the scheduled
// channels of [c0, C) -- all of them when la_all > 0 -- in whole XCD rounds
// of 8 for the level 2/3 anchors (la_anchor_far)
// fold (ProcArgs::la_l1in2): level-1 anchors ride in the level-2 anchor
// workgroups (one each, after the level-2 walk), so the level-2 count covers
// the level-1 channels too.
static void la_counts(ProcArgs &a, int log2b, int S, int C, bool all, bool mid_wg, bool fold = false,
                      int jw = LA_JW) {
    const LaDims d = la_dims(log2b, S, jw);
    int n1 = 0;
    for (int lv = 1; lv <= 3; ++lv) {
        const int P = d.per[lv - 1];
        const int t0 = a.la_t % P;
        const int n = all ? C - a.la_c0 : (C > t0 ? (C - t0 + P - 1) / P : 0);
        if (lv == 1) {
            n1 = n;
            a.la_n[0] = mid_wg ? (n + 7) / 8 * 8 : 0;  // (whole rounds of 8: the XF 3 grid interleave)
        } else {
            a.la_n[lv - 1] = (lv <= d.nlv) ? (n + 7) / 8 * 8 * d.wg[lv - 1] : 0;
        }
    }
    if (fold) a.la_n[1] = std::max(a.la_n[1], (n1 + 7) / 8 * 8);
    a.la_l1in2 = fold ? 1 : 0;
    a.la_nlv = d.nlv;
}

template <int LOG2B>
static hipError_t launch_la_t(const ProcArgs &a, int channels, hipStream_t s) {
    if constexpr (LOG2B < 7 || LOG2B > 9) {
        return hipErrorNotSupported;
    } else {
        using LG = LaGeo<LOG2B>;
        const bool xf3 = a.la_mix == 3;
        const size_t lsb = xf3 ? LaStep<LOG2B, 3>::bytes : LaStep<LOG2B>::bytes;
        const int nch = xf3 ? 1 : LaStep<LOG2B>::NCH;  // channels per step workgroup
        constexpr size_t gen = Geo<LOG2B, LA_NT>::lds_bytes;
        const size_t lds0 = lsb > LG::anchor_bytes ? lsb : LG::anchor_bytes;
        const size_t lds1 = lds0 > gen ? lds0 : gen;
        const size_t lds = (lds1 + 15) / 16 * 16;
        if (!a.laW) return hipErrorInvalidValue;
        if (xf3 && (a.njobs != 2 || !a.laW2 || a.job[0].S != a.job[1].S || a.job[0].n != a.job[1].n ||
                    a.job[0].add0 || a.job[1].add0 || !a.mix.buf_a || !a.mix.buf_b))
            return hipErrorInvalidValue;
        // the full-pass streams: nontemporal once the whole H + FDL working
        // set exceeds the Infinity Cache
        const double stream = 16.0 * (double)channels * (double)a.job[0].S * (double)(1 << LOG2B);
        const bool ntl = !scan_variant_set() ? stream > 192.0 * 1024 * 1024 : (g_variant & VARIANT_NT) != 0;
        auto kern = a.la_mix == 1   ? (ntl ? upols_la_kernel<LOG2B, true, 1> : upols_la_kernel<LOG2B, false, 1>)
                    : a.la_mix == 2 ? (ntl ? upols_la_kernel<LOG2B, true, 2> : upols_la_kernel<LOG2B, false, 2>)
                    : xf3           ? (ntl ? upols_la_kernel<LOG2B, true, 3> : upols_la_kernel<LOG2B, false, 3>)
                                    : (ntl ? upols_la_kernel<LOG2B, true, 0> : upols_la_kernel<LOG2B, false, 0>);
        ProcArgs args = a;
        args.pipe = 0;
        args.lag = 0;
        args.la_channels = channels;
        args.la_c0 = 0;
        args.la_rebuild = 0;
        args.la_t = a.la_t % LA_PER;
        if (g_variant != VARIANT_AUTO && (g_variant & VARIANT_LAFULL)) args.la_all = -1;  // no anchors: every eligible step sums all its rows
        // standalone batches at B <= 256: level 1 in the level-2 anchor
        // workgroups (they finish their walks first); the crossfade launches
        // keep it in the step workgroups (LaStep::MIDIN)
        const bool fold = a.la_mix == 0 && LOG2B <= LA_MIDIN_MAXLOG;
        const bool midin = !fold && LOG2B <= LA_MIDIN_MAXLOG;
        la_counts(args, LOG2B, a.job[0].S, channels, args.la_all > 0, !fold && !midin, fold);
        if (args.la_all < 0) args.la_n[0] = args.la_n[1] = args.la_n[2] = 0;
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        const int nstep = (channels + nch - 1) / nch;
        if (a.la_mix == 2 && a.job[0].add0) return hipErrorInvalidValue;  // (the fused mix uses the add buffers' LDS)
        const int xwg = a.la_mix == 1 ? LA_XWG : 0;  // A's launch: the mix_value walk workgroups
        const int nanch = (xf3 ? 2 : 1) * (args.la_n[0] + args.la_n[1] + args.la_n[2]);
        hipLaunchKernelGGL(kern, dim3(nanch + nstep + xwg), dim3(LA_NT), lds, s, args);
        return hipGetLastError();
    }
}

hipError_t launch_process_la(int log2b, const ProcArgs &a, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    if (a.njobs != (a.la_mix == 3 ? 2 : 1) || !a.laW) return hipErrorInvalidValue;
    FFTCONV_DISPATCH(launch_la_t, log2b, a, channels, s)
}

int la_trace_grid(int log2b, int S, int channels) {  // (steady-state launches: la_t = 0 has the most anchors)
    if (log2b < 7 || log2b > 9) return 0;
    ProcArgs a{};
    la_counts(a, log2b, S, channels, false, true, true);
    return 2 * (a.la_n[0] + a.la_n[1] + a.la_n[2]) + channels + LA_XWG;  // (XF 3: A's and B's anchors)
}

// ---------------------------------------------------------------------------
// Window rebuild after update() / reset / init (FFTConvolver::update
// :174-213 keeps the FDL but replaces H, so every partial-sum window is
// stale).  Instead of the next process launch re-anchoring every channel on
// its latency-critical path, the update enqueues this anchors-only launch:
// each channel's windows of every level, as the anchors of the previous
// launch would have left them (la_anchor_state, la_rebuild), then the state
// words pointing at them.  The next process launch is a steady-state launch.
// ---------------------------------------------------------------------------
#ifndef FFTCONV_RB_WPC
#define FFTCONV_RB_WPC 4
#endif
#ifndef FFTCONV_RB_UF
#define FFTCONV_RB_UF LA_UF
#endif
// window steps per level-2/3 rebuild workgroup (LA_JW in the process launches):
// each workgroup walks its rows once for RB_JW steps, so the rows' L2
// requests scale with P / RB_JW; same rows in the same order per step
#ifndef FFTCONV_RB_JW
#define FFTCONV_RB_JW LA_JW
#endif
constexpr int RB_JW = FFTCONV_RB_JW;
static_assert(LA_JW == 8, "la_dims' default window slice (kernels.hpp)");
template <int LOG2B, bool NTL>
__global__ __launch_bounds__(LA_NT, FFTCONV_RB_WPC) void la_rebuild_kernel(ProcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    la_anchor<LOG2B, NTL, FFTCONV_RB_UF, RB_JW>(a, 0, (int)blockIdx.x, smem);
}

// the state words of the rebuilt windows (same eligibility test as the
// anchors: both read the state word the update left)
template <int LOG2B>
__global__ void la_rebuild_state_kernel(ProcArgs a) {
    const int c = a.la_c0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (c >= a.la_channels) return;
    const int4 st = a.job[0].state[c];
    // (vnext, when the host passes it: the next lookahead launch's copy of
    // every word, la.hpp la_anchor_state -- no separate refresh copy)
    int4 *vn = a.job[0].vnext;
    if (!la_eligible<LOG2B>(st, a.job[0].n)) {
        if (vn) vn[c] = st;
        return;
    }
    int nf = st.w & ~(LA_MASK | SEQ_MASK);  // (launch tag 0: no process launch wrote it)
    // (the anchors wrote the other window of each level: toggle its flag)
    for (int lv = 1; lv <= a.la_nlv; ++lv) nf = (nf ^ la_flag_win(lv)) | la_flag_live(lv);
    a.job[0].state[c].w = nf;
    if (vn) vn[c] = make_int4(st.x, st.y, st.z, nf);
}

template <int LOG2B>
static hipError_t launch_rebuild_t(const ProcArgs &a, int channels, hipStream_t s) {
    if constexpr (LOG2B < 7 || LOG2B > 9) {
        return hipErrorNotSupported;
    } else {
        using LG = LaGeo<LOG2B>;
        constexpr size_t anchor_bytes = (size_t)(LA_NG - 1) * RB_JW * LG::FS * 16;  // (LaGeo::anchor_bytes at RB_JW)
        constexpr size_t lds = (anchor_bytes + 15) / 16 * 16 + 16;
        if (!a.laW || a.njobs != 1 || a.job[0].n != (1 << LOG2B)) return hipErrorInvalidValue;
        const double stream = 16.0 * (double)channels * (double)a.job[0].S * (double)(1 << LOG2B);
        const bool ntl = !scan_variant_set() ? stream > 192.0 * 1024 * 1024 : (g_variant & VARIANT_NT) != 0;
        auto kern = ntl ? la_rebuild_kernel<LOG2B, true> : la_rebuild_kernel<LOG2B, false>;
        ProcArgs args = a;
        args.la_channels = channels;
        args.la_all = 1;
        args.la_rebuild = 1;
        args.la_seq = 0;
        args.la_t = a.la_t % LA_PER;
        const int nch = channels - a.la_c0;
        if (nch <= 0) return hipSuccess;
        la_counts(args, LOG2B, a.job[0].S, channels, true, true, false, RB_JW);  // (level 1 in workgroups of its own)
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(kern, dim3(args.la_n[0] + args.la_n[1] + args.la_n[2]), dim3(LA_NT), lds, s, args);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        hipLaunchKernelGGL(la_rebuild_state_kernel<LOG2B>, dim3((nch + 255) / 256), dim3(256), 0, s, args);
        return hipGetLastError();
    }
}

hipError_t launch_la_rebuild(int log2b, const ProcArgs &a, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    FFTCONV_DISPATCH(launch_rebuild_t, log2b, a, channels, s)
}

bool la_full_variant() { return g_variant != VARIANT_AUTO && (g_variant & VARIANT_LAFULL); }

hipError_t launch_ir_segments(int log2b, const IrArgs &a, int channels, hipStream_t s) {
    if (channels <= 0 || a.S <= 0) return hipSuccess;
    FFTCONV_DISPATCH(launch_ir_t, log2b, a, channels, s)
}

hipError_t launch_fft_rows(int log2m, bool inverse, const FftArgs &a, int rows, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    FFTCONV_DISPATCH(launch_fft_t, log2m, inverse, a, rows, s)
}

hipError_t launch_twostage_accum(const TwoStageAccumArgs &a, int channels, hipStream_t s) {
    if (channels <= 0 || a.cnt <= 0) return hipSuccess;
    hipLaunchKernelGGL(twostage_accum_kernel, dim3(channels), dim3(a.cnt >= 256 ? 256 : 64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_crossfade_mix(const CrossfadeMixArgs &a, int channels, hipStream_t s) {
    if (channels <= 0 || a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(crossfade_mix_kernel, dim3(channels), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_crossfade_walk(const CrossfadeMixArgs &a, float *vtab, hipStream_t s) {
    if (a.n <= 0 || !a.approaching) return hipSuccess;
    hipLaunchKernelGGL(crossfade_walk_kernel, dim3(1), dim3(64), 0, s, a, vtab);
    return hipGetLastError();
}

template <int LOG2B>
static hipError_t launch_pair_t(const ProcArgs &a, int channels, hipStream_t s) {
    if constexpr (LOG2B < 1 || LOG2B > 9) {
        return hipErrorNotSupported;
    } else {
        constexpr int PNT = proc_nt(LOG2B);
        using PG = PairGeo<LOG2B, PNT>;
        const int var = pick_variant(a, channels, LOG2B);
        if (var & (VARIANT_ZIGZAG | VARIANT_NOPAIR)) return hipErrorNotSupported;  // the pair scan is the plain order only
        ProcArgs args = a;
        args.pipe = 0;
        args.lag = 0;
        auto kern = (var & VARIANT_NT) ? upols_pair_kernel<LOG2B, PNT, true> : upols_pair_kernel<LOG2B, PNT, false>;
        if (PG::lds_bytes > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)PG::lds_bytes);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(kern, dim3(channels), dim3(PNT), PG::lds_bytes, s, args);
        return hipGetLastError();
    }
}

bool pair_supported(int log2b, int S) {
    // long FDLs only: there the step is HBM-bound and the shared stream saves
    // a quarter of the bytes; short ones are latency-bound and run better as
    // two pipelined workgroups
    return log2b >= 1 && log2b <= 9 && ((long long)S << log2b) > 16384 &&
           (g_variant == VARIANT_AUTO || !(g_variant & (VARIANT_ZIGZAG | VARIANT_NOPAIR)));
}

hipError_t launch_process_pair(int log2b, const ProcArgs &a, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    if (a.njobs != 2) return hipErrorInvalidValue;
    FFTCONV_DISPATCH(launch_pair_t, log2b, a, channels, s)
}

__global__ void state_flags_kernel(int4 *state, int channels, int set, int clear) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < channels) state[c].w = (state[c].w & ~clear) | set;
}

hipError_t launch_state_flags(int4 *state, int channels, int set, int clear, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    hipLaunchKernelGGL(state_flags_kernel, dim3((channels + 255) / 256), dim3(256), 0, s, state, channels, set, clear);
    return hipGetLastError();
}

void set_variant(int v) { g_variant = v < 0 ? VARIANT_AUTO : (v & 4095); }
bool gw_windows_allowed() { return g_variant == VARIANT_AUTO || !(g_variant & VARIANT_NOGW); }
bool tail0_defer_allowed() { return g_variant == VARIANT_AUTO || !(g_variant & VARIANT_T0BLOCK); }
bool la_fuse_mix_allowed() { return g_variant == VARIANT_AUTO || !(g_variant & VARIANT_NOFMIX); }
void set_pipeline_lag(int rows) { g_lag = rows < 0 ? -1 : rows; }
int get_pipeline_lag() { return g_lag; }
int get_variant() { return g_variant == VARIANT_AUTO ? -1 : g_variant; }

hipError_t launch_reset_state(int4 *state, int channels, hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    hipLaunchKernelGGL(reset_state_kernel, dim3((channels + 255) / 256), dim3(256), 0, s, state, channels);
    return hipGetLastError();
}

size_t process_lds_bytes(int log2b) {
    switch (log2b) {
#define LDSCASE(L) case L: return Geo<L, proc_nt(L)>::lds_bytes;
        LDSCASE(0) LDSCASE(1) LDSCASE(2) LDSCASE(3) LDSCASE(4) LDSCASE(5) LDSCASE(6)
        LDSCASE(7) LDSCASE(8) LDSCASE(9) LDSCASE(10) LDSCASE(11) LDSCASE(12) LDSCASE(13)
#undef LDSCASE
        default: return 0;
    }
}

}  // namespace fftconv
