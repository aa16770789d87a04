// large.hip -- the long-block path: FFTConvolver / Fft for block sizes past
// the fused kernel's LDS (B >= 16384, i.e. transforms of N = 2B >= 32768
// reals, up to B = 2^22).
//
// The reference takes any block size (src/fft_convolver.rs:115-117); its
// two-stage tail block grows with the response (:520-526: head 512 / IR
// 200,000 -> T = 16,384; head 1024 / IR 1M -> T = 32,768).  One workgroup can
// no longer hold a block's B-point complex FFT in LDS, so a block's transforms
// are split four-step over the chip, M = B = M1 x M2 (M2 <= 2048):
//
//   pass A  (columns, lg_cols_fwd): for each n2 < M2, the M1-point FFT over
//           n1 of z[M2 n1 + n2] (the packed zero-padded block), times
//           W_M^(n2 k1), stored as row k1 of a [M1][M2] array
//   pass B  (row pairs, lg_rows): for each k1, the M2-point FFT over n2 gives
//           Z[k1 + M1 k2] at position k1 M2 + k2
//
// Spectra rows (H, FDL, pre) are kept in that *transposed* bin order: bin
// k = k1 + M1 k2 lives at position k1 M2 + k2.  The spectral MAC is pointwise,
// so any fixed bin order serves it, and both halves of realfft's post-twiddle
// pair (bin k and bin M - k) sit in the row pair {k1, M1 - k1}: one pass-B
// workgroup owns both rows, so it runs the post-twiddle, the whole FDL MAC
// (:244-261) of its bins, realfft's C2R pre-twiddle, and the inverse row FFT
// in one go.  Pass C (lg_cols_inv, columns again) finishes the inverse and
// runs the overlap-add epilogue (:270-292) on its samples.  Position 0 is
// bin 0, so the packed (DC, Nyquist) slot stays slot 0 of a row.
//
// Per process() call: one (A, B, C) triple per chunk of the reference's chunk
// loop (:222-294), every channel deriving its chunk from its own device state
// and a per-call progress word; then lg_call_end (the zero-filled output of a
// failed C2R, the two-stage epilogue, the progress reset).  The block state is
// written once per chunk by the last pass-C workgroup of the channel to
// finish (an arrival counter), after every workgroup of the pass has read it.
//
// Arithmetic: explicit FMAs (built with -ffp-contract=off), twiddles from
// f64-rounded f32 tables; the same code runs the IR transform (init/update)
// and the public Fft, so a handle's IR spectrum and Fft::forward of its
// segment are bit-identical here too.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft_lds.hpp"
#include "kernels.hpp"

namespace fftconv {
namespace {

constexpr int LG_NT = 256;
// threads of a column-pass workgroup of a convolution pass (A and C: one
// 4096-point tile per workgroup).  With fewer tiles than two per CU the pass
// runs one wave per SIMD at 256 threads; LG_CNT_WIDE threads per tile then
// hide its latency (lgu, 256 tiles: 113.7 -> 101.7 us per step, A/B
// r5aa_ab_lg_cnt.log); larger grids keep 256.
constexpr int LG_CNT_WIDE = 1024;
constexpr int LG_WIDE_MAX_TILES = 512;
constexpr int LG_E = 4096;  // complex points per column tile (passes A and C), at most
// tiles per transform, at least: 8 (B = 16384: 2048-point tiles of 256-byte
// column runs).  With the per-tile agent-scope release in pass C, 8 or 16
// tiles were 2-20 % slower than 4 (r5y_ab_lg_tiles.log); without it 8 tiles
// are 1.4 % faster at lgu and 1.2 % at lgt, 16 slower (r5av_ab_lg_tiles.log)
#ifndef FFTCONV_LG_TILES
#define FFTCONV_LG_TILES 8
#endif

template <int LM>
struct LgGeo {
    static constexpr int L2 = LM - 6 < 11 ? LM - 6 : 11;  // row length M2 = 2^L2 (256..2048)
    static constexpr int L1 = LM - L2;                     // column length M1 = 2^L1 (64..2048)
    static constexpr int M = 1 << LM, M1 = 1 << L1, M2 = 1 << L2;
    // complex points per pass-A / pass-C tile: LG_E, or fewer for FFTCONV_LG_TILES tiles (>= 2 columns)
    static constexpr int E0 = M / FFTCONV_LG_TILES < LG_E ? M / FFTCONV_LG_TILES : LG_E;
    static constexpr int E = E0 > 2 * M1 ? E0 : 2 * M1;
    static constexpr int TC = E / M1;                      // columns per pass-A / pass-C tile
    static constexpr int NTILE = M2 / TC;                  // tiles per row of the [M1][M2] array
    static constexpr int NPAIR = M1 / 2;                   // pass-B workgroups per transform
    static constexpr int EP = 2 * M2 / (2 * LG_NT);        // pass B: element pairs per thread
    static constexpr size_t col_lds = 2 * (size_t)E * sizeof(float2);
    static constexpr size_t row_lds = 2 * 2 * (size_t)M2 * sizeof(float2);
    static_assert(LM >= 14 && LM <= 22, "long-block path: 2^14 <= B <= 2^22");
    static_assert(TC >= 2 && TC <= M2 && EP >= 1 && E % LG_NT == 0 && E % LG_CNT_WIDE == 0 && E <= LG_E, "tile shape");
};

// ---------------------------------------------------------------------------
// Batched Stockham FFT in LDS: NB transforms of FL = 2^LF points, element
// (b, pos) at pos * NB + b (IL, interleaved: a tile of columns loaded row by
// row) or b * FL + pos (contiguous rows).  Radix-4 stages, then one radix-2
// stage when LF is odd.  tw = W_{2FL}^i, i < 2FL (f64-rounded f32).
// ---------------------------------------------------------------------------
template <int LF, int NB, bool IL>
__device__ __forceinline__ int bat(int b, int pos) {
    return IL ? pos * NB + b : (b << LF) + pos;
}

template <int LF, int NB, bool IL, bool INV, int NT, int S>
__device__ __forceinline__ void bstage(const float2 *src, float2 *dst, const float2 *__restrict__ tw, int tid) {
    constexpr int FL = 1 << LF, R4 = LF / 2;
    if constexpr (S < R4) {
        constexpr int Ns = 1 << (2 * S), Q = FL / 4;
        constexpr int step = FL / (2 * Ns);  // W_{2FL}^(m k step) = W_{4Ns}^(m k)
        for (int e = tid; e < NB * Q; e += NT) {
            const int b = IL ? (e & (NB - 1)) : e / Q;
            const int j = IL ? e / NB : (e & (Q - 1));
            const int k = j & (Ns - 1);
            float2 v0 = src[bat<LF, NB, IL>(b, j)];
            float2 v1 = src[bat<LF, NB, IL>(b, j + Q)];
            float2 v2 = src[bat<LF, NB, IL>(b, j + 2 * Q)];
            float2 v3 = src[bat<LF, NB, IL>(b, j + 3 * Q)];
            if constexpr (S > 0) {
                v1 = twmul<INV>(v1, tw[k * step]);
                v2 = twmul<INV>(v2, tw[2 * k * step]);
                v3 = twmul<INV>(v3, tw[3 * k * step]);
            }
            const float2 a02 = cadd(v0, v2), s02 = csub(v0, v2);
            const float2 a13 = cadd(v1, v3), s13 = mul_mi<INV>(csub(v1, v3));
            const int base = (j - k) * 4 + k;
            dst[bat<LF, NB, IL>(b, base)] = cadd(a02, a13);
            dst[bat<LF, NB, IL>(b, base + Ns)] = cadd(s02, s13);
            dst[bat<LF, NB, IL>(b, base + 2 * Ns)] = csub(a02, a13);
            dst[bat<LF, NB, IL>(b, base + 3 * Ns)] = csub(s02, s13);
        }
    } else {
        constexpr int H = FL / 2;  // the final radix-2 stage: Ns = FL / 2, k = j
        for (int e = tid; e < NB * H; e += NT) {
            const int b = IL ? (e & (NB - 1)) : e / H;
            const int j = IL ? e / NB : (e & (H - 1));
            const float2 v0 = src[bat<LF, NB, IL>(b, j)];
            const float2 v1 = twmul<INV>(src[bat<LF, NB, IL>(b, j + H)], tw[2 * j]);  // W_FL^j
            dst[bat<LF, NB, IL>(b, j)] = cadd(v0, v1);
            dst[bat<LF, NB, IL>(b, j + H)] = csub(v0, v1);
        }
    }
}

// all stages from src (ping-pong with dst); returns the buffer holding the
// naturally ordered result.  Every thread of the workgroup calls it.
template <int LF, int NB, bool IL, bool INV, int NT = LG_NT, int S = 0>
__device__ __forceinline__ float2 *bfft(float2 *src, float2 *dst, const float2 *__restrict__ tw, int tid) {
    constexpr int NS = LF / 2 + (LF & 1);
    if constexpr (S >= NS) {
        return src;
    } else {
        bstage<LF, NB, IL, INV, NT, S>(src, dst, tw, tid);
        __syncthreads();
        return bfft<LF, NB, IL, INV, NT, S + 1>(dst, src, tw, tid);
    }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ntload(const float4 *p) {  // streaming read: H / FDL rows are used once per block
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ bool finite2(float2 v) { return isfinite(v.x) && isfinite(v.y); }

// complex_multiply_accumulate (:62-74) on a pair of positions; position 0 is
// the packed (DC, Nyquist) slot (two real products)
__device__ __forceinline__ float4 mac4(float4 acc, float4 h, float4 x, bool slot0) {
    float4 r;
    if (slot0) {
        r.x = fmaf(h.x, x.x, acc.x);
        r.y = fmaf(h.y, x.y, acc.y);
    } else {
        r.x = fmaf(-h.y, x.y, fmaf(h.x, x.x, acc.x));
        r.y = fmaf(h.y, x.x, fmaf(h.x, x.y, acc.y));
    }
    r.z = fmaf(-h.w, x.w, fmaf(h.z, x.z, acc.z));
    r.w = fmaf(h.w, x.z, fmaf(h.z, x.w, acc.w));
    return r;
}
__device__ __forceinline__ float4 vadd4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// one channel's chunk of the reference's chunk loop (:222-232), from its
// block state and the call's progress word {processed, done, c2r failed,
// arrival counter}
struct Chunk {
    int cur, act, fill, flags, processed, k;
    bool go;
};
template <int LM>
__device__ __forceinline__ Chunk lg_chunk(const ProcJob &J, size_t c) {
    constexpr int B = 1 << LM;
    const int4 st = J.state[c];
    const int *pg = reinterpret_cast<const int *>(J.lg_prog + c);
    Chunk ch;
    ch.cur = st.x;
    ch.act = st.y;
    ch.fill = st.z;
    ch.flags = st.w;
    ch.processed = pg[0];
    ch.go = st.y > 0 && pg[1] == 0 && ch.processed < J.n;
    ch.k = min(J.n - ch.processed, B - ch.fill);
    return ch;
}

enum { LG_CONV = 0, LG_IR = 1, LG_RAW = 2, LG_RAWINV = 3 };

struct LgPass {
    ProcJob J;              // LG_CONV
    LgTab tb;
    // LG_IR: rows (c, s < nseg) of channel chan0 + c; samples src + c * src_stride
    const float *src;
    long long src_stride, len_data;
    float2 *H;
    int S, chan0, nseg;
    // LG_RAW / LG_RAWINV: the public Fft's rows
    const float *in;
    long long in_stride;
    float *out;
    long long out_stride;
    int *status;
    float2 *Y;              // [rows][M] scratch
    int row0;               // first row of this batch
    // LG_CONV far-row windows (ProcArgs::gw_p / gw / gw_t)
    const float2 *gw;
    int gw_p, gw_t;
    // LG_CONV: a one-chunk call with no two-stage epilogue -- pass C ends it
    // (what lg_call_end does otherwise: zero output for a channel without
    // active segments or with a failed C2R, progress words reset)
    int end_fused;
};

// the far-row split of a channel's pre_multiplied (0 = one sum) and whether
// this chunk reads its window row: the generic step's rule (kernels.hip
// process_job) -- a one-block call from an empty input buffer, window live
__device__ __forceinline__ int lg_split(const LgPass &p, const Chunk &ch) {
    return p.gw_p > 0 && ch.act > p.gw_p ? p.gw_p : 0;
}
__device__ __forceinline__ bool lg_window(const LgPass &p, const Chunk &ch, int sp, int B) {
    return sp && p.gw && ch.fill == 0 && ch.processed == 0 && p.J.n == B &&
           !(ch.flags & (FLAG_INBUF | FLAG_PRE)) && (ch.flags & FLAG_GW);
}

// ---------------------------------------------------------------------------
// pass A: packed input -> column FFTs -> x W_M^(n2 k1) -> rows of Y
// (LG_CONV: Y is the FDL row `current`, overwritten by pass B's spectrum;
// LG_IR: the H row itself; LG_RAW: scratch)
// ---------------------------------------------------------------------------
template <int LM, int MODE, int NT = LG_NT>
__global__ __launch_bounds__(NT) void lg_cols_fwd(LgPass p) {
    using G = LgGeo<LM>;
    constexpr int M = G::M, M1 = G::M1, M2 = G::M2, TC = G::TC;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + G::E;
    const int tid = threadIdx.x;
    const int tile = blockIdx.x % G::NTILE;
    const size_t row = blockIdx.x / G::NTILE;
    const int c0 = tile * TC;
    float2 *Y;
    if constexpr (MODE == LG_CONV) {
        const ProcJob &J = p.J;
        const Chunk ch = lg_chunk<LM>(J, row);
        if (!ch.go) return;
        DBG_CHECK(ch.cur >= 0 && ch.cur < J.S && ch.act <= J.S && ch.k > 0 && ch.fill + ch.k <= M, 50, ch.cur, ch.act,
                  ch.fill, ch.k);  // (site 50: pass A's chunk and FDL row)
        Y = J.X + (row * (size_t)J.S + (size_t)ch.cur) * M;
        // copy_and_pad of the input buffer (:229-234): sample i is the chunk's
        // input inside [fill, fill + k), else the buffered sample (or 0)
        const float *inc = J.in + row * J.in_stride;
        const float *ibc = J.inbuf + row * M;
        const bool inb = (ch.flags & FLAG_INBUF) != 0;
        auto x = [&](int i) -> float {
            if (i >= ch.fill && i < ch.fill + ch.k) return inc[ch.processed + i - ch.fill];
            return inb ? ibc[i] : 0.f;
        };
        for (int e = tid; e < G::E; e += NT) {
            const int t = e & (TC - 1), n1 = e / TC;
            const int n = n1 * M2 + c0 + t;
            b0[e] = n1 < M1 / 2 ? make_float2(x(2 * n), x(2 * n + 1)) : make_float2(0.f, 0.f);
        }
    } else if constexpr (MODE == LG_IR) {
        const size_t ch = row / p.nseg, s = row % p.nseg;
        DBG_CHECK(p.nseg <= p.S, 51, (int)s, p.nseg, p.S, p.chan0);  // (site 51: an IR segment row)
        Y = p.H + ((p.chan0 + ch) * (size_t)p.S + s) * M;
        const float *src = p.src + ch * p.src_stride;
        const long long base = (long long)s * M;  // (B = M samples per segment)
        auto x = [&](int i) -> float { return base + i < p.len_data ? src[base + i] : 0.f; };
        for (int e = tid; e < G::E; e += NT) {
            const int t = e & (TC - 1), n1 = e / TC;
            const int n = n1 * M2 + c0 + t;
            b0[e] = n1 < M1 / 2 ? make_float2(x(2 * n), x(2 * n + 1)) : make_float2(0.f, 0.f);
        }
    } else {
        Y = p.Y + row * M;
        const float *in = p.in + (p.row0 + row) * p.in_stride;
        for (int e = tid; e < G::E; e += NT) {
            const int t = e & (TC - 1), n1 = e / TC;
            const int n = n1 * M2 + c0 + t;
            b0[e] = make_float2(in[2 * n], in[2 * n + 1]);
        }
    }
    __syncthreads();
    const float2 *R = bfft<G::L1, TC, true, false, NT>(b0, b1, p.tb.twA, tid);
    for (int e = tid; e < G::E; e += NT) {
        const int t = e & (TC - 1), k1 = e / TC;
        const int n2 = c0 + t;
        DBG_CHECK(k1 < M1 && n2 < M2, 52, k1, n2, tile, (int)row);  // (site 52: pass A's Y position)
        Y[(size_t)k1 * M2 + n2] = cmul(R[e], p.tb.twM[(n2 * k1) & (M - 1)]);
    }
}

// element e of a pass-B workgroup (rows r0 = w, r1 = the mirror row, at
// [0, M2) and [M2, 2 M2) of LDS): its row, column k2 and the element holding
// bin M - k (realfft's post/pre-twiddle partner)
template <int LM>
struct RowPair {
    int w, r0, r1;
    __device__ __forceinline__ explicit RowPair(int w_) : w(w_), r0(w_), r1(w_ ? LgGeo<LM>::M1 - w_ : LgGeo<LM>::M1 / 2) {}
    __device__ __forceinline__ int row(int e) const { return e < LgGeo<LM>::M2 ? r0 : r1; }
    __device__ __forceinline__ int mirror(int e) const {
        constexpr int M2 = LgGeo<LM>::M2;
        const int b = e >= M2, k2 = e & (M2 - 1);
        if (w == 0) return b ? M2 + (M2 - 1 - k2) : ((M2 - k2) & (M2 - 1));  // rows 0 and M1/2 mirror themselves
        return (1 - b) * M2 + (M2 - 1 - k2);
    }
    __device__ __forceinline__ size_t pos(int e) const {  // position in a spectrum row
        constexpr int M2 = LgGeo<LM>::M2;
        return (size_t)row(e) * M2 + (e & (M2 - 1));
    }
    __device__ __forceinline__ int bin(int e) const {
        constexpr int M1 = LgGeo<LM>::M1, M2 = LgGeo<LM>::M2;
        return row(e) + M1 * (e & (M2 - 1));
    }
};

// realfft's C2R pre-twiddle (real_pre) of bin k from X[k] (a) and X[M - k] (xb)
__device__ __forceinline__ float2 real_pre_pair(float2 a, float2 xb, int k, const float2 *__restrict__ twN) {
    if (k == 0) return make_float2(a.x + a.y, a.x - a.y);
    const float2 b = make_float2(xb.x, -xb.y);
    const float2 e = cadd(a, b);
    const float2 o = cmulc(csub(a, b), twN[k]);
    return make_float2(e.x - o.y, e.y + o.x);
}

// ---------------------------------------------------------------------------
// pass B: row pair {w, mirror}.
//  LG_CONV: forward row FFTs, post-twiddle -> FDL row `current` (:233-241);
//           pre_multiplied (:244-255, when the chunk starts a block) or the
//           stored one; conv = pre + X H[0] (:256-261); realfft's C2R error
//           check (:264-267); pre-twiddle, inverse row FFTs, x W_M^-(n2 k1)
//           -> the call's V scratch
//  LG_IR:   forward row FFTs + post-twiddle -> the H row (in place)
//  LG_RAW:  forward row FFTs + post-twiddle -> natural-order bins
//  LG_RAWINV: natural-order bins -> pre-twiddle, inverse rows -> scratch
// ---------------------------------------------------------------------------
template <int LM, int MODE>
__global__ __launch_bounds__(LG_NT) void lg_rows(LgPass p) {
    using G = LgGeo<LM>;
    constexpr int M = G::M, M2 = G::M2, EP = G::EP;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + 2 * M2;
    const int tid = threadIdx.x;
    const RowPair<LM> rp((int)(blockIdx.x % G::NPAIR));
    const size_t row = blockIdx.x / G::NPAIR;
    const float2 *__restrict__ twN = p.tb.twN;

    Chunk ch{};
    const float2 *Yr;  // pass A's rows
    if constexpr (MODE == LG_CONV) {
        ch = lg_chunk<LM>(p.J, row);
        if (!ch.go) return;
        DBG_CHECK(ch.cur >= 0 && ch.cur < p.J.S && ch.act <= p.J.S, 53, ch.cur, ch.act, p.J.S, (int)row);  // (site 53)
        Yr = p.J.X + (row * (size_t)p.J.S + (size_t)ch.cur) * M;
    } else if constexpr (MODE == LG_IR) {
        const size_t c = row / p.nseg, s = row % p.nseg;
        Yr = p.H + ((p.chan0 + c) * (size_t)p.S + s) * M;
    } else {
        Yr = p.Y + row * M;
    }

    float2 *F, *Gb;  // Gb: the other buffer
    if constexpr (MODE != LG_RAWINV) {
        for (int e = tid; e < 2 * M2; e += LG_NT) b0[e] = Yr[rp.pos(e)];
        __syncthreads();
        F = bfft<G::L2, 2, false, false>(b0, b1, p.tb.twB, tid);
        Gb = F == b0 ? b1 : b0;
        // realfft's post-twiddle: bin k from Z[k] and Z[M - k]
        for (int e = tid; e < 2 * M2; e += LG_NT) Gb[e] = real_post_pair(F[e], F[rp.mirror(e)], rp.bin(e), twN);
        __syncthreads();
        if constexpr (MODE == LG_IR) {
            float2 *Hr = p.H + (p.chan0 + row / p.nseg) * (size_t)p.S * M + (row % p.nseg) * (size_t)M;
            for (int e = tid; e < 2 * M2; e += LG_NT) Hr[rp.pos(e)] = Gb[e];
            return;
        } else if constexpr (MODE == LG_RAW) {
            float *o = p.out + (p.row0 + row) * p.out_stride;
            for (int e = tid; e < 2 * M2; e += LG_NT) {
                const int k = rp.bin(e);
                const float2 v = Gb[e];
                if (k == 0) {  // packed (DC, Nyquist)
                    o[0] = v.x;
                    o[1] = 0.f;
                    o[2 * M] = v.y;
                    o[2 * M + 1] = 0.f;
                } else {
                    o[2 * k] = v.x;
                    o[2 * k + 1] = v.y;
                }
            }
            return;
        }
    }

    if constexpr (MODE == LG_CONV) {
        const ProcJob &J = p.J;
        const size_t rows = (size_t)J.S * M;
        const float2 *Hc = J.H + row * rows;
        float2 *Xc = J.X + row * rows;
        float2 *Xcur = Xc + (size_t)ch.cur * M;
        float2 *prec = J.pre + row * M;
        // this thread's element pairs: e = 2 tid + 2 LG_NT u (two adjacent
        // positions of one row: 16-byte accesses)
        float4 acc[EP];
#pragma unroll
        for (int u = 0; u < EP; ++u) {
            const int e = 2 * tid + 2 * LG_NT * u;
            reinterpret_cast<float4 *>(Xcur + rp.pos(e))[0] =
                make_float4(Gb[e].x, Gb[e].y, Gb[e + 1].x, Gb[e + 1].y);  // segments[current] (:237)
        }
        if (ch.fill == 0) {
            // pre_multiplied = sum_{i=1}^{act-1} H[i] (.) X[(current + i) % act] (:244-255)
#ifdef FFTCONV_LG_RU
            constexpr int RU = FFTCONV_LG_RU;  // (A/B builds)
#else
            constexpr int RU = EP >= 8 ? 1 : 8 / EP;
#endif
            size_t q[EP];
#pragma unroll
            for (int u = 0; u < EP; ++u) q[u] = rp.pos(2 * tid + 2 * LG_NT * u) / 2;
            const float4 *H4 = reinterpret_cast<const float4 *>(Hc);
            const float4 *X4 = reinterpret_cast<const float4 *>(Xc);
            constexpr size_t RF = (size_t)M / 2;  // float4 per row
            // rows [i0, i1) summed from zero into r: RU rows in flight per
            // thread (RU x EP x 2 float4 loads issued before their MACs), then
            // the MACs in row order -- the same sums in the same order as one
            // row at a time
            auto mac_range = [&](float4 (&r)[EP], int i0, int i1) {
#pragma unroll
                for (int u = 0; u < EP; ++u) r[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                int xi = (ch.cur + i0) % ch.act;  // (current may exceed act after an update shrank it)
                int i = i0;
                for (; i + RU <= i1; i += RU) {
                    float4 hv[RU][EP], xv[RU][EP];
                    int xr = xi;
#pragma unroll
                    for (int t = 0; t < RU; ++t) {
#pragma unroll
                        for (int u = 0; u < EP; ++u) {
                            DBG_CHECK(xr >= 0 && xr < ch.act && 2 * q[u] + 1 < (size_t)M, 54, xr, ch.act, (int)q[u],
                                      i + t);  // (site 54: a MAC row)
                            hv[t][u] = ntload(H4 + (size_t)(i + t) * RF + q[u]);
                            xv[t][u] = ntload(X4 + (size_t)xr * RF + q[u]);
                        }
                        if (++xr == ch.act) xr = 0;
                    }
#pragma unroll
                    for (int t = 0; t < RU; ++t)
#pragma unroll
                        for (int u = 0; u < EP; ++u)
                            r[u] = mac4(r[u], hv[t][u], xv[t][u], tid == 0 && u == 0 && rp.w == 0);
                    xi = xr;
                }
                for (; i < i1; ++i) {
                    float4 hv[EP], xv[EP];
#pragma unroll
                    for (int u = 0; u < EP; ++u) {
                        DBG_CHECK(xi >= 0 && xi < ch.act, 54, xi, ch.act, (int)q[u], i);
                        hv[u] = ntload(H4 + (size_t)i * RF + q[u]);
                        xv[u] = ntload(X4 + (size_t)xi * RF + q[u]);
                    }
#pragma unroll
                    for (int u = 0; u < EP; ++u) r[u] = mac4(r[u], hv[u], xv[u], tid == 0 && u == 0 && rp.w == 0);
                    if (++xi == ch.act) xi = 0;
                }
            };
            // far-row windows (as the generic step): rows 1..sp-1
            // plus rows sp..act-1 in every launch of such a batch; a one-block
            // call of a channel whose window is live reads the far part from
            // its window row (gw_anchor_kernel summed it with the same
            // arithmetic), else sums it here
            const int sp = lg_split(p, ch);
            mac_range(acc, 1, sp ? sp : ch.act);
            if (lg_window(p, ch, sp, M)) {
                const int k = (int)(((long long)p.gw_t - 1 - (long long)row) % sp + sp) % sp;
                DBG_CHECK(k >= 0 && k < sp, 60, k, p.gw_t, sp, (int)row);  // (site 60: the window row)
                const float4 *wr = reinterpret_cast<const float4 *>(p.gw + (row * sp + k) * (size_t)M);
#pragma unroll
                for (int u = 0; u < EP; ++u) acc[u] = vadd4(acc[u], ntload(wr + q[u]));
            } else if (sp) {
                float4 far[EP];
                mac_range(far, sp, ch.act);
#pragma unroll
                for (int u = 0; u < EP; ++u) acc[u] = vadd4(acc[u], far[u]);
            }
#pragma unroll
            for (int u = 0; u < EP; ++u)
                reinterpret_cast<float4 *>(prec + rp.pos(2 * tid + 2 * LG_NT * u))[0] = acc[u];
        } else {
#pragma unroll
            for (int u = 0; u < EP; ++u)
                acc[u] = reinterpret_cast<const float4 *>(prec + rp.pos(2 * tid + 2 * LG_NT * u))[0];
        }
        // conv = pre_multiplied + segments[current] (.) segments_ir[0] -> F
        // (free: every post-twiddle read of it is behind the barrier above)
#pragma unroll
        for (int u = 0; u < EP; ++u) {
            const int e = 2 * tid + 2 * LG_NT * u;
            const float4 h0 = reinterpret_cast<const float4 *>(Hc + rp.pos(e))[0];
            const float4 x = make_float4(Gb[e].x, Gb[e].y, Gb[e + 1].x, Gb[e + 1].y);
            const bool s0 = tid == 0 && u == 0 && rp.w == 0;
            const float4 cv = mac4(acc[u], h0, x, s0);
            F[e] = make_float2(cv.x, cv.y);
            F[e + 1] = make_float2(cv.z, cv.w);
            if (s0 && !(isfinite(cv.x) && isfinite(cv.y))) {
                // realfft's C2R rejects a non-zero DC / Nyquist imaginary part
                // (:264-267).  The reference's imaginary part there is a sum of
                // re * 0 + 0 * re products: NaN exactly when one of the
                // operand rows' (DC, Nyquist) parts is not finite, while a
                // finite overflow leaves it 0 (and runs the C2R on inf).  A
                // carried pre_multiplied was summed from the same rows.
                bool bad = !finite2(make_float2(x.x, x.y)) || !finite2(make_float2(h0.x, h0.y));
                if (!bad && !finite2(make_float2(acc[0].x, acc[0].y))) {
                    for (int i = 1; i < ch.act && !bad; ++i) {
                        const int xi = (ch.cur + i) % ch.act;
                        bad = !finite2(Hc[(size_t)i * M]) || !finite2(Xc[(size_t)xi * M]);
                    }
                }
                if (bad) reinterpret_cast<int *>(J.lg_prog + row)[2] = 1;
            }
        }
        __syncthreads();
    } else {  // LG_RAWINV: the bins of row (row0 + row), natural order
        F = b0;
        Gb = b1;
        const float *in = p.in + (p.row0 + row) * p.in_stride;
        for (int e = tid; e < 2 * M2; e += LG_NT) {
            const int k = rp.bin(e);
            F[e] = k == 0 ? make_float2(in[0], in[2 * M]) : make_float2(in[2 * k], in[2 * k + 1]);
        }
        if (rp.w == 0 && tid == 0 && p.status)
            p.status[p.row0 + row] = (in[1] != 0.f || in[2 * M + 1] != 0.f) ? 1 : 0;  // FftError::InputValues
        __syncthreads();
    }

    // C2R: pre-twiddle -> Gb, inverse row FFTs, x W_M^-(n2 k1)
    for (int e = tid; e < 2 * M2; e += LG_NT) Gb[e] = real_pre_pair(F[e], F[rp.mirror(e)], rp.bin(e), twN);
    __syncthreads();
    const float2 *R = bfft<G::L2, 2, false, true>(Gb, F, p.tb.twB, tid);
    float2 *V = MODE == LG_CONV ? p.J.lg_v + row * M : p.Y + row * M;
    for (int e = tid; e < 2 * M2; e += LG_NT) {
        const int n2 = e & (M2 - 1), r = rp.row(e);
        V[(size_t)r * M2 + n2] = cmulc(R[e], p.tb.twM[(n2 * r) & (M - 1)]);
    }
}

// ---------------------------------------------------------------------------
// pass C: inverse column FFTs -> samples y[2n], y[2n+1] of n = M2 n1 + n2;
//  LG_CONV: overlap-add (:270-274), overlap save (:283-284), input buffer
//           (:230-231, :280), and -- by the channel's last workgroup -- the
//           block state (:277-292) and the call's progress
//  LG_RAWINV: the rows, divided by N unless realfft flagged them (:42-46)
// ---------------------------------------------------------------------------
template <int LM, int MODE, int NT = LG_NT>
__global__ __launch_bounds__(NT) void lg_cols_inv(LgPass p) {
    using G = LgGeo<LM>;
    constexpr int M = G::M, M2 = G::M2, TC = G::TC, B = M;
    constexpr float invN = 1.0f / (float)(2 * M);
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + G::E;
    const int tid = threadIdx.x;
    const int tile = blockIdx.x % G::NTILE;
    const size_t row = blockIdx.x / G::NTILE;
    const int c0 = tile * TC;
    Chunk ch{};
    const float2 *V;
    if constexpr (MODE == LG_CONV) {
        ch = lg_chunk<LM>(p.J, row);
        if (!ch.go) {
            if (p.end_fused) {  // (one chunk: !go = no active segment) output.fill(0) (:216-219), this tile's samples
                float *outc = p.J.out + row * p.J.out_stride;
                for (int e = tid; e < G::E / 2; e += NT) {
                    const int j0 = 2 * ((e / TC) * M2 + c0 + (e & (TC - 1)));
                    if (j0 < p.J.n) outc[j0] = 0.f;
                    if (j0 + 1 < p.J.n) outc[j0 + 1] = 0.f;
                }
            }
            return;
        }
        V = p.J.lg_v + row * M;
    } else {
        V = p.Y + row * M;
    }
    for (int e = tid; e < G::E; e += NT) {
        const int t = e & (TC - 1), k1 = e / TC;
        b0[e] = V[(size_t)k1 * M2 + c0 + t];
    }
    __syncthreads();
    const float2 *R = bfft<G::L1, TC, true, true, NT>(b0, b1, p.tb.twA, tid);

    if constexpr (MODE == LG_RAWINV) {
        const float *in = p.in + (p.row0 + row) * p.in_stride;
        const float sc = (in[1] != 0.f || in[2 * M + 1] != 0.f) ? 1.0f : invN;  // (flagged rows stay unscaled)
        float *o = p.out + (p.row0 + row) * p.out_stride;
        for (int e = tid; e < G::E; e += NT) {
            const int t = e & (TC - 1), n1 = e / TC;
            const size_t n = (size_t)n1 * M2 + c0 + t;
            o[2 * n] = R[e].x * sc;
            o[2 * n + 1] = R[e].y * sc;
        }
        return;
    } else {
        const ProcJob &J = p.J;
        int *pg = reinterpret_cast<int *>(J.lg_prog + row);
        const bool err = pg[2] != 0;
        const float *inc = J.in + row * J.in_stride;
        float *outc = J.out + row * J.out_stride;
        float *ovc = J.overlap + row * B;
        float *ibc = J.inbuf + row * B;
        const int lo = ch.fill, hi = ch.fill + ch.k;
        const bool complete = hi == B;
        // the first half of the tile's rows (n1 < M1/2) holds samples j < B;
        // a whole block into an 8-byte aligned output goes out as sample pairs
        const bool pairs = !err && lo == 0 && complete &&
                           (reinterpret_cast<uintptr_t>(outc + ch.processed) & 7) == 0;
        if (pairs) {
            for (int e = tid; e < G::E / 2; e += NT) {
                const int j0 = 2 * ((e / TC) * M2 + c0 + (e & (TC - 1)));
                DBG_CHECK(j0 + 1 < B && ch.processed + j0 + 1 < J.n, 56, j0, lo, hi, ch.processed);
                const float2 o = *reinterpret_cast<const float2 *>(ovc + j0);
                *reinterpret_cast<float2 *>(outc + ch.processed + j0) =
                    make_float2(R[e].x * invN + o.x, R[e].y * invN + o.y);  // :270-274
                if (ch.flags & FLAG_INBUF) *reinterpret_cast<float2 *>(ibc + j0) = make_float2(0.f, 0.f);  // :280
            }
        }
        for (int e = tid; e < (pairs ? 0 : G::E / 2); e += NT) {
            const int t = e & (TC - 1), n1 = e / TC;
            const int j0 = 2 * (n1 * M2 + c0 + t);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = j0 + q;
                if (err) {
                    // output.fill(0); return (:264-267): the chunk stays in
                    // the input buffer (lg_call_end zero-fills the output,
                    // or this pass when it ends the call)
                    if (j >= lo && j < hi) {
                        ibc[j] = inc[ch.processed + j - lo];
                        if (p.end_fused) outc[ch.processed + j - lo] = 0.f;
                    }
                    continue;
                }
                DBG_CHECK(j < B && (j < lo || j >= hi || ch.processed + j - lo < J.n), 56, j, lo, hi, ch.processed);
                if (j >= lo && j < hi) outc[ch.processed + j - lo] = (q ? R[e].y : R[e].x) * invN + ovc[j];  // :270-274
                if (complete) {
                    if (ch.flags & FLAG_INBUF) ibc[j] = 0.f;  // :280
                } else if (j >= lo && j < hi) {
                    ibc[j] = inc[ch.processed + j - lo];  // :230-231
                }
            }
        }
        if (complete && !err) {
            __syncthreads();  // every overlap read above is done (sample j and j + B share the column)
            for (int e = G::E / 2 + tid; e < G::E; e += NT) {
                const int t = e & (TC - 1), n1 = e / TC;
                const int j = 2 * (n1 * M2 + c0 + t) - B;
                *reinterpret_cast<float2 *>(ovc + j) = make_float2(R[e].x * invN, R[e].y * invN);  // :283-284
            }
        }
        // the channel's last workgroup of this pass writes the block state
        __syncthreads();
        if (tid == 0) {
#ifndef FFTCONV_LG_ARRIVE_RELAXED
#define FFTCONV_LG_ARRIVE_RELAXED 1
#endif
#if FFTCONV_LG_ARRIVE_RELAXED
            // relaxed: a tile only reports that it has consumed the progress
            // words and the state (their values were used above); the last
            // tile reads nothing another tile wrote (the outputs meet the next
            // launch at the kernel boundary), so no release -- which at agent
            // scope would write back this XCD's L2 once per tile
            const int old = __hip_atomic_fetch_add(pg + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
            __threadfence();
            const int old = __hip_atomic_fetch_add(pg + 3, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#endif
            DBG_CHECK(old >= 0 && old < G::NTILE, 55, old, G::NTILE, (int)row, 0);  // (site 55: the arrival counter)
            if (old == G::NTILE - 1) {
                pg[3] = 0;
                int cur = ch.cur, fill = ch.fill, flags = ch.flags & ~(LA_MASK | SEQ_MASK | FLAG_PRE);
                // a step that read its window keeps it live for the window's
                // next block (the generic step's rule)
                const bool gwin = lg_window(p, ch, lg_split(p, ch), B);
                if (err) {
                    flags |= FLAG_INBUF;  // fill / current unchanged
                    pg[1] = 1;
                } else {
                    if (complete) {
                        flags &= ~FLAG_INBUF;
                        flags ^= FLAG_REV;
                        fill = 0;
                        cur = cur > 0 ? cur - 1 : ch.act - 1;  // :287-291
                        if (gwin) flags |= FLAG_GW;
                    } else {
                        flags |= FLAG_INBUF;
                        fill += ch.k;
                    }
                    pg[0] = ch.processed + ch.k;
                }
                if (p.end_fused) {  // the call ends here: progress words reset (every tile has read them)
                    pg[0] = 0;
                    pg[1] = 0;
                    pg[2] = 0;
                }
                J.state[row] = make_int4(cur, ch.act, fill, flags);
            }
        }
    }
}

// after the call's chunks: a channel with no active segment (:216-219) or a
// failed C2R (:264-267) outputs zeros; the two-stage sub-chunk epilogue
// (:438-461) when the job carries it; the progress word is reset
__global__ __launch_bounds__(256) void lg_call_end(ProcJob J) {
    const size_t c = blockIdx.x;
    int *pg = reinterpret_cast<int *>(J.lg_prog + c);
    const bool zero = J.state[c].y == 0 || pg[2] != 0;
    float *outc = J.out + c * J.out_stride;
    const float *inc = J.in + c * J.in_stride;
    const float *p0 = J.add0 ? J.add0 + c * J.add_stride : nullptr;
    const float *p1 = J.add1 ? J.add1 + c * J.add_stride : nullptr;
    float *ti = J.tin ? J.tin + c * J.tin_stride : nullptr;
    // (a standalone call that produced its output: nothing to rewrite)
    const int nloop = (zero || p0 || ti) ? J.n : 0;
    for (int j = threadIdx.x; j < nloop; j += 256) {
        float v = zero ? 0.f : outc[j];
        if (p0) {
            v += p0[j];
            if (p1) v += p1[j];
        }
        if (zero || p0) outc[j] = v;
        if (ti) ti[j] = inc[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        pg[0] = 0;
        pg[1] = 0;
        pg[2] = 0;
    }
}

// update(): zero overlap / pre_multiplied, set active_seg_count (:185-190)
__global__ __launch_bounds__(256) void lg_update_state(IrArgs a, int B, int active) {
    const size_t c = a.chan0 + blockIdx.x;
    for (int j = threadIdx.x; j < B; j += 256) {
        a.overlap[c * B + j] = 0.f;
        a.pre[c * B + j] = make_float2(0.f, 0.f);
    }
    if (threadIdx.x == 0) {
        a.state[c].y = active;
        a.state[c].w &= ~(FLAG_PRE | LA_MASK | SEQ_MASK);
    }
}

template <class K>
hipError_t lds_attr(K kern, size_t lds) {
    if (lds > 64 * 1024)
        return hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return hipSuccess;
}

template <int LM>
hipError_t lg_process_t(const ProcArgs &a, const LgTab &t, int chunks, int channels, hipStream_t s) {
    using G = LgGeo<LM>;
    for (int j = 0; j < a.njobs; ++j) {
        LgPass p{};
        p.J = a.job[j];
        p.tb = t;
        p.gw = a.gw;
        p.gw_p = a.gw_p;
        p.gw_t = a.gw_t;
        if (!p.J.lg_prog || !p.J.lg_v) return hipErrorInvalidValue;
        if (p.J.n <= 0) continue;
        if (hipError_t e = lds_attr(lg_rows<LM, LG_CONV>, G::row_lds); e != hipSuccess) return e;
        const bool wide = (long long)channels * G::NTILE <= LG_WIDE_MAX_TILES;
#ifndef FFTCONV_LG_END_FUSED
#define FFTCONV_LG_END_FUSED 1
#endif
        p.end_fused = FFTCONV_LG_END_FUSED && chunks == 1 && !p.J.add0 && !p.J.tin;
        for (int it = 0; it < chunks; ++it) {
            if (wide)
                hipLaunchKernelGGL((lg_cols_fwd<LM, LG_CONV, LG_CNT_WIDE>), dim3(channels * G::NTILE), dim3(LG_CNT_WIDE),
                                   G::col_lds, s, p);
            else
                hipLaunchKernelGGL((lg_cols_fwd<LM, LG_CONV>), dim3(channels * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
            hipLaunchKernelGGL((lg_rows<LM, LG_CONV>), dim3(channels * G::NPAIR), dim3(LG_NT), G::row_lds, s, p);
            if (wide)
                hipLaunchKernelGGL((lg_cols_inv<LM, LG_CONV, LG_CNT_WIDE>), dim3(channels * G::NTILE), dim3(LG_CNT_WIDE),
                                   G::col_lds, s, p);
            else
                hipLaunchKernelGGL((lg_cols_inv<LM, LG_CONV>), dim3(channels * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
        }
        if (!p.end_fused) hipLaunchKernelGGL(lg_call_end, dim3(channels), dim3(256), 0, s, p.J);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int LM>
hipError_t lg_ir_t(const IrArgs &a, const LgTab &t, int channels, hipStream_t s) {
    using G = LgGeo<LM>;
    constexpr size_t B = (size_t)1 << LM;
    const long long active = (a.len_active + (long long)B - 1) / (long long)B;
    if (a.update_state) hipLaunchKernelGGL(lg_update_state, dim3(channels), dim3(256), 0, s, a, (int)B, (int)active);
    const int nseg = (int)std::min<long long>(a.S, active);
    if (nseg > 0) {
        LgPass p{};
        p.tb = t;
        p.src = a.src;
        p.src_stride = a.src_stride;
        p.len_data = a.len_data;
        p.H = a.H;
        p.S = a.S;
        p.chan0 = a.chan0;
        p.nseg = nseg;
        if (hipError_t e = lds_attr(lg_rows<LM, LG_IR>, G::row_lds); e != hipSuccess) return e;
        const long long rows = (long long)channels * nseg;
        if (rows * G::NPAIR > INT32_MAX) return hipErrorInvalidValue;
        hipLaunchKernelGGL((lg_cols_fwd<LM, LG_IR>), dim3((unsigned)(rows * G::NTILE)), dim3(LG_NT), G::col_lds, s, p);
        hipLaunchKernelGGL((lg_rows<LM, LG_IR>), dim3((unsigned)(rows * G::NPAIR)), dim3(LG_NT), G::row_lds, s, p);
    }
    if (nseg < a.S) {  // segments past the response: zero (:210-212)
        const size_t pitch = (size_t)a.S * B * sizeof(float2);
        float2 *base = a.H + ((size_t)a.chan0 * a.S + nseg) * B;
        if (hipError_t e = hipMemset2DAsync(base, pitch, 0, (size_t)(a.S - nseg) * B * sizeof(float2), channels, s);
            e != hipSuccess)
            return e;
    }
    return hipGetLastError();
}

template <int LM>
hipError_t lg_fft_t(bool inverse, const FftArgs &a, const LgTab &t, float2 *scratch, int rows, int batch,
                    hipStream_t s) {
    using G = LgGeo<LM>;
    auto kb = inverse ? lg_rows<LM, LG_RAWINV> : lg_rows<LM, LG_RAW>;
    if (hipError_t e = lds_attr(kb, G::row_lds); e != hipSuccess) return e;
    for (int r0 = 0; r0 < rows; r0 += batch) {
        const int n = std::min(batch, rows - r0);
        LgPass p{};
        p.tb = t;
        p.in = a.in;
        p.in_stride = a.in_stride;
        p.out = a.out;
        p.out_stride = a.out_stride;
        p.status = a.status;
        p.Y = scratch;
        p.row0 = r0;
        if (!inverse) {
            hipLaunchKernelGGL((lg_cols_fwd<LM, LG_RAW>), dim3(n * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
            hipLaunchKernelGGL(kb, dim3(n * G::NPAIR), dim3(LG_NT), G::row_lds, s, p);
        } else {
            hipLaunchKernelGGL(kb, dim3(n * G::NPAIR), dim3(LG_NT), G::row_lds, s, p);
            hipLaunchKernelGGL((lg_cols_inv<LM, LG_RAWINV>), dim3(n * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
        }
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// Fft of any length n (src/fft_convolver.rs:29-49; realfft plans every
// length, RealToComplexOdd / Even over rustfft's mixed-radix, Rader and
// Bluestein plans).  Here every non-power-of-two n runs Bluestein's chirp-z
// transform over the power-of-two complex FFTs above:
//   X[k] = conj(w_k) sum_j (s_j conj(w_j)) w_(k-j),  w_m = exp(i pi m^2 / n),
// the circular convolution of length P = 2^LP >= 2n - 1 as FFT, product with
// the chirp filter's spectrum Bf (f64 on the host, rounded), inverse FFT.
// P <= 8192: one workgroup per row in LDS (natural order); larger P: the
// four-step passes, with the spectra (A and Bf) in the transposed order.
// Forward: s = x (real), bins 0..n/2 out, DC (and an even n's Nyquist)
// imaginary part exactly 0.  Inverse: s = conj of the Hermitian spectrum
// (DC / Nyquist imaginary parts taken as 0, flagged as FftError::InputValues),
// out = Re(DFT(s)) / n -- divided, as Fft::inverse (:44-46), unless flagged.
// ---------------------------------------------------------------------------
struct BsPass {
    int n, inverse;
    const float *in;
    long long in_stride;
    float *out;
    long long out_stride;
    int *status;
    const float2 *w;    // [n] chirp
    const float2 *bf;   // [P] filter spectrum
    const float2 *twP;  // W_{2P}^i, i < 2P (one-workgroup FFT)
    LgTab tb;           // four-step tables of P (twM = W_P^j)
    float2 *Y;          // [rows][P] scratch (four-step)
    int row0;
};

// s_j of row r: the sequence whose forward DFT is wanted
__device__ __forceinline__ float2 bs_src(const BsPass &p, const float *in, int j) {
    if (!p.inverse) return make_float2(in[j], 0.f);
    const int nb = p.n / 2;  // last bin
    // conj(X_full[j]): X_full[j] = bin j (j <= n/2) or conj(bin n - j)
    DBG_CHECK(j >= 0 && j < p.n, 57, j, p.n, 0, 0);  // (site 57: a Bluestein source index)
    if (j <= nb) {
        const bool real = j == 0 || (2 * j == p.n);  // DC / Nyquist: imaginary part taken as 0
        return make_float2(in[2 * j], real ? 0.f : -in[2 * j + 1]);
    }
    return make_float2(in[2 * (p.n - j)], in[2 * (p.n - j) + 1]);
}
__device__ __forceinline__ bool bs_flagged(const BsPass &p, const float *in) {
    return p.inverse && (in[1] != 0.f || (p.n % 2 == 0 && in[p.n + 1] != 0.f));
}
// X_m = conj(w_m) c_m / P written out (forward: bins m <= n/2; inverse: sample m)
__device__ __forceinline__ void bs_out(const BsPass &p, float *o, int m, float2 c, float invP, bool flagged) {
    DBG_CHECK(m >= 0 && m < p.n, 58, m, p.n, 0, 0);  // (site 58: a Bluestein output index)
    const float2 x = cmulc(make_float2(c.x * invP, c.y * invP), p.w[m]);
    if (!p.inverse) {
        if (2 * m > p.n) return;
        const bool real = m == 0 || 2 * m == p.n;
        o[2 * m] = x.x;
        o[2 * m + 1] = real ? 0.f : x.y;
    } else {
        o[m] = flagged ? x.x : x.x / (float)p.n;
    }
}

template <int LP>
__global__ __launch_bounds__(LG_NT) void bs_small(BsPass p) {
    constexpr int P = 1 << LP;
    constexpr float invP = 1.0f / (float)P;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + P;
    const int tid = threadIdx.x;
    const size_t r = p.row0 + blockIdx.x;
    const float *in = p.in + r * p.in_stride;
    for (int j = tid; j < P; j += LG_NT) b0[j] = j < p.n ? cmulc(bs_src(p, in, j), p.w[j]) : make_float2(0.f, 0.f);
    __syncthreads();
    float2 *A = bfft<LP, 1, false, false>(b0, b1, p.twP, tid);
    float2 *Bq = A == b0 ? b1 : b0;
    for (int k = tid; k < P; k += LG_NT) Bq[k] = cmul(A[k], p.bf[k]);
    __syncthreads();
    const float2 *c = bfft<LP, 1, false, true>(Bq, A, p.twP, tid);
    const bool flagged = bs_flagged(p, in);
    if (p.status && tid == 0) p.status[r] = flagged ? 1 : 0;
    float *o = p.out + r * p.out_stride;
    for (int m = tid; m < p.n; m += LG_NT) bs_out(p, o, m, c[m], invP, flagged);
}

// four-step, pass A: pre-chirp, column FFTs, x W_P^(n2 k1) -> Y
template <int LP>
__global__ __launch_bounds__(LG_NT) void bs_cols_fwd(BsPass p) {
    using G = LgGeo<LP>;
    constexpr int M2 = G::M2, TC = G::TC, P = G::M;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + G::E;
    const int tid = threadIdx.x, c0 = (int)(blockIdx.x % G::NTILE) * TC;
    const size_t row = blockIdx.x / G::NTILE;
    const float *in = p.in + (p.row0 + row) * p.in_stride;
    for (int e = tid; e < G::E; e += LG_NT) {
        const int j = (e / TC) * M2 + c0 + (e & (TC - 1));
        b0[e] = j < p.n ? cmulc(bs_src(p, in, j), p.w[j]) : make_float2(0.f, 0.f);
    }
    __syncthreads();
    const float2 *R = bfft<G::L1, TC, true, false>(b0, b1, p.tb.twA, tid);
    float2 *Y = p.Y + row * P;
    for (int e = tid; e < G::E; e += LG_NT) {
        const int t = e & (TC - 1), k1 = e / TC, n2 = c0 + t;
        Y[(size_t)k1 * M2 + n2] = cmul(R[e], p.tb.twM[(n2 * k1) & (P - 1)]);
    }
}

// pass B: one row k1: row FFT, x Bf (transposed order), inverse row FFT,
// x W_P^-(n2 k1), in place
template <int LP>
__global__ __launch_bounds__(LG_NT) void bs_rows(BsPass p) {
    using G = LgGeo<LP>;
    constexpr int M1 = G::M1, M2 = G::M2, P = G::M;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + M2;
    const int tid = threadIdx.x, k1 = (int)(blockIdx.x % M1);
    const size_t row = blockIdx.x / M1;
    float2 *Y = p.Y + row * P + (size_t)k1 * M2;
    for (int e = tid; e < M2; e += LG_NT) b0[e] = Y[e];
    __syncthreads();
    float2 *F = bfft<G::L2, 1, false, false>(b0, b1, p.tb.twB, tid);
    float2 *Gb = F == b0 ? b1 : b0;
    for (int e = tid; e < M2; e += LG_NT) {
        DBG_CHECK((size_t)k1 * M2 + e < (size_t)P, 59, k1, e, M2, P);  // (site 59: the filter spectrum)
        Gb[e] = cmul(F[e], p.bf[(size_t)k1 * M2 + e]);
    }
    __syncthreads();
    const float2 *R = bfft<G::L2, 1, false, true>(Gb, F, p.tb.twB, tid);
    for (int e = tid; e < M2; e += LG_NT) Y[e] = cmulc(R[e], p.tb.twM[(e * k1) & (P - 1)]);
}

// pass C: inverse column FFTs -> c_m, m = M2 n1 + n2; post-chirp and out
template <int LP>
__global__ __launch_bounds__(LG_NT) void bs_cols_inv(BsPass p) {
    using G = LgGeo<LP>;
    constexpr int M2 = G::M2, TC = G::TC, P = G::M;
    constexpr float invP = 1.0f / (float)P;
    extern __shared__ __attribute__((aligned(16))) unsigned char lg_smem[];
    float2 *b0 = reinterpret_cast<float2 *>(lg_smem), *b1 = b0 + G::E;
    const int tid = threadIdx.x, c0 = (int)(blockIdx.x % G::NTILE) * TC;
    const size_t row = blockIdx.x / G::NTILE;
    const float2 *V = p.Y + row * P;
    for (int e = tid; e < G::E; e += LG_NT) b0[e] = V[(size_t)(e / TC) * M2 + c0 + (e & (TC - 1))];
    __syncthreads();
    const float2 *R = bfft<G::L1, TC, true, true>(b0, b1, p.tb.twA, tid);
    const size_t r = p.row0 + row;
    const float *in = p.in + r * p.in_stride;
    const bool flagged = bs_flagged(p, in);
    if (p.status && blockIdx.x % G::NTILE == 0 && tid == 0) p.status[r] = flagged ? 1 : 0;
    float *o = p.out + r * p.out_stride;
    for (int e = tid; e < G::E; e += LG_NT) {
        const int m = (e / TC) * M2 + c0 + (e & (TC - 1));
        if (m < p.n) bs_out(p, o, m, R[e], invP, flagged);
    }
}

template <int LP>
hipError_t bs_launch_t(const BsPass &p0, int rows, int batch, hipStream_t s) {
    if constexpr (LP <= 13) {
        constexpr size_t lds = 2 * ((size_t)1 << LP) * sizeof(float2);
        if (hipError_t e = lds_attr(bs_small<LP>, lds); e != hipSuccess) return e;
        BsPass p = p0;
        p.row0 = 0;
        hipLaunchKernelGGL(bs_small<LP>, dim3(rows), dim3(LG_NT), lds, s, p);
        return hipGetLastError();
    } else {
        using G = LgGeo<LP>;
        for (int r0 = 0; r0 < rows; r0 += batch) {
            const int nr = std::min(batch, rows - r0);
            BsPass p = p0;
            p.row0 = r0;
            hipLaunchKernelGGL(bs_cols_fwd<LP>, dim3(nr * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
            hipLaunchKernelGGL(bs_rows<LP>, dim3(nr * G::M1), dim3(LG_NT), 2 * (size_t)G::M2 * sizeof(float2), s, p);
            hipLaunchKernelGGL(bs_cols_inv<LP>, dim3(nr * G::NTILE), dim3(LG_NT), G::col_lds, s, p);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        }
        return hipSuccess;
    }
}

}  // namespace

#define LG_DISPATCH(FN, LM, ...)                     \
    switch (LM) {                                    \
        case 14: return FN<14>(__VA_ARGS__);         \
        case 15: return FN<15>(__VA_ARGS__);         \
        case 16: return FN<16>(__VA_ARGS__);         \
        case 17: return FN<17>(__VA_ARGS__);         \
        case 18: return FN<18>(__VA_ARGS__);         \
        case 19: return FN<19>(__VA_ARGS__);         \
        case 20: return FN<20>(__VA_ARGS__);         \
        case 21: return FN<21>(__VA_ARGS__);         \
        case 22: return FN<22>(__VA_ARGS__);         \
        default: return hipErrorInvalidValue;        \
    }

void lg_split(int log2b, int *l1, int *l2) {
    *l2 = log2b - 6 < 11 ? log2b - 6 : 11;
    *l1 = log2b - *l2;
}

size_t lg_position(int log2b, size_t k) {
    int l1, l2;
    lg_split(log2b, &l1, &l2);
    const size_t m1 = (size_t)1 << l1;
    return (k & (m1 - 1)) * ((size_t)1 << l2) + (k >> l1);
}

hipError_t launch_process_large(int log2b, const ProcArgs &a, const LgTab &t, int chunks, int channels,
                                hipStream_t s) {
    if (channels <= 0) return hipSuccess;
    LG_DISPATCH(lg_process_t, log2b, a, t, chunks, channels, s)
}

hipError_t launch_ir_large(int log2b, const IrArgs &a, const LgTab &t, int channels, hipStream_t s) {
    if (channels <= 0 || a.S <= 0) return hipSuccess;
    LG_DISPATCH(lg_ir_t, log2b, a, t, channels, s)
}

hipError_t launch_fft_large(int log2m, bool inverse, const FftArgs &a, const LgTab &t, float2 *scratch, int rows,
                            int batch, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    LG_DISPATCH(lg_fft_t, log2m, inverse, a, t, scratch, rows, batch, s)
}

hipError_t launch_fft_bluestein(size_t n, int log2p, bool inverse, const FftArgs &a, const float2 *chirp,
                                const float2 *filt, const float2 *twP, const LgTab &t, float2 *scratch, int rows,
                                int batch, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    if (n < 1 || n > INT32_MAX) return hipErrorInvalidValue;
    BsPass p{};
    p.n = (int)n;
    p.inverse = inverse ? 1 : 0;
    p.in = a.in;
    p.in_stride = a.in_stride;
    p.out = a.out;
    p.out_stride = a.out_stride;
    p.status = a.status;
    p.w = chirp;
    p.bf = filt;
    p.twP = twP;
    p.tb = t;
    p.Y = scratch;
    switch (log2p) {
#define BSC(L) case L: return bs_launch_t<L>(p, rows, batch, s);
        BSC(1) BSC(2) BSC(3) BSC(4) BSC(5) BSC(6) BSC(7) BSC(8) BSC(9) BSC(10) BSC(11) BSC(12) BSC(13)
        BSC(14) BSC(15) BSC(16) BSC(17) BSC(18) BSC(19) BSC(20) BSC(21) BSC(22)
#undef BSC
        default: return hipErrorInvalidValue;
    }
}

}  // namespace fftconv
