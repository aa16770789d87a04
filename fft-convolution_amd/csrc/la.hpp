// la.hpp -- lookahead step: FFTConvolver::process with the FDL sum
// re-associated in time (included by kernels.hip after its helpers).
//
// The reference computes, for every block s of a channel (src/fft_convolver.rs
// :258-275),
//     conv_s = sum_{i=1}^{act-1} H[i] (.) X_{s-i}  +  H[0] (.) X_s
// where X_b is the spectrum of block b (FDL row (current + age) % act).  Every
// step re-reads all act rows of H and of the FDL: 16 B per bin-row, the whole
// 773 KB per channel-block at cfg2.  But a far row i > D only meets blocks
// that are at least i - D steps old, so the terms of the next D steps that
// use far rows are known D steps ahead.  An *anchor* at step a computes them
// all in ONE pass over H and the FDL, keeping a window of D X rows in
// registers:
//     P_j = sum_{i > D} H[i] (.) X_{a+j-i},    j = 1..D
// and the D steps that follow only add their D near rows (H[1..D] and the
// last D blocks: 32 KB per channel, hot in the Infinity Cache) and H[0] X_s.
// The far-row bytes per channel-block drop from 16 S B to ~16 S B / D; the
// per-step work stays zero-latency (step s needs nothing after block s).
//
// Anchors are staggered over channels (channel c anchors when (c - t) % D
// == 0, t = launch counter), so every launch carries C / D anchors and the
// per-launch bytes are even.  Anchor and step workgroups of one launch touch
// disjoint memory: an anchor reads FDL ages >= 1 (the step writes age 0) and
// writes the other P window (two windows per channel, FLAG_PWIN).
//
// Summation order (canonical, phase independent).  The far rows [D+1, act)
// split into NG fixed groups; each group is ONE sequential chain over its
// rows (even groups descending, odd ascending -- neighbouring groups then
// read their shared window rows at the same time); groups combine in a
// fixed tree (sequentially within an anchor workgroup's lanesets, then over
// the workgroups).  The near rows D..1 form their own chain, then
//     pre = near + A,    conv = pre + H[0] (.) X_s     (slot_mac, as :270-275).
// An anchor's j-th accumulator visits exactly the rows and the blocks the
// step a+j would, in the same order, so a step served from a window and a
// step that computes everything itself (entry, after update / reset /
// partial calls) produce the same bits.  Results therefore do not depend on
// the stagger, the channel index or the shard size.
#pragma once
// (no namespace of its own: included inside namespace fftconv)

constexpr int LA_D = 8;             // steps served per anchor (window)
constexpr int LA_U = 2;             // anchor: H / X rows in flight per lane
constexpr int LA_RS = LA_D + LA_U;  // anchor: X register ring (window + prefetch)
constexpr int LA_NT = 256;          // threads per workgroup (anchor and step roles)
constexpr int LA_NG = 8;            // far-row groups
constexpr int LA_CU = 8;            // full-pass chain: rows in flight per lane
constexpr int LA_OOB = 0x7ffffff0;  // a buffer voffset past every stream's range

typedef float f2v __attribute__((ext_vector_type(2)));

// Per-row operands of one float4 slot (2 bins).  Bin 0 of slot 0 is the packed
// (DC, Nyquist) pair, multiplied component-wise; operand selection makes the
// same two packed FMAs do both (q0 = 0 adds a signed zero there).
struct LaH {
    f2v p0, q0, p1, q1;
};
__device__ __forceinline__ LaH la_ops(float4 h, bool z0) {
    LaH o;
    o.p0 = f2v{h.x, z0 ? h.y : h.x};
    o.q0 = z0 ? f2v{0.f, 0.f} : f2v{-h.y, h.y};
    o.p1 = f2v{h.z, h.z};
    o.q1 = f2v{-h.w, h.w};
    return o;
}
// complex_multiply_accumulate (src/fft_convolver.rs:76-88) over 2 bins:
// re = fma(-h.im, x.im, fma(h.re, x.re, re)), im = fma(h.im, x.re, fma(h.re, x.im, im))
struct LaAcc {
    f2v a01, a23;
    __device__ __forceinline__ void zero() { a01 = f2v{0.f, 0.f}; a23 = f2v{0.f, 0.f}; }
    __device__ __forceinline__ void mac(const LaH &h, float4 x) {
        a01 = __builtin_elementwise_fma(h.p0, f2v{x.x, x.y}, a01);
        a01 = __builtin_elementwise_fma(h.q0, f2v{x.y, x.x}, a01);
        a23 = __builtin_elementwise_fma(h.p1, f2v{x.z, x.w}, a23);
        a23 = __builtin_elementwise_fma(h.q1, f2v{x.w, x.z}, a23);
    }
    __device__ __forceinline__ float4 get() const { return make_float4(a01.x, a01.y, a23.x, a23.y); }
};

__device__ __forceinline__ int la_jget(int w) { return (w >> LA_J_SHIFT) & 15; }
__device__ __forceinline__ int la_dget(int w) { return (w >> LA_D_SHIFT) & 15; }

// the lookahead step applies: one whole block from an empty input buffer, at
// least one far row
template <int LOG2B>
__device__ __forceinline__ bool la_eligible(int4 st, int n) {
    return n == (1 << LOG2B) && st.z == 0 && !(st.w & FLAG_INBUF) && st.y >= LA_D + 2 && st.x < st.y;
}
__device__ __forceinline__ int la_phase(int c, const ProcArgs &a) {
    const int r = (c - a.la_t) % LA_D;
    return r < 0 ? r + LA_D : r;
}
__device__ __forceinline__ bool la_sched(int c, const ProcArgs &a) {
    return a.la_all > 0 || (a.la_all == 0 && la_phase(c, a) == 0);
}
// window of a new anchor: up to the channel's next stagger slot
__device__ __forceinline__ int la_dnew(int c, const ProcArgs &a) {
    const int r = la_phase(c, a);
    return r == 0 ? LA_D : r;
}
// far-row group g of NG: rows [lo, hi) of [D+1, act)
__device__ __forceinline__ void la_group(int g, int NG, int act, int &lo, int &hi) {
    const int nf = act - LA_D - 1;
    lo = LA_D + 1 + (g * nf) / NG;
    hi = LA_D + 1 + ((g + 1) * nf) / NG;
}
// P row of (channel, window, step j of the window, anchor part w)
__device__ __forceinline__ float4 *la_prow(const ProcArgs &a, size_t c, int win, int j, int w, int B) {
    return reinterpret_cast<float4 *>(a.laP + ((((c * 2 + win) * LA_D + j) * (size_t)a.la_W + w) * (size_t)B));
}

// ---------------------------------------------------------------------------
// Anchor walk over one far-row group [lo, hi) in direction ASC: for window
// steps j = 1..D, acc[j-1] += H[i] (.) X(age i - j at the anchor), rows in
// the group's order.  X rows live in a register ring indexed by the walk
// position e (age lo - D + e ascending, hi - 2 - e descending); each row of H
// and of the FDL is loaded once, LA_U rows ahead.
// ---------------------------------------------------------------------------
template <int LOG2B, bool ASC, bool NTL>
__device__ __forceinline__ void la_walk(LaAcc (&acc)[LA_D], const RowStream &hs, const RowStream &xs, int voff,
                                        bool z0, int lo, int hi, int cur, int act) {
    constexpr int ROWB = (1 << LOG2B) * (int)sizeof(float2);
    const int n = hi - lo;
    const int ne = n + LA_D - 1;
    auto xoff = [&](int e) {
        const int age = ASC ? lo - LA_D + e : hi - 2 - e;
        int r = cur + age;
        if (r >= act) r -= act;
        return r * ROWB;
    };
    auto hoff = [&](int k) { return (ASC ? lo + k : hi - 1 - k) * ROWB; };
    // rows past the walk are loaded from an out-of-range buffer offset (zero,
    // no memory access): no branches around the loads, no register copies
    auto vo = [&](bool in) { return in ? voff : LA_OOB; };
    float4 xr[LA_RS], hr[LA_U];
#pragma unroll
    for (int e = 0; e < LA_RS - 1; ++e) xr[e] = xs.ld4<NTL>(vo(e < ne), xoff(e < ne ? e : 0));
#pragma unroll
    for (int k = 0; k < LA_U; ++k) hr[k] = hs.ld4<NTL>(vo(k < n), hoff(k < n ? k : 0));
    for (int k0 = 0; k0 < n; k0 += LA_RS) {
#pragma unroll
        for (int u = 0; u < LA_RS; ++u) {
            const int k = k0 + u;
            if (k >= n) break;
            const LaH h = la_ops(hr[u % LA_U], z0);
#pragma unroll
            for (int j = 0; j < LA_D; ++j) acc[j].mac(h, xr[(ASC ? u + LA_D - 1 - j : u + j) % LA_RS]);
            const bool hin = k + LA_U < n, xin = k + LA_RS - 1 < ne;
            hr[u % LA_U] = hs.ld4<NTL>(vo(hin), hoff(hin ? k + LA_U : 0));
            xr[(u + LA_RS - 1) % LA_RS] = xs.ld4<NTL>(vo(xin), xoff(xin ? k + LA_RS - 1 : 0));
            // keep the issue order: the scheduler would otherwise hoist the
            // loads of later rows and run out of registers
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// One group's chain for the current step (window step 0: X age i), the same
// rows in the same order as an anchor's accumulators.
template <int LOG2B, bool ASC, bool NTL>
__device__ __forceinline__ void la_chain(LaAcc &acc, const RowStream &hs, const RowStream &xs, int voff, bool z0,
                                         int lo, int hi, int cur, int act) {
    constexpr int ROWB = (1 << LOG2B) * (int)sizeof(float2);
    const int n = hi - lo;
    for (int k0 = 0; k0 < n; k0 += LA_CU) {
        float4 hv[LA_CU], xv[LA_CU];
#pragma unroll
        for (int u = 0; u < LA_CU; ++u) {
            const bool in = k0 + u < n;
            const int i = in ? (ASC ? lo + k0 + u : hi - 1 - k0 - u) : lo;
            int r = cur + i;
            if (r >= act) r -= act;
            hv[u] = hs.ld4<NTL>(in ? voff : LA_OOB, i * ROWB);
            xv[u] = xs.ld4<NTL>(in ? voff : LA_OOB, r * ROWB);
        }
#pragma unroll
        for (int u = 0; u < LA_CU; ++u)
            if (k0 + u < n) acc.mac(la_ops(hv[u], z0), xv[u]);
    }
}

template <int LOG2B>
struct LaGeo {
    static constexpr int B = 1 << LOG2B, F = B / 2, LPW = LA_NT / F;
    static constexpr size_t anchor_bytes = (size_t)(LPW - 1) * LA_D * F * 16;
};

// ---------------------------------------------------------------------------
// Anchor workgroup b: part w of channel c's anchor (groups w*LPW .. +LPW-1,
// one per laneset of F lanes), combined in laneset order and stored as
// window rows P[win][j][w], j < d.
// ---------------------------------------------------------------------------
template <int LOG2B, bool NTL>
__device__ __forceinline__ void la_anchor(const ProcArgs &a, int b, unsigned char *smem) {
    using LG = LaGeo<LOG2B>;
    constexpr int B = LG::B, F = LG::F, LPW = LG::LPW;
    const ProcJob &J = a.job[0];
    const int W = a.la_W;
    const int ci = b / W, w = b - ci * W;
    const int c = a.la_all > 0 ? ci : a.la_t + LA_D * ci;
    const int4 st = J.state[c];
    const int sx = __builtin_amdgcn_readfirstlane(st.x), sy = __builtin_amdgcn_readfirstlane(st.y);
    const int sz = __builtin_amdgcn_readfirstlane(st.z), sw = __builtin_amdgcn_readfirstlane(st.w);
    const int act = sy;
    int cur, win, d;
    if (((sw & SEQ_MASK) >> SEQ_SHIFT) == a.la_seq) {
        // this launch's step has already stored the channel's state: it
        // opened a window iff the state says so (j = 0)
        if (!(sw & FLAG_LA) || la_jget(sw) != 0) return;
        cur = sx + 1 == act ? 0 : sx + 1;
        win = (sw & FLAG_PWIN) ? 1 : 0;
        d = la_dget(sw);
    } else {
        if (!la_eligible<LOG2B>(make_int4(sx, sy, sz, sw), J.n)) return;
        cur = sx;
        win = (sw & FLAG_PWIN) ? 0 : 1;
        d = la_dnew(c, a);
    }

    const int tid = threadIdx.x;
    const int l = __builtin_amdgcn_readfirstlane(tid / F), f = tid % F;
    const int NG = W * LPW, g = w * LPW + l;
    int lo, hi;
    la_group(g, NG, act, lo, hi);
    const size_t rows = (size_t)J.S * B;
    const size_t bytes = rows * sizeof(float2);
    const RowStream hs(J.H + (size_t)c * rows, bytes), xs(J.X + (size_t)c * rows, bytes);
    LaAcc acc[LA_D];
#pragma unroll
    for (int j = 0; j < LA_D; ++j) acc[j].zero();
    if (hi > lo) {
        if (g & 1) la_walk<LOG2B, true, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
        else la_walk<LOG2B, false, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
    }
    if constexpr (LPW > 1) {
        float4 *red = reinterpret_cast<float4 *>(smem);  // [LPW-1][D][F]
        if (l > 0) {
#pragma unroll
            for (int j = 0; j < LA_D; ++j) red[((l - 1) * LA_D + j) * F + f] = acc[j].get();
        }
        __syncthreads();
        if (l == 0) {
#pragma unroll
            for (int j = 0; j < LA_D; ++j) {
                if (j < d) {
                    float4 p = acc[j].get();
#pragma unroll
                    for (int q = 1; q < LPW; ++q) p = vadd(p, red[((q - 1) * LA_D + j) * F + f]);
                    la_prow(a, c, win, j, w, B)[f] = p;
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < LA_D; ++j)
            if (j < d) la_prow(a, c, win, j, w, B)[f] = acc[j].get();
    }
}

// ---------------------------------------------------------------------------
// Step workgroup: one full block of each of NCH channels (FFTConvolver::
// process :229-309 for the common call).  Wave k < NCH runs channel k's
// transform chain (R2C of the block into FDL row `current`, then conv, C2R,
// overlap-add) while the other waves form every channel's
// pre = near rows D..1 + far partials (from the window, or -- `full` -- from
// the far-row groups all four waves sum first).  Two channels per workgroup
// at B <= 256: the step and anchor workgroups of a launch then fit the CUs
// together (4 workgroups per CU at 128 VGPRs), so the anchors' stream runs
// under the steps' transform chains instead of after them.
// ---------------------------------------------------------------------------
template <int LOG2B>
struct LaStep {
    static constexpr int B = 1 << LOG2B, F = B / 2, LPW = LA_NT / F;
    static constexpr int NCH = LOG2B <= 8 ? 2 : 1;           // channels per step workgroup
    static constexpr int HL = LA_NT - 64 * NCH;               // helper lanes
    static constexpr int TPL = (NCH * F + HL - 1) / HL;       // pre slots per helper lane
    // tw (2B float2) | per channel: bufA | bufB | H0 | pre (float2) | overlap | tail0 | tail1 (float)
    static constexpr size_t ch_bytes = 4 * 8 * (size_t)B + 3 * 4 * (size_t)B;
    static constexpr size_t chain_bytes = 16 * (size_t)B + NCH * ch_bytes;
    // the full pass's group partials alias the chain buffers (done before them)
    static constexpr size_t grp_bytes = (size_t)NCH * LA_NG * F * 16;
    static constexpr size_t bytes = chain_bytes > grp_bytes ? chain_bytes : grp_bytes;
};

template <int LOG2B, bool NTL, int NCH>
__device__ __forceinline__ void la_step(const ProcArgs &a, const ProcJob &J, const int (&cs)[NCH],
                                        const int4 (&st)[NCH], const bool (&full)[NCH], const bool (&sched)[NCH],
                                        int nvalid, unsigned char *smem) {
    using LS = LaStep<LOG2B>;
    constexpr int B = LS::B, F = LS::F, LPW = LS::LPW;
    constexpr int HL = LA_NT - 64 * NCH;
    constexpr int TPL = (NCH * F + HL - 1) / HL;
    constexpr int ROWB = B * (int)sizeof(float2);
    constexpr float invN = 1.0f / (float)(2 * B);
    constexpr size_t chb = 4 * 8 * (size_t)B + 3 * 4 * (size_t)B;
    float2 *twl = reinterpret_cast<float2 *>(smem);
    auto chan_lds = [&](int k) { return smem + 16 * (size_t)B + (size_t)k * chb; };
    float4 *grp = reinterpret_cast<float4 *>(smem);  // [NCH][NG][F], full pass only

    static_assert(NCH == 1 || NCH == 2, "one or two channels per step workgroup");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = a.la_W, NG = W * LPW;
    // per-channel values by a runtime channel index without private-array
    // indexing (which would put the arrays in scratch)
    auto ST = [&](int k) { return (NCH == 1 || k == 0) ? st[0] : st[NCH - 1]; };
    auto CS = [&](int k) { return (NCH == 1 || k == 0) ? cs[0] : cs[NCH - 1]; };
    auto FULL = [&](int k) { return (NCH == 1 || k == 0) ? full[0] : full[NCH - 1]; };
    auto SCHED = [&](int k) { return (NCH == 1 || k == 0) ? sched[0] : sched[NCH - 1]; };
    const size_t rows = (size_t)J.S * B;
    const size_t bytes = rows * sizeof(float2);
    bool anyfull = false;
#pragma unroll
    for (int k = 0; k < NCH; ++k) anyfull |= k < nvalid && FULL(k);

    // helper slot t of this lane: channel k, slot f (valid if k < nvalid)
    auto task = [&](int t, int &k, int &f) {
        const int idx = (tid - 64 * NCH) + t * HL;
        k = idx / F;
        f = idx - k * F;
        return idx < NCH * F && k < nvalid;
    };
    float4 Areg[TPL];
    if (anyfull) {
        // every far-row group's chain of the channels that sum everything, into LDS
        const int l = __builtin_amdgcn_readfirstlane(tid / F), f = tid % F;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            if (k >= nvalid || !FULL(k)) continue;
            const int cur = __builtin_amdgcn_readfirstlane(ST(k).x), act = __builtin_amdgcn_readfirstlane(ST(k).y);
            const RowStream hs(J.H + (size_t)CS(k) * rows, bytes), xs(J.X + (size_t)CS(k) * rows, bytes);
            for (int g = l; g < NG; g += LPW) {
                int lo, hi;
                la_group(g, NG, act, lo, hi);
                LaAcc acc;
                acc.zero();
                if (g & 1) la_chain<LOG2B, true, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
                else la_chain<LOG2B, false, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
                grp[(k * NG + g) * F + f] = acc.get();
            }
        }
        __syncthreads();
        if (wave >= NCH) {  // each helper slot's A, in the anchors' tree order
#pragma unroll
            for (int t = 0; t < TPL; ++t) {
                int k, f;
                if (!task(t, k, f) || !FULL(k)) continue;
                float4 A;
                for (int w = 0; w < W; ++w) {
                    float4 pw = grp[(k * NG + w * LPW) * F + f];
#pragma unroll
                    for (int q = 1; q < LPW; ++q) pw = vadd(pw, grp[(k * NG + w * LPW + q) * F + f]);
                    A = w == 0 ? pw : vadd(A, pw);
                }
                Areg[t] = A;
            }
        }
        __syncthreads();  // the chain buffers below overwrite the group partials
    }

    float2 *Z = nullptr, *Q = nullptr;
    if (wave < NCH) {
        if (wave >= nvalid) return;
        // ---- transform chain of channel k = wave: the block -> R2C -> FDL row `current`
        const int k = wave;
        const size_t c = (size_t)CS(k);
        const int cur = __builtin_amdgcn_readfirstlane(ST(k).x);
        float2 *bufA = reinterpret_cast<float2 *>(chan_lds(k));
        float2 *bufB = bufA + B, *h0l = bufB + B;
        float *ovl = reinterpret_cast<float *>(h0l + 2 * B);
        float *p0l = ovl + B, *p1l = p0l + B;
        const float *inc = J.in + c * J.in_stride;
        dma_f32<64>(reinterpret_cast<float *>(bufA), inc, B);  // x[0..B) as packed z[0..B/2)
        for (int m = B / 2 + lane; m < B; m += 64) bufA[m] = make_float2(0.f, 0.f);
        if (k == 0) dma_16b<64>(twl, a.tw, 2 * B * (int)sizeof(float2));
        dma_16b<64>(h0l, J.H + c * rows, B * (int)sizeof(float2));
        dma_f32<64>(ovl, J.overlap + c * B, B);
        if (J.add0) dma_f32<64>(p0l, J.add0 + c * J.add_stride, B);
        if (J.add1) dma_f32<64>(p1l, J.add1 + c * J.add_stride, B);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (NCH > 1) {
            __syncthreads();  // wave 0's twiddle table is in LDS
        } else {
            wave_sync();
        }
        if (J.tin) {  // two-stage: append the block to tail_input (:473-475)
            const float *xb = reinterpret_cast<const float *>(bufA);
            float *ti = J.tin + c * J.tin_stride;
            for (int j = lane; j < B; j += 64) ti[j] = xb[j];
        }
        wave_sync();
        Z = lds_cfft<LOG2B, 64, false, true>(bufA, bufB, twl);  // :243-255
        Q = Z == bufA ? bufB : bufA;
        float2 *Xcur = J.X + c * rows + (size_t)cur * B;
        for (int m = lane; m < B; m += 64) {
            const float2 v = real_post<LOG2B, 64>(Z, m, twl);
            Q[m] = v;
            Xcur[m] = v;
        }
    } else {
        if constexpr (NCH > 1) __syncthreads();  // (the chain waves' twiddle barrier)
        // ---- pre = near chain (rows D..1) + far partials A, canonical order
#pragma unroll
        for (int t = 0; t < TPL; ++t) {
            int k, f;
            if (!task(t, k, f)) continue;
            const size_t c = (size_t)CS(k);
            const int cur = ST(k).x, act = ST(k).y, flags = ST(k).w;
            const RowStream hs(J.H + c * rows, bytes), xs(J.X + c * rows, bytes);
            float4 hv[LA_D], xv[LA_D];
#pragma unroll
            for (int i = LA_D; i >= 1; --i) {
                int r = cur + i;
                if (r >= act) r -= act;
                hv[i - 1] = hs.ld4<false>(f * 16, i * ROWB);
                xv[i - 1] = xs.ld4<false>(f * 16, r * ROWB);
            }
            float4 A;
            if (FULL(k)) {
                A = Areg[t];
            } else {
                const int win = (flags & FLAG_PWIN) ? 1 : 0;
                const float4 *P0 = la_prow(a, c, win, la_jget(flags), 0, B);
                A = P0[f];
                for (int w = 1; w < W; ++w) A = vadd(A, P0[(size_t)w * F + f]);
            }
            LaAcc acc;
            acc.zero();
#pragma unroll
            for (int i = LA_D; i >= 1; --i) acc.mac(la_ops(hv[i - 1], f == 0), xv[i - 1]);
            float2 *prel = reinterpret_cast<float2 *>(chan_lds(k)) + 3 * B;
            reinterpret_cast<float4 *>(prel)[f] = vadd(acc.get(), A);
            __builtin_amdgcn_sched_barrier(0);  // one slot's 2D + W rows in flight at a time
        }
    }
    __syncthreads();
    if (wave >= NCH) return;

    const int k = wave;
    const size_t c = (size_t)CS(k);
    const int cur = __builtin_amdgcn_readfirstlane(ST(k).x), act = __builtin_amdgcn_readfirstlane(ST(k).y);
    const int flags = __builtin_amdgcn_readfirstlane(ST(k).w);
    float2 *bufA = reinterpret_cast<float2 *>(chan_lds(k));
    float2 *h0l = bufA + 2 * B, *prel = bufA + 3 * B;
    float *ovl = reinterpret_cast<float *>(bufA + 4 * B);
    float *p0l = ovl + B, *p1l = p0l + B;
    float *outc = J.out + c * J.out_stride;
    float *ovc = J.overlap + c * B;
    bool bad = false;  // conv = pre + X (.) H[0] (:270-275), then the C2R error check
    for (int f = lane; f < F; f += 64) {
        const float4 cv = slot_mac(reinterpret_cast<const float4 *>(prel)[f], reinterpret_cast<const float4 *>(Q)[f],
                                   reinterpret_cast<const float4 *>(h0l)[f], f);
        reinterpret_cast<float4 *>(Z)[f] = cv;
        if (f == 0 && !slot0_finite(cv)) bad = true;
    }
    const bool err = __ballot(bad) != 0ull;
    wave_sync();
    const int keep = flags & ~(FLAG_INBUF | FLAG_PRE | LA_MASK | SEQ_MASK);
    const int tag = a.la_seq << SEQ_SHIFT;
    if (!err) {
        for (int m = lane; m < B; m += 64) Q[m] = real_pre<LOG2B, 64>(Z, m, twl);
        wave_sync();
        const float *y = reinterpret_cast<const float *>(lds_cfft<LOG2B, 64, true, true>(Q, Z, twl));
        for (int j = lane; j < B; j += 64) {  // overlap-add (:284-288) + two-stage adds (:453-468)
            float v = y[j] * invN + ovl[j];
            if (J.add0) {
                v += p0l[j];
                if (J.add1) v += p1l[j];
            }
            outc[j] = v;
            ovc[j] = y[B + j] * invN;  // :297-298
        }
        if (lane == 0) {
            const int curp = cur > 0 ? cur - 1 : act - 1;  // :301-305
            int nf = (keep ^ FLAG_REV) | tag;
            if (SCHED(k)) nf = (nf ^ FLAG_PWIN) | FLAG_LA | (la_dnew((int)c, a) << LA_D_SHIFT);
            else if (!FULL(k)) nf |= FLAG_LA | ((la_jget(flags) + 1) << LA_J_SHIFT) | (la_dget(flags) << LA_D_SHIFT);
            J.state[c] = make_int4(curp, act, 0, nf);
        }
    } else {
        // output.fill(0); return (:278-281): the block stays in the input
        // buffer, fill / current unchanged; the window is dropped
        const float *inc = J.in + c * J.in_stride;
        float *ibc = J.inbuf + c * B;
        for (int j = lane; j < B; j += 64) {
            float v = 0.f;
            if (J.add0) {
                v += p0l[j];
                if (J.add1) v += p1l[j];
            }
            outc[j] = v;
            ibc[j] = inc[j];
        }
        if (lane == 0) J.state[c] = make_int4(cur, act, 0, keep | FLAG_INBUF | tag);
    }
}

// a channel off the lookahead path (partial block, buffered input, short
// response) in the workgroup: its channels run one at a time, out of line
// (the rare fallback keeps its registers out of the step's allocation)
template <int LOG2B, bool NTL>
__device__ __attribute__((noinline)) void la_fallback(const ProcArgs *ap, int c0, int nvalid, unsigned char *smem) {
    const ProcArgs &a = *ap;
    const ProcJob &J = a.job[0];
    for (int k = 0; k < nvalid; ++k) {
        if (k) __syncthreads();
        const int c = c0 + k;
        const int4 st = J.state[c];
        if (la_eligible<LOG2B>(st, J.n)) {
            const int c1[1] = {c};
            const int4 s1[1] = {st};
            const bool f1[1] = {!((st.w & FLAG_LA) && la_jget(st.w) < la_dget(st.w))};
            const bool h1[1] = {la_sched(c, a)};
            la_step<LOG2B, NTL, 1>(a, J, c1, s1, f1, h1, 1, smem);
        } else {
            process_job<LOG2B, LA_NT, false, NTL>(a, J, (size_t)c, st, smem);
        }
    }
}

template <int LOG2B, bool NTL>
__global__ __launch_bounds__(LA_NT, 4) void upols_la_kernel(ProcArgs a) {
    using LS = LaStep<LOG2B>;
    constexpr int NCH = LS::NCH;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nstep = (int)gridDim.x - a.la_nanchor;  // step workgroups
    const int b = blockIdx.x;
    const int ba = a.la_steps_first ? b - nstep : b;  // anchor index, < 0 for a step
    if (ba >= 0 && ba < a.la_nanchor) {
        if (a.la_probe != 1) la_anchor<LOG2B, NTL>(a, ba, smem);
        return;
    }
    if (a.la_probe == 2) return;
    const int c0 = (a.la_steps_first ? b : b - a.la_nanchor) * NCH;
    const ProcJob &J = a.job[0];
    const int nvalid = min(NCH, a.la_channels - c0);
    int cs[NCH];
    int4 st[NCH];
    bool full[NCH], sched[NCH];
    bool all = true;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        cs[k] = c0 + k;
        int4 v = k < nvalid ? J.state[cs[k]] : make_int4(0, 0, 0, 0);
        // wave-uniform: keep the state words in scalar registers
        st[k] = make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                          __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
        all &= k >= nvalid || la_eligible<LOG2B>(st[k], J.n);
        full[k] = !((st[k].w & FLAG_LA) && la_jget(st[k].w) < la_dget(st[k].w));
        sched[k] = la_sched(cs[k], a);
    }
    if (all) la_step<LOG2B, NTL, NCH>(a, J, cs, st, full, sched, nvalid, smem);
    else  // (the arguments by their kernarg address: no private copy of the block)
        la_fallback<LOG2B, NTL>((const ProcArgs *)__builtin_amdgcn_kernarg_segment_ptr(), c0, nvalid, smem);
}
