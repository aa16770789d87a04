// la.hpp -- lookahead step: FFTConvolver::process with the FDL sum
// re-associated in time (included by kernels.hip, inside namespace fftconv,
// after its helpers).
//
// The reference computes, for every block s of a channel (src/fft_convolver.rs
// :244-261),
//     conv_s = sum_{i=1}^{act-1} H[i] (.) X_{s-i}  +  H[0] (.) X_s
// where X_b is the spectrum of block b (FDL row (current + age) % act).  Every
// step re-reads all act rows of H and of the FDL: 16 B per bin-row, 773 KB
// per channel-block at cfg2.  But a row i only meets blocks at least i steps
// old, so its terms for the next j < i steps are known now.  The rows split
// into a near level and three anchor levels by that horizon:
//   near rows 1..D0          summed by each step itself;
//   level 1  rows D0+1..R1   summed by an anchor every P1 <= D0 steps for the
//                            P1 steps after it (X ages >= 1 at the anchor);
//   level 2  rows R1+1..R2   every P2 <= R1 steps, for the P2 steps after it;
//   level 3  rows R2+1..     every P3 <= R2 steps, for the P3 steps after it.
// (D0 = P1 = 4, R1 = P2 = 16, R2 = P3 = 64: geometric periods.  Against the
// three levels of round 2 -- near 1..5, 6..32 every 5, 33.. every 32 -- the
// row transfers per cfg2 channel-block drop from 40.3 to 36.5 and the
// longest walks from 27 (in-step) / 39 (far) rows to 12 / 31.)
// An anchor walks its rows once, keeping a window of X rows in registers, and
// leaves one partial-sum row per future step (the level's window in HBM).
// Per channel-block level L costs 16 B (2 n_L + P_L - 1) / (2 P_L) per bin
// for its n_L rows, plus one window row written and one read.  The step stays
// zero-latency: step s needs nothing after block s.
//
// Anchors are staggered over channels (channel c anchors at level L when
// (c - t) % P_L == 0, t = launch counter), so every launch carries C/P_L
// anchors of each level and the per-launch bytes are even.  Anchor and step
// workgroups of one launch touch disjoint memory: an anchor reads FDL ages
// >= 1 (the step writes age 0) and writes the other window of its level (two
// per channel and level).  A window row is stored at the position of the
// step it serves: the step of launch t reads row (t - 1 - c) mod P_L, so an
// anchor that opens a short window (entry, rebuild: up to the channel's next
// stagger slot) writes the tail of the window and no step counter is kept.
//
// Summation order (canonical, phase independent).  Each level is a fixed set
// of sequential chains: near rows D0..1; level 1 rows R1..D0+1; levels 2 and
// 3 in NG fixed groups (even groups descending, odd ascending, so that
// neighbouring groups read their shared window rows at the same time)
// combined in group order.  Then
//     pre = near + (W1 + (W2 + W3)),   conv = pre + H[0] (.) X_s  (slot_mac, :256-261).
// An anchor's accumulator for step a+j visits exactly the rows and blocks the
// step a+j would, in the same order, so a step served from windows and a step
// that sums everything itself (entry, after update / reset / partial calls,
// VARIANT_LAFULL) give the same bits: results do not depend on the stagger,
// the channel index or the shard size.
#pragma once
// (no namespace of its own: included inside namespace fftconv)

constexpr int LA_D0 = 4;                     // near rows 1..D0, summed by the step
constexpr int LA_P1 = 4, LA_R1 = 16;         // level 1: rows D0+1..R1, period P1
constexpr int LA_P2 = 16, LA_R2 = 64;        // level 2: rows R1+1..R2, period P2
constexpr int LA_P3 = 64;                    // level 3: rows R2+1..act-1, period P3
constexpr int LA_PT = LA_P1 + LA_P2 + LA_P3;  // window rows per channel and window
constexpr int LA_PER = 64;                   // stagger clock modulus (every period divides it)
constexpr int LA_JW = 8;                     // far-style window steps per workgroup (register window)
constexpr int LA_U = 2;                      // anchor: H / X rows in flight per lane
constexpr int LA_UF = 2;                     // level 2/3 anchors: H / X rows in flight per lane
// level-1 walks: H / X rows in flight per lane for a window of JM steps per
// laneset -- 4 where the X ring (JM + U rows) is a whole number of U-row
// turns (the 4-step in-step walk at B = 256: 16.60 vs 17.19 us per cfg2
// step with 2, r3), else 2 or 3, so the unrolled ring stays short
__host__ __device__ constexpr int la_um(int JM) { return JM >= 4 ? 4 : (JM == 2 ? 2 : 3); }
constexpr int LA_NT = 256;                   // threads per workgroup (anchor and step roles)
constexpr int LA_NG = 4;                     // row groups of a level 2/3 anchor (one wave each)
constexpr int LA_CU = 8;                     // full-pass chain: rows in flight per lane
constexpr int LA_OOB = 0x7ffffff0;           // a buffer voffset past every stream's range
// launch shape: the largest log2 B whose step workgroups run the level-1
// anchors (else level-1 anchor workgroups); the smallest log2 B whose helpers
// store the next block's near sum (round-3 A/Bs)
constexpr int LA_MIDIN_MAXLOG = 8;
constexpr int LA_NEARNEXT_MINLOG = 9;
static_assert(LA_P1 <= LA_D0 && LA_P2 <= LA_R1 && LA_P3 <= LA_R2, "a level's rows are older than its window");
static_assert(LA_PER % LA_P1 == 0 && LA_PER % LA_P2 == 0 && LA_PER % LA_P3 == 0, "stagger clock");
static_assert(LA_P2 % LA_JW == 0 && LA_P3 % LA_JW == 0 && LA_P1 <= 8, "window slices");

// level lv (1..3): period, first row, end of its rows for an FDL of act
// segments, offset of its window rows
__host__ __device__ constexpr int la_per(int lv) { return lv == 1 ? LA_P1 : (lv == 2 ? LA_P2 : LA_P3); }
__host__ __device__ constexpr int la_lo(int lv) { return lv == 1 ? LA_D0 + 1 : (lv == 2 ? LA_R1 + 1 : LA_R2 + 1); }
__host__ __device__ constexpr int la_hi(int lv, int act) {
    return lv == 1 ? (act < LA_R1 + 1 ? act : LA_R1 + 1) : (lv == 2 ? (act < LA_R2 + 1 ? act : LA_R2 + 1) : act);
}
__host__ __device__ constexpr int la_off(int lv) { return lv == 1 ? 0 : (lv == 2 ? LA_P1 : LA_P1 + LA_P2); }
__host__ __device__ constexpr int la_flag_live(int lv) { return FLAG_LA1 << (2 * (lv - 1)); }
__host__ __device__ constexpr int la_flag_win(int lv) { return FLAG_PW1 << (2 * (lv - 1)); }
// anchor levels of a geometry: level 3 only when some FDL row reaches it
__host__ __device__ constexpr int la_nlv(int S) { return S > LA_R2 + 1 ? 3 : 2; }

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
// complex_multiply_accumulate (src/fft_convolver.rs:62-74) over 2 bins:
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

__device__ __forceinline__ bool la_live(int w, int lv) { return (w & la_flag_live(lv)) != 0; }

// the lookahead step applies: one whole block from an empty input buffer, at
// least one level-1 row
template <int LOG2B>
__device__ __forceinline__ bool la_eligible(int4 st, int n) {
    return n == (1 << LOG2B) && st.z == 0 && !(st.w & (FLAG_INBUF | FLAG_CALLDONE)) && st.y >= LA_D0 + 2 &&
           st.x < st.y;
}
// stagger phase of channel c at level period P (la_t = launch counter mod LA_PER)
__device__ __forceinline__ int la_phase(int c, const ProcArgs &a, int P) {
    const int r = (c - a.la_t) % P;
    return r < 0 ? r + P : r;
}
__device__ __forceinline__ bool la_sched(int c, const ProcArgs &a, int P) {
    return a.la_all > 0 || (a.la_all == 0 && la_phase(c, a, P) == 0);
}
// window of a new anchor: up to the channel's next stagger slot
__device__ __forceinline__ int la_dnew(int c, const ProcArgs &a, int P) {
    const int r = la_phase(c, a, P);
    return r == 0 ? P : r;
}
// the window row the step of this launch reads: (t - 1 - c) mod P
__device__ __forceinline__ int la_pos(int c, const ProcArgs &a, int P) {
    const int r = (a.la_t - 1 - c) % P;
    return r < 0 ? r + P : r;
}
// level-1 window split over L lanesets: ceil(P1 / L) steps each; the last
// laneset's run is shifted back to end at step P1 (no step past the window:
// its rows would meet blocks not yet written) and stores only the steps it owns
__host__ __device__ constexpr int la_mid_per(int L) { return (LA_P1 + (L < LA_P1 ? L : LA_P1) - 1) / (L < LA_P1 ? L : LA_P1); }
__device__ __forceinline__ int la_mid_j0(int l, int JM) { return min(l * JM, LA_P1 - JM); }
// row group g (of NG) of level lv walks descending, or ascending for odd g
// (neighbouring groups then read their shared X rows at the same time)
__host__ __device__ constexpr bool la_asc(int g) { return (g & 1) != 0; }
// level lv's row group g of LA_NG: rows [lo, hi) (empty when act is short)
__device__ __forceinline__ void la_group(int lv, int g, int act, int &lo, int &hi) {
    const int l0 = la_lo(lv), h0 = la_hi(lv, act);
    const int nf = h0 > l0 ? h0 - l0 : 0;
    lo = l0 + (g * nf) / LA_NG;
    hi = l0 + ((g + 1) * nf) / LA_NG;
}
// window row `pos` of level lv: W[c][win][off(lv) + pos]
__device__ __forceinline__ float4 *la_win(const ProcArgs &a, int jb, size_t c, int win, int lv, int pos, int B) {
#ifdef FFTCONV_DEBUG_BOUNDS
    if (!(c < (size_t)a.la_channels && win >= 0 && win < 2 && lv >= 1 && lv <= 3 && pos >= 0 && pos < la_per(lv))) {
        dbg_bounds(4, (int)c, win, lv, pos);  // (site 4: a window row index)
        c = 0; win = 0; lv = 1; pos = 0;
    }
#endif
    return reinterpret_cast<float4 *>((jb ? a.laW2 : a.laW) + (((c * 2 + win) * LA_PT + la_off(lv) + pos) * (size_t)B));
}

// Crossfade A and B in one launch (XF 3, CrossfadeConvolver::process
// :72-77): both convolvers see the same input, so while their ring states
// agree and FLAG_XSYNC says they always have, their FDLs are equal row for
// row.  B's FDL reads then go to A's copy: A's and B's walkers of a channel run
// side by side on one XCD (la_kernel_body's XF 3 grid), and the second read
// of each row is an L2 hit -- one X stream for both windows.  (The anchors
// read the pair from the launch-start copies, ProcJob::sview.)
__device__ __forceinline__ bool la_xf_paired(int4 sa, int4 sb) {
    return (sa.w & sb.w & FLAG_XSYNC) && sa.x == sb.x && sa.y == sb.y && sa.z == sb.z &&
           !((sa.w ^ sb.w) & FLAG_INBUF);
}
__device__ __forceinline__ const float2 *la_xsrc(const ProcArgs &a, int jb, size_t c) {
    if (jb == 0 || a.la_mix != 3) return a.job[jb].X;
    // (the anchors' copies of the words: the steps of this launch rewrite `state`)
    const int4 *va = a.job[0].sview ? a.job[0].sview : a.job[0].state;
    const int4 *vb = a.job[1].sview ? a.job[1].sview : a.job[1].state;
    const int4 sa = va[c], sb = vb[c];
    const int4 ua = make_int4(__builtin_amdgcn_readfirstlane(sa.x), __builtin_amdgcn_readfirstlane(sa.y),
                              __builtin_amdgcn_readfirstlane(sa.z), __builtin_amdgcn_readfirstlane(sa.w));
    const int4 ub = make_int4(__builtin_amdgcn_readfirstlane(sb.x), __builtin_amdgcn_readfirstlane(sb.y),
                              __builtin_amdgcn_readfirstlane(sb.z), __builtin_amdgcn_readfirstlane(sb.w));
    return la_xf_paired(ua, ub) ? a.job[0].X : a.job[1].X;
}

// ---------------------------------------------------------------------------
// Anchor walk over rows [lo, hi) in direction ASC for window steps
// j = j0+1 .. j0+JW: acc[jj] += H[i] (.) X(age i - j0 - 1 - jj at the anchor),
// rows in the chain's order.  X rows live in a register ring indexed by the
// walk position e; each row of H and of the FDL is loaded once, LA_U ahead.
// (Callers pass hi > lo.)
// ---------------------------------------------------------------------------
template <int LOG2B, bool ASC, bool NTL, int JW, int U = LA_U>
__device__ __forceinline__ void la_walk(LaAcc (&acc)[JW], const RowStream &hs, const RowStream &xs, int voff,
                                        bool z0, int lo, int hi, int j0, int cur, int act) {
    constexpr int ROWB = (1 << LOG2B) * (int)sizeof(float2);
    constexpr int RS = JW + U;                         // X ring: window + prefetch
    constexpr int UNR = RS % U == 0 ? RS : RS * U;  // static ring slots
    const int n = hi - lo;
    const int ne = n + JW - 1;
    auto xoff = [&](int e) {
        const int age = ASC ? lo - j0 - JW + e : hi - 2 - j0 - e;
        int r = cur + age;
        if (r >= act) r -= act;
        return r * ROWB;
    };
    auto hoff = [&](int k) { return (ASC ? lo + k : hi - 1 - k) * ROWB; };
    // rows past the walk are loaded from an out-of-range buffer offset (zero,
    // no memory access): no branches around the loads, no register copies
    auto vo = [&](bool in) { return in ? voff : LA_OOB; };
    float4 xr[RS], hr[U];
#pragma unroll
    for (int e = 0; e < RS - 1; ++e) xr[e] = xs.ld4<NTL>(vo(e < ne), xoff(e < ne ? e : 0));
#pragma unroll
    for (int k = 0; k < U; ++k) hr[k] = hs.ld4<NTL>(vo(k < n), hoff(k < n ? k : 0));
#pragma nounroll
    for (int k0 = 0; k0 < n; k0 += UNR) {  // (not unrolled: a constant walk would hoist every load)
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int k = k0 + u;
            if (k >= n) break;
            const LaH h = la_ops(hr[u % U], z0);
#pragma unroll
            for (int jj = 0; jj < JW; ++jj) acc[jj].mac(h, xr[(ASC ? u + JW - 1 - jj : u + jj) % RS]);
            const bool hin = k + U < n, xin = k + RS - 1 < ne;
            hr[u % U] = hs.ld4<NTL>(vo(hin), hoff(hin ? k + U : 0));
            xr[(u + RS - 1) % RS] = xs.ld4<NTL>(vo(xin), xoff(xin ? k + RS - 1 : 0));
            // keep the issue order: the scheduler would otherwise hoist the
            // loads of later rows and run out of registers
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// One chain for the current step (X age i), the same rows in the same order
// as an anchor's accumulators.
template <int LOG2B, bool ASC, bool NTL>
__device__ __forceinline__ void la_chain(LaAcc &acc, const RowStream &hs, const RowStream &xs, int voff, bool z0,
                                         int lo, int hi, int cur, int act) {
    constexpr int ROWB = (1 << LOG2B) * (int)sizeof(float2);
    const int n = hi - lo;
#pragma nounroll
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
    static constexpr int B = 1 << LOG2B, F = B / 2, LPW = LA_NT / F;  // lanesets of F lanes per workgroup
    // level 2/3 anchor workgroup: one bin slice of FS lanes (bins are
    // independent), the NG row groups (one wave-sized laneset each) of one
    // window slice of JW steps, combined in LDS into one window row per step;
    // one anchor = NSL bin slices x (P / JW) window slices, XCD-aligned (see
    // la_anchor_far)
    static constexpr int FS = F < 64 ? F : 64, NSL = F / FS, LPF = LA_NT / FS;
    static_assert(LPF == LA_NG, "one row group per wave-sized laneset");
    static constexpr int WG2 = NSL * (LA_P2 / LA_JW), WG3 = NSL * (LA_P3 / LA_JW);  // workgroups per anchor
    static constexpr int JM = la_mid_per(LPW);                  // level-1 window steps per laneset
    static constexpr size_t anchor_bytes = (size_t)(LA_NG - 1) * LA_JW * FS * 16;
};

// store policy of the launch's outputs (FFTCONV_LA_NTST bit 0 = window rows,
// bit 1 = the step's FDL row, bit 2 = output and overlap samples,
// nontemporal; the rows are read by later launches, on other XCDs)
#ifndef FFTCONV_LA_NTST
#define FFTCONV_LA_NTST 1  // (cfg2 A/B: window rows nontemporal 16.78 -> 16.44 us per step, r5h)
#endif
__device__ __forceinline__ void la_wst(float4 *p, float4 v) {
    if constexpr ((FFTCONV_LA_NTST & 1) != 0) ntst4(p, v);
    else *p = v;
}
__device__ __forceinline__ void la_ost(float *p, float v) {
    if constexpr ((FFTCONV_LA_NTST & 4) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// the anchor's view of channel c at level lv: its ring position, window and
// length, or false if this launch opens no window of the level at c.
//
// No word is read while it is written.  A lookahead launch's step rewrites
// its channels' state words while the launch's anchors run, so the anchors
// read ProcJob::sview instead: the words as the previous lookahead launch's
// steps left them (every step stores its final word to ProcJob::vnext as
// well as to `state`, la_step / la_fallback), or as the host copied them from
// `state` before a lookahead launch that follows any other state writer
// (update, reset, a partial or off-path call, clone; UniformCore::la_view).
// One launch writes the copy and a later one reads it, so the kernel boundary
// orders them (plain loads and stores, no atomicity assumed).  The copy is
// the word at the start of this launch: window step 0 serves this launch's
// step, whose row i meets FDL row (current + i) % act = age i.  The window
// rebuild runs no steps and reads `state`.
template <int LOG2B>
__device__ __forceinline__ bool la_anchor_state(const ProcArgs &a, int jb, int c, int lv, int &cur, int &act, int &win,
                                                int &d) {
    const ProcJob &J = a.job[jb];
    DBG_CHECK(c >= 0 && c < a.la_channels, 1, c, lv, a.la_channels, 0);  // (site 1: an anchor's channel)
    if (a.la_probe_cnt && !a.la_rebuild) {
        // (tests: FFTCONV_LA_PROBE) let the steps of this launch store their
        // words (each step fences its store out to memory), then read the
        // live word past this XCD's L2 and count the ones the step already
        // rewrote: the race the copy keeps the anchors out of
        for (int i = 0; i < 24; ++i) __builtin_amdgcn_s_sleep(127);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (threadIdx.x == 0) {
            const int lw = __hip_atomic_load(&J.state[c].w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (((lw & SEQ_MASK) >> SEQ_SHIFT) == a.la_seq) atomicAdd(a.la_probe_cnt, 1);
        }
    }
    const int4 st = (J.sview && !a.la_rebuild) ? J.sview[c] : J.state[c];
    const int sx = __builtin_amdgcn_readfirstlane(st.x), sy = __builtin_amdgcn_readfirstlane(st.y);
    const int sz = __builtin_amdgcn_readfirstlane(st.z), sw = __builtin_amdgcn_readfirstlane(st.w);
    const int pw = la_flag_win(lv);
    act = sy;
    d = la_dnew(c, a, la_per(lv));
    if (!la_eligible<LOG2B>(make_int4(sx, sy, sz, sw), J.n)) return false;
    if (a.la_rebuild) {
        // window rebuild (no steps in this launch): the window an anchor of
        // the previous launch would have opened, i.e. as after that launch's
        // step -- window step 0 serves the next step (current = sx), whose
        // row i meets FDL row (sx + i) % act = age i - 1 from sx + 1
        cur = sx + 1 == act ? 0 : sx + 1;
        win = (sw & pw) ? 0 : 1;
        return true;
    }
    cur = sx;
    win = (sw & pw) ? 0 : 1;
    return true;
}

// ---------------------------------------------------------------------------
// Level LV (2 or 3) anchor workgroup b: bin slice and window slice of one
// channel's anchor; the NG row groups (one per wave) combined in group order
// and stored as one window row per step.
// ---------------------------------------------------------------------------
template <int LOG2B, int LV, bool NTL, int UF = LA_UF, int JW = LA_JW>
__device__ __forceinline__ void la_anchor_far(const ProcArgs &a, int jb, int b, unsigned char *smem) {
    using LG = LaGeo<LOG2B>;
    constexpr int B = LG::B, P = la_per(LV), FS = LG::FS, NSL = LG::NSL;
    constexpr int WGA = NSL * (P / JW);
    static_assert(P % JW == 0, "window slices");
    const ProcJob &J = a.job[jb];
    // XCD-aware: workgroups are dealt to the 8 XCDs round-robin, so the WGA
    // workgroups of one anchor sit 8 apart -- on one XCD, whose L2 then
    // serves the rows the window slices and neighbouring groups share
    const int x = b & 7, y = b >> 3;
    const int ci = (y / WGA) * 8 + x, r = y % WGA;
    const int c = a.la_all > 0 ? a.la_c0 + ci : (a.la_t % P) + P * ci;
    if (c >= a.la_channels) return;  // (padding of the last XCD round)
    int cur, act, win, d;
    if (!la_anchor_state<LOG2B>(a, jb, c, LV, cur, act, win, d)) return;
    const int h = r / NSL;                   // window slice: steps h*JW .. h*JW+JW-1
    if (h * JW >= d) return;              // (wholly past the window)

    const int tid = threadIdx.x;
    const int l = __builtin_amdgcn_readfirstlane(tid / FS), fl = tid % FS;
    const int f = (r % NSL) * FS + fl;       // bin slice
    int lo, hi;
    la_group(LV, l, act, lo, hi);
    const size_t rows = (size_t)J.S * B;
    const size_t bytes = rows * sizeof(float2);
    const RowStream hs(J.H + (size_t)c * rows, bytes), xs(la_xsrc(a, jb, (size_t)c) + (size_t)c * rows, bytes);
    LaAcc acc[JW];
#pragma unroll
    for (int j = 0; j < JW; ++j) acc[j].zero();
    // (plain loads: the nontemporal policy streamed no faster here and cost the
    // step workgroups' cache-resident near rows ~8 % of the launch, r1i_la15_ab)
    if (hi > lo) {
        if (la_asc(l)) la_walk<LOG2B, true, false, JW, UF>(acc, hs, xs, f * 16, f == 0, lo, hi, h * JW, cur, act);
        else la_walk<LOG2B, false, false, JW, UF>(acc, hs, xs, f * 16, f == 0, lo, hi, h * JW, cur, act);
    }
    float4 *red = reinterpret_cast<float4 *>(smem);  // [NG-1][JW][FS]
    if (l > 0) {
#pragma unroll
        for (int j = 0; j < JW; ++j) red[((l - 1) * JW + j) * FS + fl] = acc[j].get();
    }
    __syncthreads();
    if (l == 0) {
#pragma unroll
        for (int j = 0; j < JW; ++j) {
            const int jj = h * JW + j;
            if (jj < d) {
                float4 p = acc[j].get();
#pragma unroll
                for (int q = 1; q < LA_NG; ++q) p = vadd(p, red[((q - 1) * JW + j) * FS + fl]);
                la_wst(la_win(a, jb, c, win, LV, P - d + jj, B) + f, p);
            }
        }
    }
}

// Level-1 anchor: channel c's rows R1..D0+1 (one descending chain per window
// step), the window steps split over the lanesets of l0 .. (l0 + L) with
// threads [t0, t0 + L*F).  Used by the level-1 anchor workgroups (B = 512)
// and by the step workgroups' helper waves (in-step, B <= 256).
template <int LOG2B, int JM>
__device__ __forceinline__ void la_level1(const ProcArgs &a, int jb, const float2 *X, int c, int cur, int act, int win,
                                          int d, int l, int f) {
    constexpr int B = 1 << LOG2B;
    const ProcJob &J = a.job[jb];
    const int hi = la_hi(1, act);
    if (hi <= LA_D0 + 1) return;
    const size_t rows = (size_t)J.S * B;
    const size_t bytes = rows * sizeof(float2);
    const RowStream hs(J.H + (size_t)c * rows, bytes), xs(X + (size_t)c * rows, bytes);
    const int j0 = la_mid_j0(l, JM);
    LaAcc acc[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) acc[j].zero();
    la_walk<LOG2B, false, false, JM, la_um(JM)>(acc, hs, xs, f * 16, f == 0, LA_D0 + 1, hi, j0, cur, act);
#pragma unroll
    for (int j = 0; j < JM; ++j)
        if (j0 + j >= l * JM && j0 + j < d) la_wst(la_win(a, jb, c, win, 1, LA_P1 - d + j0 + j, B) + f, acc[j].get());
}

// Level-1 anchor workgroup b (B = 512: the step workgroups have no helper
// laneset to spare).
template <int LOG2B>
__device__ __forceinline__ void la_anchor_mid(const ProcArgs &a, int jb, int b) {
    using LG = LaGeo<LOG2B>;
    constexpr int F = LG::F, JM = LG::JM;
    const int c = a.la_all > 0 ? a.la_c0 + b : (a.la_t % LA_P1) + LA_P1 * b;
    if (c >= a.la_channels) return;
    int cur, act, win, d;
    if (!la_anchor_state<LOG2B>(a, jb, c, 1, cur, act, win, d)) return;
    const int tid = threadIdx.x;
    const int l = __builtin_amdgcn_readfirstlane(tid / F), f = tid % F;
    if (l * JM >= LA_P1) return;  // (more lanesets than window steps)
    la_level1<LOG2B, JM>(a, jb, la_xsrc(a, jb, (size_t)c), c, cur, act, win, d, l, f);
}

// ---------------------------------------------------------------------------
// Step workgroup: one full block of each of NCH channels (FFTConvolver::
// process :215-295 for the common call).  Wave k < NCH runs channel k's
// transform chain (R2C of the block into FDL row `current`, then conv, C2R,
// overlap-add) while the other waves form every channel's
// pre = near + (W1 + (W2 + W3)), each level's partial from its window or --
// when the level has no live window (entry, after update / reset / partial
// calls) -- from chains all four waves sum first.  Two channels per
// workgroup at B <= 256: the step and anchor workgroups of a launch then fit
// the CUs together, so the anchors' stream runs under the transform chains.
// ---------------------------------------------------------------------------
template <int LOG2B, int XF = 0>
struct LaStep {
    static constexpr int B = 1 << LOG2B, F = B / 2, LPW = LA_NT / F;
    // channels per step workgroup (XF 3: A's and B's instance of one channel)
    static constexpr int NCH = (XF == 3 || LOG2B <= 8) ? 2 : 1;
    // B <= 256: the step workgroup's helper waves (>= one laneset of F lanes
    // after the pre) also run the level-1 anchors of its channels, after the
    // pre, under the transform chains; B = 512 launches level-1 anchor
    // workgroups
    // (XF 0: level 1 in the level-2 anchor workgroups instead, la_l1in2)
    static constexpr bool MIDIN = LOG2B <= LA_MIDIN_MAXLOG && XF != 0;
    static constexpr bool NEARNEXT = LOG2B >= LA_NEARNEXT_MINLOG;
    // tw (the 3N/4 = 1.5B float2 the transforms index) | per channel:
    // bufA | bufB | pre (float2) | tail0 | tail1 (float) -- H[0] and the
    // overlap stay in the chain wave's registers (XF 3 at B = 512: 38 KB, so
    // four workgroups fit a CU's 160 KB instead of three)
    static constexpr size_t tw_bytes = 12 * (size_t)B;
    static constexpr size_t ch_bytes = 3 * 8 * (size_t)B + 2 * 4 * (size_t)B;
    static constexpr size_t chain_bytes = tw_bytes + NCH * ch_bytes;
    // the full pass's chain results alias the chain buffers (they are
    // consumed before the chains start): per channel the level-1 chain and
    // the NG groups of levels 2 and 3 -- or, where one laneset runs every
    // chain of a channel in order (LPW == 1), one slot per level, folded
    // group by group as the anchors combine them
    static constexpr bool FOLD = LPW == 1;
    static constexpr int GSLOTS = FOLD ? 3 : 1 + 2 * LA_NG;
    static constexpr size_t grp_bytes = (size_t)NCH * GSLOTS * F * 16;
    // (+ the XF 3 mix counter after the chain buffers; it may alias the
    // full pass's results, which are consumed before the counter is set)
    static constexpr size_t cnt_off = chain_bytes;
    static constexpr size_t bytes = chain_bytes + 16 > grp_bytes ? chain_bytes + 16 : grp_bytes;
};

// A register value the compiler must treat as produced here.  The pre's
// "full-pass result (registers) or window row (HBM)" would otherwise be folded
// into ONE load through a selected pointer, which moves the full-pass
// registers to scratch: a scratch zero-fill in every step workgroup of every
// launch (4 MB of writes per cfg2 launch in round 2, left dirty at the kernel
// boundary) and flat loads for every window row.
__device__ __forceinline__ float4 la_opaque(float4 v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return v;
}

// launch timeline phase stamp k (0..3) of this wave (FFTCONV_LA_TRACE)
__device__ __forceinline__ void la_stamp(const ProcArgs &a, int k) {
    if (a.la_trace && (threadIdx.x & 63) == 0) {
        int *p = reinterpret_cast<int *>(a.la_trace + ((size_t)a.la_trace_grid * 4 + (size_t)blockIdx.x * 4 + (threadIdx.x >> 6)));
        p[k] = (int)(unsigned)__builtin_amdgcn_s_memrealtime();
    }
}

// XF 3 (crossfade A and B in one launch): a participant of the channel's mix
// (A's chain, B's chain, the helper that walks mix_value) has stored its part
// in LDS; the last of the three mixes the block into the output
// (Crossfader::mix, src/crossfade_convolver.rs:75-77, 242-278) -- no
// workgroup barrier, so the chain waves never wait for one another.
__device__ __forceinline__ void la_xf_arrive(const ProcArgs &a, int *cnt, const float *yA, const float *yB,
                                             const float *vtab, size_t c) {
    wave_sync();  // this wave's LDS stores are complete
    int old = 0;
    if ((threadIdx.x & 63) == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != 2) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const CrossfadeMixArgs &m = a.mix;
    float *o = a.job[0].out + c * a.job[0].out_stride;
    for (int j = (int)(threadIdx.x & 63); j < m.n; j += 64) o[j] = mix_select(yA[j], yB[j], mix_selector(m, j, vtab));
}

template <int LOG2B, bool NTL, int NCH, int XF>
__device__ __forceinline__ void la_step(const ProcArgs &a, const ProcJob &J, const int (&cs)[NCH],
                                        const int4 (&st)[NCH], int nvalid, unsigned char *smem) {
    using LS = LaStep<LOG2B, XF>;
    constexpr int B = LS::B, F = LS::F, LPW = LS::LPW, NG = LA_NG;
    constexpr int HL = LA_NT - 64 * NCH;
    constexpr int TPL = (NCH * F + HL - 1) / HL;
    constexpr int NCHAIN = 1 + 2 * NG;  // full pass: level-1 chain + the groups of levels 2 and 3, per channel
    constexpr int GS = LS::GSLOTS;      // LDS result slots per channel (LS::FOLD: one per level)
    constexpr int ROWB = B * (int)sizeof(float2);
    constexpr float invN = 1.0f / (float)(2 * B);
    constexpr size_t chb = LS::ch_bytes;
    static_assert(NCH == 1 || NCH == 2, "one or two channels per step workgroup");
    // a workgroup barrier after the chains' prologue (XF 3 only: the twiddle
    // table staged by wave 0 and the mix counter); otherwise the helpers issue
    // their near and window rows with the launch instead of after the chains'
    // prologue DMA has landed (r3 timeline: pre at 10.5 us, R2C done at 7.3)
    constexpr bool TWBAR = NCH > 1 && XF == 3;
    float2 *twl = reinterpret_cast<float2 *>(smem);
    auto chan_lds = [&](int k) { return smem + LS::tw_bytes + (size_t)k * chb; };
    float4 *grp = reinterpret_cast<float4 *>(smem);  // [NCH][GS][F], full pass only
    const int nlv = a.la_nlv;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const size_t rows = (size_t)J.S * B;
    const size_t bytes = rows * sizeof(float2);
    // per-channel values by a runtime channel index without private-array
    // indexing (which would put the arrays in scratch)
    auto ST = [&](int k) { return (NCH == 1 || k == 0) ? st[0] : st[NCH - 1]; };
    auto CS = [&](int k) { return (NCH == 1 || k == 0) ? cs[0] : cs[NCH - 1]; };
    // the instance of slot k: XF 3 runs A's (job 0) and B's (job 1) instance
    // of one channel; otherwise every slot is a channel of job 0
    auto JK = [&](int k) -> const ProcJob & { return (XF == 3 && k == 1) ? a.job[1] : J; };
    auto JB = [&](int k) { return (XF == 3 && k == 1) ? 1 : 0; };
    // the FDL the helpers read for slot k (XF 3: B's rows from A's copy when
    // the two are in step, la_xf_paired)
    const bool xpair = XF == 3 && la_xf_paired(st[0], st[NCH - 1]);
    auto XK = [&](int k) -> const float2 * { return (XF == 3 && k == 1 && xpair) ? a.job[0].X : JK(k).X; };
    // XF 3: A's / B's block and the mix_value walk in LDS (the two-stage add
    // buffers, unused by a crossfade), and the mix's arrival counter
    float *yA = reinterpret_cast<float *>(chan_lds(0) + 24 * (size_t)B), *yB = yA + B;
    float *vtab = reinterpret_cast<float *>(chan_lds(1) + 24 * (size_t)B);  // (B + 1 floats)
    // the chain wave's H[0] row slots and overlap samples (registers)
    float4 h0r[F / 64];
    float ovr[B / 64];
    int *xcnt = reinterpret_cast<int *>(smem + LS::cnt_off);
    // the helpers leave the next block's near sum (FLAG_NEAR) where the
    // step's pre is the launch's critical path: B = 512 (no in-step level-1
    // anchors; the crossfade's A + B pair: helper pre 13.9 -> 9.7 us, cfg5
    // 47.8 -> 45.8 us per step, r2j).  With in-step anchors (B <= 256) the
    // extra helper work after the barrier lengthens the anchor workgroups
    // (cfg2 18.97 -> 19.57 us, r2j), so those steps sum their near rows
    // themselves.
    auto near_next = [&](int) { return LS::NEARNEXT; };
    // a level without a live window is summed by the full pass
    auto full = [&](int k, int lv) { return lv <= nlv && !la_live(ST(k).w, lv); };
    bool anyfull = false;
#pragma unroll
    for (int k = 0; k < NCH; ++k) anyfull |= k < nvalid && (full(k, 1) || full(k, 2) || full(k, 3));

    // helper slot t of this lane: channel k, slot f (valid if k < nvalid)
    // (F is a multiple of 64 for B >= 128: k is wave-uniform; kept in an SGPR
    // where a lane has more than two tasks -- at two, the scheduler would then
    // overlap both tasks' rows and spill)
    auto task = [&](int t, int &k, int &f) {
        const int idx = (tid - 64 * NCH) + t * HL;
        k = TPL > 2 ? __builtin_amdgcn_readfirstlane(idx / F) : idx / F;
        f = idx - k * F;
        return idx < NCH * F && k < nvalid;
    };
    // the full pass's level sums: level 1, and the full ones of levels 2 / 3
    // (both: W2 + W3; one: that level's sum) -- two register sets, not three
    float4 W1reg[TPL], W23reg[TPL];
#pragma unroll
    for (int t = 0; t < TPL; ++t) W1reg[t] = W23reg[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (anyfull) {
        // the chains of the levels without a live window, into LDS
        const int l = __builtin_amdgcn_readfirstlane(tid / F), f = tid % F;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            if (k >= nvalid) continue;
            const int cur = __builtin_amdgcn_readfirstlane(ST(k).x), act = __builtin_amdgcn_readfirstlane(ST(k).y);
            const RowStream hs(JK(k).H + (size_t)CS(k) * rows, bytes), xs(JK(k).X + (size_t)CS(k) * rows, bytes);
            for (int q = l; q < NCHAIN; q += LPW) {
                const int lv = q == 0 ? 1 : (q <= NG ? 2 : 3);
                const int g = q == 0 ? 0 : (q - 1) % NG;
                if (!full(k, lv)) continue;
                int lo, hi;
                if (q == 0) {
                    lo = LA_D0 + 1;
                    hi = la_hi(1, act);
                } else {
                    la_group(lv, g, act, lo, hi);
                }
                LaAcc acc;
                acc.zero();
                if (hi > lo) {
                    if (q > 0 && la_asc(g)) la_chain<LOG2B, true, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
                    else la_chain<LOG2B, false, NTL>(acc, hs, xs, f * 16, f == 0, lo, hi, cur, act);
                }
                if constexpr (LS::FOLD) {
                    // this thread ran the level's earlier groups: fold in the
                    // anchors' order (group 0, then + each next)
                    float4 *slot = &grp[(k * GS + lv - 1) * F + f];
                    *slot = g == 0 ? acc.get() : vadd(*slot, acc.get());
                } else {
                    grp[(k * GS + q) * F + f] = acc.get();
                }
            }
        }
        __syncthreads();
        if (wave >= NCH) {  // each helper slot's level sums (the anchors' group order)
#pragma unroll
            for (int t = 0; t < TPL; ++t) {
                int k, f;
                if (!task(t, k, f)) continue;
                auto level = [&](int lv) {
                    if constexpr (LS::FOLD) {
                        return grp[(k * GS + lv - 1) * F + f];
                    } else {
                        if (lv == 1) return grp[(k * GS) * F + f];
                        const int q0 = 1 + (lv - 2) * NG;
                        float4 p = grp[(k * GS + q0) * F + f];
#pragma unroll
                        for (int g = 1; g < NG; ++g) p = vadd(p, grp[(k * GS + q0 + g) * F + f]);
                        return p;
                    }
                };
                if (full(k, 1)) W1reg[t] = level(1);
                if (full(k, 2) && full(k, 3)) W23reg[t] = vadd(level(2), level(3));
                else if (full(k, 2)) W23reg[t] = level(2);
                else if (full(k, 3)) W23reg[t] = level(3);
            }
        }
        __syncthreads();  // the chain buffers below overwrite the chain results
    }

    float2 *Z = reinterpret_cast<float2 *>(chan_lds(0)), *Q = Z + B;
    if (wave < NCH && wave >= nvalid) {
        // (no channel for this chain wave: it still takes part in the barriers)
        if constexpr (TWBAR) __syncthreads();
    } else if (wave < NCH) {
        // ---- transform chain of channel k = wave: the block -> R2C -> FDL row `current`
        const int k = wave;
        const ProcJob &JC = JK(k);
        const size_t c = (size_t)CS(k);
        const int cur = __builtin_amdgcn_readfirstlane(ST(k).x);
        DBG_CHECK(c < (size_t)a.la_channels && cur >= 0 && cur < J.S, 2, (int)c, cur, nvalid, 0);  // (site 2: a step chain)
        float2 *bufA = reinterpret_cast<float2 *>(chan_lds(k));
        float2 *bufB = bufA + B;
        float *p0l = reinterpret_cast<float *>(bufA + 3 * B), *p1l = p0l + B;
        const float *inc = JC.in + c * JC.in_stride;
        dma_f32<64>(reinterpret_cast<float *>(bufA), inc, B);  // x[0..B) as packed z[0..B/2)
        for (int m = B / 2 + lane; m < B; m += 64) bufA[m] = make_float2(0.f, 0.f);
        // the twiddle table: every chain wave stages it (the same bytes), so
        // no workgroup barrier holds the helpers' first loads behind the
        // chains' prologue (XF 3: wave 0, then the barrier that also
        // publishes the mix counter)
        if (!TWBAR || k == 0) dma_16b<64>(twl, a.tw, (int)LS::tw_bytes);
        if (XF == 3 && k == 0 && lane == 0) *xcnt = 0;  // (visible to all after the barrier below)
#pragma unroll
        for (int i = 0; i < F / 64; ++i) h0r[i] = reinterpret_cast<const float4 *>(JC.H + c * rows)[lane + 64 * i];
#pragma unroll
        for (int i = 0; i < B / 64; ++i) ovr[i] = JC.overlap[c * B + lane + 64 * i];
        if (JC.add0) dma_f32<64>(p0l, JC.add0 + c * JC.add_stride, B);
        if (JC.add1) dma_f32<64>(p1l, JC.add1 + c * JC.add_stride, B);
        if constexpr (XF == 2) {
            // crossfade, B's launch (no two-stage adds): A's block and the
            // per-sample mix selectors (la_mix_walk) in p0l / p1l
            dma_f32<64>(p0l, a.mix.buf_a + c * a.mix.buf_stride, B);
            dma_f32<64>(p1l, a.mix_tab, B);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        la_stamp(a, 0);
        if constexpr (TWBAR) {
            __syncthreads();  // wave 0's twiddle table is in LDS
        } else {
            wave_sync();
        }
        if (JC.tin) {  // two-stage: append the block to tail_input (:459-461)
            const float *xb = reinterpret_cast<const float *>(bufA);
            float *ti = JC.tin + c * JC.tin_stride;
            for (int j = lane; j < B; j += 64) ti[j] = xb[j];
        }
        wave_sync();
        // R2C (:229-241) with the last stage and the post-twiddle in
        // registers / across the wavefront (wave_r2c_post): the spectrum to
        // Q (LDS) and FDL row `current` (HBM)
        Q = fft_r2c_q_is_buf1<LOG2B>() ? bufB : bufA;
        Z = fft_r2c_q_is_buf1<LOG2B>() ? bufA : bufB;
        wave_r2c_post<LOG2B, 0, const float2 *, false, (FFTCONV_LA_NTST & 2) != 0>(bufA, bufB, twl, Q,
                                                                              JC.X + c * rows + (size_t)cur * B);
        la_stamp(a, 1);
    } else {
        if constexpr (TWBAR) __syncthreads();  // (the chain waves' twiddle barrier)
        // ---- pre = near chain (rows D0..1) + (W1 + (W2 + W3)), canonical order
#pragma unroll
        for (int t = 0; t < TPL; ++t) {
            int k, f;
            if (!task(t, k, f)) continue;
            const size_t c = (size_t)CS(k);
            const int cur = ST(k).x, act = ST(k).y, flags = ST(k).w;
            const bool nearp = (flags & FLAG_NEAR) != 0;  // the previous step left this block's near sum
            const RowStream hs(JK(k).H + c * rows, bytes), xs(XK(k) + c * rows, bytes);
            float4 hv[LA_D0], xv[LA_D0], N0;
            if (nearp) {
                N0 = reinterpret_cast<const float4 *>(JK(k).pre + c * B)[f];
            } else {
#pragma unroll
                for (int i = LA_D0; i >= 1; --i) {
                    int r = cur + i;
                    if (r >= act) r -= act;
                    hv[i - 1] = hs.ld4<false>(f * 16, i * ROWB);
                    xv[i - 1] = xs.ld4<false>(f * 16, r * ROWB);
                }
            }
            auto wrow = [&](int lv) {
                return la_win(a, JB(k), c, (flags & la_flag_win(lv)) ? 1 : 0, lv, la_pos((int)c, a, la_per(lv)), B)[f];
            };
            const float4 W1 = full(k, 1) ? la_opaque(W1reg[t]) : wrow(1);
            const bool f2 = full(k, 2), f3 = full(k, 3);
            float4 W23;
            if (nlv < 3) W23 = f2 ? la_opaque(W23reg[t]) : wrow(2);
            else if (f2 && f3) W23 = la_opaque(W23reg[t]);
            else if (f2) W23 = vadd(la_opaque(W23reg[t]), wrow(3));
            else if (f3) W23 = vadd(wrow(2), la_opaque(W23reg[t]));
            else W23 = vadd(wrow(2), wrow(3));
            if (!nearp) {
                LaAcc acc;
                acc.zero();
#pragma unroll
                for (int i = LA_D0; i >= 1; --i) acc.mac(la_ops(hv[i - 1], f == 0), xv[i - 1]);
                N0 = acc.get();
            }
            float2 *prel = reinterpret_cast<float2 *>(chan_lds(k)) + 2 * B;
            reinterpret_cast<float4 *>(prel)[f] = vadd(N0, vadd(W1, W23));
            if constexpr (TPL > 2) __builtin_amdgcn_sched_barrier(0);  // (one task's rows in flight at a time)
        }
        la_stamp(a, 0);
    }
    __syncthreads();
    la_stamp(a, 2);
    if (wave >= NCH) {
        if constexpr (XF == 3) {
            if (wave == NCH) {  // this call's mix_value walk (:259), one lane, then arrive
                if (a.mix.approaching && lane == 0)  // one f32 rounding each, as the reference
                    mix_walk_lane(vtab, a.mix.mix_value0, a.mix.step, a.mix.n);
                la_xf_arrive(a, xcnt, yA, yB, vtab, (size_t)CS(0));
            }
        }
        // the NEXT block's near sum, rows D0..1 in the canonical order, while
        // the chains run their C2R: rows D0..2 meet the blocks this step's
        // near rows met one age earlier, row 1 meets this step's block (the
        // chain's spectrum Q, kept in LDS) -- stored in pre[] (FLAG_NEAR)
        if constexpr (LS::NEARNEXT) {
            constexpr int QOFF = fft_r2c_q_is_buf1<LOG2B>() ? B : 0;  // (the chain's Q: wave_r2c_post)
#pragma unroll
            for (int t = 0; t < TPL; ++t) {
                int k, f;
                if (!task(t, k, f) || !near_next(k)) continue;
                const size_t c = (size_t)CS(k);
                const int cur = ST(k).x, act = ST(k).y;
                const RowStream hs(JK(k).H + c * rows, bytes), xs(XK(k) + c * rows, bytes);
                float4 hv[LA_D0], xv[LA_D0 - 1];
#pragma unroll
                for (int i = LA_D0; i >= 1; --i) {
                    hv[i - 1] = hs.ld4<false>(f * 16, i * ROWB);
                    if (i >= 2) {
                        int r = cur + i - 1;
                        if (r >= act) r -= act;
                        xv[i - 2] = xs.ld4<false>(f * 16, r * ROWB);
                    }
                }
                const float4 xq = reinterpret_cast<const float4 *>(reinterpret_cast<float2 *>(chan_lds(k)) + QOFF)[f];
                LaAcc acc;
                acc.zero();
#pragma unroll
                for (int i = LA_D0; i >= 2; --i) acc.mac(la_ops(hv[i - 1], f == 0), xv[i - 2]);
                acc.mac(la_ops(hv[0], f == 0), xq);
                reinterpret_cast<float4 *>(JK(k).pre + c * B)[f] = acc.get();
                if constexpr (TPL > 2) __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (LS::MIDIN) {
            // level-1 anchors of this workgroup's scheduled channels: rows
            // R1..D0+1 for the next P1 steps (the pre-launch ring position is
            // at hand)
            constexpr int LH = HL / F;  // helper lanesets
            constexpr int JMS = la_mid_per(LH);
            const int hl = tid - 64 * NCH;
            const int l = __builtin_amdgcn_readfirstlane(hl / F), f = hl % F;
            if (l * JMS < LA_P1) {
#pragma unroll
                for (int k = 0; k < NCH; ++k) {
                    if (k >= nvalid || !la_sched(CS(k), a, LA_P1)) continue;
                    const int c = CS(k);
                    const int cur = __builtin_amdgcn_readfirstlane(ST(k).x);
                    const int act = __builtin_amdgcn_readfirstlane(ST(k).y);
                    const int flags = __builtin_amdgcn_readfirstlane(ST(k).w);
                    const int win = (flags & FLAG_PW1) ? 0 : 1, d = la_dnew(c, a, LA_P1);
                    la_level1<LOG2B, JMS>(a, JB(k), XK(k), c, cur, act, win, d, l, f);
                }
            }
        }
        return;
    }
    if (wave >= nvalid) return;

    const int k = wave;
    const ProcJob &JC = JK(k);
    const size_t c = (size_t)CS(k);
    const int cur = __builtin_amdgcn_readfirstlane(ST(k).x), act = __builtin_amdgcn_readfirstlane(ST(k).y);
    const int flags = __builtin_amdgcn_readfirstlane(ST(k).w);
    float2 *bufA = reinterpret_cast<float2 *>(chan_lds(k));
    float2 *prel = bufA + 2 * B;
    float *p0l = reinterpret_cast<float *>(bufA + 3 * B), *p1l = p0l + B;
    // (XF 3: this instance's block goes to LDS, the mix writes the output)
    float *outc = XF == 3 ? (k == 0 ? yA : yB) : JC.out + c * JC.out_stride;
    float *ovc = JC.overlap + c * B;
    // crossfade, B's launch: out = mix(A's block, this block) (:75-77)
    bool bad = false;  // conv = pre + X (.) H[0] (:256-261), then the C2R error check
    la_stamp(a, 3);
#pragma unroll
    for (int i = 0; i < F / 64; ++i) {
        const int f = lane + 64 * i;
        const float4 cv = slot_mac(reinterpret_cast<const float4 *>(prel)[f], reinterpret_cast<const float4 *>(Q)[f],
                                   h0r[i], f);
        reinterpret_cast<float4 *>(Z)[f] = cv;
        if (f == 0 && !slot0_finite(cv) &&
            c2r_rejects(JC.H + c * rows, XK(k) + c * rows, B, cur, act, slot0_of(reinterpret_cast<const float4 *>(prel)[0]),
                        slot0_of(reinterpret_cast<const float4 *>(Q)[0]), slot0_of(h0r[0])))
            bad = true;
    }
    const bool err = __ballot(bad) != 0ull;
    wave_sync();
    const int keep = flags & ~(FLAG_INBUF | FLAG_PRE | LA_MASK | SEQ_MASK);
    const int tag = a.la_seq << SEQ_SHIFT;
    if (!err) {
        // C2R with the pre-twiddle fused into its first stage (wave_c2r),
        // ping-ponging through prel and Z: Q -- this block's spectrum --
        // stays intact for the helpers' next near sum
        const float *y = wave_c2r<LOG2B>(Z, prel, Z, twl);
#pragma unroll
        for (int i = 0; i < B / 64; ++i) {  // overlap-add (:270-274) + two-stage adds (:439-454)
            const int j = lane + 64 * i;
            float v = y[j] * invN + ovr[i];
            if (JC.add0) {
                v += p0l[j];
                if (JC.add1) v += p1l[j];
            }
            if constexpr (XF == 2) v = mix_select(p0l[j], v, p1l[j]);
            la_ost(outc + j, v);
            la_ost(ovc + j, y[B + j] * invN);  // :283-284
        }
        if (lane == 0) {
            const int curp = cur > 0 ? cur - 1 : act - 1;  // :287-291
            int nf = (keep ^ FLAG_REV) | tag | (near_next(k) ? FLAG_NEAR : 0);  // (the helpers stored it)
            // per level: open a window (an anchor this launch), keep it, or drop it
            for (int lv = 1; lv <= nlv; ++lv) {
                if (la_sched((int)c, a, la_per(lv))) nf = (nf ^ la_flag_win(lv)) | la_flag_live(lv);
                else if (la_live(flags, lv)) nf |= la_flag_live(lv);
            }
            JC.state[c] = make_int4(curp, act, 0, nf);
            if (JC.vnext) JC.vnext[c] = make_int4(curp, act, 0, nf);  // (the next launch's anchors)
            if (a.la_probe_cnt) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (tests: the probe)
        }
    } else {
        // output.fill(0); return (:264-267): the block stays in the input
        // buffer, fill / current unchanged; the windows are dropped
        const float *inc = JC.in + c * JC.in_stride;
        float *ibc = JC.inbuf + c * B;
        for (int j = lane; j < B; j += 64) {
            float v = 0.f;
            if (JC.add0) {
                v += p0l[j];
                if (JC.add1) v += p1l[j];
            }
            if constexpr (XF == 2) v = mix_select(p0l[j], v, p1l[j]);
            ibc[j] = inc[j];  // (before the output: a caller's output may alias its input)
            outc[j] = v;
        }
        // a multi-block call (:222-294 over mcall blocks) returns here: the
        // whole call's output is zero, its later blocks are not processed
        const bool rest = XF == 0 && JC.mcall > 1;
        if (rest) {
            float *o0 = outc - (size_t)JC.mk * B;
            for (int j = lane; j < JC.mcall * B; j += 64)
                if (j < JC.mk * B || j >= (JC.mk + 1) * B) o0[j] = 0.f;
        }
        const int done = rest && JC.mk < JC.mcall - 1 ? FLAG_CALLDONE : 0;
        if (lane == 0) {
            JC.state[c] = make_int4(cur, act, 0, keep | FLAG_INBUF | tag | done);
            if (JC.vnext) JC.vnext[c] = make_int4(cur, act, 0, keep | FLAG_INBUF | tag | done);
        }
    }
    if constexpr (XF == 3) la_xf_arrive(a, xcnt, yA, yB, vtab, c);
}

// a channel off the lookahead path (partial block, buffered input, short
// response) in the workgroup: its channels run one at a time, out of line
// (the rare fallback keeps its registers out of the step's allocation)
template <int LOG2B, bool NTL, int XF>
__device__ __attribute__((noinline)) void la_fallback(const ProcArgs *ap, int c0, int nvalid, unsigned char *smem) {
    const ProcArgs &a = *ap;
    const ProcJob &J = a.job[0];
    for (int k = 0; k < nvalid; ++k) {
        if (k) __syncthreads();
        const int c = c0 + k;
        int4 st = J.state[c];
        bool done = false;
        if (XF == 0 && (st.w & FLAG_CALLDONE)) {
            if (J.mcall > 1 && J.mk > 0) {
                // done with this multi-block call; its last launch clears the flag
                if (J.mk == J.mcall - 1 && threadIdx.x == 0) J.state[c] = make_int4(st.x, st.y, st.z, la_clear(st.w & ~FLAG_CALLDONE, a));
                done = true;
            } else {
                // a stale flag: the call that set it stopped before its last
                // launch (a failed launch).  This is a new call's first
                // block: process it (the state written below drops the flag)
                st.w &= ~FLAG_CALLDONE;
            }
        }
        if (!done && XF == 0 && J.mcall > 1 && J.mk == 0 && !la_eligible<LOG2B>(st, J.n)) {
            // off the lookahead path at the start of a multi-block call
            // (buffered samples, a short response): the whole call by the
            // reference's chunk loop, here (in / out are the call's at mk 0)
            ProcJob Jw = J;
            Jw.n = J.mcall * J.n;
            process_job<LOG2B, LA_NT, false, NTL>(a, Jw, (size_t)c, st, smem);
            __syncthreads();
            if (threadIdx.x == 0) {  // (the same thread stored the state above)
                int4 s2 = J.state[c];
                s2.w |= FLAG_CALLDONE;
                J.state[c] = s2;
            }
            done = true;
        }
        if (done) {
        } else if (la_eligible<LOG2B>(st, J.n)) {
            const int c1[1] = {c};
            const int4 s1[1] = {st};
            la_step<LOG2B, NTL, 1, XF>(a, J, c1, s1, 1, smem);
        } else if (XF == 2) {
            // crossfade, B's launch: the generic step writes B's block to
            // buf_b, then the workgroup mixes it with A's (same-workgroup
            // global writes are visible after the barrier)
            ProcJob Jb = J;
            Jb.out = const_cast<float *>(a.mix.buf_b);
            Jb.out_stride = a.mix.buf_stride;
            process_job<LOG2B, LA_NT, false, NTL>(a, Jb, (size_t)c, st, smem);
            __syncthreads();
            const float *ya = a.mix.buf_a + (size_t)c * a.mix.buf_stride;
            const float *yb = a.mix.buf_b + (size_t)c * a.mix.buf_stride;
            float *o = J.out + (size_t)c * J.out_stride;
            const float *sel = a.mix_tab;
            for (int j = threadIdx.x; j < J.n; j += LA_NT) o[j] = mix_select(ya[j], yb[j], sel[j]);
        } else {
            process_job<LOG2B, LA_NT, false, NTL>(a, J, (size_t)c, st, smem);
        }
        // the channel's final word of this launch, for the next launch's
        // anchors (same-workgroup global writes are visible after the barrier)
        if (J.vnext) {
            __syncthreads();
            if (threadIdx.x == 0) J.vnext[c] = J.state[c];
        }
    }
}

// XF 3: channel c of A or B off the lookahead path -- both instances take the
// generic step (out to buf_a / buf_b), then the workgroup walks mix_value and
// mixes (the same arithmetic as the lookahead mix)
template <int LOG2B, bool NTL>
__device__ __attribute__((noinline)) void la_fallback_xf(const ProcArgs *ap, int c, unsigned char *smem) {
    const ProcArgs &a = *ap;
    const CrossfadeMixArgs m = a.mix;
    ProcJob Ja = a.job[0], Jb = a.job[1];
    Ja.out = const_cast<float *>(m.buf_a);
    Ja.out_stride = m.buf_stride;
    Jb.out = const_cast<float *>(m.buf_b);
    Jb.out_stride = m.buf_stride;
    const int4 sa = Ja.state[c], sb = Jb.state[c];
    process_job<LOG2B, LA_NT, false, NTL>(a, Ja, (size_t)c, sa, smem);
    __syncthreads();
    process_job<LOG2B, LA_NT, false, NTL>(a, Jb, (size_t)c, sb, smem);
    __syncthreads();
    if (threadIdx.x == 0) {
        // (thread 0 stored both states) the rings have diverged -- a C2R
        // error in one of them: the FDLs differ from here on, never pair again
        int4 ta = Ja.state[c], tb = Jb.state[c];
        if (!(ta.x == tb.x && ta.y == tb.y && ta.z == tb.z && !((ta.w ^ tb.w) & FLAG_INBUF))) {
            ta.w &= ~FLAG_XSYNC;
            tb.w &= ~FLAG_XSYNC;
            Ja.state[c] = ta;
            Jb.state[c] = tb;
        }
        if (Ja.vnext) Ja.vnext[c] = ta;  // (the next launch's anchors)
        if (Jb.vnext) Jb.vnext[c] = tb;
    }
    float *t = reinterpret_cast<float *>(smem);
    if (m.approaching) {
        if (threadIdx.x == 0) mix_walk_lane(t, m.mix_value0, m.step, m.n);
        __syncthreads();
    }
    const float *ya = m.buf_a + (size_t)c * m.buf_stride, *yb = m.buf_b + (size_t)c * m.buf_stride;
    float *o = a.job[0].out + (size_t)c * a.job[0].out_stride;
    for (int j = threadIdx.x; j < m.n; j += LA_NT) o[j] = mix_select(ya[j], yb[j], mix_selector(m, j, t));
}

constexpr int LA_XWG = 8;  // A's launch: leading workgroups (the first writes the mix_value walk)

// crossfade, A's launch: per-sample mix selectors of this call for B's
// launch (mix_select): Crossfader::mix (:242-278) for sample j is A's sample,
// B's sample, or the raised-cosine blend with gain g1 of the mix_value walk
// entry it has reached -- the reference's sequential f32 additions, one lane,
// into LDS -- so B's epilogue reads one word per sample and no crossfader
// state.  (Out of line: keeps its registers out of the step's allocation.)
__device__ __attribute__((noinline)) void la_mix_walk(const ProcArgs *ap, unsigned char *smem) {
    // (the walk's operands in registers: stores through the LDS pointer could
    // otherwise alias the kernel arguments and reload them every entry)
    const CrossfadeMixArgs m = ap->mix;
    float *mt = ap->mix_tab;
    float *t = reinterpret_cast<float *>(smem);
    if (m.approaching) {
        if (threadIdx.x == 0) mix_walk_lane(t, m.mix_value0, m.step, m.n);  // mix_value += step (:259)
        __syncthreads();
    }
    for (int j = threadIdx.x; j < m.n; j += LA_NT) mt[j] = mix_selector(m, j, t);
}

// Anchor workgroup ba of the grid's anchor block [level 3 | level 2 | level 1]
// (la_n[2], la_n[1], la_n[0] workgroups) of instance jb; false if ba is past it.
// The level-3 and level-2 counts are whole XCD rounds (multiples of 8), so
// every anchor keeps its XCD placement.
template <int LOG2B, bool NTL, int UF = LA_UF, int JW = LA_JW>
__device__ __forceinline__ bool la_anchor(const ProcArgs &a, int jb, int ba, unsigned char *smem) {
    if (ba < a.la_n[2]) {
        la_anchor_far<LOG2B, 3, NTL, UF, JW>(a, jb, ba, smem);
        return true;
    }
    ba -= a.la_n[2];
    if (ba < a.la_n[1]) {
        la_anchor_far<LOG2B, 2, NTL, UF, JW>(a, jb, ba, smem);
        // level-1 anchor ba after the level-2 walk: the level-2 workgroups
        // finish first (r4 timeline: 8.9 us median against 13.4 for level 3
        // and ~15 for the in-step level-1 walks they replace)
        if (a.la_l1in2) la_anchor_mid<LOG2B>(a, jb, ba);
        return true;
    }
    ba -= a.la_n[1];
    if (ba < a.la_n[0]) {
        la_anchor_mid<LOG2B>(a, jb, ba);
        return true;
    }
    return false;
}

// grid (XF 0 / 1 / 2): [the 8 mix-walk workgroups (XF 1) | level 3 | level 2 |
// level 1 anchors | step workgroups].  XF 3: [one step workgroup per channel |
// A's level 3 | B's level 3 | A's level 2 | B's level 2 | A's level 1 | B's
// level 1] -- the latency-critical chains get the CUs first, the anchors fill
// in (each level's count is a multiple of 8: B's anchors keep their XCD
// placement).
// XF: crossfade role of the launch (ProcArgs::la_mix): 0 none; 1 = A's launch,
// whose first workgroup also writes the gains of this call's mix_value walk to mix_tab;
// 2 = B's launch, whose steps mix A's block with their own
template <int LOG2B, bool NTL, int XF>
__device__ __forceinline__ void la_kernel_body(const ProcArgs &a, unsigned char *smem) {
    using LS = LaStep<LOG2B, XF>;
    constexpr int NCH = LS::NCH;
    if constexpr (XF == 3) {
        int b = (int)blockIdx.x;
        if (b >= a.la_channels) {
            b -= a.la_channels;
            for (int lv = 3; lv >= 1; --lv) {
                const int n = a.la_n[lv - 1];
                if (b < 2 * n) {
                    // A's and B's workgroup of the same anchor slice 8 apart:
                    // on one XCD, at the same time (la_xsrc: B reads A's rows)
                    const int jb = (b >> 3) & 1, ba = ((b >> 4) << 3) | (b & 7);
                    if (lv == 3) la_anchor_far<LOG2B, 3, NTL>(a, jb, ba, smem);
                    else if (lv == 2) la_anchor_far<LOG2B, 2, NTL>(a, jb, ba, smem);
                    else la_anchor_mid<LOG2B>(a, jb, ba);
                    return;
                }
                b -= 2 * n;
            }
            return;
        }
        const int c = b;
        const int4 va = a.job[0].state[c], vb = a.job[1].state[c];
        const int4 st[2] = {make_int4(__builtin_amdgcn_readfirstlane(va.x), __builtin_amdgcn_readfirstlane(va.y),
                                      __builtin_amdgcn_readfirstlane(va.z), __builtin_amdgcn_readfirstlane(va.w)),
                            make_int4(__builtin_amdgcn_readfirstlane(vb.x), __builtin_amdgcn_readfirstlane(vb.y),
                                      __builtin_amdgcn_readfirstlane(vb.z), __builtin_amdgcn_readfirstlane(vb.w))};
        const int cs[2] = {c, c};
        if (la_eligible<LOG2B>(st[0], a.job[0].n) && la_eligible<LOG2B>(st[1], a.job[1].n))
            la_step<LOG2B, NTL, 2, 3>(a, a.job[0], cs, st, 2, smem);
        else
            la_fallback_xf<LOG2B, NTL>((const ProcArgs *)__builtin_amdgcn_kernarg_segment_ptr(), c, smem);
        return;
    }
    if constexpr (XF == 1) {
        // 8 extra workgroups at the front of the grid (one per XCD: the
        // anchors' XCD placement behind them is unchanged); the first walks,
        // so the walk starts with the launch and runs beside the steps
        if (blockIdx.x < LA_XWG) {
            if (blockIdx.x == 0) la_mix_walk((const ProcArgs *)__builtin_amdgcn_kernarg_segment_ptr(), smem);
            return;
        }
    }
    const int nanchor = a.la_n[0] + a.la_n[1] + a.la_n[2];
    const int b = (int)blockIdx.x - (XF == 1 ? LA_XWG : 0);
    if (b < nanchor) {
        la_anchor<LOG2B, NTL>(a, 0, b, smem);
        return;
    }
    const int c0 = (b - nanchor) * NCH;
    const ProcJob &J = a.job[0];
    const int nvalid = min(NCH, a.la_channels - c0);
    int cs[NCH];
    int4 st[NCH];
    bool all = true;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        cs[k] = c0 + k;
        int4 v = k < nvalid ? J.state[cs[k]] : make_int4(0, 0, 0, 0);
        // wave-uniform: keep the state words in scalar registers
        st[k] = make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                          __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
        all &= k >= nvalid || la_eligible<LOG2B>(st[k], J.n);
    }
    if (all)
        la_step<LOG2B, NTL, NCH, XF>(a, J, cs, st, nvalid, smem);
    else  // (the arguments by their kernarg address: no private copy of the block)
        la_fallback<LOG2B, NTL, XF>((const ProcArgs *)__builtin_amdgcn_kernarg_segment_ptr(), c0, nvalid, smem);
}

// the role of workgroup blockIdx.x in a lookahead launch (for the timeline):
// 0 level-3 anchor, 1 level-2 anchor, 2 step, 3 level-1 anchor, 4 mix walk, 5 padding
template <int XF>
__device__ __forceinline__ int la_role(const ProcArgs &a) {
    int b = (int)blockIdx.x;
    if (XF == 3) {
        if (b < a.la_channels) return 2;
        b -= a.la_channels;
        if (b < 2 * a.la_n[2]) return 0;
        b -= 2 * a.la_n[2];
        if (b < 2 * a.la_n[1]) return 1;
        b -= 2 * a.la_n[1];
        return b < 2 * a.la_n[0] ? 3 : 5;
    }
    if (XF == 1) {
        if (b < LA_XWG) return 4;
        b -= LA_XWG;
    }
    if (b < a.la_n[2]) return 0;
    b -= a.la_n[2];
    if (b < a.la_n[1]) return 1;
    b -= a.la_n[1];
    return b < a.la_n[0] ? 3 : 2;
}

template <int LOG2B, bool NTL, int XF>
__global__ __launch_bounds__(LA_NT, 4) void upols_la_kernel(ProcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned t0 = 0;
    if (a.la_trace) t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
    la_kernel_body<LOG2B, NTL, XF>(a, smem);
    if (a.la_trace) {
        const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
        const int wave = (int)(threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0) {
            const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(0xF804);   // HW_REG_HW_ID
            const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
            a.la_trace[(size_t)blockIdx.x * 4 + wave] =
                make_int4(la_role<XF>(a) | (wave << 4), (int)((hw & 0xffffu) | ((xcc & 0xffu) << 24)), (int)t0, (int)t1);
        }
    }
}
