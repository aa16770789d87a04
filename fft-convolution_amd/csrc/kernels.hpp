// kernels.hpp -- host-visible kernel argument blocks and launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

// FFTCONV_DEBUG_BOUNDS (debug builds only, Makefile target debug-bounds):
// DBG_CHECK(cond, site, v0..v3) reports a failed index check with printf.
// One out-of-line report per translation unit (a printf inlined at each of
// the hundreds of inlined load sites made the debug build compile for hours).
#ifdef FFTCONV_DEBUG_BOUNDS
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
static __device__ __attribute__((noinline)) void dbg_bounds(int site, int v0, int v1, int v2, int v3) {
    printf("BOUNDS site %d blk %d tid %d: %d %d %d %d\n", site, (int)blockIdx.x, (int)threadIdx.x, v0, v1, v2, v3);
}
#endif
#define DBG_CHECK(cond, site, v0, v1, v2, v3)          \
    do {                                               \
        if (!(cond)) dbg_bounds(site, v0, v1, v2, v3); \
    } while (0)
#else
#define DBG_CHECK(cond, site, v0, v1, v2, v3) do {} while (0)
#endif

namespace fftconv {

enum : int {
    FLAG_INBUF = 1,  // the HBM input buffer holds live samples
    FLAG_REV = 2,    // scan parity of the segment MAC (toggled per completed block)
    FLAG_PRE = 4,    // pre[] holds pre_multiplied of the block that starts at `current`
    FLAG_XSYNC = 8,  // crossfade pair: this FDL has always equalled its partner's
    // lookahead (time-blocked FDL, see la.hpp): per anchor level lv = 1..3 the
    // window of partial sums is live (FLAG_LA1 << 2(lv-1)) in window
    // FLAG_PW1 << 2(lv-1) of the two; a step at launch t reads the row at
    // position (t - 1 - c) mod P_lv.  Bits 24-25 = the launch tag of the last
    // process launch that wrote this state word
    FLAG_LA1 = 16,
    FLAG_PW1 = 32,
    FLAG_LA2 = 64,
    FLAG_PW2 = 128,
    FLAG_LA3 = 256,
    FLAG_PW3 = 512,
    // a multi-block call on the lookahead path (ProcJob::mcall > 1) is done
    // for this channel before its last launch: it ran the whole call by the
    // generic chunk loop in the first launch (off the lookahead path), or a
    // block's C2R failed (the call's output is zero-filled, :264-267); the
    // call's remaining launches skip it, the last one clears the flag
    FLAG_CALLDONE = 1 << 10,
    // far-row windows of the generic step (B >= 1024, gw_anchor_kernel): the
    // channel's P windows were anchored after the step of its class and every
    // step since read one and advanced
    FLAG_GW = 1 << 11,
    SEQ_SHIFT = 24,
    // lookahead: pre[] holds the near rows' sum (rows D0..1) of the block
    // that starts at `current`, left by the previous step (la.hpp)
    FLAG_NEAR = 1 << 26,
    LA_MASK = FLAG_LA1 | FLAG_LA2 | FLAG_LA3 | FLAG_NEAR | FLAG_GW,
    SEQ_MASK = 3 << SEQ_SHIFT,
};

// fused-kernel variants (bit mask): 1 = zig-zag segment scan, 2 = nontemporal H/X loads
enum : int {
    VARIANT_ZIGZAG = 1, VARIANT_NT = 2, VARIANT_NOPIPE = 4, VARIANT_NOPAIR = 8, VARIANT_NOLA = 16,
    VARIANT_LAFULL = 32,  // lookahead launches without anchors: every step sums all rows itself (tests)
    VARIANT_NOFMIX = 64,  // crossfade on the lookahead step: stand-alone mix kernel instead of B's epilogue
    VARIANT_IRBLOCK = 128,  // IR transforms: one segment per workgroup (else one per wave, 64 <= B <= 1024)
    VARIANT_T0BLOCK = 256,  // two-stage: tail0 per block (else deferred to the end of its period), read at create
    VARIANT_T0FUSED = 512,  // deferred tail0 at B = 64: the five-kernel flush instead of the fused one (bit-identical)
    VARIANT_NOGW = 1024,    // B >= 1024: no far-row windows, every step sums its far rows itself (tests)
    VARIANT_NORUN = 2048,   // process_device_steps: one launch per call (else a run of a period's calls per launch)
    VARIANT_NORUNLDS = 4096,  // runs stream the FDL / IR rows from memory (else from LDS copies when they fit; same bits)
    VARIANT_AUTO = 0x7fffffff
};
void set_variant(int v);
int get_variant();
void set_pipeline_lag(int rows);
int get_pipeline_lag();

// One convolver batch's call (FFTConvolver::process over `n` samples of every
// channel), optionally with the two-stage epilogue of the head block
// (src/fft_convolver.rs:438-461): out[j] += add0[j], then += add1[j], and
// tin[j] = in[j], applied after the call.
struct ProcJob {
    const float2 *H;       // [C][S][B] packed IR spectra
    float2 *X;             // [C][S][B] packed FDL
    float *overlap;        // [C][B]
    float *inbuf;          // [C][B]
    float2 *pre;           // [C][B]
    int4 *state;           // [C] {current, active, fill, flags}
    const float *in;
    long long in_stride;
    float *out;
    long long out_stride;
    const float *add0;     // tail_precalculated0 + precalculated_pos (or null)
    const float *add1;     // tail_precalculated  + precalculated_pos (or null)
    long long add_stride;
    float *tin;            // tail_input + tail_input_fill (or null)
    long long tin_stride;
    int S;                 // seg_count (row pitch of H and X in rows)
    int n;                 // output samples this call
    // lookahead launches of a multi-block call (n = mcall * B, one launch per
    // block, in / out advanced by mk * B): blocks of the whole call, this
    // launch's block (0 / 0 otherwise)
    int mcall, mk;
    // long-block path (B > 2^kMaxLog2Fused, large.hip): per channel the
    // call's progress {processed, done, C2R failed, arrival counter}, and the
    // [C][B] scratch between the row and the column passes of the inverse.
    // Lookahead launches (la.hpp, B <= 512: never long-block) use the same
    // two words for the channels' state words as of the end of the previous
    // launch, which the anchors read instead of `state` (the step of this
    // launch rewrites `state` while the anchors run), and the copy the steps
    // of this launch fill for the next one (null elsewhere).  (Shared words,
    // not new ones: a larger argument block measurably slows every launch,
    // +0.2 us per cfg2 step for 32 bytes, r6y.)
    union {
        int4 *lg_prog;
        const int4 *sview;
    };
    union {
        float2 *lg_v;
        int4 *vnext;
    };
    // two-stage head of a multi-call launch (upols_run_kernel): its block's
    // spectrum also goes to the deferred tail0's pending-block row
    // t0x + c * t0x_stride (the same R2C tail0_r2c_kernel would compute), so
    // the period's flush skips those blocks' transforms; null = none
    float2 *t0x;
    long long t0x_stride;
    // [C]: set by a run's call that did NOT write its block's spectrum to t0x
    // (a channel whose head buffer is out of step with tail_input, e.g. after
    // a C2R error on a partial call, :264-267): the flush recomputes that
    // channel's pending spectra from tail_input and clears the flag
    int *t0m;
};

// Twiddle tables of the long-block path (large.hip), f64-rounded f32:
// twN = W_N^k (k < N/2, the post/pre-twiddle), twM = W_M^j (j < M = N/2, the
// four-step's inner twiddle), twA / twB = W_{2 M1}^i / W_{2 M2}^i (the column
// and row FFTs), M = M1 x M2 (lg_split)
struct LgTab {
    const float2 *twN, *twM, *twA, *twB;
};

// Crossfader::mix over one call's samples (src/crossfade_convolver.rs:242-278),
// the crossfader state at the start of the call.
struct CrossfadeMixArgs {
    const float *buf_a;
    const float *buf_b;
    long long buf_stride;
    float *out;
    long long out_stride;
    int n;
    int approaching;       // FadingState::Approaching
    int target;            // 0 = A, 1 = B
    long long counter0;
    long long fading;
    float mix_value0;
    float step;
    const float *vtab;     // calls longer than 1024 samples: the mix_value walk (launch_crossfade_walk), or null
};

// Up to two jobs of the same block size in one launch (grid.y = job): the
// two-stage head and tail0 run together on the same input block.
struct ProcArgs {
    ProcJob job[2];
    const float2 *tw;      // W_N^k, k < N = 2B
    int njobs;
    int pipe;              // pipelined full-block step allowed (B <= 512)
    int lag;               // pipelined step: FDL rows wave 0 leaves to the stream waves
    int fuse_mix;          // crossfade pair launch: mix A and B into mix.out in-kernel
    CrossfadeMixArgs mix;  // (buf_a / buf_b unused then)
    // lookahead launch (launch_process_la; job[0] only)
    float2 *laW;           // [C][2 windows][LA_PT][B]: the partial-sum windows of levels 1..3
    float2 *laW2;          // job[1]'s windows (la_mix 3: the crossfade's B in the same launch)
    int la_n[3];           // anchor workgroups of levels 1..3 (grid: level 3, 2, 1, then the steps)
    int la_nlv;            // anchor levels: 3, or 2 when no FDL row reaches level 3 (S <= LA_R2 + 1)
    int la_all;            // 1: every channel is scheduled for anchors (entry launch); -1: none is
    int la_t;              // launch counter mod LA_PER: channel c anchors at period P when (c - t) % P == 0
    int la_seq;            // 1 or 2, alternating per lookahead launch; 0 in every other launch
    int la_channels;       // channels of the batch (step workgroups cover LaStep::NCH each)
    int la_l1in2;          // 1: level-1 anchor b runs in level-2 anchor workgroup b, after its walk
    // crossfade on the lookahead step (CrossfadeConvolver::process :72-77):
    // 1 = A's launch also writes this call's per-sample mix selectors to mix_tab;
    // 2 = B's launch mixes in its epilogue: out = mix(mix.buf_a, B's block);
    // 3 = ONE launch for A (job[0]) and B (job[1]): a step workgroup runs A's
    //     and B's chain of one channel and mixes in LDS (out = job[0].out)
    int la_mix;
    float *mix_tab;        // [n] mix_selector of each sample (la_mix 1 writes, 2 reads)
    // window rebuild (launch_la_rebuild, after update / reset / init): anchors
    // only, for channels [la_c0, la_channels), as if they had run in the
    // launch before the next one (la_t = that launch's counter)
    int la_rebuild;
    int la_c0;
    // launch timeline (tuning only, FFTCONV_LA_TRACE): per wave {role | wave
    // << 4, HW_ID low 16 bits | XCC_ID << 24, t0, t1} (s_memrealtime, 100 MHz)
    int4 *la_trace;        // this launch's record: [la_trace_grid][4 waves] + phase stamps after it
    int la_trace_grid;
    // state-word probe (tests only, FFTCONV_LA_PROBE at handle creation): the
    // anchors wait for the launch's steps and read the state past their L2,
    // so they observe the post-step word; each such observation is counted
    int *la_probe_cnt;
    // long-block path (launch_process with log2b > kMaxLog2Fused): the
    // geometry's tables and the chunks to run (an upper bound over channels)
    LgTab lg;
    int lg_chunks;
    // far-row windows of the generic step (B >= 1024, gw_anchor_kernel):
    // gw_p = the split row P (pre = rows 1..P-1 + rows P..act-1; 0 = one sum),
    // gw = [C][P][B] windows (null: no step of this launch reads one), gw_t =
    // the batch's one-block step count mod P (channel c reads row (gw_t-1-c) mod P)
    float2 *gw;
    int gw_p;
    int gw_t;
    // 2048 <= B <= 8192: 256-thread workgroups (upols_narrow_kernel) instead
    // of 512 -- a two-stage tail beside the head's multi-call run, so one
    // tail workgroup fits each CU next to a run workgroup (same bits)
    int narrow;
    // multi-call run (upols_run_kernel): the waves' issue priority (s_setprio;
    // 0 = the default) -- the latency-bound chain beside the two-stage tail
    int prio;
    // multi-call run: the FDL rows and IR rows held in LDS for the whole run
    // (the pipelined step's helpers stream them from LDS), when they fit: the
    // row count S of the job, 0 = off (the rows stream from HBM / L2)
    int run_lds_rows;
    // device-side ordering of a two-stage period's head after the previous
    // tail step, without a barrier packet on the head's stream: sig_mode 1
    // (the tail's step) -- every workgroup arrives on sig[0], the last one
    // releases sig[1] = sig_val; sig_mode 2 (a run) -- the workgroups start
    // once sig[1] has reached sig_val (acquire), or after a bounded wait that
    // counts in sig[2]
    unsigned *sig;
    unsigned sig_val;
    int sig_mode;
};

struct IrArgs {
    float2 *H;
    float *overlap;
    float2 *pre;
    int4 *state;
    const float *src;      // device IR samples of channel chan0 (+ src_stride per channel)
    long long src_stride;
    long long len_data;    // samples present in src
    long long len_active;  // length that sets active_seg_count = ceil(len_active / B)
    const float2 *tw;
    int S;
    int chan0;
    int update_state;      // 1: update() side effects (zero overlap/pre, set active)
};

struct TwoStageAccumArgs {
    float *out;
    long long out_stride;
    const float *p0;       // tail_precalculated0 [C][T]
    const float *p1;       // tail_precalculated  [C][T]
    long long T;
    int pos;               // precalculated_pos
    const float *in;
    long long in_stride;
    int sb;                // sub-chunk start within the call
    float *tail_input;     // [C][T]
    int fill;              // tail_input_fill before the append
    int cnt;               // samples in the sub-chunk
};


// Fft::forward / Fft::inverse (src/fft_convolver.rs:36-49) over rows of
// N = 2M reals / M+1 interleaved complex bins (the public Fft of the
// reference, fftconv_fft_*): one workgroup per row, the convolver's own
// transforms (lds_cfft + real_post / real_pre, the same twiddle table)
struct FftArgs {
    const float *in;
    long long in_stride;   // floats between rows
    float *out;
    long long out_stride;
    const float2 *tw;      // W_N^k, k < N
    int *status;           // inverse: per row 1 = FftError::InputValues (DC / Nyquist imag != 0), or null
};
hipError_t launch_fft_rows(int log2m, bool inverse, const FftArgs &a, int rows, hipStream_t s);

hipError_t launch_process(int log2b, const ProcArgs &a, int channels, hipStream_t s);
// a run of r.n consecutive one-job process() calls in one launch
// (upols_run_kernel, 64 <= B <= 512): call k = job[0] with in / out advanced
// by k * in_step / out_step floats and add0 / add1 / tin by k * n
struct RunSteps {
    long long in_step, out_step;
    int n;
};
bool run_supported(int log2b);
int run_lds_rows(int log2b, int S);  // a run's LDS-resident rows for this geometry (0 = none)
hipError_t launch_process_run(int log2b, const ProcArgs &a, const RunSteps &r, int channels, hipStream_t s);
hipError_t launch_ir_segments(int log2b, const IrArgs &a, int channels, hipStream_t s);
hipError_t launch_twostage_accum(const TwoStageAccumArgs &a, int channels, hipStream_t s);
hipError_t launch_crossfade_mix(const CrossfadeMixArgs &a, int channels, hipStream_t s);
bool la_fuse_mix_allowed();  // VARIANT_NOFMIX unset
hipError_t launch_reset_state(int4 *state, int channels, hipStream_t s);
// crossfade pair (A and B of one CrossfadeConvolver in one workgroup per channel)
bool pair_supported(int log2b, int S);
hipError_t launch_process_pair(int log2b, const ProcArgs &a, int channels, hipStream_t s);
hipError_t launch_state_flags(int4 *state, int channels, int set, int clear, hipStream_t s);
size_t process_lds_bytes(int log2b);
// lookahead: 1 if this geometry takes the lookahead step, else 0
int la_parts(int log2b, int S);
// the lookahead launch shape of a geometry (la.hpp): anchor levels, the
// workgroups per anchor of each level (level 1: 0 = run by the step
// workgroups), and the periods
struct LaDims {
    int nlv;
    int per[3];
    int wg[3];
    int pt;           // window rows per channel and window (all levels)
    int per_all;      // the stagger clock's modulus
};
LaDims la_dims(int log2b, int S, int jw = 8);  // (jw: window steps per level-2/3 anchor workgroup, LA_JW)
// launch timeline records per lookahead launch (FFTCONV_LA_TRACE): the largest grid
int la_trace_grid(int log2b, int S, int channels);
hipError_t launch_process_la(int log2b, const ProcArgs &a, int channels, hipStream_t s);
// every far and mid window of channels [a.la_c0, channels) rebuilt from the
// current H and FDL (anchors only), then their state words pointed at them
hipError_t launch_la_rebuild(int log2b, const ProcArgs &a, int channels, hipStream_t s);
bool la_full_variant();  // VARIANT_LAFULL: lookahead launches without anchors

// Two-stage tail0 deferred to the end of its period (src/fft_convolver.rs
// :464-475: tail_output0 is first read after the period's swap).  pa.job[0]
// is tail0's job with in = tail_input + off, out = tail_output0 + off (both
// stride T); the n pending blocks of every channel are transformed, summed
// against one pass of tail0's IR rows and FDL, inverted, and committed --
// or, for a channel whose C2R fails on any block (realfft's error path),
// replayed block by block by the generic step from the untouched state.
struct Tail0Args {
    ProcArgs pa;
    float2 *xs;            // [C][nmax][B]: spectra of the pending blocks
    float *ys;             // [C][nmax][2B]: their C2R outputs (not yet scaled)
    int *err;              // [C]: some pending block's C2R fails
    float *ov0;            // [C][B]: the overlap before the pending blocks
    float2 *cv;            // [C][nmax][B]: conv of each pending block
    int act;               // tail0's active segments (every channel: TwoStage never updates tail0)
    int n;                 // pending blocks
    int nmax;              // row pitch of xs / ys in blocks
    int k0;                // blocks [0, k0) already have their spectra in xs (the head's run wrote them)
    int *miss;             // [C]: 1 = the run missed some of this channel's spectra: recompute [0, n) (ProcJob::t0m)
};
bool tail0_defer_supported(int log2b, int act, int nmax);
bool tail0_defer_allowed();  // VARIANT_T0BLOCK unset
// done (optional): an event recorded by the flush's last kernel itself (hipExtLaunchKernel)
hipError_t launch_tail0_flush(int log2b, const Tail0Args &a, int channels, hipStream_t s, hipEvent_t done = nullptr);

// The fused one-workgroup-per-channel kernels hold two B-point complex
// buffers in LDS: B <= 8192 (128 KiB).  Larger blocks, up to 2^22, take the
// four-step long-block path (large.hip).
constexpr int kMaxLog2Fused = 13;
constexpr int kMaxLog2Block = 22;
// far-row windows (gw_anchor_kernel): window rows per channel = the split row
constexpr int kGwP = 8;
// a batch of this geometry sums far rows through windows: 1024 <= B <= 8192
// and enough far rows to pay for the anchors
bool gw_supported(int log2b, int S);
bool gw_windows_allowed();  // VARIANT_NOGW unset
// the windows of the channels of class a.gw_t mod kGwP, from the state after
// the step just launched (a.job[0]: H, X, state, S; a.la_channels channels)
hipError_t launch_gw_anchor(int log2b, const ProcArgs &a, int channels, hipStream_t s);
// M = 2^log2b = M1 x M2 of the long-block path; bin k of a spectrum row sits
// at position (k mod M1) * M2 + k / M1
void lg_split(int log2b, int *l1, int *l2);
size_t lg_position(int log2b, size_t k);
hipError_t launch_process_large(int log2b, const ProcArgs &a, const LgTab &t, int chunks, int channels,
                                hipStream_t s);
hipError_t launch_ir_large(int log2b, const IrArgs &a, const LgTab &t, int channels, hipStream_t s);
// the public Fft's rows through the same passes: rows in batches of `batch`,
// scratch [batch][N/2] complex
hipError_t launch_fft_large(int log2m, bool inverse, const FftArgs &a, const LgTab &t, float2 *scratch, int rows,
                            int batch, hipStream_t s);
// the public Fft of a length n that is not a power of two: Bluestein over
// P = 2^log2p >= 2n - 1 point FFTs (large.hip).  chirp[m] = exp(i pi m^2 / n)
// (m < n); filt = FFT_P of the chirp filter (natural order for P <= 8192,
// else the four-step's transposed order); twP = W_{2P}^i (P <= 8192); t =
// the four-step tables of P (P > 8192); scratch [batch][P] (P > 8192)
hipError_t launch_fft_bluestein(size_t n, int log2p, bool inverse, const FftArgs &a, const float2 *chirp,
                                const float2 *filt, const float2 *twP, const LgTab &t, float2 *scratch, int rows,
                                int batch, hipStream_t s);
// crossfade mix of calls longer than the in-LDS walk (n > 1024): the walk
// once into a device table (one lane), then the mix reading it
hipError_t launch_crossfade_walk(const CrossfadeMixArgs &a, float *vtab, hipStream_t s);

}  // namespace fftconv
