// host.cpp -- C++ host side of the MI355X convolver and its C ABI (include/fftconv.h).
//
// The three reference types are mirrored as batches of device-resident
// channels:
//   UniformCore   <- FFTConvolver          (src/fft_convolver.rs:86-307)
//   TwoStageCore  <- TwoStageFFTConvolver  (src/fft_convolver.rs:323-512)
//   CrossfadeCore <- CrossfadeConvolver<FFTConvolver> (src/crossfade_convolver.rs:3-105)
// Per-channel block state lives on the device (the fused kernel advances it);
// the host only keeps what the reference keeps per *instance* and what all
// channels share in lockstep (two-stage fill/position, the crossfader).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/fftconv.h"
#include "kernels.hpp"

using namespace fftconv;

namespace {

thread_local std::string g_last_error;

void set_error(const std::string &m) { g_last_error = m; }

struct Status {
    int code = FFTCONV_OK;
    explicit operator bool() const { return code != FFTCONV_OK; }
};

int fail(int code, const std::string &m) {
    set_error(m);
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e__ = (expr);                                                         \
        if (e__ != hipSuccess)                                                           \
            return fail(FFTCONV_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e__)); \
    } while (0)

size_t next_pow2(size_t v) {  // usize::next_power_of_two (0 -> 1)
    size_t p = 1;
    while (p < v) p <<= 1;
    return p;
}
int ilog2(size_t v) {
    int l = 0;
    while (((size_t)1 << l) < v) ++l;
    return l;
}
size_t ceil_div(size_t a, size_t b) { return (a + b - 1) / b; }  // == (a as f64 / b as f64).ceil()

template <class T>
struct DevPtr {
    T *p = nullptr;
    size_t n = 0;
    DevPtr() = default;
    DevPtr(const DevPtr &) = delete;
    DevPtr &operator=(const DevPtr &) = delete;
    ~DevPtr() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    int alloc(size_t count) {
        reset();
        n = count;
        if (count == 0) return FFTCONV_OK;
        hipError_t e = hipMalloc((void **)&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            n = 0;
            return fail(e == hipErrorOutOfMemory ? FFTCONV_E_NOMEM : FFTCONV_E_DEVICE,
                        std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        // (tests: FFTCONV_POISON_ALLOC=1 fills every new device buffer with NaN
        // bytes, so a read of memory the path never wrote shows in the output
        // instead of reading whatever the allocator recycled)
        static const bool poison = [] {
            const char *v = getenv("FFTCONV_POISON_ALLOC");
            return v && atoi(v) > 0;
        }();
        if (poison) {  // (done before any stream uses the buffer: null stream, then wait)
            if (hipMemset(p, 0xff, count * sizeof(T)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
                return fail(FFTCONV_E_DEVICE, "poison memset");
        }
        return FFTCONV_OK;
    }
    size_t bytes() const { return n * sizeof(T); }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int now = -1;
        (void)hipGetDevice(&now);
        if (prev >= 0 && now != prev) (void)hipSetDevice(prev);
    }
};

int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(FFTCONV_E_DEVICE, "no HIP device available (the convolver has no CPU fallback)");
    if (device < 0 || device >= n) return fail(FFTCONV_E_DEVICE, "device index out of range");
    return FFTCONV_OK;
}

// Device scratch for the host-pointer entry points (grown on demand).
struct Scratch {
    DevPtr<float> in, out;
    int ensure(size_t nin, size_t nout) {
        if (in.n < nin) { if (int r = in.alloc(nin)) return r; }
        if (out.n < nout) { if (int r = out.alloc(nout)) return r; }
        return FFTCONV_OK;
    }
};

// Cross-stream ordering of one handle's work.  Asynchronous entry points take
// a caller stream; every call must still see the state the previous call left
// (the reference's calls are sequential on one instance).  `enter(s)` before
// enqueueing on s makes s wait for the stream of the handle's previous work
// when that was another stream (an event recorded there now -- so, as with a
// library handle's stream, a caller stream must stay valid until the handle's
// next call).  Host-synchronous entry points enter their own stream and wait
// for it alone: no device-wide synchronisation, so other handles' and other
// libraries' streams are never waited for.
struct StreamOrder {
    hipStream_t last = nullptr;
    bool any = false;
    hipEvent_t ev = nullptr;
    ~StreamOrder() {
        if (ev) (void)hipEventDestroy(ev);
    }
    int enter(hipStream_t s) {
        if (any && last != s) {
            if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(ev, last));
            HIP_TRY(hipStreamWaitEvent(s, ev, 0));
        }
        last = s;
        any = true;
        return FFTCONV_OK;
    }
    // every piece of the handle's work has finished, once `own` has drained
    int drain(hipStream_t own) {
        if (int r = enter(own)) return r;
        HIP_TRY(hipStreamSynchronize(own));
        return FFTCONV_OK;
    }
};

// Pinned host staging for host-memory IR uploads: update() copies the caller's
// response into it and returns once the H2D copy and the IR transform are
// enqueued (the next call on the handle is ordered behind them).  Reserved at
// init, so update() never allocates (src/lib.rs:8); `busy` guards its reuse.
// The reservation is capped by fftconv_set_host_stage_limit, and a failed one
// falls back to smaller sizes (down to one response row): then an
// update streams its rows through the stage in chunks, each chunk waiting for
// the previous one's copy out of it -- still no allocation, but the host
// waits for all but the last chunk's DMA.
static std::atomic<size_t> g_stage_limit{0};  // bytes, 0 = none (set / read from any thread)

struct PinnedStage {
    float *p = nullptr;
    size_t n = 0;
    hipEvent_t busy = nullptr;
    bool pending = false;
    PinnedStage() = default;
    PinnedStage(const PinnedStage &) = delete;
    PinnedStage &operator=(const PinnedStage &) = delete;
    ~PinnedStage() {
        if (busy) {
            if (pending) (void)hipEventSynchronize(busy);
            (void)hipEventDestroy(busy);
        }
        if (p) (void)hipHostFree(p);
    }
    // count floats wanted, at least min_count (one response row)
    int alloc(size_t count, size_t min_count) {
        if (count == 0) return FFTCONV_OK;
        min_count = std::max<size_t>(1, std::min(min_count, count));
        const size_t lim = g_stage_limit.load(std::memory_order_relaxed);
        if (lim) count = std::max(min_count, std::min(count, lim / sizeof(float)));
        hipError_t e = hipErrorOutOfMemory;
        for (;;) {
            e = hipHostMalloc((void **)&p, count * sizeof(float), hipHostMallocDefault);
            if (e == hipSuccess || count == min_count) break;
            (void)hipGetLastError();
            count = std::max(min_count, count / 4);
        }
        if (e != hipSuccess) {
            p = nullptr;
            return fail(FFTCONV_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        }
        n = count;
        HIP_TRY(hipEventCreateWithFlags(&busy, hipEventDisableTiming));
        return FFTCONV_OK;
    }
    // wait until the previous upload has left the buffer (normally long done)
    int acquire() {
        if (pending) HIP_TRY(hipEventSynchronize(busy));
        pending = false;
        return FFTCONV_OK;
    }
    int release(hipStream_t s) {  // after the H2D copy out of the buffer is enqueued on s
        HIP_TRY(hipEventRecord(busy, s));
        pending = true;
        return FFTCONV_OK;
    }
    // rows r of the caller's responses (src + r*stride, len floats each) to
    // device rows dst + r*dpitch, in as few chunks of whole rows as the stage
    // holds (one when it was reserved for the whole batch)
    int upload(const float *src, size_t rows, size_t len, size_t stride, float *dst, size_t dpitch, hipStream_t s) {
        if (len == 0 || rows == 0) return FFTCONV_OK;
        if (!p || n < len) return fail(FFTCONV_E_INVALID, "no host staging for this update");
        const size_t per = n / len;
        for (size_t r0 = 0; r0 < rows; r0 += per) {
            const size_t k = std::min(per, rows - r0);
            if (int r = acquire()) return r;
            for (size_t c = 0; c < k; ++c) std::memcpy(p + c * len, src + (r0 + c) * stride, len * sizeof(float));
            HIP_TRY(hipMemcpy2DAsync(dst + r0 * dpitch, dpitch * sizeof(float), p, len * sizeof(float),
                                     len * sizeof(float), k, hipMemcpyHostToDevice, s));
            if (int r = release(s)) return r;
        }
        return FFTCONV_OK;
    }
};

int lg_tables(int dev, int log2m, LgTab *out);

// ---------------------------------------------------------------------------
// UniformCore -- a batch of FFTConvolver instances
// ---------------------------------------------------------------------------
struct UniformCore {
    int device = 0;
    size_t C = 0;         // channels
    size_t ir_len = 0;    // max_response_length (padded IR length)
    size_t B = 0;         // block_size.next_power_of_two()
    int log2b = 0;
    size_t S = 0;         // seg_count
    DevPtr<float2> H, X, pre, tw;
    DevPtr<float> overlap, inbuf, staging;
    DevPtr<int4> state;
    hipStream_t stream = nullptr;
    // an inner convolver (of a two-stage or a crossfade) runs on its owner's
    // stream: `parent_stream`, set before init / clone_from, is borrowed
    // instead of created, so a composite handle holds 2 HIP streams, not 5
    // (fewer streams sharing the process's hardware queues)
    hipStream_t parent_stream = nullptr;
    Scratch scratch;
    // host IR uploads (update_host), [C][ir_len]: only a standalone batch
    // owns one (own_stage, set before init).  A crossfade's a / b stage
    // through the crossfade's, and a two-stage's inner convolvers are never
    // updated (TwoStageFFTConvolver::update is todo!(), :408-410).
    PinnedStage hstage;
    bool own_stage = false;
    mutable StreamOrder order;     // (clone_from drains its source)
    // lookahead (la.hpp): standalone batches only (la_ok, set before init)
    bool la_ok = false;
    int la_W = 0;                 // far parts (partial rows per step), 0 = off
    DevPtr<float2> laW;           // windows of the three anchor levels [C][2][LA_PT][B]
    unsigned long long la_t = 0;  // lookahead launches so far (stagger clock)
    // launch timelines of the last `trace_slots` lookahead launches (tuning
    // only: FFTCONV_LA_TRACE=<slots>, written to FFTCONV_LA_TRACE_OUT at destroy)
    DevPtr<int4> trace;
    size_t trace_slots = 0, trace_grid = 0;
    std::vector<long long> trace_meta;  // per slot: la_t, grid
    int la_seq = 1;               // launch tag, alternating 1 / 2
    DevPtr<int> la_probe;         // (tests: FFTCONV_LA_PROBE) live words the anchors found rewritten
    // the anchors' copies of the state words [2][C] (ProcJob::sview / vnext):
    // copy la_seq & 1 is read by the next lookahead launch, the other filled
    // by its steps.  view_ok: that copy holds the current words -- true only
    // right after a lookahead launch; every other writer of the state words
    // (any launch built by job(), update, reset, init, clone) clears it, and
    // the next lookahead launch copies them first (la_view)
    DevPtr<int4> lav;
    mutable bool view_ok = false;
    bool la_all = true;           // next lookahead launch re-anchors every channel
    // long-block path (B > 2^kMaxLog2Fused, large.hip): per-call progress,
    // the inverse's scratch, the geometry's tables; lg_whole: every call
    // since init / reset was whole blocks, so every channel's buffer is empty
    // at a call's start (a failed C2R freezes fill at 0 then) and a call of
    // m blocks is exactly m chunks -- else one more chunk bounds any channel
    bool large = false;
    DevPtr<int4> lg_prog;
    DevPtr<float2> lg_v;
    LgTab lgt{};
    bool lg_whole = true;
    // far-row windows of the generic step (1024 <= B <= 8192):
    // standalone batches and the two-stage tail (gw_ok, set before init);
    // gw_p = the split row (0 = off), gwin = [C][P][B], gw_t = one-block
    // steps so far (the anchor class of the next one)
    bool gw_ok = false;
    bool narrow = false;  // 2048 <= B <= 8192: 256-thread step workgroups (ProcArgs::narrow)
    // (a two-stage tail's one-block step: arrive on this signal, ProcArgs::sig; null = none)
    unsigned *sig_arrive = nullptr;
    unsigned sig_arrive_val = 0;
    int gw_p = 0;
    DevPtr<float2> gwin;
    unsigned long long gw_t = 0;

    ~UniformCore() {
        if (stream) {
            DeviceGuard g(device);
            (void)order.drain(stream);  // (work still queued on a caller stream reads these buffers)
            if (trace_slots) dump_trace();
            if (!parent_stream) (void)hipStreamDestroy(stream);
        }
    }

    void dump_trace() {
        static int dumps = 0;
        bool any = false;
        for (size_t k = 0; k < trace_slots; ++k) any = any || trace_meta[2 * k] >= 0;
        if (!any) return;
        std::vector<int4> h(trace.n);
        if (hipMemcpy(h.data(), trace.p, trace.bytes(), hipMemcpyDeviceToHost) != hipSuccess) return;
        const char *path = getenv("FFTCONV_LA_TRACE_OUT");
        const std::string fn = std::string(path ? path : "/tmp/la_trace.bin") + "." + std::to_string(dumps++);
        FILE *f = fopen(fn.c_str(), "wb");
        if (!f) return;
        const long long hdr[4] = {(long long)trace_slots, (long long)trace_grid, (long long)C, (long long)B};
        fwrite(hdr, sizeof(hdr), 1, f);
        fwrite(trace_meta.data(), sizeof(long long), trace_meta.size(), f);
        fwrite(h.data(), sizeof(int4), h.size(), f);
        fclose(f);
    }

    int alloc_geometry(int dev, size_t channels, size_t max_block_size, size_t max_len) {
        device = dev;
        C = channels;
        ir_len = max_len;
        B = next_pow2(max_block_size);                             // :115
        log2b = ilog2(B);
        if (log2b > kMaxLog2Block)
            return fail(FFTCONV_E_UNSUPPORTED, "block size " + std::to_string(B) + " exceeds 2^22");
        large = log2b > kMaxLog2Fused;
        S = ceil_div(ir_len, B);                                   // :117
        if (S * B > (size_t)INT32_MAX || C > (size_t)INT32_MAX)
            return fail(FFTCONV_E_UNSUPPORTED, "geometry exceeds 32-bit indexing");
        if (parent_stream) stream = parent_stream;
        else HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        if (int r = H.alloc(C * S * B)) return r;
        if (int r = X.alloc(C * S * B)) return r;
        if (int r = pre.alloc(C * B)) return r;
        if (int r = overlap.alloc(C * B)) return r;
        if (int r = inbuf.alloc(C * B)) return r;
        if (int r = state.alloc(C)) return r;
        if (int r = tw.alloc(2 * B)) return r;
        if (int r = staging.alloc(C * ir_len)) return r;  // update() never allocates
        if (own_stage)
            if (int r = hstage.alloc(C * ir_len, ir_len)) return r;
        if (large)
            if (int r = alloc_large()) return r;
        gw_p = gw_ok && gw_supported(log2b, (int)S) ? kGwP : 0;
        if (gw_p)
            if (int r = gwin.alloc(C * (size_t)gw_p * B)) return r;
        la_W = la_ok ? la_parts(log2b, (int)S) : 0;
        if (la_W) {
            const LaDims d = la_dims(log2b, (int)S);
            if (int r = laW.alloc(C * 2 * (size_t)d.pt * B)) return r;
            // (tests: FFTCONV_LA_POISON=1 fills the windows with NaN at init, so a
            // window row read before any anchor wrote it shows in the output)
            if (const char *e = getenv("FFTCONV_LA_POISON"); e && atoi(e) > 0)
                HIP_TRY(hipMemsetAsync(laW.p, 0xff, laW.bytes(), stream));
            if (int r = lav.alloc(2 * C)) return r;
            view_ok = false;
            if (const char *e = getenv("FFTCONV_LA_PROBE"); e && atoi(e) > 0) {
                if (int r = la_probe.alloc(1)) return r;
                HIP_TRY(hipMemsetAsync(la_probe.p, 0, sizeof(int), stream));
            }
        }
        // launch timelines (tuning only): FFTCONV_LA_TRACE for the lookahead
        // launches of a batch that has them, FFTCONV_PROC_TRACE for the
        // process launches of one that has not (e.g. cfg3's head)
        if (const char *e = getenv(la_W ? "FFTCONV_LA_TRACE" : "FFTCONV_PROC_TRACE")) {
            trace_slots = (size_t)std::max(0, atoi(e));
            trace_grid = la_W ? (size_t)la_trace_grid(log2b, (int)S, (int)C) : C;
            if (trace_slots) {
                if (int r = trace.alloc(trace_slots * trace_grid * 8)) return r;
                HIP_TRY(hipMemsetAsync(trace.p, 0, trace.bytes(), stream));
                trace_meta.assign(2 * trace_slots, -1);
            }
        }
        // twiddles W_N^k in double, rounded to f32
        std::vector<float2> t(2 * B);
        const size_t N = 2 * B;
        for (size_t k = 0; k < N; ++k) {
            const double ang = -2.0 * M_PI * (double)k / (double)N;
            t[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
        }
        HIP_TRY(hipMemcpy(tw.p, t.data(), t.size() * sizeof(float2), hipMemcpyHostToDevice));
        return FFTCONV_OK;
    }

    // long-block path buffers (B > 2^kMaxLog2Fused); the tables are shared
    // per (device, geometry); W_N^k is the handle's own `tw`
    int alloc_large() {
        if (int r = lg_prog.alloc(C)) return r;
        if (C) HIP_TRY(hipMemsetAsync(lg_prog.p, 0, lg_prog.bytes(), stream));
        if (int r = lg_v.alloc(C * B)) return r;
        if (int r = lg_tables(device, log2b, &lgt)) return r;
        lgt.twN = tw.p;
        lg_whole = true;
        return FFTCONV_OK;
    }
    // chunks of an n-sample call, an upper bound over the channels
    int lg_chunks(size_t n) const {
        return (int)(lg_whole && n % B == 0 ? n / B : (n + B - 1) / B + 1);
    }
    void lg_note_call(size_t n) { lg_whole = lg_whole && n % B == 0; }

    // fresh state: zero FDL/overlap/buffers, {current 0, active S, fill 0}
    int zero_state() {
        if (X.n) HIP_TRY(hipMemsetAsync(X.p, 0, X.bytes(), stream));
        if (pre.n) HIP_TRY(hipMemsetAsync(pre.p, 0, pre.bytes(), stream));
        if (overlap.n) HIP_TRY(hipMemsetAsync(overlap.p, 0, overlap.bytes(), stream));
        if (inbuf.n) HIP_TRY(hipMemsetAsync(inbuf.p, 0, inbuf.bytes(), stream));
        std::vector<int4> st(C, make_int4(0, (int)S, 0, 0));
        if (C) HIP_TRY(hipMemcpyAsync(state.p, st.data(), C * sizeof(int4), hipMemcpyHostToDevice, stream));
        view_ok = false;
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // run the IR partition FFT from device samples (channel c at src + c*stride)
    int ir_from_device(size_t chan0, size_t nch, const float *src, size_t stride, size_t len_data,
                       size_t len_active, bool update_state, hipStream_t s) {
        IrArgs a{};
        a.H = H.p; a.overlap = overlap.p; a.pre = pre.p; a.state = state.p;
        a.src = src; a.src_stride = (long long)stride;
        a.len_data = (long long)len_data; a.len_active = (long long)len_active;
        a.tw = tw.p; a.S = (int)S; a.chan0 = (int)chan0; a.update_state = update_state ? 1 : 0;
        if (update_state) view_ok = false;
        if (large) {
            HIP_TRY(launch_ir_large(log2b, a, lgt, (int)nch, s));
            return FFTCONV_OK;
        }
        HIP_TRY(launch_ir_segments(log2b, a, (int)nch, s));
        // the updated channels dropped their windows: rebuild them now, in
        // the update, so the next process launch stays a steady-state one
        if (update_state && !la_all) return la_rebuild(s, chan0, nch);
        return FFTCONV_OK;
    }

    // lookahead windows of channels [chan0, chan0+nch) from the current H and
    // FDL (launch_la_rebuild), as if anchored by the launch before the next
    // one; without the lookahead step (or with VARIANT_LAFULL) nothing to do
    int la_rebuild(hipStream_t s, size_t chan0, size_t nch) {
        if (!la_W || la_parts(log2b, (int)S) != la_W || la_full_variant() || nch == 0) return FFTCONV_OK;
        const unsigned long long per = (unsigned long long)la_dims(log2b, (int)S).per_all;
        ProcArgs a{};
        a.job[0] = job(nullptr, 0, nullptr, 0, B);
        a.tw = tw.p;
        a.njobs = 1;
        a.laW = laW.p;
        a.la_c0 = (int)chan0;
        a.la_t = (int)((la_t + per - 1) % per);
        // a rebuild of every channel also fills the next lookahead launch's
        // copy of the state words (la_job then copies nothing)
        const bool whole = chan0 == 0 && nch == C && lav.p;
        if (whole) a.job[0].vnext = lav.p + (size_t)(la_seq & 1) * C;
        HIP_TRY(launch_la_rebuild(log2b, a, (int)(chan0 + nch), s));
        if (whole) view_ok = true;
        return FFTCONV_OK;
    }

    // upload host IRs (channel c at src + c*stride, len samples) into staging rows
    int upload(size_t chan0, size_t nch, const float *src, size_t len, size_t stride, hipStream_t s) {
        if (len == 0 || nch == 0) return FFTCONV_OK;
        float *dst = staging.p + chan0 * ir_len;
        if (stride == 0 || nch == 1) {
            HIP_TRY(hipMemcpyAsync(dst, src, len * sizeof(float), hipMemcpyHostToDevice, s));
        } else {
            HIP_TRY(hipMemcpy2DAsync(dst, ir_len * sizeof(float), src, stride * sizeof(float),
                                     len * sizeof(float), nch, hipMemcpyHostToDevice, s));
        }
        return FFTCONV_OK;
    }

    int init(int dev, size_t channels, const float *responses, size_t len, size_t stride, size_t max_block,
             size_t max_len) {
        if (max_len < len)                                          // :106-110
            return fail(FFTCONV_E_INVALID,
                        "max_response_length must be at least the length of the initial impulse response");
        if (int r = check_device(dev)) return r;
        DeviceGuard g(dev);
        if (int r = alloc_geometry(dev, channels, max_block, max_len)) return r;
        if (int r = zero_state()) return r;
        if (S > 0) {
            if (int r = upload(0, C, responses, len, stride == 0 ? 0 : stride, stream)) return r;
            // every channel reads its own staging row; a shared response reads row 0
            const size_t sst = (stride == 0 && C > 1) ? 0 : ir_len;
            if (int r = ir_from_device(0, C, staging.p, sst, len, ir_len, false, stream)) return r;
        }
        if (la_W && !la_full_variant()) {  // the first process launch is a steady-state one too
            if (int r = la_rebuild(stream, 0, C)) return r;
            la_all = false;
        }
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // FFTConvolver::update (:174-213) for channels [chan0, chan0+nch)
    int update_host(size_t chan0, size_t nch, const float *src, size_t len, size_t stride) {
        if (len > ir_len) return fail(FFTCONV_E_INVALID, "New impulse response is longer than initialized length");
        if (ir_len == 0) return FFTCONV_OK;                        // :181-183
        DeviceGuard g(device);
        // asynchronous: the response goes through the pinned stage; the copy
        // and the transform are enqueued behind the handle's previous work,
        // and every later call is ordered behind them (StreamOrder)
        if (int r = order.enter(stream)) return r;
        return update_host_on(chan0, nch, src, len, stride, stream, hstage);
    }
    // (the caller has ordered stream s behind the handle's previous work);
    // the response goes through `stage` into the staging rows
    int update_host_on(size_t chan0, size_t nch, const float *src, size_t len, size_t stride, hipStream_t s,
                       PinnedStage &stage) {
        if (len > ir_len) return fail(FFTCONV_E_INVALID, "New impulse response is longer than initialized length");
        if (ir_len == 0) return FFTCONV_OK;
        const bool shared = stride == 0 && nch > 1;  // one response for every channel: one staging row
        if (len && nch)
            if (int r = stage.upload(src, shared ? 1 : nch, len, stride, staging.p + chan0 * ir_len, ir_len, s)) return r;
        return ir_from_device(chan0, nch, staging.p + chan0 * ir_len, shared ? 0 : ir_len, len, len, true, s);
    }

    // update() from device samples, stream-ordered (used by the crossfade swap)
    int update_device(const float *src, size_t stride, size_t len, hipStream_t s) {
        if (len > ir_len) return fail(FFTCONV_E_INVALID, "New impulse response is longer than initialized length");
        if (ir_len == 0) return FFTCONV_OK;
        return ir_from_device(0, C, src, stride, len, len, true, s);
    }

    int reset(hipStream_t s) {  // :296-306
        if (X.n) HIP_TRY(hipMemsetAsync(X.p, 0, X.bytes(), s));
        if (overlap.n) HIP_TRY(hipMemsetAsync(overlap.p, 0, overlap.bytes(), s));
        if (inbuf.n) HIP_TRY(hipMemsetAsync(inbuf.p, 0, inbuf.bytes(), s));
        if (pre.n) HIP_TRY(hipMemsetAsync(pre.p, 0, pre.bytes(), s));
        HIP_TRY(launch_reset_state(state.p, (int)C, s));
        view_ok = false;
        lg_whole = true;
        if (la_W && !la_full_variant()) {  // windows of the zeroed FDL, in the reset
            la_all = false;
            return la_rebuild(s, 0, C);
        }
        la_all = true;
        return FFTCONV_OK;
    }

    // a launch's job: any launch but a lookahead one may write the state
    // words, so the anchors' copy is stale after it (la_job for those)
    ProcJob job(const float *din, size_t is, float *dout, size_t os, size_t n) const {
        view_ok = false;
        return job_raw(din, is, dout, os, n);
    }
    ProcJob job_raw(const float *din, size_t is, float *dout, size_t os, size_t n) const {
        ProcJob j{};
        j.H = H.p; j.X = X.p; j.overlap = overlap.p; j.inbuf = inbuf.p; j.pre = pre.p; j.state = state.p;
        j.in = din; j.in_stride = (long long)is; j.out = dout; j.out_stride = (long long)os;
        j.S = (int)S; j.n = (int)n;
        j.lg_prog = lg_prog.p; j.lg_v = lg_v.p;
        return j;
    }
    // the long-block fields of a launch of this batch's n-sample call (the
    // call is counted: a launch failure after this leaves lg_whole pessimistic)
    void lg_fill(ProcArgs &a, size_t n) {
        if (!large) return;
        a.lg = lgt;
        a.lg_chunks = std::max(a.lg_chunks, lg_chunks(n));
        lg_note_call(n);
    }

    // a call of whole blocks takes the lookahead launch, one
    // launch per block
    bool la_ready(size_t n) const { return la_W && n > 0 && n % B == 0 && la_parts(log2b, (int)S) == la_W; }

    // this batch's lookahead fields of a launch: windows, stagger clock (the
    // launcher derives the anchor workgroups from them), and the timeline
    // record, when tracing
    int la_fill(ProcArgs &a, hipStream_t s) {
        a.laW = laW.p;
        a.la_all = la_all ? 1 : 0;
        a.la_t = (int)(la_t % (unsigned long long)la_dims(log2b, (int)S).per_all);  // (every period divides it)
        a.la_seq = la_seq;
        a.la_probe_cnt = la_probe.p;
        if (!la_all) return trace_fill(a, s);  // (steady-state launches only: the record is sized for them)
        return FFTCONV_OK;
    }
    // this launch's timeline record (slot = launch count mod trace_slots)
    int trace_fill(ProcArgs &a, hipStream_t s) {
        if (!trace_slots) return FFTCONV_OK;
        const size_t slot = (size_t)(la_t % trace_slots);
        a.la_trace = trace.p + slot * trace_grid * 8;
        a.la_trace_grid = (int)trace_grid;
        trace_meta[2 * slot] = (long long)la_t;
        trace_meta[2 * slot + 1] = -1;  // (grid: the analysis counts the records)
        HIP_TRY(hipMemsetAsync(a.la_trace, 0, trace_grid * 8 * sizeof(int4), s));
        return FFTCONV_OK;
    }
    void la_advance() {
        ++la_t;
        la_seq = 3 - la_seq;
        la_all = false;
    }
    // a lookahead launch's job: the anchors read copy la_seq & 1 of the state
    // words, the steps fill the other for the next launch (la.hpp
    // la_anchor_state); after any other writer the words are copied first
    int la_job(ProcJob &j, const float *din, size_t is, float *dout, size_t os, size_t n, hipStream_t s) {
        j = job_raw(din, is, dout, os, n);
        if (!lav.p) return fail(FFTCONV_E_DEVICE, "lookahead launch without the state copies");
        int4 *rd = lav.p + (size_t)(la_seq & 1) * C, *wr = lav.p + (size_t)((la_seq & 1) ^ 1) * C;
        if (!view_ok && C) HIP_TRY(hipMemcpyAsync(rd, state.p, C * sizeof(int4), hipMemcpyDeviceToDevice, s));
        view_ok = true;  // (the launch's steps fill `wr`; la_advance makes it the next read copy)
        j.sview = rd;
        j.vnext = wr;
        return FFTCONV_OK;
    }

    // la_mix / mix / mix_tab: crossfade fusion on the lookahead step (ProcArgs::la_mix);
    // the caller only passes them when this call takes the lookahead launch
    // after_step (optional): recorded once the call's outputs are final, before
    // the far-row window anchor that follows a one-block step (the two-stage
    // head reads the tail's output, not its windows)
    int process_device(const float *din, size_t is, float *dout, size_t os, size_t n, hipStream_t s,
                       int la_mix = 0, const CrossfadeMixArgs *mix = nullptr, float *mix_tab = nullptr,
                       hipEvent_t after_step = nullptr) {
        if (n > (size_t)INT32_MAX) return fail(FFTCONV_E_UNSUPPORTED, "process length exceeds 2^31-1");
        if (n == 0 || C == 0) return FFTCONV_OK;
        ProcArgs a{};
        a.job[0] = job_raw(din, is, dout, os, n);
        a.tw = tw.p;
        a.njobs = 1;
        if (la_ready(n)) {
            // lookahead launches, one per block of the call: the step
            // workgroups behind each launch's anchors (every channel on entry,
            // else the stagger classes (c - t) % period == 0).  A multi-block
            // call keeps the windows: each launch is the step of one block,
            // bit-identical to one call per block; a channel off the lookahead
            // path runs the whole call (:222-294) in the first launch
            const size_t m = n / B;
            if (m > 1 && la_mix) return fail(FFTCONV_E_INVALID, "crossfade lookahead launch of more than one block");
            for (size_t k = 0; k < m; ++k) {
                if (int r = la_job(a.job[0], din + k * B, is, dout + k * B, os, B, s)) return r;
                a.job[0].mcall = (int)m;
                a.job[0].mk = (int)k;
                if (int r = la_fill(a, s)) return r;
                if (la_mix && mix) {
                    a.la_mix = la_mix;
                    a.mix = *mix;
                    a.mix_tab = mix_tab;
                }
                HIP_TRY(launch_process_la(log2b, a, (int)C, s));
                la_advance();
            }
            if (after_step) HIP_TRY(hipEventRecord(after_step, s));
            return FFTCONV_OK;
        }
        if (la_W) la_all = true;  // this launch drops every window
        view_ok = false;          // (and writes the state words)
        if (trace_slots && !la_W && n == B) {  // (process timelines: one-block calls)
            if (int r = trace_fill(a, s)) return r;
            ++la_t;
        }
        lg_fill(a, n);
        a.narrow = narrow ? 1 : 0;
        a.gw_p = gw_p;  // (every launch: the split order)
        if (sig_arrive && n == B && !large) {
            a.sig = sig_arrive;
            a.sig_val = sig_arrive_val;
            a.sig_mode = 1;
        }
        if (gw_p && n == B && gw_windows_allowed()) {
            // a one-block step reads the live windows, then the channels of
            // class gw_t mod P anchor theirs for their next P blocks
            a.gw = gwin.p;
            a.gw_t = (int)(gw_t % (unsigned long long)gw_p);
            HIP_TRY(launch_process(log2b, a, (int)C, s));
            if (after_step) HIP_TRY(hipEventRecord(after_step, s));
            a.sig_mode = 0;  // (the anchor does not arrive)
            HIP_TRY(launch_gw_anchor(log2b, a, (int)C, s));
            ++gw_t;
            return FFTCONV_OK;
        }
        HIP_TRY(launch_process(log2b, a, (int)C, s));
        if (after_step) HIP_TRY(hipEventRecord(after_step, s));
        return FFTCONV_OK;
    }

    // `steps` consecutive process() calls (fftconv_uniform_process_device_steps).
    // A batch on the generic / pipelined step (no lookahead, no far-row
    // windows, B <= 512) whose workgroups fit the chip twice over runs them
    // as ONE launch (upols_run_kernel: each channel loops over its calls,
    // process_job per call -- the same bits as one launch per call).
    int process_device_steps(const float *din, size_t is, size_t in_step, float *dout, size_t os, size_t out_step,
                             size_t n, size_t steps, hipStream_t s) {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 0;
        if (steps >= 2 && n > 0 && n <= (size_t)INT32_MAX && !la_W && !large && !gw_p && !trace_slots &&
            C <= 2 * (size_t)ncu && steps <= (size_t)INT32_MAX && run_supported(log2b) &&
            in_step <= (size_t)LLONG_MAX && out_step <= (size_t)LLONG_MAX) {
            ProcArgs a{};
            a.job[0] = job(din, is, dout, os, n);
            a.tw = tw.p;
            a.njobs = 1;
            a.run_lds_rows = run_lds_rows(log2b, (int)S);
            RunSteps r{(long long)in_step, (long long)out_step, (int)steps};
            HIP_TRY(launch_process_run(log2b, a, r, (int)C, s));
            return FFTCONV_OK;
        }
        for (size_t k = 0; k < steps; ++k)
            if (int r = process_device(din + k * in_step, is, dout + k * out_step, os, n, s)) return r;
        return FFTCONV_OK;
    }

    int process_host(const float *in, size_t in_len, float *out, size_t out_len) {
        if (in_len < out_len) return fail(FFTCONV_E_INVALID, "input slice shorter than output (range end index out of range)");
        if (out_len == 0 || C == 0) return FFTCONV_OK;
        DeviceGuard g(device);
        if (int r = order.enter(stream)) return r;
        if (int r = scratch.ensure(C * out_len, C * out_len)) return r;
        HIP_TRY(hipMemcpy2DAsync(scratch.in.p, out_len * sizeof(float), in, in_len * sizeof(float),
                                 out_len * sizeof(float), C, hipMemcpyHostToDevice, stream));
        if (int r = process_device(scratch.in.p, out_len, scratch.out.p, out_len, out_len, stream)) return r;
        HIP_TRY(hipMemcpyAsync(out, scratch.out.p, C * out_len * sizeof(float), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // #[derive(Clone)]
    int clone_from(const UniformCore &o, bool with_stage = true) {
        DeviceGuard g(o.device);
        if (int r = o.order.drain(o.stream)) return r;
        device = o.device;
        C = o.C; ir_len = o.ir_len; B = o.B; log2b = o.log2b; S = o.S;
        if (parent_stream) stream = parent_stream;
        else HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        auto cp = [&](auto &dst, const auto &src) -> int {
            if (int r = dst.alloc(src.n)) return r;
            if (src.n) HIP_TRY(hipMemcpyAsync(dst.p, src.p, src.bytes(), hipMemcpyDeviceToDevice, stream));
            return FFTCONV_OK;
        };
        if (int r = cp(H, o.H)) return r;
        if (int r = cp(X, o.X)) return r;
        if (int r = cp(pre, o.pre)) return r;
        if (int r = cp(tw, o.tw)) return r;
        if (int r = cp(overlap, o.overlap)) return r;
        if (int r = cp(inbuf, o.inbuf)) return r;
        if (int r = cp(state, o.state)) return r;
        if (int r = cp(laW, o.laW)) return r;
        la_ok = o.la_ok; la_W = o.la_W; la_t = o.la_t; la_seq = o.la_seq; la_all = o.la_all;
        if (o.lav.n)
            if (int r = lav.alloc(o.lav.n)) return r;
        view_ok = false;  // (copied from `state` before the clone's first lookahead launch)
        if (int r = cp(gwin, o.gwin)) return r;
        gw_ok = o.gw_ok; gw_p = o.gw_p; gw_t = o.gw_t;
        large = o.large;
        if (large) {  // (the progress words are zero between calls)
            if (int r = alloc_large()) return r;
            lg_whole = o.lg_whole;
        }
        if (o.trace_slots) {  // (tuning: a clone keeps its own timeline)
            trace_slots = o.trace_slots;
            trace_grid = o.trace_grid;
            if (int r = trace.alloc(trace_slots * trace_grid * 8)) return r;
            HIP_TRY(hipMemsetAsync(trace.p, 0, trace.bytes(), stream));
            trace_meta.assign(2 * trace_slots, -1);
        }
        if (int r = staging.alloc(o.staging.n)) return r;
        own_stage = with_stage && o.own_stage;
        if (own_stage)
            if (int r = hstage.alloc(o.hstage.n, ir_len)) return r;
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // segments_ir[seg] of channel c as the reference holds it: B+1 bins,
    // interleaved (re, im), unpacked from the (DC, Nyquist) slot
    int ir_spectrum(size_t c, size_t seg, float *out) {
        if (c >= C || seg >= S) return fail(FFTCONV_E_INVALID, "channel or segment out of range");
        DeviceGuard g(device);
        if (int r = order.drain(stream)) return r;
        std::vector<float2> row(B);
        HIP_TRY(hipMemcpy(row.data(), H.p + (c * S + seg) * B, B * sizeof(float2), hipMemcpyDeviceToHost));
        out[0] = row[0].x;
        out[1] = 0.f;
        for (size_t k = 1; k < B; ++k) {
            const size_t p = large ? lg_position(log2b, k) : k;  // (long blocks: transposed bin order)
            out[2 * k] = row[p].x;
            out[2 * k + 1] = row[p].y;
        }
        out[2 * B] = row[0].y;
        out[2 * B + 1] = 0.f;
        return FFTCONV_OK;
    }

    int channel_state(size_t c, size_t out3[3]) {
        if (c >= C) return fail(FFTCONV_E_INVALID, "channel out of range");
        DeviceGuard g(device);
        if (int r = order.drain(stream)) return r;
        int4 st;
        HIP_TRY(hipMemcpy(&st, state.p + c, sizeof(int4), hipMemcpyDeviceToHost));
        out3[0] = (size_t)st.x; out3[1] = (size_t)st.y; out3[2] = (size_t)st.z;
        return FFTCONV_OK;
    }
};

// ---------------------------------------------------------------------------
// TwoStageCore -- TwoStageFFTConvolver (src/fft_convolver.rs:323-512)
// ---------------------------------------------------------------------------
struct TwoStageCore {
    int device = 0;
    size_t C = 0, head_bs = 0, T = 0;
    std::unique_ptr<UniformCore> head, tail0, tail;  // null tail = Default (zeros)
    DevPtr<float> out0, pre0, out1, pre1;            // [C][T] each
    DevPtr<float> tin_buf[2];                        // tail_input, double-buffered per tail period
    int tin_idx = 0;
    float *tail_output0 = nullptr, *tail_precalculated0 = nullptr;
    float *tail_output = nullptr, *tail_precalculated = nullptr;
    size_t tail_input_fill = 0, precalculated_pos = 0;
    hipStream_t stream = nullptr;
    // The T-sized tail convolution runs on its own stream: its result is first
    // read one whole tail period later (after the next swap), which is the
    // reference's "might be done in some background thread" (:478).
    hipStream_t side = nullptr;
    // an unmasked side stream for the tail of a period whose calls ran as
    // multi-call launches (process_device_steps, upols_run_kernel): those
    // head workgroups stay resident for the whole run, so the tail may use
    // every CU beside them (cfg3: 5.34 us per step unmasked vs 9.26 on one
    // unit, while one launch per call is fastest on one unit: 7.18 vs 8.07;
    // profiles/r5/r5f_*).  null when `side` is unmasked already.
    hipStream_t side_open = nullptr;
    bool period_runs = false;  // this period's calls went through multi-call launches
    hipStream_t last_ts = nullptr;  // the side stream of the last tail
    // ev_tail: the tail's step (its output, what the next period reads);
    // ev_tail_done: everything of it, its window anchor included (quiesce)
    hipEvent_t ev_main = nullptr, ev_tail = nullptr, ev_tail_done = nullptr;
    bool tail_in_flight = false;
    // The head of the period after a tail's period reads that tail's output.
    // Instead of a barrier packet on the head's stream at every period end
    // (hipStreamWaitEvent: ~7 us of cfg3's ~240 us period, r6p), the next
    // run waits on the device (ProcArgs::sig): tail step k releases
    // tsig[1] = k, and `pend` names the tail the next head work must follow
    // (0 = none); every other path waits on that tail's event ev_tk[k & 1].
    DevPtr<unsigned> tsig;  // {arrivals, last tail done, wait timeouts, -}
    hipEvent_t ev_tk[2] = {nullptr, nullptr};
    bool tk_sig[2] = {false, false};  // tail k arrives on tsig
    unsigned tseq = 0, pend = 0;
    // the event wait for a pending tail, on stream s (every path but a run)
    int resolve_pend(hipStream_t s) {
        if (pend) HIP_TRY(hipStreamWaitEvent(s, ev_tk[pend & 1], 0));
        pend = 0;
        return FFTCONV_OK;
    }
    int ts_exp = 0;  // (timing probes, FFTCONV_TS_EXP at creation; never in tests)
    // the tail's step on 256-thread workgroups: 0 never, 1 in periods that ran
    // as multi-call runs, 2 always (FFTCONV_TAIL_NARROW at creation)
    int tail_narrow = 2;
    // the side stream confined to the tail's byte share of the CUs (off: the
    // tail's step runs on 256-thread workgroups that fit beside the head's,
    // and a CU-masked side stream held one handle's one-launch-per-call head
    // launches for 456 us at a time, 21.5-22.9 us per cfg3 call, against
    // 7.55 unmasked: profiles/r6/r6b, r6c).  FFTCONV_TAIL_MASKED=1 at creation
    bool tail_masked = false;
    // the side stream at the device's highest stream priority: HIP maps
    // streams onto at most GPU_MAX_HW_QUEUES (4) hardware queues, and a side
    // stream that shared its queue with the head's caller stream serialised
    // the tail behind the head (the third cfg3 handle of a process ran at
    // 5.1 us per call against 3.8); high-priority streams get queues of their
    // own (three handles 3.75 / 3.75 / 3.75 us, profiles/r6/r6m).
    // FFTCONV_TAIL_PRIO=0 at creation: a normal-priority side stream
    bool tail_prio = true;
    int run_prio = 0;  // (tuning, FFTCONV_RUN_PRIO at creation: ProcArgs::prio of the runs)
    int run_min = 2;   // (tuning, FFTCONV_RUN_MIN at creation: shortest run of calls taken as one launch)
    // tail0 deferred to the end of its period (launch_tail0_flush): the
    // aligned calls' blocks [t0_off, t0_off + t0_n * head_bs) of tail_input
    // still to be convolved by tail_convolver0 (FFTCONV_TAIL0_DEFER=0: off)
    bool t0_defer = false;
    mutable size_t t0_off = 0, t0_n = 0;
    // pending blocks [0, t0_have) whose spectra a run already wrote to t0_xs
    mutable size_t t0_have = 0;
    size_t t0_nmax = 0;
    DevPtr<float2> t0_xs;
    DevPtr<float> t0_ys;
    DevPtr<int> t0_err;
    DevPtr<float> t0_ov;
    DevPtr<float2> t0_cv;
    // [C]: a run's call of this channel wrote no spectrum to t0_xs (its head
    // buffer out of step with tail_input); the flush recomputes and clears it
    DevPtr<int> t0_miss;
    DevPtr<int> t0_trace;  // (tuning, FFTCONV_T0_TRACE: the fused flush's phase stamps, [C][8], last flush)
    Scratch scratch;
    mutable StreamOrder order;

    ~TwoStageCore() {
        DeviceGuard g(device);
        if (t0_trace.n) {  // (FFTCONV_T0_TRACE: per-phase medians of the last flush, us)
            (void)hipDeviceSynchronize();
            std::vector<int> h(t0_trace.n);
            if (hipMemcpy(h.data(), t0_trace.p, t0_trace.bytes(), hipMemcpyDeviceToHost) == hipSuccess) {
                std::vector<double> ph[5];
                for (size_t c = 0; c < C; ++c)
                    for (int k = 0; k < 5; ++k) ph[k].push_back((double)(unsigned)(h[c * 8 + k + 1] - h[c * 8]) / 100.0);
                fprintf(stderr, "t0 flush phases (us from the workgroup's start, median over channels):");
                for (auto &v : ph) {
                    std::sort(v.begin(), v.end());
                    fprintf(stderr, " %.2f", v[v.size() / 2]);
                }
                fprintf(stderr, "\n");
            }
        }
        if (side) { (void)hipStreamSynchronize(side); (void)hipStreamDestroy(side); }
        if (side_open) { (void)hipStreamSynchronize(side_open); (void)hipStreamDestroy(side_open); }
        if (stream) (void)order.drain(stream);
        head.reset(); tail0.reset(); tail.reset();  // (they borrow `stream`)
        if (stream) (void)hipStreamDestroy(stream);
        if (ev_main) (void)hipEventDestroy(ev_main);
        if (ev_tail) (void)hipEventDestroy(ev_tail);
        for (auto &e : ev_tk)
            if (e) (void)hipEventDestroy(e);
        if (ev_tail_done) (void)hipEventDestroy(ev_tail_done);
    }

    float *tail_input() const { return tin_buf[tin_idx].p; }

    // every piece of the handle's work has finished: the caller-stream work
    // (StreamOrder) and the tail convolution on the side stream
    int quiesce() const {
        if (int r = order.enter(stream)) return r;
        if (tail_in_flight) HIP_TRY(hipStreamWaitEvent(stream, ev_tail_done, 0));
        HIP_TRY(hipStreamSynchronize(stream));
        if (tsig.n) {  // (a run that gave up waiting for its tail: never expected)
            unsigned to = 0;
            HIP_TRY(hipMemcpy(&to, tsig.p + 2, sizeof(unsigned), hipMemcpyDeviceToHost));
            if (to) return fail(FFTCONV_E_DEVICE, "a two-stage run timed out waiting for its tail step");
        }
        return FFTCONV_OK;
    }

    // The side stream is confined to the first CUs of the mask, in units of
    // ncu/8 (one XCD's worth of CUs; how the mask's CU numbering maps onto
    // XCDs is not documented): as many units as the tail's share of the
    // bytes streamed per tail period, at least one.  A T-block
    // tail workgroup fills a whole CU (512 lanes x 197 VGPRs), and unconfined
    // it locks the latency-critical head steps out of the chip for its whole
    // duration (measured: a 197 us head step behind a 193 us tail).  With the
    // tail's far-row windows cfg3's tail fits one unit (32 CUs):
    // the head steps keep the rest of the chip (6.92 us per
    // step, vs 7.29 on 36 CUs, 7.23 on 64, 7.54 on 85, and the tail no longer
    // fits a period on 25 or fewer: profiles/r4/r4w_*, r4x_*).  Contiguous
    // masks only: power-of-two strided masks read back fine but did not
    // constrain dispatch (scripts/cumask_probe.hip).
    int create_side_stream() {
        int ncu = 0;
        HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        int cus = 0;  // 0 = unmasked
        // A long-block tail (T > 2^kMaxLog2Fused, large.hip) is unmasked: its
        // passes are many short 256-lane workgroups that leave room for the
        // head steps, and confined by its byte share its row pass ran at a
        // fraction of the chip's bandwidth (head 512 / IR 200,000: 59.6 us per
        // step on one unit of 32 CUs, 28.7 on 3 units, 21.4 unmasked;
        // profiles/r5/r5d_lgt_tail_units.log)
        if (tail && ncu >= 8 && !tail->large && tail_masked) {
            // bytes per tail period in B-bin rows: the tail's step (with windows:
            // P-1 near rows of H and X, one window row, and 1/P of an anchor's
            // S H rows, S X rows and P window rows) against T/h head steps
            const double P = tail->gw_p;
            const double tail_rows = P > 0 ? (2 * (P - 1) + 1 + (2 * tail->S + P) / P) / 2 : (double)tail->S;
            const double tail_b = tail_rows * (double)tail->B;
            const double per_b = tail_b + (double)(T / std::max<size_t>(head_bs, 1)) *
                                              (double)((head ? head->S * head->B : 0) + (tail0 ? tail0->S * tail0->B : 0));
            const int nx = std::min(7, std::max(1, (int)std::lround(8.0 * tail_b / std::max(per_b, 1.0))));
            cus = nx * (ncu / 8);
        }
        // (tuning, read once per handle at creation: FFTCONV_TAIL_CU_DIV=k
        // confines the tail to ncu/k CUs instead, 1 = unmasked;
        // FFTCONV_TAIL_CU_UNITS=n to n units of ncu/8, 8 = unmasked)
        if (const char *e = getenv("FFTCONV_TAIL_CU_DIV")) {
            const int k = std::max(1, atoi(e));
            cus = k <= 1 ? 0 : std::max(1, ncu / k);
        }
        const bool knob = getenv("FFTCONV_TAIL_CU_DIV") || getenv("FFTCONV_TAIL_CU_UNITS");
        if (const char *e = getenv("FFTCONV_TAIL_CU_UNITS")) {
            const int n = std::min(8, std::max(1, atoi(e)));
            cus = n >= 8 ? 0 : n * (ncu / 8);
        }
        if (cus > 0 && cus < ncu && !knob)  // (a tuning knob governs every period)
            HIP_TRY(hipStreamCreateWithFlags(&side_open, hipStreamNonBlocking));
        if (cus <= 0 || cus >= ncu) {
            if (tail_prio) {
                int least = 0, greatest = 0;
                HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
                HIP_TRY(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, greatest));
            } else {
                HIP_TRY(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
            }
            return FFTCONV_OK;
        }
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int cu = 0; cu < cus; ++cu) mask[cu / 32] |= 1u << (cu % 32);
        HIP_TRY(hipExtStreamCreateWithCUMask(&side, (uint32_t)mask.size(), mask.data()));
        return FFTCONV_OK;
    }

    int alloc_buffers() {
        if (const char *e = getenv("FFTCONV_TS_EXP")) ts_exp = atoi(e);
        if (const char *e = getenv("FFTCONV_TAIL_NARROW")) tail_narrow = atoi(e);
        if (const char *e = getenv("FFTCONV_TAIL_MASKED")) tail_masked = atoi(e) != 0;
        if (const char *e = getenv("FFTCONV_TAIL_PRIO")) tail_prio = atoi(e) != 0;
        if (const char *e = getenv("FFTCONV_RUN_PRIO")) run_prio = atoi(e);
        if (const char *e = getenv("FFTCONV_RUN_MIN")) run_min = std::max(1, atoi(e));
        if (int r = create_side_stream()) return r;
        // The period events order kernels on this device only (no host wait
        // reads what they guard), so they carry no system-scope fence: with
        // it, cfg3 one-launch-per-call periods ran at 21.5 us per call on one
        // box (head launches held for 456 us beside the tail), without it
        // 6.6 us (profiles/r6/r6b).  (FFTCONV_TS_EXP bit 2: the fence back)
        const unsigned evf = hipEventDisableTiming | ((ts_exp & 4) ? 0u : hipEventDisableSystemFence);
        HIP_TRY(hipEventCreateWithFlags(&ev_main, evf));
        HIP_TRY(hipEventCreateWithFlags(&ev_tail, evf));
        for (auto &e : ev_tk) HIP_TRY(hipEventCreateWithFlags(&e, evf));
        if (int r = tsig.alloc(4)) return r;
        HIP_TRY(hipMemsetAsync(tsig.p, 0, tsig.bytes(), stream));
        tseq = pend = 0;
        HIP_TRY(hipEventCreateWithFlags(&ev_tail_done, evf));
        for (auto *b : {&out0, &pre0, &out1, &pre1, &tin_buf[0], &tin_buf[1]}) {
            if (int r = b->alloc(C * T)) return r;
            if (b->n) HIP_TRY(hipMemsetAsync(b->p, 0, b->bytes(), stream));
        }
        tail_output0 = out0.p; tail_precalculated0 = pre0.p;
        tail_output = out1.p; tail_precalculated = pre1.p;
        tin_idx = 0;
        const bool defer = tail0_defer_allowed();  // (VARIANT_T0BLOCK: per-block tail0, tests)
        t0_nmax = T / std::max<size_t>(head_bs, 1);
        t0_defer = defer && tail0 && tail0->B == head_bs &&
                   tail0_defer_supported(tail0->log2b, (int)tail0->S, (int)t0_nmax);
        if (t0_defer) {
            if (int r = t0_xs.alloc(C * t0_nmax * head_bs)) return r;
            if (int r = t0_ys.alloc(C * t0_nmax * 2 * head_bs)) return r;
            if (int r = t0_err.alloc(C)) return r;
            if (int r = t0_ov.alloc(C * head_bs)) return r;
            if (int r = t0_cv.alloc(C * t0_nmax * head_bs)) return r;
            if (int r = t0_miss.alloc(C)) return r;
            if (getenv("FFTCONV_T0_TRACE"))
                if (int r = t0_trace.alloc(C * 16)) return r;  // (C x 4 int4: the replay's proc_stamp too)
            HIP_TRY(hipMemsetAsync(t0_err.p, 0, t0_err.bytes(), stream));
            if (t0_miss.n) HIP_TRY(hipMemsetAsync(t0_miss.p, 0, t0_miss.bytes(), stream));
        }
        t0_off = t0_n = t0_have = 0;
        return FFTCONV_OK;
    }

    // tail_convolver0.process (:464-472) of the deferred blocks, in one pass
    int flush_t0(hipStream_t s, hipEvent_t done = nullptr) const {
        if (t0_n == 0) return FFTCONV_OK;
        Tail0Args a{};
        a.pa.job[0] = tail0->job(tail_input() + t0_off, T, tail_output0 + t0_off, T, head_bs);
        a.pa.tw = tail0->tw.p;
        a.pa.njobs = 1;
        a.xs = t0_xs.p; a.ys = t0_ys.p; a.err = t0_err.p; a.ov0 = t0_ov.p; a.cv = t0_cv.p;
        a.act = (int)tail0->S;
        a.n = (int)t0_n; a.nmax = (int)t0_nmax;
        a.k0 = (int)std::min(t0_have, t0_n);
        a.miss = t0_miss.p;
        if (t0_trace.n) a.pa.la_trace = reinterpret_cast<int4 *>(t0_trace.p);  // (FFTCONV_T0_TRACE)
        HIP_TRY(launch_tail0_flush(tail0->log2b, a, (int)C, s, done));
        t0_n = t0_have = 0;  // (only once the flush is enqueued: a failed launch keeps the blocks pending)
        return FFTCONV_OK;
    }

    int init(int dev, size_t channels, const float *responses, size_t len, size_t stride, size_t block_size,
             size_t max_len) {
        head_bs = block_size;                                                   // :341
        T = fftconv_compute_tail_block_size(block_size, max_len);              // :342
        if (max_len < len)                                                      // :344-348
            return fail(FFTCONV_E_INVALID,
                        "max_response_length must be at least the length of the initial impulse response");
        if (int r = check_device(dev)) return r;
        if (ilog2(T) > kMaxLog2Block)
            return fail(FFTCONV_E_UNSUPPORTED, "tail block size " + std::to_string(T) + " exceeds 2^22");
        device = dev;
        C = channels;
        DeviceGuard g(dev);
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        // padded_ir = response zero-extended to max_len (:349-350); sub-ranges
        // are cut on the host so each stage sees exactly its reference slice
        const size_t sstride = stride == 0 ? 0 : stride;
        auto slice = [&](size_t off, size_t cnt, std::vector<float> &buf) -> size_t {
            const size_t rows = (sstride == 0) ? 1 : C;
            buf.assign(rows * std::max<size_t>(cnt, 1), 0.f);
            for (size_t c = 0; c < rows; ++c)
                for (size_t j = 0; j < cnt; ++j) {
                    const size_t p = off + j;
                    buf[c * cnt + j] = p < len ? responses[c * sstride + p] : 0.f;
                }
            return sstride == 0 ? 0 : cnt;
        };
        std::vector<float> tmp;
        const size_t head_ir_len = std::min(max_len, T);                        // :352-354
        head.reset(new (std::nothrow) UniformCore());
        if (!head) return fail(FFTCONV_E_NOMEM, "out of host memory");
        head->parent_stream = stream;
        size_t st = slice(0, head_ir_len, tmp);
        if (int r = head->init(dev, C, tmp.data(), head_ir_len, st, head_bs, head_ir_len)) return r;
        if (max_len > T) {                                                      // :356-368
            const size_t tl = std::min(max_len - T, T);
            tail0.reset(new (std::nothrow) UniformCore());
            if (!tail0) return fail(FFTCONV_E_NOMEM, "out of host memory");
            tail0->parent_stream = stream;
            st = slice(T, tl, tmp);
            if (int r = tail0->init(dev, C, tmp.data(), tl, st, head_bs, tl)) return r;
        }
        if (max_len > 2 * T) {                                                  // :373-384
            const size_t tl = max_len - 2 * T;
            tail.reset(new (std::nothrow) UniformCore());
            if (!tail) return fail(FFTCONV_E_NOMEM, "out of host memory");
            tail->parent_stream = stream;
            // one full-block call per period: far-row windows (tuning, read at
            // creation: FFTCONV_TAIL_GW=0 turns them off)
            const char *gwe = getenv("FFTCONV_TAIL_GW");
            tail->gw_ok = !gwe || atoi(gwe) != 0;
            st = slice(2 * T, tl, tmp);
            if (int r = tail->init(dev, C, tmp.data(), tl, st, T, tl)) return r;
        }
        if (int r = alloc_buffers()) return r;
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // fill reached T (:464-491): swap the tail0 buffers, swap the tail buffers,
    // and start the tail convolution of this period on the side stream.
    // (Starting the tail before the flush, beside it, was slower: 8.17 vs
    // 7.62 us per cfg3 step, profiles/r4/r4u_ab_cfg3_tail_early_rejected.log.)
    int end_of_period(hipStream_t s) {
        // ev_main (the tail may start) recorded by the flush kernel's own
        // completion (hipExtLaunchKernel) instead of a marker packet after it
        // (cfg3 A/B 3.669 -> 3.645 us per call, r6p); FFTCONV_TS_EXP bit 4: the marker
        const bool ev_on_flush = !(ts_exp & 16) && t0_n > 0 && tail && !(ts_exp & 8);
        if (int r = flush_t0(s, ev_on_flush ? ev_main : nullptr)) return r;  // (tail_output0 is complete before the swap)
        std::swap(tail_precalculated0, tail_output0);                         // :473-475
        std::swap(tail_precalculated, tail_output);                           // :483
        // work after this point reads the swapped-in tail_precalculated: it is
        // the previous period's tail result, which the next head work waits
        // for (`pend`: a run on the device, every other path on its event)
        // (FFTCONV_TS_EXP bit 0, timing probes only: no wait -- racy)
        if (int r = resolve_pend(s)) return r;  // (a period of one call: the previous one's)
        if (tail_in_flight && !(ts_exp & 1)) pend = tseq;
        if (tail && !(ts_exp & 8)) {  // :484-485 (FFTCONV_TS_EXP bit 3, timing probes only: no tail at all)
            hipStream_t ts = period_runs && side_open ? side_open : side;
            if (!ev_on_flush) HIP_TRY(hipEventRecord(ev_main, s));  // this period's tail_input is complete
            HIP_TRY(hipStreamWaitEvent(ts, ev_main, 0));
            // ev_main follows the previous tail's step only (ev_tail): its
            // window anchor ran on its own side stream, so a tail on the other
            // one starts after that too
            if (tail_in_flight && ts != last_ts) HIP_TRY(hipStreamWaitEvent(ts, ev_tail_done, 0));
            // (the next period waits for the tail's output only, not for its
            // window anchor: 19 us of cross-queue wait behind the anchor, r5p;
            // starting the tail before the flush gained nothing, r5s)
            tail->narrow = (tail_narrow == 2 || (tail_narrow == 1 && period_runs)) && !tail->large;
            const unsigned seq = tseq + 1 == 0 ? 1 : tseq + 1;  // (0 = none)
            const bool use_sig = !tail->large && !(ts_exp & 32);  // (FFTCONV_TS_EXP bit 5: events only)
            tail->sig_arrive = use_sig ? tsig.p : nullptr;
            tail->sig_arrive_val = seq;
            const int rr = tail->process_device(tail_input(), T, tail_output, T, T, ts, 0, nullptr, nullptr, ev_tk[seq & 1]);
            tail->sig_arrive = nullptr;
            if (rr) return rr;
            tk_sig[seq & 1] = use_sig;
            tseq = seq;
            HIP_TRY(hipEventRecord(ev_tail_done, ts));
            tail_in_flight = true;
            last_ts = ts;
        }
        period_runs = false;
        tin_idx ^= 1;  // the next period fills the other buffer while the tail reads this one
        tail_input_fill = 0;                                                   // :488-491
        precalculated_pos = 0;
        return FFTCONV_OK;
    }

    // TwoStageFFTConvolver::process (:412-495)
    int process_device(const float *din, size_t is, float *dout, size_t os, size_t len, hipStream_t s) {
        if (len > head_bs) return fail(FFTCONV_E_INVALID, "assertion failed: input.len() <= self.head_block_size");
        if (len == 0 || C == 0) return FFTCONV_OK;
        if (int r = resolve_pend(s)) return r;
        if (len == head_bs && tail_input_fill % head_bs == 0 && tail_input_fill + len <= T &&
            head->log2b <= kMaxLog2Fused) {
            // aligned call: one sub-chunk, and tail0 consumes exactly this block.
            // One launch: head (+ the sub-chunk epilogue) and tail0 as two jobs.
            ProcArgs a{};
            a.job[0] = head->job(din, is, dout, os, len);                       // :417
            a.job[0].add0 = tail_precalculated0 + precalculated_pos;            // :439-445
            a.job[0].add1 = tail_precalculated + precalculated_pos;             // :448-454
            a.job[0].add_stride = (long long)T;
            a.job[0].tin = tail_input() + tail_input_fill;                     // :459-461
            a.job[0].tin_stride = (long long)T;
            a.njobs = 1;
            const bool defer_block = tail0 && t0_defer;                        // :464-472, deferred
            if (tail0 && !defer_block) {                                        // :464-472
                a.job[1] = tail0->job(din, is, tail_output0 + tail_input_fill, T, head_bs);
                a.njobs = 2;
            }
            a.tw = head->tw.p;
            if (head->trace_slots && !head->la_W) {  // (FFTCONV_PROC_TRACE timelines)
                if (int r = head->trace_fill(a, s)) return r;
                ++head->la_t;
            }
            HIP_TRY(launch_process(head->log2b, a, (int)C, s));
            if (defer_block) {  // (counted once the head launch that writes its tail_input is enqueued)
                if (t0_n == 0) t0_off = tail_input_fill;
                ++t0_n;
            }
            precalculated_pos += len;
            tail_input_fill += len;
            if (tail_input_fill == T) {
                if (int r = end_of_period(s)) return r;
            }
            return FFTCONV_OK;
        }
        if (int r = flush_t0(s)) return r;  // (the sub-chunk loop runs tail0 per block)
        if (int r = head->process_device(din, is, dout, os, len, s)) return r;   // :417
        size_t processed = 0;
        while (processed < len) {                                                 // :427
            const size_t processing = std::min(len - processed, head_bs - (tail_input_fill % head_bs));
            if (tail_input_fill + processing > T)  // tail_input[fill..fill+processing] out of range (:459-460)
                return fail(FFTCONV_E_INVALID, "range end index out of range for slice of length tail_block_size");
            TwoStageAccumArgs a{};
            a.out = dout; a.out_stride = (long long)os;
            a.p0 = tail_precalculated0; a.p1 = tail_precalculated; a.T = (long long)T;
            a.pos = (int)precalculated_pos; a.in = din; a.in_stride = (long long)is;
            a.sb = (int)processed; a.tail_input = tail_input(); a.fill = (int)tail_input_fill;
            a.cnt = (int)processing;
            HIP_TRY(launch_twostage_accum(a, (int)C, s));                        // :438-461
            precalculated_pos += processing;
            tail_input_fill += processing;
            if (tail_input_fill % head_bs == 0 && tail0) {                        // :464-472
                const size_t off = tail_input_fill - head_bs;
                if (int r = tail0->process_device(tail_input() + off, T, tail_output0 + off, T, head_bs, s)) return r;
            }
            if (tail_input_fill == T) {
                if (int r = end_of_period(s)) return r;
            }
            processed += processing;
        }
        return FFTCONV_OK;
    }

    // `steps` consecutive process() calls (fftconv_twostage_process_device_steps).
    // Aligned head-block calls inside one tail period, with tail0 deferred,
    // run as ONE launch (upols_run_kernel: each channel loops over the calls,
    // process_job per call -- the same bits as one launch per call); the
    // period's end and every other call shape go through process_device.
    int process_device_steps(const float *din, size_t is, size_t in_step, float *dout, size_t os, size_t out_step,
                             size_t len, size_t steps, hipStream_t s) {
        size_t k = 0;
        while (k < steps) {
            const bool aligned = len == head_bs && tail_input_fill % head_bs == 0 && tail_input_fill + len <= T &&
                                 head->log2b <= kMaxLog2Fused;
            const size_t left = aligned ? (T - tail_input_fill) / head_bs : 0;
            const size_t nrun = std::min(steps - k, left);
            if (aligned && nrun >= (size_t)run_min && t0_defer && tail0 && run_supported(head->log2b) &&
                nrun <= (size_t)INT32_MAX && in_step <= (size_t)LLONG_MAX && out_step <= (size_t)LLONG_MAX) {
                ProcArgs a{};
                a.job[0] = head->job(din + k * in_step, is, dout + k * out_step, os, len);  // :417
                a.job[0].add0 = tail_precalculated0 + precalculated_pos;                // :439-445
                a.job[0].add1 = tail_precalculated + precalculated_pos;                 // :448-454
                a.job[0].add_stride = (long long)T;
                a.job[0].tin = tail_input() + tail_input_fill;                         // :459-461
                a.job[0].tin_stride = (long long)T;
                a.njobs = 1;
                a.tw = head->tw.p;
                // the run's block spectra double as tail0's pending-block
                // spectra while every pending block so far has one
                const bool t0spec = t0_have == t0_n && t0_n + nrun <= t0_nmax;
                if (t0spec) {
                    a.job[0].t0x = t0_xs.p + t0_n * head_bs;
                    a.job[0].t0x_stride = (long long)(t0_nmax * head_bs);
                    a.job[0].t0m = t0_miss.p;  // (a call that cannot write its spectrum flags the channel)
                }
                a.prio = run_prio;
                a.run_lds_rows = run_lds_rows(head->log2b, (int)head->S);
                if (pend && tk_sig[pend & 1]) {  // (the run waits for the tail on the device)
                    a.sig = tsig.p;
                    a.sig_val = pend;
                    a.sig_mode = 2;
                    pend = 0;
                } else if (int r = resolve_pend(s)) {
                    return r;
                }
                if (head->trace_slots) {  // (FFTCONV_PROC_TRACE: the run's last call, per wave)
                    if (int r = head->trace_fill(a, s)) return r;
                    ++head->la_t;
                }
                RunSteps r{(long long)in_step, (long long)out_step, (int)nrun};
                HIP_TRY(launch_process_run(head->log2b, a, r, (int)C, s));
                period_runs = true;
                if (t0_n == 0) t0_off = tail_input_fill;  // :464-472, deferred
                t0_n += nrun;
                if (t0spec) t0_have += nrun;
                precalculated_pos += nrun * len;
                tail_input_fill += nrun * len;
                k += nrun;
                // a run that ends the period ends it as a per-call aligned call does
                if (tail_input_fill == T) {
                    if (int r = end_of_period(s)) return r;
                }
                continue;
            }
            if (int r = process_device(din + k * in_step, is, dout + k * out_step, os, len, s)) return r;
            ++k;
        }
        return FFTCONV_OK;
    }

    int process_host(const float *in, float *out, size_t len) {
        if (len > head_bs) return fail(FFTCONV_E_INVALID, "assertion failed: input.len() <= self.head_block_size");
        if (len == 0 || C == 0) return FFTCONV_OK;
        DeviceGuard g(device);
        if (int r = order.enter(stream)) return r;
        if (int r = scratch.ensure(C * len, C * len)) return r;
        HIP_TRY(hipMemcpyAsync(scratch.in.p, in, C * len * sizeof(float), hipMemcpyHostToDevice, stream));
        if (int r = process_device(scratch.in.p, len, scratch.out.p, len, len, stream)) return r;
        HIP_TRY(hipMemcpyAsync(out, scratch.out.p, C * len * sizeof(float), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    int reset() {  // :497-511
        DeviceGuard g(device);
        if (int r = quiesce()) return r;
        if (int r = head->reset(stream)) return r;
        if (tail0) { if (int r = tail0->reset(stream)) return r; }
        if (tail) { if (int r = tail->reset(stream)) return r; }
        for (auto *b : {&out0, &pre0, &out1, &pre1, &tin_buf[0], &tin_buf[1]})
            if (b->n) HIP_TRY(hipMemsetAsync(b->p, 0, b->bytes(), stream));
        tail_input_fill = 0;
        precalculated_pos = 0;
        tail_in_flight = false;
        pend = 0;  // (quiesce waited for every tail)
        t0_n = t0_have = 0;  // (the deferred blocks' state is reset with everything else)
        if (t0_miss.n) HIP_TRY(hipMemsetAsync(t0_miss.p, 0, t0_miss.bytes(), stream));
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    int clone_from(const TwoStageCore &o) {
        DeviceGuard g(o.device);
        if (int r = o.quiesce()) return r;
        if (o.t0_n) {  // the source's deferred tail0 blocks first: the copy starts with none
            if (int r = o.flush_t0(o.stream)) return r;
            HIP_TRY(hipStreamSynchronize(o.stream));
        }
        device = o.device; C = o.C; head_bs = o.head_bs; T = o.T;
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        auto cl = [&](std::unique_ptr<UniformCore> &dst, const std::unique_ptr<UniformCore> &src) -> int {
            if (!src) return FFTCONV_OK;
            dst.reset(new (std::nothrow) UniformCore());
            if (!dst) return fail(FFTCONV_E_NOMEM, "out of host memory");
            dst->parent_stream = stream;
            return dst->clone_from(*src);
        };
        if (int r = cl(head, o.head)) return r;
        if (int r = cl(tail0, o.tail0)) return r;
        if (int r = cl(tail, o.tail)) return r;
        if (int r = alloc_buffers()) return r;
        auto map = [&](const float *p) -> float * {  // same role, this instance's buffer
            if (p == o.out0.p) return out0.p;
            if (p == o.pre0.p) return pre0.p;
            if (p == o.out1.p) return out1.p;
            return pre1.p;
        };
        tail_output0 = map(o.tail_output0); tail_precalculated0 = map(o.tail_precalculated0);
        tail_output = map(o.tail_output); tail_precalculated = map(o.tail_precalculated);
        tin_idx = o.tin_idx;
        const std::pair<DevPtr<float> *, const DevPtr<float> *> pairs[] = {
            {&out0, &o.out0}, {&pre0, &o.pre0}, {&out1, &o.out1}, {&pre1, &o.pre1},
            {&tin_buf[0], &o.tin_buf[0]}, {&tin_buf[1], &o.tin_buf[1]}};
        for (auto &pr : pairs)
            if (pr.second->n)
                HIP_TRY(hipMemcpyAsync(pr.first->p, pr.second->p, pr.second->bytes(), hipMemcpyDeviceToDevice, stream));
        tail_input_fill = o.tail_input_fill;
        precalculated_pos = o.precalculated_pos;
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }
};

// ---------------------------------------------------------------------------
// Crossfader<RaisedCosineMixer> host state (src/crossfade_convolver.rs:192-279);
// the per-sample gains are evaluated on the device by crossfade_mix_kernel.
// ---------------------------------------------------------------------------
struct Crossfader {
    int64_t fading_samples = 0, hold_samples = 0, counter = 0;
    float mix_value_step = 0.f, mix_value = 0.f;
    bool approaching = false;
    int target = 0;  // 0 = A, 1 = B

    void init(size_t fading, size_t hold) {  // :204-214
        fading_samples = (int64_t)fading;
        hold_samples = (int64_t)hold;
        counter = 0;
        mix_value_step = 1.0f / (float)fading;
        mix_value = 0.f;
        approaching = false;
        target = 0;
    }
    void fade_into(int t) {  // :216-240
        if (target == t) return;
        if (!approaching) {
            counter = -hold_samples;
            approaching = true;
            target = t;
            mix_value_step = -mix_value_step;
        } else if (counter >= 0) {
            counter = fading_samples - counter;
            target = t;
            mix_value_step = -mix_value_step;
        } else {
            approaching = false;
            target = t;
        }
    }
    // advance the state machine over n samples exactly as n calls of mix() (:242-278)
    void advance(size_t n) {
        for (size_t i = 0; i < n && approaching; ++i) {
            counter += 1;
            if (counter <= 0) continue;
            volatile float v = mix_value + mix_value_step;  // one f32 rounding per step
            mix_value = v;
            if (counter == fading_samples) {
                approaching = false;
                mix_value = target == 0 ? 0.0f : 1.0f;
            }
        }
    }
};

// ---------------------------------------------------------------------------
// CrossfadeCore -- CrossfadeConvolver<FFTConvolver> (src/crossfade_convolver.rs:3-105)
// ---------------------------------------------------------------------------
struct CrossfadeCore {
    int device = 0;
    size_t C = 0, max_buffer_size = 0, stored_len = 0, stored_stride = 0;
    size_t stage_row = 0;  // hstage row: the stored response, or a direct update of a / b
    std::unique_ptr<UniformCore> a, b;
    Crossfader xf;
    DevPtr<float> buf_a, buf_b, stored;
    DevPtr<float> mix_tab;  // [max_buffer_size + 1] mix_value walk (lookahead-fused mix)
    bool response_pending = false;
    hipStream_t stream = nullptr;
    Scratch scratch;
    // crossfade pair launch (one FDL stream for A and B): allowed while A and B
    // have had the same active_seg_count at every call; act[] as far as the
    // host knows (-1: channels differ), sticky off once they disagree
    long long act[2] = {-1, -1};
    bool pair_ok = false;
    // A's launch of a fused crossfade step ran but B's failed: A is a block
    // ahead of B and the crossfader did not advance.  Every later call fails
    // instead of silently mixing convolvers that are out of step.
    bool poisoned = false;
    mutable StreamOrder order;
    PinnedStage hstage;  // host responses for the pending path (stored_response)
    // CrossfadeConvolver<TwoStageFFTConvolver> (the reference is generic over
    // Convolution, :11,45-49): convolver_a only.  B starts as A's clone and is
    // never switched to: every swap (:94-105) reaches TwoStageFFTConvolver::
    // update, todo!() (src/fft_convolver.rs:408-410), before fade_into, so the
    // crossfader stays Reached(A) and mix() returns A's sample (:244-247).  B
    // would run the same work on the same state and is never observable.
    std::unique_ptr<TwoStageCore> ts;
    int check_poisoned() const {
        return poisoned ? fail(FFTCONV_E_DEVICE, "crossfade handle unusable: an earlier process() failed between "
                                                  "its two convolvers' launches")
                        : FFTCONV_OK;
    }

    ~CrossfadeCore() {
        if (stream) {
            DeviceGuard g(device);
            (void)order.drain(stream);
            a.reset(); b.reset();  // (they borrow `stream`)
            (void)hipStreamDestroy(stream);
        }
    }

    // CrossfadeConvolver::new (:19-43)
    int init_new(const UniformCore &conv, size_t max_response_length, size_t mbs, size_t crossfade_samples) {
        device = conv.device;
        C = conv.C;
        DeviceGuard g(device);
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        a.reset(new (std::nothrow) UniformCore());
        b.reset(new (std::nothrow) UniformCore());
        if (!a || !b) return fail(FFTCONV_E_NOMEM, "out of host memory");
        a->parent_stream = b->parent_stream = stream;
        if (int r = a->clone_from(conv, false)) return r;  // (update() stages through hstage below)
        if (int r = b->clone_from(conv, false)) return r;
        // A and B start as copies: equal FDLs (FLAG_XSYNC), and one
        // active_seg_count if every channel of `conv` has the same
        if (C) {
            std::vector<int4> st(C);
            HIP_TRY(hipMemcpy(st.data(), a->state.p, C * sizeof(int4), hipMemcpyDeviceToHost));
            bool uniform = true;
            for (size_t c = 1; c < C; ++c) uniform = uniform && st[c].y == st[0].y;
            act[0] = act[1] = uniform ? st[0].y : -1;
            pair_ok = uniform && pair_supported(a->log2b, (int)a->S);
            HIP_TRY(launch_state_flags(a->state.p, (int)C, FLAG_XSYNC, 0, stream));
            HIP_TRY(launch_state_flags(b->state.p, (int)C, FLAG_XSYNC, 0, stream));
            a->view_ok = b->view_ok = false;
        }
        stored_len = max_response_length;
        stored_stride = stored_len;
        if (int r = stored.alloc(C * stored_len)) return r;
        if (stored.n) HIP_TRY(hipMemsetAsync(stored.p, 0, stored.bytes(), stream));
        stage_row = std::max(stored_len, a->ir_len);
        if (int r = hstage.alloc(C * stage_row, stage_row)) return r;
        xf.init(crossfade_samples, std::min(mbs, max_response_length));
        max_buffer_size = mbs;
        if (int r = buf_a.alloc(C * mbs)) return r;
        if (int r = buf_b.alloc(C * mbs)) return r;
        if (int r = mix_tab.alloc(mbs + 1)) return r;
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    // CrossfadeConvolver::<TwoStageFFTConvolver>::new (:19-43), taking
    // ownership of the (already cloned / freshly initialised) inner convolver
    int init_new_ts(std::unique_ptr<TwoStageCore> inner, size_t max_response_length, size_t mbs,
                    size_t crossfade_samples) {
        device = inner->device;
        C = inner->C;
        DeviceGuard g(device);
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        ts = std::move(inner);
        stored_len = max_response_length;  // (stored_response is never written: no swap can start)
        stored_stride = stored_len;
        xf.init(crossfade_samples, std::min(mbs, max_response_length));
        max_buffer_size = mbs;
        return buf_a.alloc(C * mbs);
    }

    int ts_update_unimplemented() const {
        return fail(FFTCONV_E_UNIMPLEMENTED, "not yet implemented (the swap calls TwoStageFFTConvolver::update, "
                                             "which is todo!())");
    }

    // :66-78 over a TwoStageFFTConvolver: convolver_a.process(input, buffer_a)
    // on max_buffer_size samples, then mix() = A's samples (Reached(A))
    int process_ts(const float *din, size_t is, float *dout, size_t os, size_t out_len, hipStream_t s) {
        const size_t m = max_buffer_size;
        if (m > ts->head_bs) return fail(FFTCONV_E_INVALID, "assertion failed: input.len() <= self.head_block_size");
        if (m == 0 || C == 0) return FFTCONV_OK;
        const bool direct = out_len == m;
        if (int r = ts->process_device(din, is, direct ? dout : buf_a.p, direct ? os : m, m, s)) return r;
        if (!direct && out_len)
            HIP_TRY(hipMemcpy2DAsync(dout, os * sizeof(float), buf_a.p, m * sizeof(float), out_len * sizeof(float), C,
                                     hipMemcpyDeviceToDevice, s));
        xf.advance(out_len);
        return FFTCONV_OK;
    }

    // every piece of the handle's work has finished (incl. a TwoStage inner's
    // tail convolution on its side stream)
    int quiesce() const {
        if (int r = order.drain(stream)) return r;
        return ts ? ts->quiesce() : FFTCONV_OK;
    }

    bool is_crossfading() const { return xf.approaching; }  // :85-92

    // swap (:94-105) from device samples
    int swap_device(const float *src, size_t stride, size_t len, hipStream_t s) {
        if (xf.target == 0) {
            if (int r = b->update_device(src, stride, len, s)) return r;
            note_update(1, len);
            xf.fade_into(1);
        } else {
            if (int r = a->update_device(src, stride, len, s)) return r;
            note_update(0, len);
            xf.fade_into(0);
        }
        return FFTCONV_OK;
    }

    // FFTConvolver::update sets active_seg_count = ceil(len / B) on every
    // channel (:185-190), unless the convolver is empty (:181-183)
    void note_update(int which, size_t len) {
        const UniformCore &u = which ? *b : *a;
        if (u.ir_len == 0) return;
        act[which] = (long long)ceil_div(len, u.B);
        if (act[0] < 0 || act[0] != act[1]) pair_ok = false;
    }

    // Convolution::update (:51-64); host samples, channel c at src + c*stride
    // (stride 0 = shared).  Asynchronous like FFTConvolver's: the response is
    // staged in pinned memory and the work enqueued behind the handle's.
    int update_host(const float *src, size_t len, size_t stride) {
        if (int r = check_poisoned()) return r;
        if (ts) return ts_update_unimplemented();
        DeviceGuard g(device);
        if (int r = order.enter(stream)) return r;
        if (!is_crossfading()) {
            UniformCore &t = xf.target == 0 ? *b : *a;
            if (len > t.ir_len) return fail(FFTCONV_E_INVALID, "New impulse response is longer than initialized length");
            if (int r = t.update_host_on(0, C, src, len, stride, stream, hstage)) return r;
            note_update(xf.target == 0 ? 1 : 0, len);
            xf.fade_into(xf.target == 0 ? 1 : 0);
            response_pending = false;
            return FFTCONV_OK;
        }
        if (len > stored_len) return fail(FFTCONV_E_INVALID, "assertion failed: response_len <= self.stored_response.len()");
        // stored_response[..len] = response; stored_response[len..] = 0
        if (stored.n) HIP_TRY(hipMemsetAsync(stored.p, 0, stored.bytes(), stream));
        if (len) {
            const bool shared = stride == 0 || C == 1;
            if (int r = hstage.upload(src, shared ? 1 : C, len, stride, stored.p, stored_len, stream)) return r;
            stored_stride = shared ? (C == 1 ? stored_len : 0) : stored_len;
        }
        response_pending = true;
        return FFTCONV_OK;
    }

    // Convolution::update (:51-64) from device samples, stream-ordered
    int update_device(const float *src, size_t len, size_t stride, hipStream_t s) {
        if (int r = check_poisoned()) return r;
        if (ts) return ts_update_unimplemented();
        if (!is_crossfading()) {
            UniformCore &t = xf.target == 0 ? *b : *a;
            if (len > t.ir_len) return fail(FFTCONV_E_INVALID, "New impulse response is longer than initialized length");
            if (int r = swap_device(src, stride, len, s)) return r;
            response_pending = false;
            return FFTCONV_OK;
        }
        if (len > stored_len) return fail(FFTCONV_E_INVALID, "assertion failed: response_len <= self.stored_response.len()");
        if (stored.n) HIP_TRY(hipMemsetAsync(stored.p, 0, stored.bytes(), s));
        if (len) {
            if (stride == 0 || C == 1) {
                HIP_TRY(hipMemcpyAsync(stored.p, src, len * sizeof(float), hipMemcpyDeviceToDevice, s));
                stored_stride = C == 1 ? stored_len : 0;
            } else {
                HIP_TRY(hipMemcpy2DAsync(stored.p, stored_len * sizeof(float), src, stride * sizeof(float),
                                         len * sizeof(float), C, hipMemcpyDeviceToDevice, s));
                stored_stride = stored_len;
            }
        }
        response_pending = true;
        return FFTCONV_OK;
    }

    CrossfadeMixArgs mix_args(float *dout, size_t os, size_t out_len) const {
        CrossfadeMixArgs x{};
        x.buf_a = buf_a.p; x.buf_b = buf_b.p; x.buf_stride = (long long)max_buffer_size;
        x.out = dout; x.out_stride = (long long)os; x.n = (int)out_len;
        x.approaching = xf.approaching ? 1 : 0; x.target = xf.target;
        x.counter0 = xf.counter; x.fading = xf.fading_samples;
        x.mix_value0 = xf.mix_value; x.step = xf.mix_value_step;
        return x;
    }

    // Convolution::process (:66-78)
    int process_device(const float *din, size_t is, float *dout, size_t os, size_t out_len, hipStream_t s) {
        if (int r = check_poisoned()) return r;
        if (out_len > max_buffer_size) return fail(FFTCONV_E_INVALID, "output longer than max_buffer_size (index out of bounds)");
        if (ts) return process_ts(din, is, dout, os, out_len, s);
        if (!is_crossfading() && response_pending) {                    // :67-70
            if (int r = swap_device(stored.p, stored_stride, stored_len, s)) return r;
            response_pending = false;
        }
        const size_t m = max_buffer_size;
        if (m > (size_t)INT32_MAX) return fail(FFTCONV_E_UNSUPPORTED, "process length exceeds 2^31-1");
        if (m > 0 && C > 0 && m == a->B && a->la_W && b->la_W && la_parts(a->log2b, (int)a->S) == a->la_W &&
            la_parts(b->log2b, (int)b->S) == b->la_W) {
            // :72-73 on the lookahead step: each convolver's full
            // block runs its own launch of far / mid anchors and steps; then
            // the mix (:75-77)
            if (out_len == m && la_fuse_mix_allowed() && a->la_t == b->la_t && a->la_seq == b->la_seq &&
                a->la_all == b->la_all) {
                // :72-77 in ONE launch: A's and B's anchors, and per channel
                // one workgroup running A's and B's step (two chain waves)
                // that mixes the two blocks in LDS -- A's and B's clocks
                // agree (they step together), so one stagger serves both
                ProcArgs pa{};
                if (int r = a->la_job(pa.job[0], din, is, dout, os, m, s)) return r;
                if (int r = b->la_job(pa.job[1], din, is, nullptr, 0, m, s)) return r;
                pa.tw = a->tw.p;
                pa.njobs = 2;
                if (int r = a->la_fill(pa, s)) return r;
                pa.laW2 = b->laW.p;
                pa.la_mix = 3;
                pa.mix = mix_args(dout, os, out_len);  // (buf_a / buf_b: the generic-step fallback)
                HIP_TRY(launch_process_la(a->log2b, pa, (int)C, s));
                a->la_advance();
                b->la_advance();
                xf.advance(out_len);
                return FFTCONV_OK;
            }
            if (out_len == m && la_fuse_mix_allowed()) {
                // the mix fused into B's launch: A's launch walks mix_value
                // once into mix_tab, B's epilogue mixes A's block (buf_a) with
                // its own straight into the output -- no mix launch, no buf_b
                const CrossfadeMixArgs mx = mix_args(dout, os, out_len);
                if (int r = a->process_device(din, is, buf_a.p, m, m, s, 1, &mx, mix_tab.p)) return r;
                if (int r = b->process_device(din, is, dout, os, m, s, 2, &mx, mix_tab.p)) {
                    poisoned = true;
                    return r;
                }
                xf.advance(out_len);
                return FFTCONV_OK;
            }
            if (int r = a->process_device(din, is, buf_a.p, m, m, s)) return r;
            if (int r = b->process_device(din, is, buf_b.p, m, m, s)) {
                poisoned = true;
                return r;
            }
            if (int r = launch_mix(dout, os, out_len, s)) return r;
            xf.advance(out_len);
            return FFTCONV_OK;
        }
        if (m > 0 && C > 0) {
            // :72-73 -- A and B are two jobs of ONE launch (same block size):
            // 2C workgroups fill the chip where C alone leaves it half occupied
            ProcArgs pa{};
            pa.job[0] = a->job(din, is, buf_a.p, m, m);
            pa.job[1] = b->job(din, is, buf_b.p, m, m);
            pa.njobs = 2;
            pa.tw = a->tw.p;
            // while A's and B's rings agree: one workgroup per channel reads
            // the FDL once for both (bit-identical to the two-job launch)
            pa.mix = mix_args(dout, os, out_len);
            if (pair_ok && pair_supported(a->log2b, (int)a->S) && m == a->B && out_len > 0) {
                // :72-77 in one launch: A, B and the mix (no buf_a / buf_b round trip)
                pa.fuse_mix = 1;
                HIP_TRY(launch_process_pair(a->log2b, pa, (int)C, s));
                xf.advance(out_len);
                return FFTCONV_OK;
            }
            a->lg_fill(pa, m);
            b->lg_fill(pa, m);
            HIP_TRY(launch_process(a->log2b, pa, (int)C, s));
        }
        if (int r = launch_mix(dout, os, out_len, s)) return r;  // :75-77
        xf.advance(out_len);
        return FFTCONV_OK;
    }

    // the stand-alone mix (:75-77); a call longer than the mix kernel's LDS
    // walk first walks mix_value once into mix_tab
    int launch_mix(float *dout, size_t os, size_t out_len, hipStream_t s) {
        CrossfadeMixArgs x = mix_args(dout, os, out_len);
        if (out_len > 1024 && x.approaching) {
            HIP_TRY(launch_crossfade_walk(x, mix_tab.p, s));
            x.vtab = mix_tab.p;
        }
        HIP_TRY(launch_crossfade_mix(x, (int)C, s));
        return FFTCONV_OK;
    }

    int process_host(const float *in, size_t in_len, float *out, size_t out_len) {
        if (in_len < max_buffer_size) return fail(FFTCONV_E_INVALID, "input shorter than max_buffer_size (range end index out of range)");
        if (ts && in_len > max_buffer_size)  // TwoStage: assert (:414), then output[i] past buffer_a (:441)
            return fail(FFTCONV_E_INVALID, in_len > ts->head_bs ? "assertion failed: input.len() <= self.head_block_size"
                                                                : "index out of bounds (input longer than max_buffer_size)");
        if (out_len > max_buffer_size) return fail(FFTCONV_E_INVALID, "output longer than max_buffer_size (index out of bounds)");
        if (C == 0) return FFTCONV_OK;
        DeviceGuard g(device);
        if (int r = order.enter(stream)) return r;
        const size_t m = max_buffer_size;
        if (int r = scratch.ensure(C * m, C * std::max<size_t>(out_len, 1))) return r;
        if (m)
            HIP_TRY(hipMemcpy2DAsync(scratch.in.p, m * sizeof(float), in, in_len * sizeof(float), m * sizeof(float), C,
                                     hipMemcpyHostToDevice, stream));
        if (int r = process_device(scratch.in.p, m, scratch.out.p, std::max<size_t>(out_len, 1), out_len, stream)) return r;
        if (out_len)
            HIP_TRY(hipMemcpy2DAsync(out, out_len * sizeof(float), scratch.out.p, out_len * sizeof(float),
                                     out_len * sizeof(float), C, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }

    int clone_from(const CrossfadeCore &o) {
        DeviceGuard g(o.device);
        if (int r = o.order.drain(o.stream)) return r;
        device = o.device; C = o.C; max_buffer_size = o.max_buffer_size;
        stored_len = o.stored_len; stored_stride = o.stored_stride;
        xf = o.xf; response_pending = o.response_pending;
        act[0] = o.act[0]; act[1] = o.act[1]; pair_ok = o.pair_ok; poisoned = o.poisoned;
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        if (o.ts) {
            ts.reset(new (std::nothrow) TwoStageCore());
            if (!ts) return fail(FFTCONV_E_NOMEM, "out of host memory");
            if (int r = ts->clone_from(*o.ts)) return r;
            return buf_a.alloc(o.buf_a.n);
        }
        a.reset(new (std::nothrow) UniformCore());
        b.reset(new (std::nothrow) UniformCore());
        if (!a || !b) return fail(FFTCONV_E_NOMEM, "out of host memory");
        a->parent_stream = b->parent_stream = stream;
        if (int r = a->clone_from(*o.a)) return r;
        if (int r = b->clone_from(*o.b)) return r;
        if (int r = buf_a.alloc(o.buf_a.n)) return r;
        if (int r = buf_b.alloc(o.buf_b.n)) return r;
        if (int r = mix_tab.alloc(o.mix_tab.n)) return r;
        if (int r = stored.alloc(o.stored.n)) return r;
        stage_row = o.stage_row;
        if (int r = hstage.alloc(o.hstage.n, stage_row)) return r;
        if (stored.n) HIP_TRY(hipMemcpyAsync(stored.p, o.stored.p, stored.bytes(), hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        return FFTCONV_OK;
    }
};

// W_N^k tables of the stand-alone Fft entry points, one per (device, N),
// built on first use in f64 and kept for the process (the handles keep
// their own); the same values as every handle's table for that N.  The first
// use uploads on the caller's stream and waits for that stream only (no
// legacy-stream synchronisation).
int fft_twiddles(int dev, int log2n, hipStream_t s, const float2 **out) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, float2 *> tabs;
    std::lock_guard<std::mutex> lk(mu);
    auto it = tabs.find({dev, log2n});
    if (it != tabs.end()) {
        *out = it->second;
        return FFTCONV_OK;
    }
    const size_t N = (size_t)1 << log2n;
    std::vector<float2> t(N);
    for (size_t k = 0; k < N; ++k) {
        const double ang = -2.0 * M_PI * (double)k / (double)N;
        t[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
    }
    float2 *p = nullptr;
    HIP_TRY(hipMalloc((void **)&p, N * sizeof(float2)));
    hipError_t e = hipMemcpyAsync(p, t.data(), N * sizeof(float2), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // (t is freed on return)
    if (e != hipSuccess) {
        (void)hipFree(p);
        return fail(FFTCONV_E_DEVICE, std::string("twiddle upload: ") + hipGetErrorString(e));
    }
    tabs[{dev, log2n}] = p;
    *out = p;
    return FFTCONV_OK;
}

// The long-block path's tables for M = 2^log2m (lg_split: M = M1 x M2), one
// set per (device, M), built in f64 and rounded to f32 like every other
// table: W_M^j (j < M), W_{2 M1}^i (i < 2 M1), W_{2 M2}^i (i < 2 M2).  The
// caller sets twN (its W_N table).  Synchronous upload on first use.
int lg_tables(int dev, int log2m, LgTab *out) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, float2 *> tabs;
    std::lock_guard<std::mutex> lk(mu);
    int l1 = 0, l2 = 0;
    lg_split(log2m, &l1, &l2);
    const size_t M = (size_t)1 << log2m, A = (size_t)2 << l1, Bt = (size_t)2 << l2;
    auto it = tabs.find({dev, log2m});
    float2 *p = nullptr;
    if (it != tabs.end()) {
        p = it->second;
    } else {
        std::vector<float2> t(M + A + Bt);
        auto fill = [&](float2 *dst, size_t n, size_t period) {
            for (size_t k = 0; k < n; ++k) {
                const double ang = -2.0 * M_PI * (double)k / (double)period;
                dst[k] = make_float2((float)std::cos(ang), (float)std::sin(ang));
            }
        };
        fill(t.data(), M, M);
        fill(t.data() + M, A, A);
        fill(t.data() + M + A, Bt, Bt);
        HIP_TRY(hipMalloc((void **)&p, t.size() * sizeof(float2)));
        hipError_t e = hipMemcpy(p, t.data(), t.size() * sizeof(float2), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return fail(FFTCONV_E_DEVICE, std::string("twiddle upload: ") + hipGetErrorString(e));
        }
        tabs[{dev, log2m}] = p;
    }
    out->twN = nullptr;
    out->twM = p;
    out->twA = p + M;
    out->twB = p + M + A;
    return FFTCONV_OK;
}

// Bluestein tables of a length n that is not a power of two (the public Fft
// of any length, launch_fft_bluestein): the chirp w_m = exp(i pi m^2 / n)
// (m^2 mod 2n in integers, the angle in f64) and the spectrum of the chirp
// filter b (b_m = b_{P-m} = w_m, m < n) by an f64 FFT on the host, both
// rounded to f32 once; the filter in the device FFT's bin order.  One set per
// (device, n) in a cache of at most kBluesteinCacheBytes of device memory:
// the least recently used sets are freed when a new length would pass it.
// The caller holds bluestein_mutex() from this lookup until its kernels are
// enqueued, so a set being freed was last used by work already on a stream,
// and the eviction waits for that device before hipFree.  The first use of a
// length uploads on the caller's stream and waits for that stream only.
constexpr size_t kMaxBluestein = (size_t)1 << 21;  // P = 2^22 at most
constexpr size_t kBluesteinCacheBytes = (size_t)256 << 20;
std::mutex &bluestein_mutex() {
    static std::mutex mu;
    return mu;
}
int bluestein_tables(int dev, size_t n, int log2p, hipStream_t s, const float2 **chirp, const float2 **filt) {
    struct Tab { float2 *p; size_t bytes; unsigned long long used; };
    static std::map<std::pair<int, size_t>, Tab> tabs;
    static size_t total = 0;
    static unsigned long long clock = 0;
    const size_t P = (size_t)1 << log2p;
    auto it = tabs.find({dev, n});
    if (it == tabs.end()) {
        const size_t bytes = (n + P) * sizeof(float2);
        while (!tabs.empty() && total + bytes > kBluesteinCacheBytes) {
            auto lru = tabs.begin();
            for (auto j = tabs.begin(); j != tabs.end(); ++j)
                if (j->second.used < lru->second.used) lru = j;
            DeviceGuard g(lru->first.first);
            (void)hipDeviceSynchronize();  // kernels enqueued with this set have finished
            (void)hipFree(lru->second.p);
            total -= lru->second.bytes;
            tabs.erase(lru);
        }
        std::vector<double> wr(n), wi(n);
        for (size_t m = 0; m < n; ++m) {
            const unsigned long long q = ((unsigned long long)m * m) % (2ull * n);
            const double ang = M_PI * (double)q / (double)n;
            wr[m] = std::cos(ang);
            wi[m] = std::sin(ang);
        }
        std::vector<double> br(P, 0.0), bi(P, 0.0);
        for (size_t m = 0; m < n; ++m) {
            br[m] = wr[m];
            bi[m] = wi[m];
            if (m) {
                br[P - m] = wr[m];
                bi[P - m] = wi[m];
            }
        }
        // forward DFT of b in f64: iterative radix-2, exp(-2 pi i / len) per stage
        for (size_t i = 1, j = 0; i < P; ++i) {
            size_t bit = P >> 1;
            for (; j & bit; bit >>= 1) j ^= bit;
            j ^= bit;
            if (i < j) {
                std::swap(br[i], br[j]);
                std::swap(bi[i], bi[j]);
            }
        }
        for (size_t len = 2; len <= P; len <<= 1) {
            const size_t h = len / 2;
            for (size_t k = 0; k < h; ++k) {
                const double ang = -2.0 * M_PI * (double)k / (double)len;
                const double c = std::cos(ang), sn = std::sin(ang);
                for (size_t b0 = 0; b0 < P; b0 += len) {
                    const size_t u = b0 + k, v = u + h;
                    const double tr = br[v] * c - bi[v] * sn, ti = br[v] * sn + bi[v] * c;
                    br[v] = br[u] - tr;
                    bi[v] = bi[u] - ti;
                    br[u] += tr;
                    bi[u] += ti;
                }
            }
        }
        std::vector<float2> t(n + P);
        for (size_t m = 0; m < n; ++m) t[m] = make_float2((float)wr[m], (float)wi[m]);
        for (size_t k = 0; k < P; ++k) {
            const size_t pos = log2p > kMaxLog2Fused ? lg_position(log2p, k) : k;
            t[n + pos] = make_float2((float)br[k], (float)bi[k]);
        }
        float2 *d = nullptr;
        HIP_TRY(hipMalloc((void **)&d, bytes));
        hipError_t e = hipMemcpyAsync(d, t.data(), bytes, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);  // (t is freed on return)
        if (e != hipSuccess) {
            (void)hipFree(d);
            return fail(FFTCONV_E_DEVICE, std::string("Bluestein tables: ") + hipGetErrorString(e));
        }
        it = tabs.emplace(std::make_pair(dev, n), Tab{d, bytes, 0}).first;
        total += bytes;
    }
    it->second.used = ++clock;
    *chirp = it->second.p;
    *filt = it->second.p + n;
    return FFTCONV_OK;
}

// Fft::forward / inverse on device rows (src/fft_convolver.rs:36-49)
int fft_rows(int device, size_t n, size_t rows, const float *din, size_t is, float *dout, size_t os, int *status,
             bool inverse, hipStream_t s) {
    if (int r = check_device(device)) return r;
    const bool pow2 = n >= 2 && !(n & (n - 1));
    if (n < 1 || (pow2 && n > ((size_t)2 << kMaxLog2Block)) || (!pow2 && n > kMaxBluestein))
        return fail(FFTCONV_E_UNSUPPORTED, "Fft length must be 1..2^21, or a power of two up to 2^23");
    const size_t nbf = 2 * (n / 2 + 1);  // floats of the n/2 + 1 interleaved bins
    const size_t cin = inverse ? nbf : n, cout = inverse ? n : nbf;
    if (rows > (size_t)INT32_MAX || (rows > 1 && (is < cin || os < cout)))
        return fail(FFTCONV_E_INVALID, "row strides shorter than a row");
    if (rows == 0) return FFTCONV_OK;
    DeviceGuard g(device);
    const float2 *tw = nullptr;
    if (pow2)
        if (int r = fft_twiddles(device, ilog2(n), s, &tw)) return r;
    FftArgs a{};
    a.in = din; a.in_stride = (long long)is; a.out = dout; a.out_stride = (long long)os; a.tw = tw; a.status = status;
    if (!pow2) {
        // any other length: Bluestein over P >= 2n - 1 point FFTs (large.hip)
        const size_t P = std::max<size_t>(2, next_pow2(2 * n - 1));
        const int lp = ilog2(P);
        const float2 *chirp = nullptr, *filt = nullptr, *twP = nullptr;
        std::lock_guard<std::mutex> lk(bluestein_mutex());  // until the kernels are enqueued
        if (int r = bluestein_tables(device, n, lp, s, &chirp, &filt)) return r;
        LgTab t{};
        float2 *scr = nullptr;
        size_t batch = rows;
        if (lp > kMaxLog2Fused) {
            if (int r = lg_tables(device, lp, &t)) return r;
            batch = std::max<size_t>(1, std::min(rows, ((size_t)64 << 20) / (P * sizeof(float2))));
            HIP_TRY(hipMallocAsync((void **)&scr, batch * P * sizeof(float2), s));
        } else {
            if (int r = fft_twiddles(device, lp + 1, s, &twP)) return r;  // W_{2P}
        }
        const hipError_t e = launch_fft_bluestein(n, lp, inverse, a, chirp, filt, twP, t, scr, (int)rows, (int)batch, s);
        if (scr) HIP_TRY(hipFreeAsync(scr, s));
        HIP_TRY(e);
        return FFTCONV_OK;
    }
    const int log2m = ilog2(n) - 1;
    if (log2m > kMaxLog2Fused) {
        // the long-block passes (large.hip) through a stream-ordered scratch
        // of up to 64 MiB of rows (the public Fft is not the real-time path)
        LgTab t{};
        if (int r = lg_tables(device, log2m, &t)) return r;
        t.twN = tw;
        const size_t m = n / 2;
        const size_t batch = std::max<size_t>(1, std::min(rows, ((size_t)64 << 20) / (m * sizeof(float2))));
        float2 *scr = nullptr;
        HIP_TRY(hipMallocAsync((void **)&scr, batch * m * sizeof(float2), s));
        const hipError_t e = launch_fft_large(log2m, inverse, a, t, scr, (int)rows, (int)batch, s);
        HIP_TRY(hipFreeAsync(scr, s));
        HIP_TRY(e);
        return FFTCONV_OK;
    }
    HIP_TRY(launch_fft_rows(log2m, inverse, a, (int)rows, s));
    return FFTCONV_OK;
}

// host-memory form: rows packed ([rows][n] reals, [rows][n + 2] bin floats),
// through temporary device buffers on a private stream; synchronous
int fft_rows_host(int device, size_t n, size_t rows, const float *in, float *out, int *status, bool inverse) {
    if (int r = check_device(device)) return r;
    if (rows == 0) return FFTCONV_OK;
    DeviceGuard g(device);
    const size_t nbf = 2 * (n / 2 + 1);
    const size_t cin = inverse ? nbf : n, cout = inverse ? n : nbf;
    DevPtr<float> din, dout;
    DevPtr<int> dst;
    if (int r = din.alloc(rows * cin)) return r;
    if (int r = dout.alloc(rows * cout)) return r;
    if (status) { if (int r = dst.alloc(rows)) return r; }
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct Del { hipStream_t s; ~Del() { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); } } del{s};
    HIP_TRY(hipMemcpyAsync(din.p, in, rows * cin * sizeof(float), hipMemcpyHostToDevice, s));
    if (int r = fft_rows(device, n, rows, din.p, cin, dout.p, cout, status ? dst.p : nullptr, inverse, s)) return r;
    HIP_TRY(hipMemcpyAsync(out, dout.p, rows * cout * sizeof(float), hipMemcpyDeviceToHost, s));
    if (status) HIP_TRY(hipMemcpyAsync(status, dst.p, rows * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFTCONV_OK;
}

template <class T>
T *make_or_null(int r, T *p) {
    if (r != FFTCONV_OK) {
        delete p;
        return nullptr;
    }
    return p;
}

// A caller's stream argument: NULL is HIP's null (legacy default) stream, as
// in every HIP API (fftconv.h "Streams"); StreamOrder orders it after the
// handle's own non-blocking streams, and nothing on it runs ahead of them.
hipStream_t pick(void *s, hipStream_t) { return (hipStream_t)s; }

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
struct fftconv_uniform { UniformCore core; };
struct fftconv_twostage { TwoStageCore core; };
struct fftconv_crossfade { CrossfadeCore core; };

extern "C" {

int fftconv_abi_version(void) { return FFTCONV_ABI_VERSION; }
const char *fftconv_last_error(void) { return g_last_error.c_str(); }
int fftconv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
size_t fftconv_complex_size(size_t size) { return size / 2 + 1; }

// ---- Fft (src/fft_convolver.rs:7-50) ---------------------------------------
int fftconv_fft_forward(int device, size_t n, size_t rows, const float *d_in, size_t in_stride, float *d_out,
                        size_t out_stride, void *hip_stream) {
    return fft_rows(device, n, rows, d_in, in_stride, d_out, out_stride, nullptr, false, (hipStream_t)hip_stream);
}
int fftconv_fft_inverse(int device, size_t n, size_t rows, const float *d_in, size_t in_stride, float *d_out,
                        size_t out_stride, int *d_status, void *hip_stream) {
    return fft_rows(device, n, rows, d_in, in_stride, d_out, out_stride, d_status, true, (hipStream_t)hip_stream);
}
int fftconv_fft_forward_host(int device, size_t n, size_t rows, const float *input, float *output) {
    return fft_rows_host(device, n, rows, input, output, nullptr, false);
}
int fftconv_fft_inverse_host(int device, size_t n, size_t rows, const float *input, float *output, int *status) {
    return fft_rows_host(device, n, rows, input, output, status, true);
}

// compute_tail_block_size, src/fft_convolver.rs:514-526, in f32 exactly as written
size_t fftconv_compute_tail_block_size(size_t head_len, size_t response_len) {
    const volatile float FFT_K = 1.5f;
    const volatile float ln2 = logf(2.0f);
    volatile float kn = (FFT_K * (float)head_len);
    kn = kn / (2.0f * ln2);
    volatile float kk = kn * kn;
    volatile float lh = (float)response_len * (float)head_len;
    volatile float sum = kk + lh;
    volatile float b = -kn + sqrtf(sum);
    const float h = (float)head_len;
    float bb = (b != b) ? h : (b > h ? b : h);
    size_t bi;
    if (!(bb > 0.0f)) bi = 0;
    else if (bb >= 18446744073709551615.0f) bi = SIZE_MAX;
    else bi = (size_t)bb;
    return next_pow2(bi);
}

int fftconv_set_kernel_variant(int variant) {
    if (variant > 4095 || variant < -1) return fail(FFTCONV_E_INVALID, "variant must be 0..4095 (or -1 = auto)");
    set_variant(variant);
    return FFTCONV_OK;
}
int fftconv_get_kernel_variant(void) { return get_variant(); }
int fftconv_set_pipeline_lag(int rows) {
    set_pipeline_lag(rows);
    return FFTCONV_OK;
}
int fftconv_get_pipeline_lag(void) { return get_pipeline_lag(); }
int fftconv_set_host_stage_limit(size_t bytes) {
    g_stage_limit.store(bytes, std::memory_order_relaxed);
    return FFTCONV_OK;
}
size_t fftconv_get_host_stage_limit(void) { return g_stage_limit.load(std::memory_order_relaxed); }

// ---- uniform --------------------------------------------------------------
fftconv_uniform *fftconv_uniform_init(const float *response, size_t response_len, size_t max_block_size,
                                      size_t max_response_length) {
    return fftconv_uniform_init_batch(0, 1, response, response_len, response_len, max_block_size,
                                      max_response_length);
}

fftconv_uniform *fftconv_uniform_init_batch(int device, size_t channels, const float *responses,
                                            size_t response_len, size_t response_stride, size_t max_block_size,
                                            size_t max_response_length) {
    set_error("");
    auto *h = new (std::nothrow) fftconv_uniform();
    if (!h) { set_error("out of host memory"); return nullptr; }
    h->core.la_ok = true;
    h->core.gw_ok = true;
    h->core.own_stage = true;
    int r = h->core.init(device, channels, responses, response_len, response_stride, max_block_size,
                         max_response_length);
    return make_or_null(r, h);
}

int fftconv_uniform_update(fftconv_uniform *h, const float *response, size_t len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.update_host(0, h->core.C, response, len, 0);
}
int fftconv_uniform_update_batch(fftconv_uniform *h, const float *responses, size_t len, size_t stride) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.update_host(0, h->core.C, responses, len, h->core.C == 1 ? 0 : stride);
}
int fftconv_uniform_update_channel(fftconv_uniform *h, size_t channel, const float *response, size_t len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    if (channel >= h->core.C) return fail(FFTCONV_E_INVALID, "channel out of range");
    return h->core.update_host(channel, 1, response, len, 0);
}
int fftconv_uniform_update_device(fftconv_uniform *h, const float *d_responses, size_t len, size_t stride,
                                  void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.update_device(d_responses, h->core.C == 1 ? 0 : stride, len, s);
}
int fftconv_uniform_reset(fftconv_uniform *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    if (int r = h->core.order.enter(h->core.stream)) return r;
    if (int r = h->core.reset(h->core.stream)) return r;
    HIP_TRY(hipStreamSynchronize(h->core.stream));
    return FFTCONV_OK;
}
int fftconv_uniform_process(fftconv_uniform *h, const float *input, size_t input_len, float *output,
                            size_t output_len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.process_host(input, input_len, output, output_len);
}
int fftconv_uniform_process_device(fftconv_uniform *h, const float *d_input, size_t in_stride, float *d_output,
                                   size_t out_stride, size_t len, void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.process_device(d_input, in_stride, d_output, out_stride, len, s);
}
int fftconv_uniform_process_device_steps(fftconv_uniform *h, const float *d_input, size_t in_stride, size_t in_step,
                                   float *d_output, size_t out_stride, size_t out_step, size_t len, size_t steps,
                                   void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.process_device_steps(d_input, in_stride, in_step, d_output, out_stride, out_step, len, steps, s);
}
fftconv_uniform *fftconv_uniform_clone(const fftconv_uniform *h) {
    if (!h) { set_error("null handle"); return nullptr; }
    auto *c = new (std::nothrow) fftconv_uniform();
    if (!c) { set_error("out of host memory"); return nullptr; }
    return make_or_null(c->core.clone_from(h->core), c);
}
void fftconv_uniform_destroy(fftconv_uniform *h) { delete h; }
int fftconv_uniform_synchronize(fftconv_uniform *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    return h->core.order.drain(h->core.stream);
}
size_t fftconv_uniform_channels(const fftconv_uniform *h) { return h ? h->core.C : 0; }
int fftconv_uniform_lookahead_parts(const fftconv_uniform *h) { return h ? h->core.la_W : 0; }
int fftconv_uniform_far_windows(const fftconv_uniform *h) { return h ? h->core.gw_p : 0; }
int fftconv_uniform_lookahead_probe(const fftconv_uniform *h) {
    if (!h || !h->core.la_probe.p) return -1;
    DeviceGuard g(h->core.device);
    if (h->core.order.drain(h->core.stream) != FFTCONV_OK) return -1;
    int n = 0;
    if (hipMemcpy(&n, h->core.la_probe.p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return n;
}
size_t fftconv_uniform_block_size(const fftconv_uniform *h) { return h ? h->core.B : 0; }
size_t fftconv_uniform_seg_count(const fftconv_uniform *h) { return h ? h->core.S : 0; }
int fftconv_uniform_ir_spectrum(const fftconv_uniform *h, size_t channel, size_t segment, float *out) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return const_cast<UniformCore &>(h->core).ir_spectrum(channel, segment, out);
}
int fftconv_uniform_channel_state(const fftconv_uniform *h, size_t channel, size_t out3[3]) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return const_cast<UniformCore &>(h->core).channel_state(channel, out3);
}

// ---- two-stage ------------------------------------------------------------
fftconv_twostage *fftconv_twostage_init(const float *response, size_t response_len, size_t max_block_size,
                                        size_t max_response_length) {
    return fftconv_twostage_init_batch(0, 1, response, response_len, response_len, max_block_size,
                                       max_response_length);
}
fftconv_twostage *fftconv_twostage_init_batch(int device, size_t channels, const float *responses,
                                              size_t response_len, size_t response_stride, size_t max_block_size,
                                              size_t max_response_length) {
    set_error("");
    auto *h = new (std::nothrow) fftconv_twostage();
    if (!h) { set_error("out of host memory"); return nullptr; }
    int r = h->core.init(device, channels, responses, response_len, channels == 1 ? response_len : response_stride,
                         max_block_size, max_response_length);
    return make_or_null(r, h);
}
int fftconv_twostage_update(fftconv_twostage *h, const float *, size_t) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return fail(FFTCONV_E_UNIMPLEMENTED, "not yet implemented (TwoStageFFTConvolver::update is todo!())");
}
int fftconv_twostage_reset(fftconv_twostage *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.reset();
}
int fftconv_twostage_process(fftconv_twostage *h, const float *input, float *output, size_t len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.process_host(input, output, len);
}
int fftconv_twostage_process_device(fftconv_twostage *h, const float *d_input, size_t in_stride, float *d_output,
                                    size_t out_stride, size_t len, void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.process_device(d_input, in_stride, d_output, out_stride, len, s);
}
int fftconv_twostage_process_device_steps(fftconv_twostage *h, const float *d_input, size_t in_stride, size_t in_step,
                                   float *d_output, size_t out_stride, size_t out_step, size_t len, size_t steps,
                                   void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.process_device_steps(d_input, in_stride, in_step, d_output, out_stride, out_step, len, steps, s);
}
fftconv_twostage *fftconv_twostage_clone(const fftconv_twostage *h) {
    if (!h) { set_error("null handle"); return nullptr; }
    auto *c = new (std::nothrow) fftconv_twostage();
    if (!c) { set_error("out of host memory"); return nullptr; }
    return make_or_null(c->core.clone_from(h->core), c);
}
void fftconv_twostage_destroy(fftconv_twostage *h) { delete h; }
int fftconv_twostage_synchronize(fftconv_twostage *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    return h->core.quiesce();
}
size_t fftconv_twostage_tail_block_size(const fftconv_twostage *h) { return h ? h->core.T : 0; }

// ---- crossfade ------------------------------------------------------------
fftconv_crossfade *fftconv_crossfade_init(const float *response, size_t response_len, size_t max_block_size,
                                          size_t max_response_length) {
    return fftconv_crossfade_init_batch(0, 1, response, response_len, response_len, max_block_size,
                                        max_response_length);
}
fftconv_crossfade *fftconv_crossfade_init_batch(int device, size_t channels, const float *responses,
                                                size_t response_len, size_t response_stride, size_t max_block_size,
                                                size_t max_response_length) {
    set_error("");
    fftconv_uniform *conv = fftconv_uniform_init_batch(device, channels, responses, response_len, response_stride,
                                                       max_block_size, max_response_length);
    if (!conv) return nullptr;
    // Convolution::init (src/crossfade_convolver.rs:46-49)
    fftconv_crossfade *h = fftconv_crossfade_new(conv, response_len, max_block_size, response_len);
    fftconv_uniform_destroy(conv);
    return h;
}
fftconv_crossfade *fftconv_crossfade_new(const fftconv_uniform *convolver, size_t max_response_length,
                                         size_t max_buffer_size, size_t crossfade_samples) {
    if (!convolver) { set_error("null handle"); return nullptr; }
    auto *h = new (std::nothrow) fftconv_crossfade();
    if (!h) { set_error("out of host memory"); return nullptr; }
    int r = h->core.init_new(convolver->core, max_response_length, max_buffer_size, crossfade_samples);
    return make_or_null(r, h);
}
// CrossfadeConvolver<TwoStageFFTConvolver>: init (:46-49) / new (:19-43)
fftconv_crossfade *fftconv_crossfade_init_twostage(const float *response, size_t response_len, size_t max_block_size,
                                                   size_t max_response_length) {
    return fftconv_crossfade_init_twostage_batch(0, 1, response, response_len, response_len, max_block_size,
                                                 max_response_length);
}
fftconv_crossfade *fftconv_crossfade_init_twostage_batch(int device, size_t channels, const float *responses,
                                                         size_t response_len, size_t response_stride,
                                                         size_t max_block_size, size_t max_response_length) {
    set_error("");
    std::unique_ptr<TwoStageCore> inner(new (std::nothrow) TwoStageCore());
    auto *h = new (std::nothrow) fftconv_crossfade();
    if (!inner || !h) { delete h; set_error("out of host memory"); return nullptr; }
    int r = inner->init(device, channels, responses, response_len, channels == 1 ? response_len : response_stride,
                        max_block_size, max_response_length);
    if (r == FFTCONV_OK) r = h->core.init_new_ts(std::move(inner), response_len, max_block_size, response_len);
    return make_or_null(r, h);
}
fftconv_crossfade *fftconv_crossfade_new_twostage(const fftconv_twostage *convolver, size_t max_response_length,
                                                  size_t max_buffer_size, size_t crossfade_samples) {
    if (!convolver) { set_error("null handle"); return nullptr; }
    std::unique_ptr<TwoStageCore> inner(new (std::nothrow) TwoStageCore());
    auto *h = new (std::nothrow) fftconv_crossfade();
    if (!inner || !h) { delete h; set_error("out of host memory"); return nullptr; }
    int r = inner->clone_from(convolver->core);
    if (r == FFTCONV_OK) r = h->core.init_new_ts(std::move(inner), max_response_length, max_buffer_size, crossfade_samples);
    return make_or_null(r, h);
}
int fftconv_crossfade_update(fftconv_crossfade *h, const float *response, size_t len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.update_host(response, len, 0);
}
int fftconv_crossfade_update_batch(fftconv_crossfade *h, const float *responses, size_t len, size_t stride) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.update_host(responses, len, h->core.C == 1 ? 0 : stride);
}
int fftconv_crossfade_update_device(fftconv_crossfade *h, const float *d_responses, size_t len, size_t stride,
                                    void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.update_device(d_responses, len, h->core.C == 1 ? 0 : stride, s);
}
int fftconv_crossfade_reset(fftconv_crossfade *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return fail(FFTCONV_E_UNIMPLEMENTED, "not yet implemented (CrossfadeConvolver::reset is todo!())");
}
int fftconv_crossfade_process(fftconv_crossfade *h, const float *input, size_t input_len, float *output,
                              size_t output_len) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    return h->core.process_host(input, input_len, output, output_len);
}
int fftconv_crossfade_process_device(fftconv_crossfade *h, const float *d_input, size_t in_stride, float *d_output,
                                     size_t out_stride, size_t output_len, void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    return h->core.process_device(d_input, in_stride, d_output, out_stride, output_len, s);
}
int fftconv_crossfade_is_crossfading(const fftconv_crossfade *h) { return h && h->core.is_crossfading() ? 1 : 0; }
int fftconv_crossfade_process_device_steps(fftconv_crossfade *h, const float *d_input, size_t in_stride, size_t in_step,
                                   float *d_output, size_t out_stride, size_t out_step, size_t len, size_t steps,
                                   void *hip_stream) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    hipStream_t s = pick(hip_stream, h->core.stream);
    if (int r = h->core.order.enter(s)) return r;
    for (size_t k = 0; k < steps; ++k) {
        if (int r = h->core.process_device(d_input + k * in_step, in_stride, d_output + k * out_step, out_stride, len, s))
            return r;
    }
    return FFTCONV_OK;
}
fftconv_crossfade *fftconv_crossfade_clone(const fftconv_crossfade *h) {
    if (!h) { set_error("null handle"); return nullptr; }
    auto *c = new (std::nothrow) fftconv_crossfade();
    if (!c) { set_error("out of host memory"); return nullptr; }
    return make_or_null(c->core.clone_from(h->core), c);
}
void fftconv_crossfade_destroy(fftconv_crossfade *h) { delete h; }
int fftconv_crossfade_synchronize(fftconv_crossfade *h) {
    if (!h) return fail(FFTCONV_E_INVALID, "null handle");
    DeviceGuard g(h->core.device);
    return h->core.quiesce();
}

}  // extern "C"
