/*
 * fftconv_oracle.c -- CPU restatement of the reference convolvers.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker*: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (fft-convolution_amd/, libfftconv_amd.so) never links it and
 * has no CPU fallback.
 *
 * It restates, line by line, the state machines of Sin-tel/fft-convolution
 * (paths relative to the reference checkout):
 *   src/fft_convolver.rs:1-84    Fft wrapper + primitives (complex_size,
 *                                 copy_and_pad, complex_multiply_accumulate, sum)
 *   src/fft_convolver.rs:86-307  FFTConvolver (init/update/process/reset)
 *   src/fft_convolver.rs:323-526  TwoStageFFTConvolver + compute_tail_block_size
 *   src/crossfade_convolver.rs    CrossfadeConvolver, Crossfader, RaisedCosineMixer
 *
 * The reference's FFT arithmetic lives in the third-party crates realfft ^3.3
 * and rustfft ^6.1 (Cargo.toml:7-8, no lockfile, not vendored, no Rust
 * toolchain in this image).  Their published algorithm is restated here: a
 * real FFT of length N computed as a complex FFT of length N/2 over the packed
 * even/odd samples plus a post-twiddle (realfft's RealToComplexEven), twiddles
 * computed in f64 and rounded to f32 (rustfft's compute_twiddle).  The C2R
 * rejects a non-zero imaginary part in the DC/Nyquist bin with an error after
 * computing (realfft ComplexToRealEven::process); the reference then zero-fills
 * its output (src/fft_convolver.rs:264-267).  Bit-level parity with rustfft is
 * unpinned (crate absent); the oracle is pinned by the reference's own
 * known-answer / self-consistency tests (src/tests.rs, inline #[test]s) and by
 * an independent f64 direct convolution (see tests/test_oracle.py).
 *
 * Build: oracle/Makefile -> oracle/liboracle.so (gcc, -ffp-contract=off so
 * that, like rustc, no multiply-add is fused).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { float re, im; } cpx;

/* ------------------------------------------------------------------------ */
/* realfft/rustfft restatement                                               */
/* ------------------------------------------------------------------------ */
typedef struct {
    size_t n;     /* real length N (0 = the reference's Default plan)       */
    size_t m;     /* N/2 complex points                                      */
    cpx *tw;      /* W_m^k = exp(-2 pi i k / m), k < m/2                     */
    cpx *rtw;     /* W_N^k = exp(-2 pi i k / N), k <= m                      */
    size_t *rev;  /* bit reversal permutation of m                           */
    cpx *z;       /* scratch m                                               */
} rfft_t;

static size_t next_pow2(size_t v) {            /* usize::next_power_of_two */
    size_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

static void rfft_free(rfft_t *f) {
    free(f->tw); free(f->rtw); free(f->rev); free(f->z);
    memset(f, 0, sizeof(*f));
}

/* Fft::init (src/fft_convolver.rs:30-34); N is always even here (2*B). */
static int rfft_init(rfft_t *f, size_t n) {
    memset(f, 0, sizeof(*f));
    f->n = n;
    if (n == 0) return 0;
    size_t m = n / 2;
    f->m = m;
    f->tw = (cpx *)calloc(m / 2 + 1, sizeof(cpx));
    f->rtw = (cpx *)calloc(m + 1, sizeof(cpx));
    f->rev = (size_t *)calloc(m, sizeof(size_t));
    f->z = (cpx *)calloc(m, sizeof(cpx));
    if (!f->tw || !f->rtw || !f->rev || !f->z) { rfft_free(f); return -1; }
    for (size_t k = 0; k < m / 2 + 1; k++) {
        double a = -2.0 * M_PI * (double)k / (double)m;
        f->tw[k].re = (float)cos(a);
        f->tw[k].im = (float)sin(a);
    }
    for (size_t k = 0; k <= m; k++) {
        double a = -2.0 * M_PI * (double)k / (double)n;
        f->rtw[k].re = (float)cos(a);
        f->rtw[k].im = (float)sin(a);
    }
    size_t bits = 0;
    while (((size_t)1 << bits) < m) bits++;
    for (size_t i = 0; i < m; i++) {
        size_t r = 0;
        for (size_t b = 0; b < bits; b++)
            if (i & ((size_t)1 << b)) r |= (size_t)1 << (bits - 1 - b);
        f->rev[i] = r;
    }
    return 0;
}

static int rfft_clone(rfft_t *dst, const rfft_t *src) { return rfft_init(dst, src->n); }

/* In-place radix-2 DIT complex FFT of length m; sign -1 forward, +1 inverse
 * (unnormalised). */
static void cfft(const rfft_t *f, cpx *z, int inverse) {
    size_t m = f->m;
    for (size_t i = 0; i < m; i++) {
        size_t r = f->rev[i];
        if (r > i) { cpx t = z[i]; z[i] = z[r]; z[r] = t; }
    }
    for (size_t len = 2; len <= m; len <<= 1) {
        size_t half = len / 2, step = m / len;
        for (size_t s = 0; s < m; s += len) {
            for (size_t j = 0; j < half; j++) {
                cpx w = f->tw[j * step];
                if (inverse) w.im = -w.im;
                cpx a = z[s + j], b = z[s + j + half];
                cpx t = { b.re * w.re - b.im * w.im, b.re * w.im + b.im * w.re };
                z[s + j].re = a.re + t.re;        z[s + j].im = a.im + t.im;
                z[s + j + half].re = a.re - t.re; z[s + j + half].im = a.im - t.im;
            }
        }
    }
}

/* Fft::forward (src/fft_convolver.rs:36-39): unnormalised R2C, N -> N/2+1. */
static void rfft_forward(const rfft_t *f, const float *x, cpx *out) {
    size_t m = f->m;
    if (f->n == 0) return;
    cpx *z = f->z;
    for (size_t k = 0; k < m; k++) { z[k].re = x[2 * k]; z[k].im = x[2 * k + 1]; }
    cfft(f, z, 0);
    out[0].re = z[0].re + z[0].im; out[0].im = 0.0f;
    out[m].re = z[0].re - z[0].im; out[m].im = 0.0f;
    for (size_t k = 1; k < m; k++) {
        cpx a = z[k], b = { z[m - k].re, -z[m - k].im };
        cpx e = { (a.re + b.re) * 0.5f, (a.im + b.im) * 0.5f };
        cpx o = { (a.im - b.im) * 0.5f, -(a.re - b.re) * 0.5f };
        cpx w = f->rtw[k];
        out[k].re = e.re + (w.re * o.re - w.im * o.im);
        out[k].im = e.im + (w.re * o.im + w.im * o.re);
    }
}

/* Fft::inverse minus the 1/N (src/fft_convolver.rs:41-49): unnormalised C2R.
 * Returns 1 (FftError::InputValues) when DC or Nyquist carries a non-zero
 * imaginary part; the output is still computed, as realfft does. */
static int rfft_inverse(const rfft_t *f, cpx *in, float *x) {
    size_t m = f->m;
    if (f->n == 0) return 0;
    int bad = 0;
    if (in[0].im != 0.0f) { in[0].im = 0.0f; bad = 1; }
    if (in[m].im != 0.0f) { in[m].im = 0.0f; bad = 1; }
    cpx *z = f->z;
    for (size_t k = 0; k < m; k++) {
        cpx a = in[k], b = { in[m - k].re, -in[m - k].im };
        cpx e = { a.re + b.re, a.im + b.im };
        cpx d = { a.re - b.re, a.im - b.im };
        cpx w = { f->rtw[k].re, -f->rtw[k].im };
        cpx o = { d.re * w.re - d.im * w.im, d.re * w.im + d.im * w.re };
        z[k].re = e.re - o.im;
        z[k].im = e.im + o.re;
    }
    cfft(f, z, 1);
    for (size_t k = 0; k < m; k++) { x[2 * k] = z[k].re; x[2 * k + 1] = z[k].im; }
    return bad;
}

/* Fft::forward / Fft::inverse (src/fft_convolver.rs:36-49) of one row of even
 * length n, for the tests (the checker of fftconv_fft_*).  Complex arrays are
 * n/2+1 interleaved (re, im).  The inverse divides by n like the reference
 * (:44-46) and returns 1 where realfft returns FftError::InputValues. */
int oracle_rfft_forward(size_t n, const float *x, float *out) {
    rfft_t f;
    if (n == 0 || (n & 1) || rfft_init(&f, n)) return -1;
    rfft_forward(&f, x, (cpx *)out);
    rfft_free(&f);
    return 0;
}
int oracle_rfft_inverse(size_t n, const float *in, float *x) {
    rfft_t f;
    if (n == 0 || (n & 1) || rfft_init(&f, n)) return -1;
    cpx *tmp = (cpx *)malloc((n / 2 + 1) * sizeof(cpx));
    if (!tmp) { rfft_free(&f); return -1; }
    memcpy(tmp, in, (n / 2 + 1) * sizeof(cpx));
    int bad = rfft_inverse(&f, tmp, x);
    /* :42 returns FftError::InputValues through `?` before the normalisation
       loop :44-46 (realfft has written the transform with those imaginary
       parts as 0), so a flagged row stays unscaled */
    if (!bad)
        for (size_t i = 0; i < n; i++) x[i] /= (float)n; /* :44-46 */
    free(tmp);
    rfft_free(&f);
    return bad;
}

/* ------------------------------------------------------------------------ */
/* primitives: src/fft_convolver.rs:52-84                                    */
/* ------------------------------------------------------------------------ */
size_t oracle_complex_size(size_t size) { return size / 2 + 1; }

static void copy_and_pad(float *dst, size_t dst_len, const float *src, size_t src_size) {
    memcpy(dst, src, src_size * sizeof(float));
    memset(dst + src_size, 0, (dst_len - src_size) * sizeof(float));
}

static void complex_multiply_accumulate(cpx *r, const cpx *a, const cpx *b, size_t len) {
    for (size_t i = 0; i < len; i++) {
        /* num_complex Mul: (a.re*b.re - a.im*b.im, a.re*b.im + a.im*b.re) */
        float re = a[i].re * b[i].re - a[i].im * b[i].im;
        float im = a[i].re * b[i].im + a[i].im * b[i].re;
        r[i].re += re;
        r[i].im += im;
    }
}

static void vsum(float *r, const float *a, const float *b, size_t len) {
    for (size_t i = 0; i < len; i++) r[i] = a[i] + b[i];
}

/* ------------------------------------------------------------------------ */
/* FFTConvolver: src/fft_convolver.rs:86-307                                */
/* ------------------------------------------------------------------------ */
typedef struct {
    size_t ir_len, block_size, seg_count, active_seg_count;
    cpx *segments;     /* seg_count x K */
    cpx *segments_ir;  /* seg_count x K */
    float *fft_buffer; /* 2B */
    rfft_t fft;
    cpx *pre_multiplied, *conv; /* K */
    float *overlap;    /* B */
    size_t current;
    float *input_buffer; /* B */
    size_t input_buffer_fill;
} ou_t;

static size_t ou_K(const ou_t *c) { return c->block_size ? oracle_complex_size(2 * c->block_size) : 0; }

void ou_free(ou_t *c) {
    if (!c) return;
    free(c->segments); free(c->segments_ir); free(c->fft_buffer);
    free(c->pre_multiplied); free(c->conv); free(c->overlap); free(c->input_buffer);
    rfft_free(&c->fft);
    free(c);
}

/* Default::default() -- every field zero / empty, length-0 FFT plans. */
ou_t *ou_default(void) { return (ou_t *)calloc(1, sizeof(ou_t)); }

/* FFTConvolver::init (src/fft_convolver.rs:105-172).  NULL = panic. */
ou_t *ou_init(const float *ir, size_t ir_len_in, size_t block_size_in, size_t max_len) {
    if (max_len < ir_len_in) return NULL; /* :106-110 */
    ou_t *c = (ou_t *)calloc(1, sizeof(ou_t));
    if (!c) return NULL;
    float *padded = (float *)calloc(max_len ? max_len : 1, sizeof(float)); /* :111-112 */
    if (ir_len_in) memcpy(padded, ir, ir_len_in * sizeof(float));
    size_t ir_len = max_len;
    size_t B = next_pow2(block_size_in);                            /* :115 */
    size_t N = 2 * B;                                               /* :116 */
    size_t S = (size_t)ceil((double)ir_len / (double)B);            /* :117 */
    size_t K = oracle_complex_size(N);                              /* :119 */
    c->ir_len = ir_len; c->block_size = B; c->seg_count = S; c->active_seg_count = S;
    if (rfft_init(&c->fft, N)) goto fail;                           /* :122-123 */
    c->fft_buffer = (float *)calloc(N, sizeof(float));
    c->segments = (cpx *)calloc(S * K + 1, sizeof(cpx));             /* :127 */
    c->segments_ir = (cpx *)calloc(S * K + 1, sizeof(cpx));
    c->pre_multiplied = (cpx *)calloc(K, sizeof(cpx));
    c->conv = (cpx *)calloc(K, sizeof(cpx));
    c->overlap = (float *)calloc(B, sizeof(float));
    c->input_buffer = (float *)calloc(B, sizeof(float));
    if (!c->fft_buffer || !c->segments || !c->segments_ir || !c->pre_multiplied || !c->conv ||
        !c->overlap || !c->input_buffer) goto fail;
    for (size_t i = 0; i < S; i++) {                                /* :131-142 */
        size_t remaining = ir_len - i * B;
        size_t size_copy = remaining >= B ? B : remaining;
        copy_and_pad(c->fft_buffer, N, padded + i * B, size_copy);
        rfft_forward(&c->fft, c->fft_buffer, c->segments_ir + i * K);
    }
    free(padded);
    return c;
fail:
    free(padded);
    ou_free(c);
    return NULL;
}

/* FFTConvolver::update (src/fft_convolver.rs:174-213).  -1 = panic. */
int ou_update(ou_t *c, const float *response, size_t new_ir_len) {
    if (new_ir_len > c->ir_len) return -1;                          /* :177-179 */
    if (c->ir_len == 0) return 0;                                   /* :181-183 */
    size_t B = c->block_size, N = 2 * B, K = ou_K(c);
    memset(c->fft_buffer, 0, N * sizeof(float));                    /* :185-188 */
    memset(c->conv, 0, K * sizeof(cpx));
    memset(c->pre_multiplied, 0, K * sizeof(cpx));
    memset(c->overlap, 0, B * sizeof(float));
    c->active_seg_count = (size_t)ceil((double)new_ir_len / (double)B); /* :190 */
    for (size_t i = 0; i < c->active_seg_count; i++) {              /* :193-207 */
        size_t remaining = new_ir_len - i * B;
        size_t size_copy = remaining >= B ? B : remaining;
        copy_and_pad(c->fft_buffer, N, response + i * B, size_copy);
        rfft_forward(&c->fft, c->fft_buffer, c->segments_ir + i * K);
    }
    for (size_t i = c->active_seg_count; i < c->seg_count; i++)     /* :210-212 */
        memset(c->segments_ir + i * K, 0, K * sizeof(cpx));
    return 0;
}

/* FFTConvolver::process (src/fft_convolver.rs:215-295).  Reads
 * input[0..out_len]; the caller guarantees input holds that many samples. */
void ou_process(ou_t *c, const float *input, float *output, size_t out_len) {
    if (c->active_seg_count == 0) {                                 /* :216-219 */
        memset(output, 0, out_len * sizeof(float));
        return;
    }
    size_t B = c->block_size, N = 2 * B, K = ou_K(c);
    size_t processed = 0;
    while (processed < out_len) {                                   /* :222 */
        int was_empty = c->input_buffer_fill == 0;                  /* :223 */
        size_t processing = out_len - processed;                    /* :224-227 */
        if (B - c->input_buffer_fill < processing) processing = B - c->input_buffer_fill;
        size_t pos = c->input_buffer_fill;                          /* :229-231 */
        memcpy(c->input_buffer + pos, input + processed, processing * sizeof(float));
        copy_and_pad(c->fft_buffer, N, c->input_buffer, B);         /* :234 */
        rfft_forward(&c->fft, c->fft_buffer, c->segments + c->current * K); /* :235-241 */
        if (was_empty) {                                            /* :244-255 */
            memset(c->pre_multiplied, 0, K * sizeof(cpx));
            for (size_t i = 1; i < c->active_seg_count; i++) {
                size_t index_ir = i;
                size_t index_audio = (c->current + i) % c->active_seg_count;
                complex_multiply_accumulate(c->pre_multiplied, c->segments_ir + index_ir * K,
                                            c->segments + index_audio * K, K);
            }
        }
        memcpy(c->conv, c->pre_multiplied, K * sizeof(cpx));        /* :256 */
        complex_multiply_accumulate(c->conv, c->segments + c->current * K, c->segments_ir, K); /* :257-261 */
        if (rfft_inverse(&c->fft, c->conv, c->fft_buffer)) {        /* :264-267 */
            memset(output, 0, out_len * sizeof(float));
            return;
        }
        for (size_t i = 0; i < N; i++) c->fft_buffer[i] /= (float)N; /* Fft::inverse :44-46 */
        vsum(output + processed, c->fft_buffer + pos, c->overlap + pos, processing); /* :270-274 */
        c->input_buffer_fill += processing;                         /* :277 */
        if (c->input_buffer_fill == B) {                            /* :278-292 */
            memset(c->input_buffer, 0, B * sizeof(float));
            c->input_buffer_fill = 0;
            memcpy(c->overlap, c->fft_buffer + B, B * sizeof(float));
            c->current = c->current > 0 ? c->current - 1 : c->active_seg_count - 1;
        }
        processed += processing;
    }
}

/* FFTConvolver::reset (src/fft_convolver.rs:296-306). */
void ou_reset(ou_t *c) {
    size_t B = c->block_size, K = ou_K(c);
    if (c->overlap) memset(c->overlap, 0, B * sizeof(float));
    if (c->segments) memset(c->segments, 0, c->seg_count * K * sizeof(cpx));
    c->current = 0;
    if (c->input_buffer) memset(c->input_buffer, 0, B * sizeof(float));
    if (c->pre_multiplied) memset(c->pre_multiplied, 0, K * sizeof(cpx));
    if (c->conv) memset(c->conv, 0, K * sizeof(cpx));
    c->input_buffer_fill = 0;
}

/* #[derive(Clone)] */
ou_t *ou_clone(const ou_t *s) {
    ou_t *c = (ou_t *)calloc(1, sizeof(ou_t));
    if (!c) return NULL;
    *c = *s;
    memset(&c->fft, 0, sizeof(c->fft));
    c->segments = c->segments_ir = c->pre_multiplied = c->conv = NULL;
    c->fft_buffer = c->overlap = c->input_buffer = NULL;
    if (s->block_size == 0) return c; /* Default */
    size_t B = s->block_size, N = 2 * B, K = ou_K(s), S = s->seg_count;
    if (rfft_clone(&c->fft, &s->fft)) goto fail;
    c->segments = (cpx *)malloc((S * K + 1) * sizeof(cpx));
    c->segments_ir = (cpx *)malloc((S * K + 1) * sizeof(cpx));
    c->pre_multiplied = (cpx *)malloc(K * sizeof(cpx));
    c->conv = (cpx *)malloc(K * sizeof(cpx));
    c->fft_buffer = (float *)malloc(N * sizeof(float));
    c->overlap = (float *)malloc(B * sizeof(float));
    c->input_buffer = (float *)malloc(B * sizeof(float));
    if (!c->segments || !c->segments_ir || !c->pre_multiplied || !c->conv || !c->fft_buffer ||
        !c->overlap || !c->input_buffer) goto fail;
    memcpy(c->segments, s->segments, (S * K + 1) * sizeof(cpx));
    memcpy(c->segments_ir, s->segments_ir, (S * K + 1) * sizeof(cpx));
    memcpy(c->pre_multiplied, s->pre_multiplied, K * sizeof(cpx));
    memcpy(c->conv, s->conv, K * sizeof(cpx));
    memcpy(c->fft_buffer, s->fft_buffer, N * sizeof(float));
    memcpy(c->overlap, s->overlap, B * sizeof(float));
    memcpy(c->input_buffer, s->input_buffer, B * sizeof(float));
    return c;
fail:
    ou_free(c);
    return NULL;
}

/* introspection used by the tests */
size_t ou_block_size(const ou_t *c) { return c->block_size; }
size_t ou_seg_count(const ou_t *c) { return c->seg_count; }
size_t ou_active_seg_count(const ou_t *c) { return c->active_seg_count; }
size_t ou_current(const ou_t *c) { return c->current; }
size_t ou_fill(const ou_t *c) { return c->input_buffer_fill; }

/* ------------------------------------------------------------------------ */
/* compute_tail_block_size: src/fft_convolver.rs:514-526 (f32 arithmetic)    */
/* ------------------------------------------------------------------------ */
size_t oracle_compute_tail_block_size(size_t head_len, size_t response_len) {
    const float FFT_K = 1.5f;
    float kn = (FFT_K * (float)head_len) / (2.0f * logf(2.0f));
    float b = -kn + sqrtf(kn * kn + (float)response_len * (float)head_len);
    float h = (float)head_len;
    b = (b != b) ? h : (b > h ? b : h); /* f32::max ignores NaN */
    size_t bi;
    if (!(b > 0.0f)) bi = 0;            /* saturating `as usize` */
    else if (b >= 18446744073709551615.0f) bi = (size_t)-1;
    else bi = (size_t)b;
    return next_pow2(bi);
}

/* ------------------------------------------------------------------------ */
/* TwoStageFFTConvolver: src/fft_convolver.rs:323-512                        */
/* ------------------------------------------------------------------------ */
typedef struct {
    size_t head_block_size, tail_block_size;
    ou_t *head, *tail0, *tail;
    float *tail_output0, *tail_precalculated0, *tail_output, *tail_precalculated, *tail_input;
    size_t tail_input_fill, precalculated_pos;
} ots_t;

void ots_free(ots_t *t) {
    if (!t) return;
    ou_free(t->head); ou_free(t->tail0); ou_free(t->tail);
    free(t->tail_output0); free(t->tail_precalculated0); free(t->tail_output);
    free(t->tail_precalculated); free(t->tail_input);
    free(t);
}

/* TwoStageFFTConvolver::init (:340-406).  NULL = panic. */
ots_t *ots_init(const float *ir, size_t ir_len_in, size_t block_size, size_t max_len) {
    size_t head_bs = block_size;                                     /* :341 */
    size_t T = oracle_compute_tail_block_size(block_size, max_len);  /* :342 */
    if (max_len < ir_len_in) return NULL;                            /* :344-348 */
    ots_t *t = (ots_t *)calloc(1, sizeof(ots_t));
    if (!t) return NULL;
    float *padded = (float *)calloc(max_len ? max_len : 1, sizeof(float)); /* :349-350 */
    if (ir_len_in) memcpy(padded, ir, ir_len_in * sizeof(float));
    t->head_block_size = head_bs;
    t->tail_block_size = T;
    size_t head_ir_len = max_len < T ? max_len : T;                  /* :352-354 */
    t->head = ou_init(padded, head_ir_len, head_bs, head_ir_len);
    if (max_len > T) {                                               /* :356-368 */
        size_t tl = max_len - T < T ? max_len - T : T;
        t->tail0 = ou_init(padded + T, tl, head_bs, tl);
    } else {
        t->tail0 = ou_default();
    }
    if (max_len > 2 * T) {                                           /* :373-384 */
        size_t tl = max_len - 2 * T;
        t->tail = ou_init(padded + 2 * T, tl, T, tl);
    } else {
        t->tail = ou_default();
    }
    t->tail_output0 = (float *)calloc(T, sizeof(float));             /* :370-388 */
    t->tail_precalculated0 = (float *)calloc(T, sizeof(float));
    t->tail_output = (float *)calloc(T, sizeof(float));
    t->tail_precalculated = (float *)calloc(T, sizeof(float));
    t->tail_input = (float *)calloc(T, sizeof(float));
    free(padded);
    if (!t->head || !t->tail0 || !t->tail || !t->tail_output0 || !t->tail_precalculated0 ||
        !t->tail_output || !t->tail_precalculated || !t->tail_input) {
        ots_free(t);
        return NULL;
    }
    return t;
}

/* TwoStageFFTConvolver::process (:412-495).  -1 = the assert at :428. */
int ots_process(ots_t *t, const float *input, float *output, size_t len) {
    size_t H = t->head_block_size, T = t->tail_block_size;
    if (len > H) return -1;                                          /* :414 */
    ou_process(t->head, input, output, len);                         /* :417 */
    /* :420 tail_input.is_empty() is false for T >= 1 */
    size_t processed = 0;
    while (processed < len) {                                        /* :427 */
        size_t remaining = len - processed;
        size_t processing = H - (t->tail_input_fill % H);
        if (remaining < processing) processing = remaining;
        size_t sb = processed, se = processed + processing;
        /* a head that does not divide T runs past the tail buffers: the
           reference panics at its first out-of-range index (:442, before the
           :459-460 slice); check before touching them (ASan, r4) */
        if (t->precalculated_pos + processing > T || t->tail_input_fill + processing > T) return -1;
        {   /* :439-445 */
            size_t p = t->precalculated_pos;
            for (size_t i = sb; i < se; i++) output[i] += t->tail_precalculated0[p++];
        }
        {   /* :448-454 */
            size_t p = t->precalculated_pos;
            for (size_t i = sb; i < se; i++) output[i] += t->tail_precalculated[p++];
        }
        t->precalculated_pos += processing;                           /* :456 */
        memcpy(t->tail_input + t->tail_input_fill, input + processed, processing * sizeof(float));
        t->tail_input_fill += processing;                             /* :459-461 */
        if (t->tail_input_fill % H == 0) {                            /* :464-476 */
            size_t off = t->tail_input_fill - H;
            ou_process(t->tail0, t->tail_input + off, t->tail_output0 + off, H);
            if (t->tail_input_fill == T) {
                float *s = t->tail_precalculated0;
                t->tail_precalculated0 = t->tail_output0;
                t->tail_output0 = s;
            }
        }
        if (t->tail_input_fill == T) {                                /* :479-486 */
            float *s = t->tail_precalculated;
            t->tail_precalculated = t->tail_output;
            t->tail_output = s;
            ou_process(t->tail, t->tail_input, t->tail_output, T);
        }
        if (t->tail_input_fill == T) {                                /* :488-491 */
            t->tail_input_fill = 0;
            t->precalculated_pos = 0;
        }
        processed += processing;
    }
    return 0;
}

/* TwoStageFFTConvolver::reset (:497-511). */
void ots_reset(ots_t *t) {
    size_t T = t->tail_block_size;
    ou_reset(t->head);
    ou_reset(t->tail0);
    memset(t->tail_output0, 0, T * sizeof(float));
    memset(t->tail_precalculated0, 0, T * sizeof(float));
    ou_reset(t->tail);
    memset(t->tail_output, 0, T * sizeof(float));
    memset(t->tail_precalculated, 0, T * sizeof(float));
    memset(t->tail_input, 0, T * sizeof(float));
    t->tail_input_fill = 0;
    t->precalculated_pos = 0;
}

ots_t *ots_clone(const ots_t *s) {
    size_t T = s->tail_block_size;
    ots_t *t = (ots_t *)calloc(1, sizeof(ots_t));
    if (!t) return NULL;
    *t = *s;
    t->head = ou_clone(s->head); t->tail0 = ou_clone(s->tail0); t->tail = ou_clone(s->tail);
    t->tail_output0 = (float *)malloc(T * sizeof(float));
    t->tail_precalculated0 = (float *)malloc(T * sizeof(float));
    t->tail_output = (float *)malloc(T * sizeof(float));
    t->tail_precalculated = (float *)malloc(T * sizeof(float));
    t->tail_input = (float *)malloc(T * sizeof(float));
    if (!t->head || !t->tail0 || !t->tail || !t->tail_output0 || !t->tail_precalculated0 ||
        !t->tail_output || !t->tail_precalculated || !t->tail_input) { ots_free(t); return NULL; }
    memcpy(t->tail_output0, s->tail_output0, T * sizeof(float));
    memcpy(t->tail_precalculated0, s->tail_precalculated0, T * sizeof(float));
    memcpy(t->tail_output, s->tail_output, T * sizeof(float));
    memcpy(t->tail_precalculated, s->tail_precalculated, T * sizeof(float));
    memcpy(t->tail_input, s->tail_input, T * sizeof(float));
    return t;
}

size_t ots_tail_block_size(const ots_t *t) { return t->tail_block_size; }

/* ------------------------------------------------------------------------ */
/* Crossfader + RaisedCosineMixer: src/crossfade_convolver.rs:160-279        */
/* ------------------------------------------------------------------------ */
enum { TGT_A = 0, TGT_B = 1 };
enum { ST_REACHED = 0, ST_APPROACHING = 1 };

typedef struct {
    int64_t fading_samples, hold_samples, counter;
    float mix_value_step, mix_value;
    int state, target;
} xfader_t;

static float raised_cosine_mix(float a, float b, float value) { /* :163-168 */
    const float PI_HALF = 3.14159265358979323846f * 0.5f;
    float rad = PI_HALF * value;
    float c = cosf(rad);
    float gain1 = c * c;
    float gain2 = 1.0f - gain1;
    return a * gain1 + b * gain2;
}

static void xfader_new(xfader_t *x, size_t fading_samples, size_t hold_samples) { /* :204-214 */
    x->fading_samples = (int64_t)fading_samples;
    x->hold_samples = (int64_t)hold_samples;
    x->counter = 0;
    x->mix_value_step = 1.0f / (float)fading_samples;
    x->mix_value = 0.0f;
    x->state = ST_REACHED;
    x->target = TGT_A;
}

static void xfader_fade_into(xfader_t *x, int target) { /* :216-240 */
    if (x->target == target) return;
    if (x->state == ST_REACHED) {
        x->counter = -x->hold_samples;
        x->state = ST_APPROACHING;
        x->target = target;
        x->mix_value_step = -x->mix_value_step;
    } else {
        if (x->counter >= 0) {
            x->counter = x->fading_samples - x->counter;
            x->state = ST_APPROACHING;
            x->target = target;
            x->mix_value_step = -x->mix_value_step;
        } else {
            x->state = ST_REACHED;
            x->target = target;
        }
    }
}

static float xfader_mix(xfader_t *x, float a, float b) { /* :242-278 */
    if (x->state == ST_REACHED) return x->target == TGT_A ? a : b;
    x->counter += 1;
    if (x->counter <= 0) return x->target == TGT_A ? b : a;
    x->mix_value += x->mix_value_step;
    if (x->counter == x->fading_samples) {
        x->state = ST_REACHED;
        if (x->target == TGT_A) { x->mix_value = 0.0f; return a; }
        x->mix_value = 1.0f;
        return b;
    }
    return raised_cosine_mix(a, b, x->mix_value);
}

/* exposed so tests can port test_crossfader (src/crossfade_convolver.rs:281-316) */
xfader_t *oracle_xfader_new(size_t fading, size_t hold) {
    xfader_t *x = (xfader_t *)calloc(1, sizeof(xfader_t));
    if (x) xfader_new(x, fading, hold);
    return x;
}
void oracle_xfader_free(xfader_t *x) { free(x); }
void oracle_xfader_fade_into(xfader_t *x, int target) { xfader_fade_into(x, target); }
float oracle_xfader_mix(xfader_t *x, float a, float b) { return xfader_mix(x, a, b); }
int oracle_xfader_state(const xfader_t *x) { return x->state * 2 + x->target; }

/* ------------------------------------------------------------------------ */
/* CrossfadeConvolver<FFTConvolver>: src/crossfade_convolver.rs:3-105         */
/* ------------------------------------------------------------------------ */
typedef struct {
    ou_t *a, *b;
    xfader_t xf;
    float *buffer_a, *buffer_b;
    size_t max_buffer_size;
    float *stored_response;
    size_t stored_len;
    int response_pending;
} ocf_t;

void ocf_free(ocf_t *c) {
    if (!c) return;
    ou_free(c->a); ou_free(c->b);
    free(c->buffer_a); free(c->buffer_b); free(c->stored_response);
    free(c);
}

/* CrossfadeConvolver::new (:19-43); takes ownership of `conv`. */
ocf_t *ocf_new(ou_t *conv, size_t max_response_length, size_t max_buffer_size, size_t crossfade_samples) {
    ocf_t *c = (ocf_t *)calloc(1, sizeof(ocf_t));
    if (!c) return NULL;
    c->stored_response = (float *)calloc(max_response_length ? max_response_length : 1, sizeof(float));
    c->stored_len = max_response_length;
    c->a = ou_clone(conv);
    c->b = conv;
    xfader_new(&c->xf, crossfade_samples,
               max_buffer_size < max_response_length ? max_buffer_size : max_response_length);
    c->buffer_a = (float *)calloc(max_buffer_size ? max_buffer_size : 1, sizeof(float));
    c->buffer_b = (float *)calloc(max_buffer_size ? max_buffer_size : 1, sizeof(float));
    c->max_buffer_size = max_buffer_size;
    if (!c->stored_response || !c->a || !c->buffer_a || !c->buffer_b) { ocf_free(c); return NULL; }
    return c;
}

/* Convolution::init (:46-49) */
ocf_t *ocf_init(const float *response, size_t len, size_t max_block_size, size_t max_len) {
    ou_t *conv = ou_init(response, len, max_block_size, max_len);
    if (!conv) return NULL;
    return ocf_new(conv, len, max_block_size, len);
}

int ocf_is_crossfading(const ocf_t *c) { return c->xf.state == ST_APPROACHING; } /* :85-92 */

static int ocf_swap(ocf_t *c, const float *response, size_t len) { /* :94-105 */
    if (c->xf.target == TGT_A) {
        if (ou_update(c->b, response, len)) return -1;
        xfader_fade_into(&c->xf, TGT_B);
    } else {
        if (ou_update(c->a, response, len)) return -1;
        xfader_fade_into(&c->xf, TGT_A);
    }
    return 0;
}

/* Convolution::update (:51-64).  -1 = panic. */
int ocf_update(ocf_t *c, const float *response, size_t len) {
    if (!ocf_is_crossfading(c)) {
        if (ocf_swap(c, response, len)) return -1;
        c->response_pending = 0;
        return 0;
    }
    if (len > c->stored_len) return -1;
    memcpy(c->stored_response, response, len * sizeof(float));
    memset(c->stored_response + len, 0, (c->stored_len - len) * sizeof(float));
    c->response_pending = 1;
    return 0;
}

/* Convolution::process (:66-78).  Input must hold >= max_buffer_size samples
 * and out_len <= max_buffer_size (else the reference panics on a slice). */
int ocf_process(ocf_t *c, const float *input, size_t in_len, float *output, size_t out_len) {
    if (in_len < c->max_buffer_size || out_len > c->max_buffer_size) return -1;
    if (!ocf_is_crossfading(c) && c->response_pending) {
        if (ocf_swap(c, c->stored_response, c->stored_len)) return -1;
        c->response_pending = 0;
    }
    ou_process(c->a, input, c->buffer_a, c->max_buffer_size);
    ou_process(c->b, input, c->buffer_b, c->max_buffer_size);
    for (size_t i = 0; i < out_len; i++) output[i] = xfader_mix(&c->xf, c->buffer_a[i], c->buffer_b[i]);
    return 0;
}

int ocf_response_pending(const ocf_t *c) { return c->response_pending; }

/* ------------------------------------------------------------------------ */
/* CPU baseline: C independent uniform convolvers (one per channel, as the    */
/* reference is one instance per channel), split over `threads` pthreads.    */
/* Synthetic white noise, distinct IR per channel.  Returns seconds spent in */
/* the timed process() loop (the init is untimed).                           */
/* ------------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static float urand(uint64_t *s) { /* U[-1, 1) */
    return (float)((double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
}

typedef struct {
    int kind; /* 0 FFTConvolver, 1 TwoStageFFTConvolver (block = head), 2 CrossfadeConvolver */
    size_t c0, c1, block, ir_len, nblocks, warm, every;
    uint64_t seed;
    double secs;
    int err;
} bench_job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* One instance per channel (the reference is one instance per channel), each
 * fed its own white-noise block every call.  kind 2 swaps in a fresh response
 * on every channel every `every` blocks (update(), timed like process()). */
static void *bench_worker(void *arg) {
    bench_job_t *j = (bench_job_t *)arg;
    size_t nc = j->c1 - j->c0;
    void **cv = (void **)calloc(nc ? nc : 1, sizeof(void *));
    float *ir = (float *)malloc(j->ir_len * sizeof(float));
    float *ir2 = (float *)malloc(j->ir_len * sizeof(float));
    float *in = (float *)malloc(nc * j->block * sizeof(float) + 4);
    float *out = (float *)malloc(j->block * sizeof(float));
    if (!cv || !ir || !ir2 || !in || !out) { j->err = 1; goto done; }
    float g = 1.0f / sqrtf((float)j->ir_len);
    for (size_t c = 0; c < nc; c++) {
        uint64_t s = j->seed + (j->c0 + c) * 7919u;
        for (size_t i = 0; i < j->ir_len; i++) ir[i] = urand(&s) * g;
        cv[c] = j->kind == 0 ? (void *)ou_init(ir, j->ir_len, j->block, j->ir_len)
              : j->kind == 1 ? (void *)ots_init(ir, j->ir_len, j->block, j->ir_len)
                             : (void *)ocf_init(ir, j->ir_len, j->block, j->ir_len);
        if (!cv[c]) { j->err = 1; goto done; }
        for (size_t i = 0; i < j->block; i++) in[c * j->block + i] = urand(&s);
    }
    uint64_t s2 = j->seed ^ 0x5bd1e995u;
    for (size_t i = 0; i < j->ir_len; i++) ir2[i] = urand(&s2) * g;
    volatile float sink = 0.0f;
    double t0 = 0.0;
    for (size_t b = 0; b < j->warm + j->nblocks; b++) {
        if (b == j->warm) t0 = now_s();
        for (size_t c = 0; c < nc; c++) {
            const float *x = in + c * j->block;
            if (j->kind == 0) {
                ou_process((ou_t *)cv[c], x, out, j->block);
            } else if (j->kind == 1) {
                if (ots_process((ots_t *)cv[c], x, out, j->block)) j->err = 1;
            } else {
                if (j->every && b % j->every == j->every - 1) ocf_update((ocf_t *)cv[c], (b / j->every) & 1 ? ir : ir2, j->ir_len);
                if (ocf_process((ocf_t *)cv[c], x, j->block, out, j->block)) j->err = 1;
            }
            sink += out[0];
        }
    }
    j->secs = now_s() - t0;
done:
    if (cv)
        for (size_t c = 0; c < nc; c++) {
            if (!cv[c]) continue;
            if (j->kind == 0) ou_free((ou_t *)cv[c]);
            else if (j->kind == 1) ots_free((ots_t *)cv[c]);
            else ocf_free((ocf_t *)cv[c]);
        }
    free(cv); free(ir); free(ir2); free(in); free(out);
    return NULL;
}

/* Returns the wall seconds of the timed region (max over threads), < 0 on error. */
double oracle_bench(int kind, size_t channels, size_t block, size_t ir_len, size_t nblocks, size_t warm,
                    size_t threads, uint64_t seed, size_t every) {
    if (threads < 1) threads = 1;
    if (threads > channels) threads = channels;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    bench_job_t *jobs = (bench_job_t *)calloc(threads, sizeof(bench_job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1.0; }
    for (size_t t = 0; t < threads; t++) {
        jobs[t].kind = kind;
        jobs[t].c0 = channels * t / threads;
        jobs[t].c1 = channels * (t + 1) / threads;
        jobs[t].block = block; jobs[t].ir_len = ir_len; jobs[t].nblocks = nblocks;
        jobs[t].warm = warm; jobs[t].seed = seed; jobs[t].every = every;
        pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
    }
    double worst = 0.0;
    int err = 0;
    for (size_t t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].err) err = 1;
        if (jobs[t].secs > worst) worst = jobs[t].secs;
    }
    free(th); free(jobs);
    return err ? -1.0 : worst;
}

double oracle_bench_uniform(size_t channels, size_t block, size_t ir_len, size_t nblocks,
                            size_t warm, size_t threads, uint64_t seed) {
    return oracle_bench(0, channels, block, ir_len, nblocks, warm, threads, seed, 0);
}
