// examples/compare_partitioned.rs as a native host over the C ABI (no Python,
// no torch): the same 64-sample uniform vs two-stage comparison, one
// process() call per block (reference: examples/compare_partitioned.rs:9-68,
// examples/util/mod.rs:7-19).  This is the call pattern a Rust `impl
// Convolution` over include/fftconv.h produces.
//   make -C examples && examples/compare_partitioned [blocks]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fftconv.h"

static std::vector<float> generate_sinusoid(size_t n, double freq, unsigned sample_rate, double gain) {
    std::vector<float> out(n);
    for (size_t i = 0; i < n; ++i) {
        const double t = (double)i / (double)sample_rate;
        out[i] = (float)(gain * std::sin(2.0 * M_PI * freq * t));
    }
    return out;
}

#define CHECK(x)                                                                        \
    do {                                                                                \
        if ((x) != FFTCONV_OK) {                                                        \
            std::fprintf(stderr, "%s failed: %s\n", #x, fftconv_last_error());          \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

int main(int argc, char **argv) {
    const unsigned SAMPLE_RATE = 44100;
    const size_t block_size = 64;
    const size_t n_blocks = argc > 1 ? (size_t)std::atol(argv[1]) : 1000;
    const size_t response_len = 128000;

    const std::vector<float> response = generate_sinusoid(response_len, 1000.0, SAMPLE_RATE, 0.1);
    fftconv_uniform *a = fftconv_uniform_init(response.data(), response.size(), block_size, response.size());
    fftconv_twostage *b = fftconv_twostage_init(response.data(), response.size(), block_size, response.size());
    if (!a || !b) {
        std::fprintf(stderr, "init failed: %s\n", fftconv_last_error());
        return 1;
    }
    const std::vector<float> input = generate_sinusoid(n_blocks * block_size, 1300.0, SAMPLE_RATE, 0.1);
    std::vector<float> out_a(block_size * n_blocks), out_b(block_size * n_blocks);

    auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n_blocks; ++i)
        CHECK(fftconv_uniform_process(a, &input[i * block_size], block_size, &out_a[i * block_size], block_size));
    auto t1 = std::chrono::steady_clock::now();
    std::printf("Uniform took = %.2f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());

    t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n_blocks; ++i)
        CHECK(fftconv_twostage_process(b, &input[i * block_size], &out_b[i * block_size], block_size));
    t1 = std::chrono::steady_clock::now();
    std::printf("Partitioned took = %.2f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());

    float max_abs_diff = 0.f;
    for (size_t i = 0; i < out_a.size(); ++i) max_abs_diff = std::fmax(max_abs_diff, std::fabs(out_a[i] - out_b[i]));
    std::printf("max_abs_diff = %g\n", (double)max_abs_diff);

    fftconv_uniform_destroy(a);
    fftconv_twostage_destroy(b);
    return 0;
}
