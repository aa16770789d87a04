// hbm_probe.hip -- achievable HBM read bandwidth on this GPU for a streaming
// read of the cfg2 footprint (788 MB), float4 per lane, plain vs nontemporal.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/hbm_probe scripts/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void rd(const f4v *__restrict__ p, size_t n4, float *out) {
    f4v acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t k = i + (size_t)u * 256;
            v[u] = k < n4 ? (NT ? __builtin_nontemporal_load(p + k) : p[k]) : f4v{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

template <bool NT, int U>
float run(const f4v *p, size_t n4, float *out, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) rd<NT, U><<<grid, 256>>>(p, n4, out);
    std::vector<float> ms;
    for (int r = 0; r < 10; ++r) {
        hipEventRecord(a);
        rd<NT, U><<<grid, 256>>>(p, n4, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float t; hipEventElapsedTime(&t, a, b); ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const size_t bytes = 788ull << 20;
    const size_t n4 = bytes / 16;
    f4v *p; float *out;
    hipMalloc(&p, bytes);
    hipMalloc(&out, 65536 * 256 * sizeof(float));
    hipMemset(p, 0x3c, bytes);
    for (int grid : {1024, 2048, 4096, 8192}) {
        float t0 = run<false, 4>(p, n4, out, grid), t1 = run<true, 4>(p, n4, out, grid);
        float t2 = run<false, 8>(p, n4, out, grid), t3 = run<true, 8>(p, n4, out, grid);
        printf("grid %5d  plain/U4 %7.1f GB/s  nt/U4 %7.1f GB/s  plain/U8 %7.1f GB/s  nt/U8 %7.1f GB/s\n", grid,
               bytes / t0 / 1e6, bytes / t1 / 1e6, bytes / t2 / 1e6, bytes / t3 / 1e6);
    }
    return 0;
}
