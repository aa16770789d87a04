// cumask_probe.hip -- which CU-mask patterns does hipExtStreamCreateWithCUMask honour?
// Times a CU-filling streaming kernel on masked streams (stride k / first-N block).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(1024) void spin(const float4 *p, size_t n4, float *o) {
    float4 a = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 1024) {
        float4 v = p[i]; a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    o[blockIdx.x * 1024 + threadIdx.x] = a.x + a.y + a.z + a.w;
}
int main() {
    int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t bytes = 1ull << 30, n4 = bytes / 16;
    float4 *p; float *o; hipMalloc(&p, bytes); hipMalloc(&o, 256 * 1024 * 4); hipMemset(p, 0, bytes);
    auto run = [&](const char *name, std::vector<uint32_t> mask) {
        hipStream_t s;
        if (mask.empty()) hipStreamCreate(&s); else hipExtStreamCreateWithCUMask(&s, mask.size(), mask.data());
        std::vector<uint32_t> back((ncu + 31) / 32, 0); hipExtStreamGetCUMask(s, back.size(), back.data());
        int bits = 0; for (auto w : back) bits += __builtin_popcount(w);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        spin<<<256, 1024, 0, s>>>(p, n4, o);
        hipEventRecord(a, s); spin<<<256, 1024, 0, s>>>(p, n4, o); hipEventRecord(b, s); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-14s readback bits %3d  time %8.1f us\n", name, bits, ms * 1000);
        hipStreamDestroy(s);
    };
    run("none", {});
    for (int k : {2, 3, 4, 8}) {
        std::vector<uint32_t> m((ncu + 31) / 32, 0);
        for (int cu = 0; cu < ncu; cu += k) m[cu / 32] |= 1u << (cu % 32);
        char nm[32]; snprintf(nm, 32, "stride %d", k); run(nm, m);
    }
    for (int k : {2, 3, 4, 8}) {
        std::vector<uint32_t> m((ncu + 31) / 32, 0);
        for (int cu = 0; cu < ncu / k; ++cu) m[cu / 32] |= 1u << (cu % 32);
        char nm[32]; snprintf(nm, 32, "first 1/%d", k); run(nm, m);
    }
    return 0;
}
