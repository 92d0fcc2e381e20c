// Clock ramp probe (development tool): a fixed-work ALU kernel of ~0.3 ms launched 30 times with a
// host-side gap of G us between launches (G = 0, 200, 500, 1000, 3000); per launch the kernel's own
// duration (events) and its shader-clock cycles per real-time tick (s_memtime / s_memrealtime, 100 MHz
// constant clock) give the clock the kernel ran at. One JSON object per gap.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <algorithm>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void alu_kernel(uint64_t* clk, uint32_t iters) {
    uint64_t c0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t x = threadIdx.x + blockIdx.x;
    uint64_t a = x;
    for (uint32_t i = 0; i < iters; i++) {
        a = a * 0x9E3779B97F4A7C15ull + x;
        x ^= (uint32_t)(a >> 29);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
    if (x == 0x12345678u) clk[2] = x;
}

int main() {
    uint64_t* clk;
    CK(hipHostMalloc((void**)&clk, 64, hipHostMallocCoherent));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int gap : {0, 200, 500, 1000, 3000, 0}) {
        std::vector<float> ms;
        std::vector<double> ghz;
        for (int i = 0; i < 30; i++) {
            if (gap) std::this_thread::sleep_for(std::chrono::microseconds(gap));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(alu_kernel, dim3(2048), dim3(256), 0, s, clk, 1500u);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
            ghz.push_back(clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 0.0);
        }
        printf("{\"gap_us\": %d, \"kernel_ms\": [", gap);
        for (size_t i = 0; i < ms.size(); i++) printf("%s%.3f", i ? ", " : "", ms[i]);
        printf("], \"clock_GHz_block0\": [");
        for (size_t i = 0; i < ghz.size(); i++) printf("%s%.2f", i ? ", " : "", ghz[i]);
        printf("]}\n");
        fflush(stdout);
    }
    return 0;
}
