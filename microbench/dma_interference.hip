// Does H2D DMA slow concurrent kernels? (development probe for the pipelined host path). Two kernels
// -- an L2-resident gather (random 16 B reads from a 4 MB table per XCD, like the comb kernels' table
// reads) and a pure ALU loop -- timed alone and beside 400 MB of pinned H2D copies issued as one copy,
// as 64 MB pieces and as 4 MB pieces on another stream. One JSON object per measurement.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void gather_kernel(const uint4* __restrict__ tab, uint32_t mask, uint32_t iters, uint4* out) {
    uint32_t x = blockIdx.x * 256 + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        const uint4 v = tab[(x >> 8) & mask];
        acc.x ^= v.x;
        acc.y += v.y;
        acc.z ^= v.z + i;
        acc.w += v.w ^ x;
    }
    if (acc.x == 0x12345678u) out[0] = acc;
}

__global__ void alu_kernel(uint32_t* out, uint32_t iters) {
    uint32_t x = threadIdx.x + blockIdx.x;
    uint64_t a = x;
    for (uint32_t i = 0; i < iters; i++) {
        a = a * 0x9E3779B97F4A7C15ull + x;
        x ^= (uint32_t)(a >> 29);
    }
    if (x == 0x12345678u) out[0] = x;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t B = 400ull << 20;
    uint8_t *h, *d;
    CK(hipHostMalloc((void**)&h, B, hipHostMallocPortable));
    CK(hipMalloc((void**)&d, B));
    memset(h, 1, B);
    const uint32_t tab_entries = (uint32_t)(((size_t)atoi(getenv("TAB_MB") ? getenv("TAB_MB") : "4") << 20) / 16);
    uint4 *tab, *out;
    CK(hipMalloc((void**)&tab, tab_entries * 16));
    CK(hipMemset(tab, 3, tab_entries * 16));
    CK(hipMalloc((void**)&out, 64));
    hipStream_t ks, cs;
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipEvent_t k0, k1;
    CK(hipEventCreate(&k0));
    CK(hipEventCreate(&k1));
    const uint32_t iters = (uint32_t)atoi(getenv("ITERS") ? getenv("ITERS") : "2048");
    auto launch = [&](int which) {
        if (which == 0)
            hipLaunchKernelGGL(gather_kernel, dim3(8192), dim3(256), 0, ks, tab, tab_entries - 1, iters, out);
        else
            hipLaunchKernelGGL(alu_kernel, dim3(8192), dim3(256), 0, ks, (uint32_t*)out, 20000u);
    };
    const char* kname[2] = {"l2_gather", "alu"};
    for (int which = 0; which < 2; which++) {
        for (int mode = 0; mode < 4; mode++) {  // 0 alone, 1 one copy, 2 64 MB pieces, 3 4 MB pieces
            float best = 1e9f;
            double copy_ms = 0;
            for (int r = 0; r < 4; r++) {
                CK(hipDeviceSynchronize());
                const double t0 = now();
                if (mode) {
                    const size_t piece = mode == 1 ? B : mode == 2 ? (64ull << 20) : (4ull << 20);
                    for (size_t o = 0; o < B; o += piece)
                        CK(hipMemcpyAsync(d + o, h + o, std::min(piece, B - o), hipMemcpyHostToDevice, cs));
                }
                // a chain of 4 kernels spanning the copies
                CK(hipEventRecord(k0, ks));
                for (int q = 0; q < 4; q++) launch(which);
                CK(hipEventRecord(k1, ks));
                CK(hipStreamSynchronize(cs));
                const double t1 = now();
                CK(hipStreamSynchronize(ks));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, k0, k1));
                if (r > 0 && ms < best) best = ms;
                if (r > 0) copy_ms = (t1 - t0) * 1e3;
            }
            printf("{\"kernel\": \"%s\", \"table_MB\": %u, \"copies\": \"%s\", \"kernels_ms_for_4\": %.3f, \"copy_wall_ms\": %.3f}\n",
                   kname[which], tab_entries >> 16, mode == 0 ? "none" : mode == 1 ? "one_400MB" : mode == 2 ? "64MB_pieces" : "4MB_pieces",
                   best, copy_ms);
            fflush(stdout);
        }
    }
    return 0;
}
