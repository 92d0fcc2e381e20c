// PCIe / host-copy probe for the host-fed path (development tool): H2D bandwidth from pinned memory
// in one call and in pieces on one or two streams, D2H, pageable -> pinned memcpy on 1..16 threads,
// hipMemcpy straight from pageable memory, hipHostRegister's cost, and an H2D beside a busy kernel.
// Prints one JSON object per measurement.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void spin_kernel(uint32_t* out, uint32_t iters) {
    uint32_t x = threadIdx.x + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[0] = x;
}

int main() {
    const size_t B = 400ull << 20;
    uint8_t *h, *d;
    CK(hipHostMalloc((void**)&h, B, hipHostMallocPortable));
    CK(hipMalloc((void**)&d, B));
    memset(h, 1, B);
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        double best = 1e9;
        for (int r = 0; r < 3; r++) {
            const double t0 = now();
            fn();
            CK(hipDeviceSynchronize());
            best = std::min(best, now() - t0);
        }
        printf("{\"probe\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"GBps\": %.2f}\n", name, B, best * 1e3, B / best / 1e9);
        fflush(stdout);
    };
    timed("h2d_pinned_one_call", [&] { CK(hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s0)); });
    for (size_t piece : {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20}) {
        char name[64];
        snprintf(name, sizeof name, "h2d_pinned_pieces_%zuMB_1stream", piece >> 20);
        timed(name, [&] {
            for (size_t o = 0; o < B; o += piece) CK(hipMemcpyAsync(d + o, h + o, std::min(piece, B - o), hipMemcpyHostToDevice, s0));
        });
        snprintf(name, sizeof name, "h2d_pinned_pieces_%zuMB_2streams", piece >> 20);
        timed(name, [&] {
            int i = 0;
            for (size_t o = 0; o < B; o += piece, i++)
                CK(hipMemcpyAsync(d + o, h + o, std::min(piece, B - o), hipMemcpyHostToDevice, (i & 1) ? s1 : s0));
        });
    }
    timed("d2h_pinned_one_call", [&] { CK(hipMemcpyAsync(h, d, B, hipMemcpyDeviceToHost, s0)); });
    // pageable source
    uint8_t* p = (uint8_t*)malloc(B);
    memset(p, 2, B);
    for (int th : {1, 4, 8, 16}) {
        char name[64];
        snprintf(name, sizeof name, "memcpy_pageable_to_pinned_%dthreads", th);
        timed(name, [&] {
            std::vector<std::thread> t;
            for (int i = 0; i < th; i++)
                t.emplace_back([&, i] {
                    const size_t a = B * i / th, b = B * (i + 1) / th;
                    memcpy(h + a, p + a, b - a);
                });
            for (auto& x : t) x.join();
        });
    }
    timed("hipMemcpy_from_pageable", [&] { CK(hipMemcpy(d, p, B, hipMemcpyHostToDevice)); });
    {
        const double t0 = now();
        CK(hipHostRegister(p, B, hipHostRegisterDefault));
        const double t1 = now();
        printf("{\"probe\": \"hipHostRegister\", \"bytes\": %zu, \"ms\": %.3f}\n", B, (t1 - t0) * 1e3);
        timed("h2d_registered_one_call", [&] { CK(hipMemcpyAsync(d, p, B, hipMemcpyHostToDevice, s0)); });
        const double t2 = now();
        CK(hipHostUnregister(p));
        printf("{\"probe\": \"hipHostUnregister\", \"ms\": %.3f}\n", (now() - t2) * 1e3);
    }
    // H2D beside a kernel that occupies every CU
    uint32_t* dout;
    CK(hipMalloc((void**)&dout, 4));
    hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, s1, dout, 1u << 16);
    CK(hipEventRecord(e0, s1));
    CK(hipDeviceSynchronize());
    {
        const double t0 = now();
        hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, s1, dout, 1u << 16);
        CK(hipStreamSynchronize(s1));
        const double k_ms = (now() - t0) * 1e3;
        const double t1 = now();
        hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, s1, dout, 1u << 16);
        for (size_t o = 0; o < B; o += 8ull << 20) CK(hipMemcpyAsync(d + o, h + o, 8ull << 20, hipMemcpyHostToDevice, s0));
        CK(hipStreamSynchronize(s0));
        const double c_ms = (now() - t1) * 1e3;
        CK(hipStreamSynchronize(s1));
        const double both = (now() - t1) * 1e3;
        printf("{\"probe\": \"h2d_beside_kernel\", \"kernel_alone_ms\": %.3f, \"copy_done_ms\": %.3f, \"both_done_ms\": %.3f}\n",
               k_ms, c_ms, both);
    }
    int dev = 0;
    CK(hipGetDevice(&dev));
    char bus[64] = {0};
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, dev));
    printf("{\"probe\": \"device\", \"pci\": \"%s\", \"hw_concurrency\": %u}\n", bus, std::thread::hardware_concurrency());
    return 0;
}
