// Latency of one sc_halfsize (the half-size split of k, sc25519.h) on ONE wave, the way the latency
// kernel's signature wave runs it (development tool). Mode 0: k held per lane (VALU), mode 1: k made
// uniform first (readfirstlane; scalar unit where the compiler can). Prints microseconds per split
// (s_memrealtime, 100 MHz) and the split's block / quotient / exact-step counts for the first k.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../indy-plenum_amd/csrc/sc25519.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(64) void k_split(const uint32_t* ks, int nk, uint32_t* out, uint64_t* t) {
    uint32_t acc = 0, st[3] = {0, 0, 0};
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int j = 0; j < nk; j++) {
        uint32_t k[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            k[q] = ks[8 * j + q] ^ (acc & 1u);  // chain the splits
            if (MODE == 1) k[q] = __builtin_amdgcn_readfirstlane(k[q]);
        }
        pv_halfk h;
        sc_halfsize(h, k, j == 0 ? st : nullptr);
        acc += h.k1[0] ^ h.k2[0] ^ (h.fallback ? 1u : 0u);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        t[0] = t1 - t0;
        out[0] = acc;
        out[1] = st[0];
        out[2] = st[1];
        out[3] = st[2];
    }
}

int main() {
    const int nk = 64;
    uint32_t hk[8 * nk];
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 8 * nk; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        hk[i] = (uint32_t)(s >> 32);
        if (i % 8 == 7) hk[i] &= 0x0FFFFFFFu;  // < 2^252 < L
    }
    uint32_t *dk, *dout;
    uint64_t* dt;
    CHECK(hipMalloc(&dk, sizeof hk));
    CHECK(hipMalloc(&dout, 64));
    CHECK(hipMalloc(&dt, 8));
    CHECK(hipMemcpy(dk, hk, sizeof hk, hipMemcpyHostToDevice));
    for (int mode = 0; mode < 2; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            if (mode == 0) hipLaunchKernelGGL(k_split<0>, dim3(1), dim3(64), 0, 0, dk, nk, dout, dt);
            else hipLaunchKernelGGL(k_split<1>, dim3(1), dim3(64), 0, 0, dk, nk, dout, dt);
            CHECK(hipDeviceSynchronize());
        }
        uint64_t tt;
        uint32_t o[4];
        CHECK(hipMemcpy(&tt, dt, 8, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(o, dout, 16, hipMemcpyDeviceToHost));
        printf("{\"mode\": %d, \"us_per_split\": %.2f, \"blocks\": %u, \"block_quotients\": %u, \"exact_steps\": %u}\n",
               mode, tt / 100.0 / nk, o[1], o[2], o[3]);
    }
    return 0;
}
