// Latency of one lp_halfsize (the latency kernels' limb-parallel split of k, lp25519.h) on ONE wave,
// as the signature wave runs it (development tool). Build with -DPV_LP_SPLIT_53=0 / 1 for the 31-bit
// Knuth blocks / the 53-bit Jebelean blocks. Prints microseconds per split (s_memrealtime, 100 MHz)
// and the mean block / quotient / exact-step counts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// phase timer: [0..2] time from mark i to mark i + 1 summed over blocks (10 ns ticks)
__device__ unsigned long long g_mark[4];
__device__ unsigned long long g_phase[3];
#define LP_SPLIT_MARK(i) do { if (stats) { const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); \
    if ((i) > 0 && threadIdx.x == 0) g_phase[(i) - 1] += t_ - g_mark[(i) - 1]; if (threadIdx.x == 0) g_mark[i] = t_; } } while (0)
#include "../indy-plenum_amd/csrc/lp25519.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(64) void k_split(const uint32_t* ks, int nk, uint32_t* out, uint64_t* t, int with_stats) {
#if LP_DEVICE  // the lp types are host arrays in the host pass
    const LpLane c = LpLane::make();
    uint32_t acc = 0, st[3] = {0, 0, 0};
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int j = 0; j < nk; j++) {
        uint32_t k[8];
#pragma unroll
        for (int q = 0; q < 8; q++) k[q] = __builtin_amdgcn_readfirstlane(ks[8 * j + q] ^ (acc & 1u));  // chained
        pv_halfk h;
        lp_halfsize(c, h, k, with_stats ? st : nullptr);
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
#endif
}

int main() {
    const int nk = 256;
    static uint32_t hk[8 * nk];
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
    for (int ws = 0; ws < 2; ws++) {
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(k_split, dim3(1), dim3(64), 0, 0, dk, nk, dout, dt, ws);
            CHECK(hipDeviceSynchronize());
        }
        uint64_t tt, ph[3];
        uint32_t o[4];
        CHECK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_phase), sizeof ph));
        CHECK(hipMemcpy(&tt, dt, 8, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(o, dout, 16, hipMemcpyDeviceToHost));
        printf("{\"split53\": %d, \"stats\": %d, \"us_per_split\": %.2f, \"blocks\": %.2f, \"block_quotients\": %.2f, \"exact_steps\": %.2f, \"acc\": %u, \"us_quot_mat_checks\": [%.2f, %.2f, %.2f]}\n",
               PV_LP_SPLIT_53, ws, tt / 100.0 / nk, o[1] / (double)nk, o[2] / (double)nk, o[3] / (double)nk, o[0], ph[0] / 300.0 / nk, ph[1] / 300.0 / nk, ph[2] / 300.0 / nk);
    }
    return 0;
}
