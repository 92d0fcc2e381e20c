// Field / group operation cost microbenchmark for the gfx950 verify kernels (development tool).
// Each lane runs ITERS dependent operations (x = op(x)) of the kernels' own fe25519/ge25519 code;
// the grid fills every SIMD with W waves. Reported: shader-clock cycles per operation per wave
// (s_memtime around the loop, wave 0 of each block) and the SIMD issue cost per wave-op
// (= cycles / W, the figure to compare with instruction counts x per-instruction cycle costs).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../indy-plenum_amd/csrc/ge25519.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 256;

enum Op { MUL = 0, SQ = 1, DBL = 2, ADDC = 3, CARRY = 4 };

template <int OP, int MINB>
__global__ __launch_bounds__(256, MINB) void k_op(const uint32_t* in, uint32_t* out, uint64_t* cyc) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    fe a, b, c;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        a.v[i] = in[(i * 64 + (t & 63)) & 1023] & ((i & 1) ? M25 : M26);
        b.v[i] = in[(i * 64 + 640 + (t & 63)) & 1023] & ((i & 1) ? M25 : M26);
        c.v[i] = in[(i * 64 + 320 + (t & 63)) & 1023] & ((i & 1) ? M25 : M26);
    }
    __syncthreads();
    const uint64_t t0 = clock64();
    if (OP == MUL) {
        for (int it = 0; it < ITERS; it++) fe_mul(a, a, b);
    } else if (OP == SQ) {
        for (int it = 0; it < ITERS; it++) fe_sq(a, a);
    } else if (OP == DBL) {
        for (int it = 0; it < ITERS; it++) {
            ge_p1p1 r;
            ge_p2_dbl(r, a, b, c);
            ge_p1p1_to_p2(a, b, c, r);
        }
    } else if (OP == ADDC) {
        ge_p3 p;
        p.X = a; p.Y = b; p.Z = c; p.T = a;
        ge_cached q;
        q.YplusX = b; q.YminusX = c; q.Z2 = a; q.T2d = b;
        for (int it = 0; it < ITERS; it++) {
            ge_p1p1 r;
            ge_add_cached(r, p, q);
            ge_p1p1_to_p3(p, r);
        }
        a = p.X; b = p.Y;
    } else if (OP == CARRY) {
        for (int it = 0; it < ITERS; it++) {
            fe_add(a, a, b);
            fe_carry(a, a);
        }
    }
    const uint64_t t1 = clock64();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) x ^= a.v[i] ^ b.v[i] ^ c.v[i];
    out[t] = x;
    if ((threadIdx.x & 63) == 0) cyc[t >> 6] = t1 - t0;
}

typedef void (*kfn)(const uint32_t*, uint32_t*, uint64_t*);

template <int MINB>
int run(const char* name, kfn f, int cus, const uint32_t* din, uint32_t* dout, uint64_t* dcyc) {
    const int blocks = cus * MINB;
    const int waves = blocks * 4;
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, din, dout, dcyc);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, din, dout, dcyc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    static uint64_t hc[1 << 16];
    CHECK(hipMemcpy(hc, dcyc, waves * 8, hipMemcpyDeviceToHost));
    double avg = 0;
    for (int i = 0; i < waves; i++) avg += (double)hc[i];
    avg /= waves;
    const double per_op = avg / ITERS;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_op_per_wave\": %.1f, "
           "\"simd_issue_cycles_per_wave_op\": %.1f, \"lane_ops_per_s\": %.4g}\n",
           name, MINB, ms, per_op, per_op / MINB, (double)waves * 64 * ITERS / (ms * 1e-3));
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t hin[1024];
    uint32_t s = 12345;
    for (int i = 0; i < 1024; i++) { s = s * 1664525u + 1013904223u; hin[i] = s; }
    uint32_t *din, *dout;
    uint64_t* dcyc;
    CHECK(hipMalloc(&din, sizeof hin));
    CHECK(hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dout, (size_t)cus * 4 * 256 * 4));
    CHECK(hipMalloc(&dcyc, (size_t)cus * 16 * 8));
#define RUNW(W)                                                                   \
    if (run<W>("mul", k_op<MUL, W>, cus, din, dout, dcyc)) return 1;            \
    if (run<W>("sq", k_op<SQ, W>, cus, din, dout, dcyc)) return 1;              \
    if (run<W>("carry+add", k_op<CARRY, W>, cus, din, dout, dcyc)) return 1;    \
    if (run<W>("dbl_p2", k_op<DBL, W>, cus, din, dout, dcyc)) return 1;         \
    if (run<W>("addc_p3", k_op<ADDC, W>, cus, din, dout, dcyc)) return 1;
    RUNW(1)
    RUNW(2)
    RUNW(3)
    RUNW(4)
    return 0;
}
