// Low-latency verification path for small batches (Plenum's feed points: a ZStack quota of 100
// client / 1,000 node messages per prod, stp_core/config.py:32-33; Node.verifySignature singletons,
// plenum/server/node.py:2624-2655). Same verdicts as libsodium 1.0.18 crypto_sign_open
// (stp_core/crypto/nacl_wrappers.py:108), computed by ONE workgroup of two waves per request with the
// limb-parallel arithmetic of lp25519.h, in one kernel launch:
//
//   wave 1  signature side: libsodium's checks on (R, S, smlen), k = SHA-512(R || A || M) mod L and its
//           signed radix-16 digits (every lane computes the same scalar values); then [S]B from the
//           engine's fixed-base comb T_B (16 table additions, the 16 entries fetched up front)
//   wave 0  key side, at the same time: decompression of A (row 0, negated) and of R (row 1) in one
//           x^((p-5)/8) chain, the key checks, and the table [j](-A), j = -8..8, into LDS
//   --- barrier ---
//   wave 0  [k](-A) (63 x 4 doublings + 64 additions), Q = [S]B + [k](-A), and the comparison with R
//           without an inversion (lp_final_check), then the request's verdict bit (atomic OR).
//
// The throughput paths keep one verification per lane and need ~1 ms however small the batch; here
// the serial chain of one verification is spread over a wave (lp25519.h), so a batch of up to a few
// thousand requests finishes in about the time of one.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comb.h"
#include "lp25519.h"
#include "verify_core.h"
#include "pv_internal.h"
#include "../../include/plenum_verify.h"

namespace {

constexpr int LAT_THREADS = 128;

// Request bytes at an arbitrary byte offset (aligned dword loads + v_alignbyte_b32).
struct LatMsg {
    const uint32_t* ap;
    uint32_t sh;
    __device__ __forceinline__ uint32_t dw(uint64_t i) const { return __builtin_amdgcn_alignbyte(ap[i + 1], ap[i], sh); }
    __device__ __forceinline__ uint64_t operator()(uint64_t q) const {
        return ((uint64_t)dw(2 * q + 1) << 32) | dw(2 * q);
    }
};

__global__ __launch_bounds__(LAT_THREADS) void pv_lat_kernel(const uint8_t* __restrict__ sm,
                                                              const uint64_t* __restrict__ off, uint64_t n,
                                                              const uint8_t* __restrict__ pk,
                                                              const uint32_t* __restrict__ bcomb,
                                                              unsigned long long* __restrict__ verdict) {
#if LP_DEVICE  // the lp types are 64-lane host arrays in the host pass: the body is device-only
    const uint32_t r = blockIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    __shared__ uint32_t s_k[8];            // signed radix-16 digits of k
    __shared__ uint32_t s_sig_ok;          // libsodium's checks on R, S, smlen
    __shared__ uint32_t s_sb[64];          // [S]B, ext layout, one word per lane
    __shared__ uint32_t s_tab[17][64];     // [j](-A), j = -8..8, cached layout

    const uint64_t o0 = off[r], o1 = off[r + 1];
    const uint64_t smlen = o1 - o0;
    const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
    const LatMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
    pv_sig_words in;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    {
        const uint4* p4 = reinterpret_cast<const uint4*>(pk + 32 * (uint64_t)r);
        const uint4 a0 = p4[0], a1 = p4[1];
        in.A[0] = a0.x; in.A[1] = a0.y; in.A[2] = a0.z; in.A[3] = a0.w;
        in.A[4] = a1.x; in.A[5] = a1.y; in.A[6] = a1.z; in.A[7] = a1.w;
    }
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);

    LpDecomp dec;
    bool key_ok = false, r_ok = false;
    if (wave == 1) {
        // the 16 fixed-base entries, lp cached layout [y-x, y+x, 2dxy, 2] (negated for f < 0)
        uint32_t fs[8];
        sc_recode65536(fs, in.S);
        lu ent[PV_BCOMB_POS];
#pragma unroll
        for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb, j, pv_half(fs[j >> 1], j));
        bool sig_ok = pv_sig_ok(in, smlen);
        uint32_t k[8];
        pv_hash_k(k, in, smlen, mw);
        uint32_t ek[8];
        sc_recode16(ek, k);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) s_k[q] = ek[q];
            s_sig_ok = sig_ok ? 1u : 0u;
        }
        auto entry = [&](int j) -> lu { return lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)); };
        s_sb[lane] = lp_comb_b(c, entry);
    } else {
        // rows 0 / 2: A's encoding, rows 1 / 3: R's
        lu sw[8];
        const lm odd_row = lp_eq(c.row & 1u, 1u);
#pragma unroll
        for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
        dec = lp_decompress_ar(c, K, sw);
        key_ok = pv_ge_is_canonical(in.A) && !pv_has_small_order(in.A) && dec.ok_a;
        r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
        const lu negA = lp_ext_from_xy(c, K, dec.X, dec.Y, 0);
        lp_build_a_table(c, K, negA, [&](int j, const lu& q) { s_tab[j + 8][lane] = q; });
    }
    __syncthreads();
    if (wave != 0) return;
    auto digit = [&](int i) { return pv_nibble(s_k[i >> 3], i); };
    auto load = [&](int e) -> lu { return s_tab[e + 8][lane]; };
    const lu QA = lp_straus_a(c, digit, load);
    const bool eq = lp_final_check(c, K, QA, s_sb[lane], dec.X, dec.Y);
    const bool ok = eq && key_ok && r_ok && s_sig_ok != 0;
    if (lane == 0 && ok) atomicOr(&verdict[r >> 6], 1ull << (r & 63));
#endif
}

}  // namespace

// Enqueue the latency path for n requests (device buffers as pv_verify_batch_device) on `stream`.
int pv_latency_launch(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk,
                      const void* d_bcomb, uint64_t* d_verdict, bool verdict_zeroed, hipStream_t stream) {
    if (n == 0) return PV_OK;
    if (n > 0x7FFFFFFFull) return pv_fail(PV_ERR_ARG, "pv_latency: too many requests for one launch");
    hipError_t e = hipSuccess;
    if (!verdict_zeroed) {  // the kernel ORs its bits into the words
        e = hipMemsetAsync(d_verdict, 0, (n + 63) / 64 * 8, stream);
        if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
    }
    hipLaunchKernelGGL(pv_lat_kernel, dim3((unsigned)n), dim3(LAT_THREADS), 0, stream, d_sm, d_off, n, d_pk,
                       reinterpret_cast<const uint32_t*>(d_bcomb), reinterpret_cast<unsigned long long*>(d_verdict));
    e = hipGetLastError();
    if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("pv_lat_kernel: ") + hipGetErrorString(e));
    return PV_OK;
}
