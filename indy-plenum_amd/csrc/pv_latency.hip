// Low-latency verification path for small batches (Plenum's feed points: a ZStack quota of 100
// client / 1,000 node messages per prod, stp_core/config.py:32-33; Node.verifySignature singletons,
// plenum/server/node.py:2624-2655). Same verdicts as libsodium 1.0.18 crypto_sign_open
// (stp_core/crypto/nacl_wrappers.py:108), computed by ONE workgroup of two waves per request with the
// limb-parallel arithmetic of lp25519.h, in one kernel launch:
//
//   wave 1  signature side: libsodium's checks on (R, S, smlen), k = SHA-512(R || A || M) mod L, then
//           the half-size split k = k1 / k2 (mod 8L) (sc25519.h sc_halfsize: |k1|, k2 ~ 2^128, k2
//           odd) and s2 = k2 S mod L (every lane computes the same scalar values)
//   wave 0  key side, at the same time: decompression of A (row 0, negated) and of R (row 1) in one
//           x^((p-5)/8) chain, the key checks, and the tables [j](-A) and [j]R', j = -8..8, into LDS
//   --- barrier 1 (split ready, tables ready) ---
//   wave 0  [k1](-A) (sign of k1 applied to the digits) + R': ~33 x 4 doublings + ~33 additions
//   wave 1  [k2](-R') from wave 0's R table, then + [s2]B from the engine's fixed-base comb T_B (16
//           table additions, the 16 entries fetched before the loop) -- the two halves of the old
//           single 252-doubling chain run on two waves at once
//   --- barrier 2 ---
//   wave 0  Q = [k1](-A) + R' + [k2](-R') + [s2]B, compared with R' without an inversion
//           (lp_final_check): equal iff [k2](SB - kA - R') = 0 iff libsodium's encode(SB - kA) == R
//           (sc25519.h), then the request's verdict bit (atomic OR).
//   A key in the node-side key cache (keycache.h) keeps the full scalar instead: wave 0 computes
//   [k](-A) as 32 additions from its comb table, wave 1 [S]B, and Q = [S]B + [k](-A) is compared
//   with R.
//
// The throughput paths keep one verification per lane and need ~1 ms however small the batch; here
// the serial chain of one verification is spread over a wave (lp25519.h), so a batch of up to a few
// thousand requests finishes in about the time of one.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comb.h"
#include "keycache.h"
#include "lp25519.h"
#include "verify_core.h"
#include "pv_internal.h"
#include "../../include/plenum_verify.h"

// PV_LAT_HALF = 0: the single-chain form for A/B (wave 0 runs [k](-A) as 63 x 4 doublings + 64
// additions, wave 1 [S]B); 1: the half-size split over both waves (above).
#ifndef PV_LAT_HALF
#define PV_LAT_HALF 1
#endif
// PV_LAT_TRACE (measurement builds only): block 0 stamps s_memrealtime (100 MHz) at its phase
// boundaries into pv_lat_trace, read back by pv_debug_lat_trace.
#ifdef PV_LAT_TRACE
__device__ unsigned long long pv_lat_trace_buf[20];
#define LAT_STAMP(i) do { if (blockIdx.x == 0 && (threadIdx.x & 63u) == 0) pv_lat_trace_buf[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define LAT_STAMP(i) do { } while (0)
#endif

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

[[maybe_unused]] constexpr uint32_t PV_ZC_MSG_WORDS = PV_ZC_MAX_STRIDE / 4;

// PV_LAT_SHA_CALL = 1: the four-wave form's SHA-512 (wave 1) is a real call with its own register
// allocation, so its speed does not move with the code around it (inlined, one request's hash took
// 24.0-26.4 us depending on the rest of the kernel); 0: inlined. The two-wave form keeps it inlined
// (a call raises every caller's VGPR count to the callee's, and that form runs several workgroups
// per CU).
#ifndef PV_LAT_SHA_CALL
#define PV_LAT_SHA_CALL 1
#endif
struct LatK {
    uint32_t k[8];
};
__device__ __noinline__ LatK lat_hash_k_call(pv_sig_words in, uint64_t smlen, const uint32_t* ap, uint32_t sh) {
    LatK o;
    pv_hash_k(o.k, in, smlen, LatMsg{ap, sh});
    return o;
}
[[maybe_unused]] __device__ __forceinline__ void lat_hash_k(uint32_t k[8], const pv_sig_words& in, uint64_t smlen, const LatMsg& mw) {
#if PV_LAT_SHA_CALL
    const LatK o = lat_hash_k_call(in, smlen, mw.ap, mw.sh);
#pragma unroll
    for (int q = 0; q < 8; q++) k[q] = o.k[q];
#else
    pv_hash_k(k, in, smlen, mw);
#endif
}

// ZC: zero-copy host-buffer call (pv_latency_launch_zc; slot layout and verdict bytes as in
// pv_lat4_kernel below).
template <bool ZC>
__global__ __launch_bounds__(LAT_THREADS) void pv_lat_kernel(const uint8_t* __restrict__ sm,
                                                              const uint64_t* __restrict__ off, uint64_t n,
                                                              const uint8_t* __restrict__ pk,
                                                              const uint32_t* __restrict__ bcomb, PvKeyCacheView kc,
                                                              unsigned long long* __restrict__ verdict,
                                                              uint8_t* __restrict__ vbytes, uint32_t zstride,
                                                              const uint32_t* __restrict__ run_if) {
#if LP_DEVICE  // the lp types are 64-lane host arrays in the host pass: the body is device-only
    if (run_if && *run_if == 0u) return;  // AUTO's device-side choice picked the keyed path
    const uint32_t r = blockIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    __shared__ uint32_t s_k16[8];          // signed radix-16 digits of |k1| (half-size split)
    __shared__ uint32_t s_k256[8];         // signed radix-256 digits of k (cached key's comb table)
    __shared__ uint32_t s_sig_ok;          // libsodium's checks on R, S, smlen
    __shared__ uint32_t s_nw, s_neg;       // windows of the split, k1 < 0
    __shared__ uint32_t s_sb[64];          // wave 1's result, ext layout, one word per lane
    __shared__ uint32_t s_tab[17][64];     // [j](-A), j = -8..8, cached layout
    __shared__ uint32_t s_rtab[17][64];    // [j]R', j = -8..8
    __shared__ uint32_t s_msg[ZC ? PV_ZC_MSG_WORDS : 1];

    uint64_t smlen;
    const uint32_t* ap;
    uint32_t sh;
    pv_sig_words in;
    if constexpr (ZC) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sm + (uint64_t)r * zstride);
        for (uint32_t t = threadIdx.x; t < zstride / 4; t += LAT_THREADS) s_msg[t] = src[t];
        __syncthreads();
        smlen = s_msg[0];
#pragma unroll
        for (int q = 0; q < 8; q++) in.A[q] = s_msg[PV_ZC_PK_WORD + q];
        ap = s_msg + PV_ZC_REC_WORD;
        sh = 0;
    } else {
        const uint64_t o0 = off[r], o1 = off[r + 1];
        smlen = o1 - o0;
        const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
        ap = reinterpret_cast<const uint32_t*>(raddr & ~3ull);
        sh = (uint32_t)(raddr & 3);
        const uint4* p4 = reinterpret_cast<const uint4*>(pk + 32 * (uint64_t)r);
        const uint4 a0 = p4[0], a1 = p4[1];
        in.A[0] = a0.x; in.A[1] = a0.y; in.A[2] = a0.z; in.A[3] = a0.w;
        in.A[4] = a1.x; in.A[5] = a1.y; in.A[6] = a1.z; in.A[7] = a1.w;
    }
    const LatMsg mw{ap, sh};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    // uniform: one branch per wave, the same on both waves
    const uint32_t slot = __builtin_amdgcn_readfirstlane(pv_kc_lookup(kc, in.A));
    const bool cached = slot != PV_KC_EMPTY;

    if (wave == 1) {
        LAT_STAMP(8);
        const bool sig_ok = pv_sig_ok(in, smlen);
        if (cached || !PV_LAT_HALF) {
            // [S]B: the 16 fixed-base entries are fetched first, then k, then the additions
            uint32_t fs[8];
            sc_recode65536(fs, in.S);
            lu ent[PV_BCOMB_POS];
#pragma unroll
            for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb, j, pv_half(fs[j >> 1], j));
            uint32_t k[8];
            pv_hash_k(k, in, smlen, mw);
            LAT_STAMP(9);
            uint32_t e256[8], e16[8];
            sc_recode256(e256, k);
            sc_recode16(e16, k);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    s_k256[q] = e256[q];
                    s_k16[q] = e16[q];
                }
                s_nw = 64;
                s_neg = 0;
                s_sig_ok = sig_ok ? 1u : 0u;
            }
            __syncthreads();  // 1: k is ready
            auto entry = [&](int j) -> lu { return lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)); };
            s_sb[lane] = lp_comb_b(c, entry);
            LAT_STAMP(11);
            __syncthreads();  // 2: [S]B is ready
            return;
        }
        uint32_t k[8], S[8];
        pv_hash_k(k, in, smlen, mw);
        LAT_STAMP(9);
        // every lane holds the same k: made uniform, the split runs on the scalar unit (short
        // dependent-instruction latency: this is one wave's serial chain)
#pragma unroll
        for (int q = 0; q < 8; q++) {
            k[q] = __builtin_amdgcn_readfirstlane(k[q]);
            S[q] = __builtin_amdgcn_readfirstlane(in.S[q]);
        }
        pv_halfk hk;
        lp_halfsize(c, hk, k);
        LAT_STAMP(12);
        uint32_t s2[8], fs[8], e1[8], e2[8];
        sc_mul<5>(s2, hk.k2, S);
        LAT_STAMP(13);
        sc_recode65536(fs, s2);
        lu ent[PV_BCOMB_POS];
#pragma unroll
        for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb, j, pv_half(fs[j >> 1], j));
        sc_recode16(e1, hk.k1);
        sc_recode16(e2, hk.k2);
        const int nw1 = sc_nwin16(e1), nw2 = sc_nwin16(e2);
        const int nw = __builtin_amdgcn_readfirstlane(nw1 > nw2 ? nw1 : nw2);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) s_k16[q] = e1[q];
            s_nw = (uint32_t)nw;
            s_neg = hk.neg ? 1u : 0u;
            s_sig_ok = sig_ok ? 1u : 0u;
        }
        LAT_STAMP(10);
        __syncthreads();  // 1: split ready; wave 0's tables ready
        // [k2](-R') = sum of [-e]R' entries, then + [s2]B
        lu acc = lp_straus_nw(c, nw, [&](int i) { return pv_nibble(e2[i >> 3], i); },
                              [&](int e) -> lu { return s_rtab[8 - e][lane]; });
#pragma unroll
        for (int j = PV_BCOMB_POS - 1; j >= 0; j--) acc = lp_add_cached(c, acc, lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)));
        s_sb[lane] = acc;
        LAT_STAMP(11);
        __syncthreads();  // 2
        return;
    }
    LAT_STAMP(0);
    // key side: decompression of A (row 0) and R (row 1) in one chain
    lu sw[8];
    const lm odd_row = lp_eq(c.row & 1u, 1u);
#pragma unroll
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    LAT_STAMP(1);
    const bool r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
    bool key_ok;
    lu QA;
    if (cached) {
        // cached key: libsodium's key checks ran when its table was built; [k](-A) = 32 additions
        key_ok = kc.flags[slot] != 0;
        const uint32_t* tab = reinterpret_cast<const uint32_t*>(kc.tab + (uint64_t)slot * PV_COMB_POS * PV_COMB_ENT * 10);
        __syncthreads();  // 1
        uint32_t e256[8];
#pragma unroll
        for (int q = 0; q < 8; q++) e256[q] = s_k256[q];
        lu ent[PV_COMB_POS];
#pragma unroll
        for (int i = 0; i < PV_COMB_POS; i++) ent[i] = lp_ctab_load(c, tab, i, pv_byte(e256[i >> 2], i));
        QA = lp_comb_a(c, [&](int i) { return lp_ctab_fix(c, ent[i], pv_byte(e256[i >> 2], i)); });
    } else {
        key_ok = pv_ge_is_canonical(in.A) && !pv_has_small_order(in.A) && dec.ok_a;
        const lu negA = lp_ext_from_xy(c, K, dec.X, dec.Y, 0);
        lp_build_a_table(c, K, negA, [&](int j, const lu& q) { s_tab[j + 8][lane] = q; });
        if (PV_LAT_HALF) {
            const lu Rp = lp_ext_from_xy(c, K, dec.X, dec.Y, 1);
            lp_build_a_table(c, K, Rp, [&](int j, const lu& q) { s_rtab[j + 8][lane] = q; });
        }
        LAT_STAMP(2);
        __syncthreads();  // 1
        LAT_STAMP(3);
        const int nw = __builtin_amdgcn_readfirstlane((int)s_nw);
        const int sgn = s_neg ? -1 : 1;
        auto digit = [&](int i) { return sgn * pv_nibble(s_k16[i >> 3], i); };
        auto load = [&](int e) -> lu { return s_tab[e + 8][lane]; };
        QA = lp_straus_nw(c, nw, digit, load);
        if (PV_LAT_HALF) QA = lp_add_cached(c, QA, s_rtab[9][lane]);  // + R'
    }
    LAT_STAMP(4);
    __syncthreads();  // 2
    LAT_STAMP(5);
    const bool eq = lp_final_check(c, K, QA, s_sb[lane], dec.X, dec.Y);
    const bool ok = eq && key_ok && r_ok && s_sig_ok != 0;
    if constexpr (ZC) {
        // a coherent (fine-grained) pinned byte the host spins on while the kernel runs
        // (pv_spin_verdict_bytes): a system-scope atomic store goes straight to host memory; relaxed,
        // since the byte itself is the only datum the host reads (a release would write back the
        // whole L2 once per request)
        if (lane == 0) __hip_atomic_store(&vbytes[r], (uint8_t)(ok ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        if (lane == 0 && ok) atomicOr(&verdict[r >> 6], 1ull << (r & 63));
    }
    LAT_STAMP(6);
#endif
}

// Four-wave form for small batches (PV_LAT4_MAX): each of [k1](+-A) and [k2](-R') is split once more at
// window PV_LAT4_SPLIT (2^68), k_i = lo + 2^68 hi, so four waves run ~17 windows each at the same time:
//   wave 0  decompression of A and R (one chain), -A and R' published (LDS flag), tables of -A and the lower half of R'
//           then lo(k1) on -A
//   wave 1  checks, k, the split, s2 = k2 S mod L and its digits; then lo(k2) on -R'
//   wave 2  [2^68](-A) by 68 doublings on y alone from A's encoding (lp_ydbl_chain), x once -A is
//           published, table of it; then hi(k1) on it + positions 0..7 of [s2]B
//   wave 3  the same for R': table of [2^68]R'; then hi(k2) on its negation + positions 8..15
//   waves 2, 3 also build R''s table entries 5, 6 / 7, 8 (wave 0 entries 0..4)
//   wave 0  sums the four parts, + R', compares with R' (lp_final_check).
// A cached key keeps the two-wave cached flow (waves 2 and 3 only join the barriers).
#ifndef PV_LAT4_MAX
#define PV_LAT4_MAX 512  // batches up to this size take the four-wave form (more waves, less chain)
#endif
#ifndef PV_LAT4_SPLIT
#define PV_LAT4_SPLIT 17
#endif
// PV_LAT4_RTAB_SPLIT = 1: R''s table is built by waves 0 (entries 0..4), 2 (5, 6) and 3 (7, 8); 0: all
// by wave 0
#ifndef PV_LAT4_RTAB_SPLIT
#define PV_LAT4_RTAB_SPLIT 1
#endif
constexpr int LAT4_THREADS = 256;
// ZC (zero-copy host-buffer calls, pv_latency_launch_zc): the requests sit in pinned host memory in
// fixed-stride slots (pv_internal.h: smlen, the key, the record, slack for the hash's read-ahead); the
// workgroup copies its slot into LDS in ONE PCIe round trip (no offset lookup first) and the verdict is
// one byte per request stored to host memory (vbytes) instead of OR-ed into device words: no copy
// kernels before or after the verification.

// The four-wave body; zsrc (ZC): this workgroup's request slot, in pinned host memory
// (pv_lat4_kernel) or in the kernel arguments (pv_lat4_one_kernel).
template <bool ZC>
__device__ __forceinline__ void lat4_body(const uint32_t* __restrict__ zsrc, const uint8_t* __restrict__ sm,
                                          const uint64_t* __restrict__ off, uint64_t n,
                                          const uint8_t* __restrict__ pk, const uint32_t* __restrict__ bcomb,
                                          PvKeyCacheView kc, unsigned long long* __restrict__ verdict,
                                          uint8_t* __restrict__ vbytes, uint32_t zstride,
                                          const uint32_t* __restrict__ run_if) {
#if LP_DEVICE
    if (run_if && *run_if == 0u) return;
    const uint32_t r = blockIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    __shared__ uint32_t s_k1[8], s_k2[8];   // signed radix-16 digits of |k1|, k2
    __shared__ uint32_t s_k256[8];          // radix-256 digits of k (cached key)
    __shared__ uint32_t s_sig_ok, s_nw, s_neg;
    __shared__ volatile uint32_t s_pts_ready;  // wave 0 -> waves 2, 3: -A and R' published
    __shared__ volatile uint32_t s_k_ready;    // cached key: wave 1 -> waves 2, 3: k's digits published
    __shared__ uint32_t s_pa[64], s_pr[64];    // -A, R' (ext)
    __shared__ uint32_t s_part[3][64];         // wave 1, 2, 3 results (cached form)
    __shared__ uint32_t s_fs[8];               // radix-65536 digits of s2 = k2 S mod L (waves 2, 3: [s2]B)
    __shared__ uint32_t s_tab[4][17][64];      // [j] of -A, R', [2^68](-A), [2^68]R', j = -8..8
    __shared__ uint32_t s_msg[ZC ? PV_ZC_MSG_WORDS : 1];

    if (threadIdx.x == 0) {
        s_pts_ready = 0u;
        s_k_ready = 0u;
    }
    LAT_STAMP(wave == 0 ? 16 : 19);  // kernel entry (19: unused slot for the other waves)
    uint64_t smlen;
    const uint32_t* ap;
    uint32_t sh;
    pv_sig_words in;
    if constexpr (ZC) {
        for (uint32_t t = threadIdx.x; t < zstride / 4; t += LAT4_THREADS) s_msg[t] = zsrc[t];
        __syncthreads();
        LAT_STAMP(wave == 0 ? 17 : 19);  // the slot is in LDS
        smlen = s_msg[0];
#pragma unroll
        for (int q = 0; q < 8; q++) in.A[q] = s_msg[PV_ZC_PK_WORD + q];
        ap = s_msg + PV_ZC_REC_WORD;
        sh = 0;
    } else {
        const uint64_t o0 = off[r], o1 = off[r + 1];
        smlen = o1 - o0;
        const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
        ap = reinterpret_cast<const uint32_t*>(raddr & ~3ull);
        sh = (uint32_t)(raddr & 3);
        const uint4* p4 = reinterpret_cast<const uint4*>(pk + 32 * (uint64_t)r);
        const uint4 a0 = p4[0], a1 = p4[1];
        in.A[0] = a0.x; in.A[1] = a0.y; in.A[2] = a0.z; in.A[3] = a0.w;
        in.A[4] = a1.x; in.A[5] = a1.y; in.A[6] = a1.z; in.A[7] = a1.w;
    }
    const LatMsg mw{ap, sh};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(pv_kc_lookup(kc, in.A));
    const bool cached = slot != PV_KC_EMPTY;
    const bool wide = cached && kc.wtab && slot < kc.wcap;  // the key's radix-65536 rows (comb.h PV_KW_*)
    __syncthreads();  // 0: s_pts_ready cleared
    LAT_STAMP(wave == 0 ? 0 : (wave == 1 ? 8 : 14));

    if (wave >= 2) {
        if (cached) {
            // [k](-A) in two halves beside wave 0's decompression of R (the only point a cached key still
            // needs): as soon as wave 1 has k's digits, wave 2 adds the upper, wave 3 the lower positions
            // -- 8 niels entries each from the wide rows, else 16 cached ones
            while (s_k_ready == 0u) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint32_t e256[8];
#pragma unroll
            for (int q = 0; q < 8; q++) e256[q] = s_k256[q];
            lu acc = lp_identity_ext(c);
            if (wide) {
                const uint32_t* wr =
                    reinterpret_cast<const uint32_t*>(kc.wtab + (uint64_t)slot * PV_KW_POS * PV_KW_ENT * (PV_BCOMB_STRIDE / 4));
                const int q0 = wave == 2 ? PV_KW_POS / 2 : 0;
                lu ent[PV_KW_POS / 2];
#pragma unroll
                for (int jj = 0; jj < PV_KW_POS / 2; jj++) ent[jj] = lp_kw_entry(c, wr, q0 + jj, pv_kw_digit(e256[(q0 + jj) >> 1], q0 + jj));
#pragma unroll
                for (int jj = PV_KW_POS / 2 - 1; jj >= 0; jj--)
                    acc = lp_add_cached(c, acc, lp_bcomb_fix(c, ent[jj], pv_kw_digit(e256[(q0 + jj) >> 1], q0 + jj)));
            } else {
                const uint32_t* tab = reinterpret_cast<const uint32_t*>(kc.tab + (uint64_t)slot * PV_COMB_POS * PV_COMB_ENT * 10);
                const int i0 = wave == 2 ? PV_COMB_POS / 2 : 0;
                lu ent[PV_COMB_POS / 2];
#pragma unroll
                for (int ii = 0; ii < PV_COMB_POS / 2; ii++) ent[ii] = lp_ctab_load(c, tab, i0 + ii, pv_byte(e256[(i0 + ii) >> 2], i0 + ii));
#pragma unroll
                for (int ii = PV_COMB_POS / 2 - 1; ii >= 0; ii--)
                    acc = lp_add_cached(c, acc, lp_ctab_fix(c, ent[ii], pv_byte(e256[(i0 + ii) >> 2], i0 + ii)));
            }
            s_part[wave - 1][lane] = lp_to_cached(c, acc, K.d2);
        }
        if (!cached) {
            // the 68 doublings run on y alone from the encoding (lp_ydbl_chain), beside wave 0's
            // decompression; x enters once it is published
            lu yw[8];
#pragma unroll
            for (int q = 0; q < 8; q++) yw[q] = wave == 2 ? in.A[q] : in.R[q];
            const LpYChain ch = lp_ydbl_chain(c, K, lp_from_words(c, yw), 4 * PV_LAT4_SPLIT);
            LAT_STAMP(wave == 2 ? 7 : 15);
            // wait for wave 0's decompression (a workgroup's waves are co-resident: it progresses)
            while (s_pts_ready == 0u) __builtin_amdgcn_s_sleep(2);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            lu x0, t1, t2, t3;
            lp_allrows(wave == 2 ? lu(s_pa[lane]) : lu(s_pr[lane]), x0, t1, t2, t3);  // ext rows [x, y, 1, xy]
            const lu P = lp_ydbl_finish(c, K, ch, x0);
            lp_build_a_table(c, K, P, [&](int j, const lu& q) { s_tab[wave][j + 8][lane] = q; });
            // waves 2 and 3 also build the upper entries of R''s table (wave 0 the lower ones): wave
            // 0's decompression + tables were the longest chain before barrier 1
            if (PV_LAT4_RTAB_SPLIT)
                lp_build_a_table_part(c, K, lu(s_pr[lane]), wave - 1, [&](int j, const lu& q) { s_tab[1][j + 8][lane] = q; });
        }
        __syncthreads();  // 1: split, tables ready
        if (!cached) {
            const int nw = __builtin_amdgcn_readfirstlane((int)s_nw);
            const int sgn = wave == 3 ? -1 : (s_neg ? -1 : 1);  // k2's part goes on -R''
            const uint32_t* dg = wave == 2 ? s_k1 : s_k2;
            // [s2]B in two halves: wave 2 positions 0..7, wave 3 8..15 of the fixed-base comb, the
            // entries fetched before the loop and added after it (balances wave 1's lo(k2) loop)
            const int j0 = wave == 2 ? 0 : PV_BCOMB_POS / 2;
            uint32_t fsl[PV_BCOMB_POS / 4];
#pragma unroll
            for (int q = 0; q < PV_BCOMB_POS / 4; q++) fsl[q] = s_fs[j0 / 2 + q];
            lu ent[PV_BCOMB_POS / 2];
#pragma unroll
            for (int jj = 0; jj < PV_BCOMB_POS / 2; jj++) ent[jj] = lp_bcomb_entry(c, bcomb, j0 + jj, pv_half(fsl[jj >> 1], jj));
            lu acc = lp_straus_range(c, PV_LAT4_SPLIT, nw, [&](int i) { return sgn * pv_nibble(dg[i >> 3], i); },
                                     [&](int e) -> lu { return s_tab[wave][e + 8][lane]; });
#pragma unroll
            for (int jj = PV_BCOMB_POS / 2 - 1; jj >= 0; jj--) acc = lp_add_cached(c, acc, lp_bcomb_fix(c, ent[jj], pv_half(fsl[jj >> 1], jj)));
            s_part[wave - 1][lane] = lp_to_cached(c, acc, K.d2);  // cached here, off wave 0's chain
        }
        __syncthreads();  // 2
        return;
    }
    if (wave == 1) {
        // libsodium's checks on R, S, smlen, published before the hash: evaluated here, beside the
        // SHA-512 call, instead of sunk behind it onto the critical path (2.6 us of dependent loads)
        if (lane == 0) s_sig_ok = pv_sig_ok(in, smlen) ? 1u : 0u;
        if (cached) {
            uint32_t fs[8];
            sc_recode65536(fs, in.S);
            lu ent[PV_BCOMB_POS];
#pragma unroll
            for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb, j, pv_half(fs[j >> 1], j));
            uint32_t k[8], e256[8];
            lat_hash_k(k, in, smlen, mw);
            sc_recode256(e256, k);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < 8; q++) s_k256[q] = e256[q];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                s_k_ready = 1u;  // waves 2 and 3 start [k](-A) now, not at barrier 1
            }
            // [S]B also before barrier 1: beside wave 0's decompression, off its chain
            s_part[0][lane] = lp_to_cached(c, lp_comb_b(c, [&](int j) -> lu { return lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)); }), K.d2);
            __syncthreads();  // 1
            __syncthreads();  // 2
            return;
        }
        uint32_t k[8], S[8];
        lat_hash_k(k, in, smlen, mw);
        LAT_STAMP(9);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            k[q] = __builtin_amdgcn_readfirstlane(k[q]);
            S[q] = __builtin_amdgcn_readfirstlane(in.S[q]);
        }
        pv_halfk hk;
        lp_halfsize(c, hk, k);
        LAT_STAMP(12);
        uint32_t s2[8], fs[8], e1[8], e2[8];
        sc_mul<5>(s2, hk.k2, S);
        LAT_STAMP(13);
        sc_recode65536(fs, s2);
        sc_recode16(e1, hk.k1);
        sc_recode16(e2, hk.k2);
        const int nw1 = sc_nwin16(e1), nw2 = sc_nwin16(e2);
        LAT_STAMP(18);
        const int nw = __builtin_amdgcn_readfirstlane(nw1 > nw2 ? nw1 : nw2);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                s_k1[q] = e1[q];
                s_k2[q] = e2[q];
                s_fs[q] = fs[q];
            }
            s_nw = (uint32_t)nw;
            s_neg = hk.neg ? 1u : 0u;
        }
        LAT_STAMP(10);
        __syncthreads();  // 1
        const int hi = nw < PV_LAT4_SPLIT ? nw : PV_LAT4_SPLIT;
        s_part[0][lane] = lp_to_cached(c, lp_straus_range(c, 0, hi, [&](int i) { return -pv_nibble(e2[i >> 3], i); },
                                                          [&](int e) -> lu { return s_tab[1][e + 8][lane]; }), K.d2);
        LAT_STAMP(11);
        __syncthreads();  // 2
        return;
    }
    // wave 0
    lu sw[8];
    const lm odd_row = lp_eq(c.row & 1u, 1u);
#pragma unroll
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    LAT_STAMP(1);
    const bool r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
    bool key_ok;
    lu QA;
    if (cached) {
        // waves 2 and 3 built the two halves of [k](-A) during the decompression
        key_ok = kc.flags[slot] != 0;
        __syncthreads();  // 1
        __syncthreads();  // 2
        QA = lp_add_cached(c, lp_add_cached(c, lp_identity_ext(c), lu(s_part[1][lane])), lu(s_part[2][lane]));
    } else {
        key_ok = pv_ge_is_canonical(in.A) && !pv_has_small_order(in.A) && dec.ok_a;
        const lu negA = lp_ext_from_xy(c, K, dec.X, dec.Y, 0);
        const lu Rp = lp_ext_from_xy(c, K, dec.X, dec.Y, 1);
        s_pa[lane] = negA;
        s_pr[lane] = Rp;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) s_pts_ready = 1u;
        lp_build_a_table(c, K, negA, [&](int j, const lu& q) { s_tab[0][j + 8][lane] = q; });
        if (PV_LAT4_RTAB_SPLIT)
            lp_build_a_table_part(c, K, Rp, 0, [&](int j, const lu& q) { s_tab[1][j + 8][lane] = q; });  // waves 2, 3: 5..8
        else
            lp_build_a_table(c, K, Rp, [&](int j, const lu& q) { s_tab[1][j + 8][lane] = q; });
        LAT_STAMP(2);
        __syncthreads();  // 1
        LAT_STAMP(3);
        const int nw = __builtin_amdgcn_readfirstlane((int)s_nw);
        const int sgn = s_neg ? -1 : 1;
        const int hi = nw < PV_LAT4_SPLIT ? nw : PV_LAT4_SPLIT;
        QA = lp_straus_range(c, 0, hi, [&](int i) { return sgn * pv_nibble(s_k1[i >> 3], i); },
                             [&](int e) -> lu { return s_tab[0][e + 8][lane]; });
        QA = lp_add_cached(c, QA, s_tab[1][9][lane]);  // + R'
        LAT_STAMP(4);
        __syncthreads();  // 2
        LAT_STAMP(5);
        // + the hi parts of k1 and k2 with the two halves of [s2]B (waves 2, 3); wave 1's part is added
        // by lp_final_check
        QA = lp_add_cached(c, QA, lu(s_part[1][lane]));
        QA = lp_add_cached(c, QA, lu(s_part[2][lane]));
    }
    // cached: QA = [k](-A), wave 1's part [S]B; otherwise QA = [k1](+-A) + R' + [2^68 hi(k2)](-R') +
    // [s2]B, wave 1's part [lo(k2)](-R')
    const bool eq = lp_final_check_cached(c, QA, s_part[0][lane], dec.X, dec.Y);
    const bool ok = eq && key_ok && r_ok && s_sig_ok != 0;
    if constexpr (ZC) {
        // a coherent (fine-grained) pinned byte the host spins on while the kernel runs
        // (pv_spin_verdict_bytes): a system-scope atomic store goes straight to host memory; relaxed,
        // since the byte itself is the only datum the host reads (a release would write back the
        // whole L2 once per request)
        if (lane == 0) __hip_atomic_store(&vbytes[r], (uint8_t)(ok ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        if (lane == 0 && ok) atomicOr(&verdict[r >> 6], 1ull << (r & 63));
    }
    LAT_STAMP(6);
#endif
}

template <bool ZC>
__global__ __launch_bounds__(LAT4_THREADS) void pv_lat4_kernel(const uint8_t* __restrict__ sm,
                                                               const uint64_t* __restrict__ off, uint64_t n,
                                                               const uint8_t* __restrict__ pk,
                                                               const uint32_t* __restrict__ bcomb, PvKeyCacheView kc,
                                                               unsigned long long* __restrict__ verdict,
                                                               uint8_t* __restrict__ vbytes, uint32_t zstride,
                                                               const uint32_t* __restrict__ run_if) {
    lat4_body<ZC>(ZC ? reinterpret_cast<const uint32_t*>(sm + (uint64_t)blockIdx.x * zstride) : nullptr, sm, off, n,
                  pk, bcomb, kc, verdict, vbytes, zstride, run_if);
}

// One request whose slot travels in the kernel arguments (pv_latency_launch_zc_one): the runtime
// writes them next to the dispatch, so the slot is read from there at the kernel's start instead of
// from pinned host memory over PCIe.
__global__ __launch_bounds__(LAT4_THREADS) void pv_lat4_one_kernel(PvZcOne one, const uint32_t* __restrict__ bcomb,
                                                                   PvKeyCacheView kc, uint8_t* __restrict__ vbytes,
                                                                   uint32_t zstride) {
    lat4_body<true>(one.w, nullptr, nullptr, 1, nullptr, bcomb, kc, nullptr, vbytes, zstride, nullptr);
}

}  // namespace

#ifdef PV_LAT_TRACE
extern "C" int pv_debug_lat_trace(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pv_lat_trace_buf), sizeof(pv_lat_trace_buf)) == hipSuccess ? 0 : -1;
}
#endif

// Enqueue the latency path for n requests (device buffers as pv_verify_batch_device) on `stream`.
int pv_latency_launch(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk,
                      const void* d_bcomb, const PvKeyCacheView& kc, uint64_t* d_verdict, bool verdict_zeroed,
                      hipStream_t stream, const uint32_t* run_if) {
    if (n == 0) return PV_OK;
    if (n > 0x7FFFFFFFull) return pv_fail(PV_ERR_ARG, "pv_latency: too many requests for one launch");
    hipError_t e = hipSuccess;
    if (!verdict_zeroed) {  // the kernel ORs its bits into the words
        e = hipMemsetAsync(d_verdict, 0, (n + 63) / 64 * 8, stream);
        if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
    }
    if (n <= PV_LAT4_MAX)
        hipLaunchKernelGGL(pv_lat4_kernel<false>, dim3((unsigned)n), dim3(LAT4_THREADS), 0, stream, d_sm, d_off, n,
                           d_pk, reinterpret_cast<const uint32_t*>(d_bcomb), kc,
                           reinterpret_cast<unsigned long long*>(d_verdict), nullptr, 0u, run_if);
    else
        hipLaunchKernelGGL(pv_lat_kernel<false>, dim3((unsigned)n), dim3(LAT_THREADS), 0, stream, d_sm, d_off, n,
                           d_pk, reinterpret_cast<const uint32_t*>(d_bcomb), kc,
                           reinterpret_cast<unsigned long long*>(d_verdict), nullptr, 0u, run_if);
    e = hipGetLastError();
    if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("pv_lat_kernel: ") + hipGetErrorString(e));
    return PV_OK;
}

int pv_latency_launch_zc_one(const PvZcOne& one, uint32_t stride, const void* d_bcomb, const PvKeyCacheView& kc,
                             uint8_t* h_vbytes, hipStream_t stream) {
    if (stride % 64 || stride > sizeof(PvZcOne)) return pv_fail(PV_ERR_ARG, "pv_latency_launch_zc_one: bad slot size");
    hipLaunchKernelGGL(pv_lat4_one_kernel, dim3(1), dim3(LAT4_THREADS), 0, stream, one,
                       reinterpret_cast<const uint32_t*>(d_bcomb), kc, h_vbytes, stride);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("pv_lat4_one_kernel: ") + hipGetErrorString(e));
    return PV_OK;
}

int pv_latency_launch_zc(const uint8_t* h_slots, uint32_t stride, uint64_t n, const void* d_bcomb,
                         const PvKeyCacheView& kc, uint8_t* h_vbytes, hipStream_t stream) {
    if (n == 0) return PV_OK;
    if (n > PV_ZC_MAX_REQ) return pv_fail(PV_ERR_ARG, "pv_latency_launch_zc: too many requests");
    if (stride % 64 || stride > PV_ZC_MAX_STRIDE) return pv_fail(PV_ERR_ARG, "pv_latency_launch_zc: bad slot stride");
    if (n <= PV_LAT4_MAX)
        hipLaunchKernelGGL(pv_lat4_kernel<true>, dim3((unsigned)n), dim3(LAT4_THREADS), 0, stream, h_slots, nullptr, n,
                           nullptr, reinterpret_cast<const uint32_t*>(d_bcomb), kc, nullptr, h_vbytes, stride, nullptr);
    else
        hipLaunchKernelGGL(pv_lat_kernel<true>, dim3((unsigned)n), dim3(LAT_THREADS), 0, stream, h_slots, nullptr, n,
                           nullptr, reinterpret_cast<const uint32_t*>(d_bcomb), kc, nullptr, h_vbytes, stride, nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return pv_fail(PV_ERR_LAUNCH, std::string("pv_lat4_kernel<zc>: ") + hipGetErrorString(e));
    return PV_OK;
}
