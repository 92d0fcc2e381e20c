// Scalars modulo L = 2^252 + delta (the Ed25519 group order) for the gfx950 verify kernels.
//
// Replaces libsodium's sc25519_reduce / sc25519_is_canonical (reached from the reference via
// stp_core/crypto/nacl_wrappers.py:108 -> crypto_sign_open). Own formulation: 32-bit limbs,
// folding with 2^252 = -delta (mod L), delta < 2^125, kept non-negative by adding multiples of L:
//   x1 = lo252(h)  + L*2^133 - delta*hi(h)    (hi < 2^260)  -> x1 < 2^386
//   x2 = lo252(x1) + L*2^7   - delta*hi(x1)   (hi < 2^134)  -> x2 < 2^261
//   x3 = lo252(x2) + L       - delta*hi(x2)   (hi < 2^9)    -> 0 < x3 < 3L
//   then subtract L at most twice.
// Also: the signed-digit recodings the Straus loop consumes (radix 16 for k, radix 256 for S).
#pragma once
#include "fe25519.h"

static constexpr uint32_t SC_DELTA[4] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu};
static constexpr uint32_t SC_L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                     0x0u,        0x0u,        0x0u,        0x10000000u};
// L * 2^133 (386 bits, 13 words) and L * 2^7 (260 bits, 9 words)
static constexpr uint32_t SC_L133[13] = {0x0u, 0x0u, 0x0u, 0x0u, 0x9eba7da0u, 0x024c634bu, 0x5ef39acbu,
                                         0x9bdf3bd4u, 0x2u, 0x0u, 0x0u, 0x0u, 0x2u};
static constexpr uint32_t SC_L7[9] = {0x7ae9f680u, 0x09318d2eu, 0x7bce6b2cu, 0x6f7cef51u, 0xau,
                                      0x0u,        0x0u,        0x0u,        0x8u};

// x[0..N) >> 252 into hi[0..NH)
template <int N, int NH>
PV_HD void mp_hi252(uint32_t hi[NH], const uint32_t x[N]) {
#pragma unroll
    for (int i = 0; i < NH; i++) {
        const uint32_t a = (7 + i < N) ? x[7 + i] : 0u;
        const uint32_t b = (8 + i < N) ? x[8 + i] : 0u;
        hi[i] = (a >> 28) | (b << 4);
    }
}

// r[0..NR) = base[0..NR) + lo252(x) - delta * hi[0..NH); requires the true result in [0, 2^(32 NR)).
template <int NR, int NH>
PV_HD void mp_fold(uint32_t r[NR], const uint32_t base[NR], const uint32_t x[8], const uint32_t hi[NH]) {
    // p = delta * hi  (NH + 4 words)
    uint32_t p[NH + 4];
#pragma unroll
    for (int i = 0; i < NH + 4; i++) p[i] = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < NH; j++) {
            const uint64_t t = (uint64_t)SC_DELTA[i] * hi[j] + p[i + j] + carry;
            p[i + j] = (uint32_t)t;
            carry = (uint32_t)(t >> 32);
        }
        p[i + NH] = carry;
    }
    // r = base + lo - p
    uint64_t acc = 0;
    int64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < NR; i++) {
        uint32_t lo = (i < 7) ? x[i] : (i == 7 ? (x[7] & 0x0fffffffu) : 0u);
        acc = (uint64_t)base[i] + lo + (acc >> 32);
        const uint32_t pi = (i < NH + 4) ? p[i] : 0u;
        const int64_t d = (int64_t)(uint32_t)acc - (int64_t)pi + borrow;
        r[i] = (uint32_t)d;
        borrow = d >> 32;  // 0 or -1
    }
}

// r = x mod L, x = 64 little-endian bytes given as 16 words
PV_HD void sc_reduce64(uint32_t r[8], const uint32_t x[16]) {
    uint32_t hi1[9];
    mp_hi252<16, 9>(hi1, x);
    uint32_t x1[13];
    mp_fold<13, 9>(x1, SC_L133, x, hi1);
    uint32_t hi2[5];
    mp_hi252<13, 5>(hi2, x1);
    uint32_t x2[9];
    mp_fold<9, 5>(x2, SC_L7, x1, hi2);
    uint32_t hi3[1];
    mp_hi252<9, 1>(hi3, x2);
    uint32_t base3[8];
#pragma unroll
    for (int i = 0; i < 8; i++) base3[i] = SC_L[i];
    uint32_t x3[8];
    mp_fold<8, 1>(x3, base3, x2, hi3);
    // x3 < 3L: subtract L while x3 >= L (twice, branch-free)
#pragma unroll
    for (int rep = 0; rep < 2; rep++) {
        uint32_t t[8];
        int64_t borrow = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int64_t d = (int64_t)x3[i] - (int64_t)SC_L[i] + borrow;
            t[i] = (uint32_t)d;
            borrow = d >> 32;
        }
        const bool ge = borrow == 0;
#pragma unroll
        for (int i = 0; i < 8; i++) x3[i] = ge ? t[i] : x3[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = x3[i];
}

// 1 iff s < L (libsodium sc25519_is_canonical: full 256-bit compare)
PV_HD bool sc_is_canonical(const uint32_t s[8]) {
    int64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int64_t d = (int64_t)s[i] - (int64_t)SC_L[i] + borrow;
        borrow = d >> 32;
    }
    return borrow != 0;  // s - L < 0
}

// Signed radix-2^w digits (w = 4, 8, 16: digits in [-2^(w-1), 2^(w-1)), the top one unreduced) in
// closed form: with M = 2^(w-1) in every w-bit field, field i of (a + M) mod 2^256 is
// n_i + c_i + 2^(w-1) - 2^w c_(i+1), where c is exactly the digit-by-digit recoding's carry
// (c_(i+1) = [n_i + c_i >= 2^(w-1)]), so digit i = field i of (a + M) - 2^(w-1), and its w-bit two's
// complement is field i of (a + M) xor M: one multiword addition instead of a carry loop over the
// digits (~16 instructions against ~5 per digit; the same output for every 256-bit a).
template <uint32_t M>
PV_HD void sc_recode_add(uint32_t out[8], const uint32_t a[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const uint64_t t = (uint64_t)a[w] + M + c;
        out[w] = (uint32_t)t ^ M;
        c = t >> 32;
    }
}

// Signed radix-16 digits of a < 2^253: a = sum e_i 16^i, e_i in [-8, 7] for i < 63, e_63 in [0, 2].
// Packed as 4-bit two's complement nibbles, digit i at bits [4i, 4i+4) of out[0..8).
PV_HD void sc_recode16(uint32_t out[8], const uint32_t a[8]) { sc_recode_add<0x88888888u>(out, a); }

// Signed radix-256 digits of a < 2^253: e_i in [-128, 127] for i < 31, e_31 in [0, 32].
// Packed as 8-bit two's complement bytes, digit i at bits [8i, 8i+8) of out[0..8).
PV_HD void sc_recode256(uint32_t out[8], const uint32_t a[8]) { sc_recode_add<0x80808080u>(out, a); }

// Signed radix-65536 digits of a < 2^253: e_i in [-32768, 32767] for i < 15, e_15 in [0, 2^13].
// Packed as 16-bit two's complement halfwords, digit i at bits [16i, 16i+16) of out[0..8).
PV_HD void sc_recode65536(uint32_t out[8], const uint32_t a[8]) { sc_recode_add<0x80008000u>(out, a); }

// ---------------------------------------------------------------- half-size scalars (Straus path)
// The check encode([S]B - [k]A) == R is equivalent to D = [S]B - [k]A - R' = 0 once R decodes to R'
// with encode(R') == R. For any (k1, k2) with k1 == k k2 (mod 8L) and k2 odd, 0 < k2 < L:
//   [k2] D = [k2 S mod L] B - [k1] A - [k2] R'   (8L kills every point of the curve, B has order L)
// and [k2] D = 0 iff D = 0 (the group is cyclic of order 8L: a nonzero D of order dividing k2 would
// need L | k2 or a 2-power order dividing an odd k2). The short vector (k1, k2) of the lattice
// {(x, y) : x == k y mod 8L} has |k1|, k2 ~ 2^128 (sqrt(8L) = 2^127.5), so the variable-base part
// needs ~128 doublings instead of ~253 (T. Pornin, "Optimized lattice basis reduction in dimension 2,
// and fast Schnorr and EdDSA signature verification", ePrint 2020/454, uses the same split modulo L
// for cofactored checks; the modulus 8L and the odd k2 keep libsodium's cofactorless verdict exact
// for mixed-order A and R).
//
// sc_halfsize: the extended Euclidean algorithm on (8L, k) -- remainders r_i = k t_i (mod 8L), t_0 = 0,
// t_1 = 1 -- stopped at the first r_i < 2^128 whose t_i is odd. While r_i >= 2^131 the steps are taken
// in Lehmer blocks (Knuth, TAOCP 4.5.2, Algorithm L): ~9 quotients at a time from the leading 31 bits
// of the pair (single-precision reciprocal estimates fixed in integer arithmetic; a quotient is
// accepted only when both of Knuth's bracketing quotients agree), then ONE multiword update of (r, t)
// by the block's 2x2 matrix; the last few bits go by exact single steps
// (a double-precision quotient estimate corrected in exact multiword arithmetic). Every update applies
// the same integer matrix to r and to t (t in two's complement), so r_i = k t_i (mod 8L) holds whatever
// the quotients were; a step whose estimate cannot be settled (a quotient >= 2^32, |t| >= 2^168,
// r_i = 0, too many steps, a block that breaks 0 <= r_{i+1} < r_i) sends the lane to the always-valid
// split (k1, k2) = (k, 1), which costs the full-length loop but gives the same verdict.
static constexpr uint32_t SC_8L[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u,
                                      0x0u,        0x0u,        0x0u,        0x80000000u};
#ifndef PV_HALF_MAXIT
#define PV_HALF_MAXIT 64  // exact single steps (after the Lehmer blocks: ~3-12)
#endif
#ifndef PV_HALF_BLOCKS
#define PV_HALF_BLOCKS 24  // Lehmer blocks (~9 of 31 bits / ~6 of 53 bits from 2^255 to 2^131)
#endif
// PV_SC_SPLIT_53 = 1: Lehmer blocks on 53 leading bits with one division per quotient and
// Jebelean's conditions (~6 blocks); 0: 31-bit blocks with Knuth's two-division test (~10 blocks).
// Both settle only true quotients, so both give the same split.
#ifndef PV_SC_SPLIT_53
#define PV_SC_SPLIT_53 1
#endif
struct pv_halfk {
    uint32_t k1[8];  // |k1|
    uint32_t k2[8];  // k2: odd, > 0, < 2^160 (words 5..7 zero: sc_mul<5>)
    bool neg;        // k1 = -|k1|
    bool fallback;   // (k, 1) was used
};

PV_HD double sc_to_double(const uint32_t x[8]) {
    double d = (double)x[7];
#pragma unroll
    for (int i = 6; i >= 0; i--) d = d * 4294967296.0 + (double)x[i];
    return d;
}

// true on every lane of the wave (device) / the one lane (host)
PV_HD bool pv_wave_all(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __all(p);
#else
    return p;
#endif
}

// N-word two's complement helpers (arithmetic mod 2^(32 N))
template <int N>
PV_HD void mp_mulu32(uint32_t r[N], const uint32_t a[N], uint32_t m) {  // r = a m
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint64_t t = (uint64_t)a[i] * m + c;
        r[i] = (uint32_t)t;
        c = t >> 32;
    }
}
template <int N>
PV_HD void mp_muls32(uint32_t r[N], const uint32_t a[N], int64_t m) {  // r = a m, |m| < 2^32
    const bool neg = m < 0;
    mp_mulu32<N>(r, a, (uint32_t)(neg ? -m : m));
    uint64_t c = neg ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint64_t t = (uint64_t)(neg ? ~r[i] : r[i]) + c;
        r[i] = (uint32_t)t;
        c = t >> 32;
    }
}
template <int N>
PV_HD void mp_add(uint32_t r[N], const uint32_t a[N], const uint32_t b[N]) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint64_t t = (uint64_t)a[i] + b[i] + c;
        r[i] = (uint32_t)t;
        c = t >> 32;
    }
}
template <int N>
PV_HD void mp_sub(uint32_t r[N], const uint32_t a[N], const uint32_t b[N]) {
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const int64_t d = (int64_t)a[i] - (int64_t)b[i] + br;
        r[i] = (uint32_t)d;
        br = d >> 32;
    }
}
template <int N>
PV_HD bool mp_lt(const uint32_t a[N], const uint32_t b[N]) {  // unsigned a < b
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < N; i++) br = ((int64_t)a[i] - (int64_t)b[i] + br) >> 32;
    return br != 0;
}
// |t| < 2^168 for an 8-word two's complement t (bits 168..255 all equal the sign): one more step
// (|q| < 2^32) or block (|A|, |B| < 2^31) cannot wrap mod 2^256
PV_HD bool mp_small168(const uint32_t t[8]) {
    const uint32_t s = (int32_t)t[7] >> 31;
    return t[7] == s && t[6] == s && ((t[5] ^ s) >> 8) == 0;
}

// 1 / x to 1 ulp (v_rcp_f32 on the device)
PV_HD float pv_rcpf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// floor(n / d) for 0 <= n < 2^31, 0 < d < 2^31 from a single-precision reciprocal estimate, fixed by
// one exact step each way; ok = false (the caller ends its Lehmer block) for n < 0, d <= 0, a
// quotient >= 2^20 or an estimate one step could not fix
PV_HD uint32_t pv_qdiv31(int32_t n, int32_t d, bool& ok) {
    ok = n >= 0 && d > 0;
    const uint32_t un = ok ? (uint32_t)n : 0u, ud = ok ? (uint32_t)d : 1u;
#if defined(__HIP_DEVICE_COMPILE__)
    const float qf = (float)un * __builtin_amdgcn_rcpf((float)ud);
#else
    const float qf = (float)un / (float)ud;
#endif
    uint32_t q = qf < 1048576.0f ? (uint32_t)qf : 1048576u;
    uint64_t p = (uint64_t)q * ud;
    if (p > un) {
        q--;
        p -= ud;
    }
    if (p + ud <= un) {
        q++;
        p += ud;
    }
    ok = ok && q < 1048576u && p <= un && p + ud > un;
    return q;
}

// stats (measurement only, nullptr otherwise): [0] Lehmer blocks, [1] quotients settled inside them,
// [2] exact single steps
PV_HD void sc_halfsize(pv_halfk& h, const uint32_t k[8], uint32_t* stats = nullptr) {
    uint32_t r0[9], r1[9], t0[8], t1[8];  // r: 9 words (word 8 = 0 for a valid state)
#pragma unroll
    for (int i = 0; i < 9; i++) {
        r0[i] = i < 8 ? SC_8L[i] : 0u;
        r1[i] = i < 8 ? k[i] : 0u;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        t0[i] = 0;
        t1[i] = i == 0 ? 1u : 0u;
    }
    bool bad = false;
    // ---- Lehmer blocks while r1 >= 2^131
    for (int blk = 0; blk < PV_HALF_BLOCKS; blk++) {
        const bool act = !bad && ((r1[4] >> 3) | r1[5] | r1[6] | r1[7]) != 0;
        if (pv_wave_all(!act)) break;
        if (!act) continue;
#if PV_SC_SPLIT_53
        // 53 leading bits (exact doubles), one division per quotient, Jebelean's conditions on the
        // sign-free cosequence (the same block as lp25519.h lp_halfsize, per lane)
        int w = 4;
#pragma unroll
        for (int i = 5; i < 8; i++) w = r0[i] ? i : w;
        uint32_t a1 = 0, a0 = 0, a2 = 0, b1 = 0, b0 = 0, b2 = 0;
#pragma unroll
        for (int i = 4; i < 8; i++) {
            a1 = i == w ? r0[i] : a1;
            a0 = i == w ? r0[i - 1] : a0;
            a2 = i == w ? r0[i - 2] : a2;
            b1 = i == w ? r1[i] : b1;
            b0 = i == w ? r1[i - 1] : b0;
            b2 = i == w ? r1[i - 2] : b2;
        }
        const int s = 43 - (int)__builtin_clz(a1);
        const uint64_t ah = ((uint64_t)a1 << 32) | a0, bh = ((uint64_t)b1 << 32) | b0;
        const uint64_t xi = s <= 32 ? (ah << (32 - s)) | ((uint64_t)a2 >> s) : ah >> (s - 32);
        const uint64_t yi = s <= 32 ? (bh << (32 - s)) | ((uint64_t)b2 >> s) : bh >> (s - 32);
        const int e = 32 * (w - 2) + s;
        const double ythr = e >= 130 ? 1.0 : (double)(1ull << (130 - e));
        double x = (double)xi, y = (double)yi, Px = 1.0, Nx = 0.0, Py = 1.0, Ny = 0.0;
        int n = 0;
        bool go = true;
#define SC_QSTEP(U, V, PU, NU, PV, NV)                                                                       \
    {                                                                                                        \
        double q = (double)__builtin_floorf((float)U * pv_rcpf((float)V));                                   \
        double nr = __builtin_fma(-q, V, U);                                                                 \
        const bool lo_ = nr < 0.0;                                                                           \
        q = lo_ ? q - 1.0 : q;                                                                               \
        nr = lo_ ? nr + V : nr;                                                                              \
        const bool hi_ = nr >= V;                                                                            \
        q = hi_ ? q + 1.0 : q;                                                                               \
        nr = hi_ ? nr - V : nr;                                                                              \
        const double nP = __builtin_fma(q, NV, PU), nN = __builtin_fma(q, PV, NU);                           \
        go = (q < 2097152.0) & (nr >= ythr) & (nr >= nN) & (V - nr >= NV + nP) & (nP + nN < 2147483648.0);  \
        if (go) {                                                                                            \
            U = nr;                                                                                          \
            PU = nP;                                                                                         \
            NU = nN;                                                                                         \
            n++;                                                                                             \
            if (stats) stats[1]++;                                                                           \
        }                                                                                                    \
    }
        for (int it = 0; it < 48; it++) {
            if (pv_wave_all(!go)) break;
            if (go) SC_QSTEP(x, y, Px, Nx, Py, Ny)
            if (go) SC_QSTEP(y, x, Py, Ny, Px, Nx)
        }
#undef SC_QSTEP
        // rows n (A, B) and n + 1 (C, D): slot x holds the even row (P, -N), slot y the odd (-N, P)
        const int64_t A = (n & 1) ? -(int64_t)Ny : (int64_t)Px, B = (n & 1) ? (int64_t)Py : -(int64_t)Nx;
        const int64_t C = (n & 1) ? (int64_t)Px : -(int64_t)Ny, D = (n & 1) ? -(int64_t)Nx : (int64_t)Py;
#else
        // leading bits: xh = floor(r0 / 2^e), yh = floor(r1 / 2^e), 2^30 <= xh < 2^31 (r0 >= 2^131: w >= 4)
        int w = 4;
#pragma unroll
        for (int i = 5; i < 8; i++) w = r0[i] ? i : w;
        uint32_t a1 = 0, a0 = 0, b1 = 0, b0 = 0;
#pragma unroll
        for (int i = 4; i < 8; i++) {
            a1 = i == w ? r0[i] : a1;
            a0 = i == w ? r0[i - 1] : a0;
            b1 = i == w ? r1[i] : b1;
            b0 = i == w ? r1[i - 1] : b0;
        }
        const int s = 33 - (int)__builtin_clz(a1);  // (a1:a0) has 64 - clz bits; keep the top 31
        const int32_t xh0 = (int32_t)((((uint64_t)a1 << 32) | a0) >> s);
        const int32_t yh0 = (int32_t)((((uint64_t)b1 << 32) | b0) >> s);
        // stop a block above 2^130: yh < 2^(130 - e), e = 32 (w - 1) + s (>= 100 here)
        const int e = 32 * (w - 1) + s;
        const int32_t ythr = e >= 130 ? 1 : (int32_t)(1u << (130 - e));
        int32_t xh = xh0, yh = yh0, A = 1, B = 0, C = 0, D = 1;
        bool go = true;
        for (int it = 0; it < 24; it++) {
            if (pv_wave_all(!go)) break;
            if (!go) continue;
            // Knuth's test: the quotient of (xh + A) / (yh + C) and of (xh + B) / (yh + D) agree
            const int32_t n1 = xh + A, d1 = yh + C, n2 = xh + B, d2 = yh + D;
            bool ok1, ok2;
            const uint32_t q = pv_qdiv31(n1, d1, ok1);
            const uint32_t q2 = pv_qdiv31(n2, d2, ok2);
            if (!ok1 || !ok2 || q != q2) {
                go = false;
                continue;
            }
            const int64_t ny = (int64_t)xh - (int64_t)q * yh;
            const int64_t nC = (int64_t)A - (int64_t)q * C, nD = (int64_t)B - (int64_t)q * D;
            if (ny < ythr || nC >= 32768 || nC <= -32768 || nD >= 32768 || nD <= -32768) {
                go = false;
                continue;
            }
            A = C;
            C = (int32_t)nC;
            B = D;
            D = (int32_t)nD;
            xh = yh;
            yh = (int32_t)ny;
            if (stats) stats[1]++;
        }
#endif
        if (stats) stats[0]++;
        if (B == 0) {
            // no quotient could be settled from the leading bits: one exact step below
            // (the block loop then continues from the new pair)
            const double qd = sc_to_double(r0) / sc_to_double(r1);
            bad |= !(qd < 4294967295.0);
            uint32_t q = bad ? 0u : (uint32_t)qd;
            uint32_t p[9], rn[9];
            mp_mulu32<9>(p, r1, q);
            mp_sub<9>(rn, r0, p);
            if ((int32_t)rn[8] < 0) {
                mp_add<9>(rn, rn, r1);
                q--;
            }
            if (!mp_lt<9>(rn, r1)) {
                mp_sub<9>(rn, rn, r1);
                q++;
            }
            bad |= (int32_t)rn[8] < 0 || !mp_lt<9>(rn, r1);
            uint32_t qt[8], tn[8];
            mp_mulu32<8>(qt, t1, q);
            mp_sub<8>(tn, t0, qt);
#pragma unroll
            for (int i = 0; i < 9; i++) {
                r0[i] = r1[i];
                r1[i] = rn[i];
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                t0[i] = t1[i];
                t1[i] = tn[i];
            }
        } else {
            uint32_t u[9], v[9], nr0[9], nr1[9], nt0[8], nt1[8], x[8], y[8];
            mp_muls32<9>(u, r0, A);  // |A|, |B|, |C|, |D| < 2^31
            mp_muls32<9>(v, r1, B);
            mp_add<9>(nr0, u, v);
            mp_muls32<9>(u, r0, C);
            mp_muls32<9>(v, r1, D);
            mp_add<9>(nr1, u, v);
            mp_muls32<8>(x, t0, A);
            mp_muls32<8>(y, t1, B);
            mp_add<8>(nt0, x, y);
            mp_muls32<8>(x, t0, C);
            mp_muls32<8>(y, t1, D);
            mp_add<8>(nt1, x, y);
            bad |= (int32_t)nr0[8] < 0 || (int32_t)nr1[8] < 0 || !mp_lt<9>(nr1, nr0);
#pragma unroll
            for (int i = 0; i < 9; i++) {
                r0[i] = nr0[i];
                r1[i] = nr1[i];
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                t0[i] = nt0[i];
                t1[i] = nt1[i];
            }
        }
        bad |= !mp_small168(t1) || !mp_small168(t0);
    }
    // ---- exact single steps until r1 < 2^128 with t1 odd
    bool done = ((r1[4] | r1[5] | r1[6] | r1[7]) == 0) && (t1[0] & 1u);
    for (int it = 0; it < PV_HALF_MAXIT; it++) {
        if (pv_wave_all(done || bad)) break;
        if (done || bad) continue;
        if (stats) stats[2]++;
        const double qd = sc_to_double(r0) / sc_to_double(r1);  // r1 = 0: +inf -> bad
        bad |= !(qd < 4294967295.0);
        uint32_t q = bad ? 0u : (uint32_t)qd;
        uint32_t p[9], rn[9];
        mp_mulu32<9>(p, r1, q);
        mp_sub<9>(rn, r0, p);
        // estimate one too high: rn < 0 -> rn += r1, q -= 1; one too low: rn >= r1 -> rn -= r1, q += 1
        {
            const bool lo = (int32_t)rn[8] < 0;
            uint32_t ra[9];
            mp_add<9>(ra, rn, r1);
#pragma unroll
            for (int i = 0; i < 9; i++) rn[i] = lo ? ra[i] : rn[i];
            bad |= lo && q == 0u;
            q -= lo ? 1u : 0u;
        }
        {
            uint32_t rs[9];
            mp_sub<9>(rs, rn, r1);
            const bool ge = (int32_t)rs[8] >= 0;
#pragma unroll
            for (int i = 0; i < 9; i++) rn[i] = ge ? rs[i] : rn[i];
            bad |= ge && q == 0xFFFFFFFFu;
            q += ge ? 1u : 0u;
        }
        bad |= (int32_t)rn[8] < 0 || !mp_lt<9>(rn, r1);
        uint32_t qt[8], tn[8];
        mp_mulu32<8>(qt, t1, q);
        mp_sub<8>(tn, t0, qt);
        bad |= !mp_small168(tn);
#pragma unroll
        for (int i = 0; i < 9; i++) {
            r0[i] = r1[i];
            r1[i] = rn[i];
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            t0[i] = t1[i];
            t1[i] = tn[i];
        }
        done = ((r1[4] | r1[5] | r1[6] | r1[7]) == 0) && (t1[0] & 1u);
    }
    // k2 = |t1|, k1 = r1 with t1's sign moved onto it
    const bool tneg = (int32_t)t1[7] < 0;
    uint32_t ta[8];
    {
        uint64_t c = tneg ? 1u : 0u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint64_t t = (uint64_t)(tneg ? ~t1[i] : t1[i]) + c;
            ta[i] = (uint32_t)t;
            c = t >> 32;
        }
    }
    const bool ok = done && !bad && (ta[5] | ta[6] | ta[7]) == 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        h.k1[i] = ok ? r1[i] : k[i];
        h.k2[i] = ok ? ta[i] : (i == 0 ? 1u : 0u);
    }
    h.neg = ok && tneg;
    h.fallback = !ok;
}

// r = a * b mod L (a, b < 2^256)
// NA: words of a that may be nonzero (a[NA..7] = 0: the split's k2 < 2^160 takes NA = 5, 40
// word products instead of 64)
template <int NA = 8>
PV_HD void sc_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
    for (int i = 0; i < NA; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + c;
            x[i + j] = (uint32_t)t;
            c = t >> 32;
        }
        x[i + 8] = (uint32_t)c;
    }
    sc_reduce64(r, x);
}

// Windows the radix-16 loop needs for packed digits e (sc_recode16): 1 + the highest nonzero digit.
PV_HD int sc_nwin16(const uint32_t e[8]) {
    int nw = 1;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        if (e[w]) {
            const int top = 31 - (int)__builtin_clz(e[w]);  // highest set bit
            nw = 8 * w + top / 4 + 1;
        }
    }
    return nw;
}

// Bits [lo, lo + n) of the 256-bit little-endian a (n <= 32).
PV_HD uint32_t sc_bits(const uint32_t a[8], int lo, int n) {
    const int i = lo >> 5, sh = lo & 31;
    uint32_t x = a[i] >> sh;
    if (sh && i + 1 < 8) x |= a[i + 1] << (32 - sh);
    return n < 32 ? x & ((1u << n) - 1u) : x;
}

// Signed radix-2^W digits of a scalar for the wide fixed-base comb (comb.h, PV_BC2_*): P positions,
// e_j in [-2^(W-1), 2^(W-1)) for j < P - 1 and the top digit e_{P-1} in [0, 2^TOP] for a < 2^253
// (TOP = 253 - W (P - 1)). For a >= 2^253 -- S >= L, which libsodium rejects before any point
// arithmetic (sc25519_is_canonical), so the verdict is false whatever Q is -- the top digit is clamped
// to 2^TOP so that the table lookup stays inside the top row. For W = 16 the digits are exactly
// sc_recode65536's (same carry rule).
template <int W, int P>
PV_HD void sc_recode_w(int32_t out[P], const uint32_t a[8]) {
    constexpr int TOP = 253 - W * (P - 1);
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < P - 1; j++) {
        const uint32_t v = sc_bits(a, W * j, W) + carry;
        carry = (v + (1u << (W - 1))) >> W;
        out[j] = (int32_t)v - (int32_t)(carry << W);
    }
    uint32_t top = sc_bits(a, W * (P - 1), 256 - W * (P - 1)) + carry;
    if (top > (1u << TOP)) top = 1u << TOP;
    out[P - 1] = (int32_t)top;
}
