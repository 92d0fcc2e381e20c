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

// Signed radix-16 digits of a < 2^253: a = sum e_i 16^i, e_i in [-8, 7] for i < 63, e_63 in [0, 2].
// Packed as 4-bit two's complement nibbles, digit i at bits [4i, 4i+4) of out[0..8).
PV_HD void sc_recode16(uint32_t out[8], const uint32_t a[8]) {
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t nib = (a[w] >> (4 * j)) & 15u;
            const uint32_t v = nib + carry;
            const bool last = (w == 7 && j == 7);
            carry = last ? 0u : ((v + 8u) >> 4);
            const uint32_t e = v - (carry << 4);  // mod 16 two's complement
            word |= (e & 15u) << (4 * j);
        }
        out[w] = word;
    }
}

// Signed radix-256 digits of a < 2^253: e_i in [-128, 127] for i < 31, e_31 in [0, 32].
// Packed as 8-bit two's complement bytes, digit i at bits [8i, 8i+8) of out[0..8).
PV_HD void sc_recode256(uint32_t out[8], const uint32_t a[8]) {
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t byte = (a[w] >> (8 * j)) & 255u;
            const uint32_t v = byte + carry;
            const bool last = (w == 7 && j == 3);
            carry = last ? 0u : ((v + 128u) >> 8);
            const uint32_t e = v - (carry << 8);
            word |= (e & 255u) << (8 * j);
        }
        out[w] = word;
    }
}

// Signed radix-65536 digits of a < 2^253: e_i in [-32768, 32767] for i < 15, e_15 in [0, 2^13].
// Packed as 16-bit two's complement halfwords, digit i at bits [16i, 16i+16) of out[0..8).
PV_HD void sc_recode65536(uint32_t out[8], const uint32_t a[8]) {
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint32_t h = (a[w] >> (16 * j)) & 0xFFFFu;
            const uint32_t v = h + carry;
            const bool last = (w == 7 && j == 1);
            carry = last ? 0u : ((v + 0x8000u) >> 16);
            const uint32_t e = v - (carry << 16);
            word |= (e & 0xFFFFu) << (16 * j);
        }
        out[w] = word;
    }
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
