// GF(2^255-19) arithmetic for the gfx950 Ed25519 verification kernels.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i has weight 2^ceil(25.5 i):
// even limbs carry 26 bits, odd limbs 25 bits). Products are formed with v_mad_u64_u32
// (32x32 -> 64 multiply + 64-bit accumulate in one instruction, 4 cycles per wave64 instruction
// on gfx950 - profiles/r01_isa_rates_full.jsonl). 5x51-bit limbs would need 64x64 -> 128 products
// that the VALU does not have.
//
// Multiplication is PRODUCT-SCANNING: column k of the (19-folded) schoolbook product is one
// v_mad_u64_u32 chain whose accumulator starts at the carry out of column k-1, so carrying costs
// one v_lshrrev_b64 + one v_and_b32 per limb and no separate 64-bit adds. The wrapped products
// use 19*g (computed once per operand by the caller when it is shared, fe_mul_pre) and odd x odd
// products use 2*f. Each column stays a single v_mad_u64_u32 chain on the device (PV_MAD_CHAIN
// below).
//
// Bound discipline (asserted by the PV_BOUNDS_CHECK host build, tests/test_native_host.py):
//   "R" reduced: limb < 2^width + 2^17. Output of fe_mul / fe_sq / fe_carry.
//   fe_mul(h, f, g): g limbs < PV_GMAX (19 g < 2^32); f limbs < 2^31; every column < 2^64
//                    (checked exactly in the host build; all terms are non-negative, so max-limb
//                    inputs are the worst case and the tests feed them).
//   fe_sq(h, f):     f limbs < PV_GMAX.
//   fe_add / fe_sub / fe_sub4p: plain limb arithmetic, see each function.
//   fe_carry:        any limbs < 2^32 -> R.
// This file replaces libsodium's fe25519 (ref10, radix 2^25.5 signed limbs), which the reference
// reaches via stp_core/crypto/nacl_wrappers.py:108 -> libnacl.crypto_sign_open.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PV_HD __host__ __device__ __forceinline__

struct fe {
    uint32_t v[10];
};

#ifdef PV_BOUNDS_CHECK
#include <stdio.h>
#include <stdlib.h>
#define PV_ASSERT(c, msg) do { if (!(c)) { fprintf(stderr, "bound violated: %s\n", msg); abort(); } } while (0)
#else
#define PV_ASSERT(c, msg) do { } while (0)
#endif

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;
// largest limb a 19-multiplied operand may have: 19 * PV_GMAX < 2^32
static constexpr uint32_t PV_GMAX = 0xD000000u;

PV_HD void fe_check_g(const fe& g) {
#ifdef PV_BOUNDS_CHECK
    for (int i = 0; i < 10; i++) PV_ASSERT(g.v[i] < PV_GMAX, "mul g operand");
#else
    (void)g;
#endif
}
PV_HD void fe_check_reduced(const fe& f) {
#ifdef PV_BOUNDS_CHECK
    for (int i = 0; i < 10; i++)
        PV_ASSERT(f.v[i] < ((i & 1) ? (1u << 25) : (1u << 26)) + (1u << 17), "reduced");
#else
    (void)f;
#endif
}

// ------------------------------------------------------------------ VALU primitives
// acc + a*b (64-bit) and a*b: one v_mad_u64_u32 each on the device.
// PV_MAD_CHAIN: each product-scanning column stays ONE chain of v_mad_u64_u32 (the accumulator of
// every mad is the previous mad's result). Left alone, the compiler re-associates a column into two
// chains joined by a v_lshl_add_u64 (one extra 4-cycle VOP3 per column, ~80 per point addition); an
// empty non-volatile asm on each partial sum hides the algebra from it without emitting anything or
// constraining the schedule beyond the data dependence. (PV_MAD_ASM: the mad itself as inline asm,
// kept for comparison: hipcc then pads the opaque instructions with hazard s_nops.)
#ifndef PV_MAD_CHAIN
#define PV_MAD_CHAIN 1
#endif
#ifndef PV_MAD_ASM
#define PV_MAD_ASM 0
#endif
PV_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && PV_MAD_ASM
    uint64_t r, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
    return r;
#elif defined(__HIP_DEVICE_COMPILE__) && PV_MAD_CHAIN
    uint64_t r = (uint64_t)a * b + c;
    asm("" : "+v"(r));
    return r;
#else
    return (uint64_t)a * b + c;
#endif
}
PV_HD uint64_t mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }
// PV_MAD_COLASM: each product-scanning column is ONE inline-asm block of N dependent
// v_mad_u64_u32 (accumulator in place). The per-mad empty asm of PV_MAD_CHAIN keeps the chain but
// the hazard recognizer cannot see through inline asm and pads EVERY mad that follows one with an
// `s_nop 0` (it assumes the asm may have been a transcendental op writing the VGPR: ~100 s_nop per
// field multiplication). A whole column per block leaves at most one pad per column. Device only.
#ifndef PV_MAD_COLASM
#define PV_MAD_COLASM 1
#endif
#define PV_MA(a, b) "v_mad_u64_u32 %0, %1, %" #a ", %" #b ", %0\n\t"
#define PV_M0(a, b) "v_mad_u64_u32 %0, %1, %" #a ", %" #b ", 0\n\t"
// acc (+)= sum_i a[i] * b[i], N terms; FIRST: acc starts at 0 (the first mad adds the constant 0)
template <int N, bool FIRST>
__device__ __forceinline__ void pv_madcol(uint64_t& acc, const uint32_t* a, const uint32_t* b) {
    uint64_t cc;
    if constexpr (N == 10 && FIRST) {
        asm(PV_M0(2, 12) PV_MA(3, 13) PV_MA(4, 14) PV_MA(5, 15) PV_MA(6, 16) PV_MA(7, 17) PV_MA(8, 18)
                PV_MA(9, 19) PV_MA(10, 20) PV_MA(11, 21)
            : "=&v"(acc), "=&s"(cc)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]),
              "v"(a[9]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]),
              "v"(b[8]), "v"(b[9]));
    } else if constexpr (N == 10) {
        asm(PV_MA(2, 12) PV_MA(3, 13) PV_MA(4, 14) PV_MA(5, 15) PV_MA(6, 16) PV_MA(7, 17) PV_MA(8, 18)
                PV_MA(9, 19) PV_MA(10, 20) PV_MA(11, 21)
            : "+v"(acc), "=&s"(cc)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]),
              "v"(a[9]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]),
              "v"(b[8]), "v"(b[9]));
    } else if constexpr (N == 6 && FIRST) {
        asm(PV_M0(2, 8) PV_MA(3, 9) PV_MA(4, 10) PV_MA(5, 11) PV_MA(6, 12) PV_MA(7, 13)
            : "=&v"(acc), "=&s"(cc)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(b[0]), "v"(b[1]), "v"(b[2]),
              "v"(b[3]), "v"(b[4]), "v"(b[5]));
    } else if constexpr (N == 6) {
        asm(PV_MA(2, 8) PV_MA(3, 9) PV_MA(4, 10) PV_MA(5, 11) PV_MA(6, 12) PV_MA(7, 13)
            : "+v"(acc), "=&s"(cc)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(b[0]), "v"(b[1]), "v"(b[2]),
              "v"(b[3]), "v"(b[4]), "v"(b[5]));
    } else if constexpr (N == 5 && !FIRST) {
        asm(PV_MA(2, 7) PV_MA(3, 8) PV_MA(4, 9) PV_MA(5, 10) PV_MA(6, 11)
            : "+v"(acc), "=&s"(cc)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]),
              "v"(b[4]));
    } else {
        static_assert(N == 10 || N == 6 || (N == 5 && !FIRST), "pv_madcol: unsupported column shape");
    }
}
#undef PV_MA
#undef PV_M0

// Opaque copy: stops the compiler from re-associating a column sum so that the carry from the
// previous column is added by a separate v_lshl_add_u64 instead of entering the first
// v_mad_u64_u32 of the column as its accumulator (no instruction is emitted).
PV_HD uint64_t pv_opaque64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && !PV_MAD_ASM && !PV_MAD_CHAIN
    asm volatile("" : "+v"(x));
#endif
    return x;
}
// 2x as a VOP2 add (2 cycles per wave64 instruction) rather than the VOP3-rate shift the compiler
// picks for x << 1.
PV_HD uint32_t dbl32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return x + x;
#endif
}

// Keeps the machine scheduler from interleaving too many independent field multiplications past
// the VGPR budget (each one has 55-100 mads, ample ILP at 3 waves/SIMD).
PV_HD void pv_sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// ------------------------------------------------------------------ limb helpers
PV_HD void fe_0(fe& h) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = 0;
}
PV_HD void fe_1(fe& h) {
    fe_0(h);
    h.v[0] = 1;
}
PV_HD void fe_copy(fe& h, const fe& f) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i];
}
PV_HD void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}
// h = f + 2p - g, g reduced (R)
PV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
    fe_check_reduced(g);
    h.v[0] = f.v[0] + 0x7FFFFDAu - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu) - g.v[i];
}
// h = f + 4p - g for g with even limbs < 2^28, odd < 2^27 (e.g. a sum of two R values).
PV_HD void fe_sub4p(fe& h, const fe& f, const fe& g) {
#ifdef PV_BOUNDS_CHECK
    for (int i = 0; i < 10; i++) PV_ASSERT(g.v[i] <= ((i & 1) ? 0x7FFFFFCu : 0xFFFFFB4u), "sub4p operand");
#endif
    h.v[0] = f.v[0] + 0xFFFFFB4u - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? 0x7FFFFFCu : 0xFFFFFFCu) - g.v[i];
}
// conditional negate of a reduced value: h = neg ? 2p - f : f (result < 2^27 even, valid g operand)
PV_HD void fe_cneg(fe& h, const fe& f, bool neg) {
    fe n, z;
    fe_0(z);
    fe_sub(n, z, f);
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = neg ? n.v[i] : f.v[i];
}
PV_HD void fe_cmov(fe& h, const fe& f, bool c) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = c ? f.v[i] : h.v[i];
}

// One parallel carry pass: any limbs < 2^32 -> R (every carry < 2^7, 19 * carry9 < 2^12).
PV_HD void fe_carry(fe& h, const fe& f) {
    uint32_t c[10], t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        c[i] = f.v[i] >> ((i & 1) ? 25 : 26);
        t[i] = f.v[i] & ((i & 1) ? M25 : M26);
    }
    h.v[0] = t[0] + 19u * c[9];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = t[i] + c[i - 1];
    fe_check_reduced(h);
}

// ------------------------------------------------------------------ multiplication
#ifdef PV_BOUNDS_CHECK
#define PV_COL_TRACK(k, a, b) col128[k] += (unsigned __int128)(a) * (b)
#else
#define PV_COL_TRACK(k, a, b) do { } while (0)
#endif

// Folds the carry out of limb 9 (c9 < 2^40) back into limbs 0 and 1: h0 + 19 c9 < 2^45, its carry
// into limb 1 < 2^19, so the result is R.
PV_HD void fe_wrap_carry(fe& h, uint64_t c9) {
    uint64_t r = mad64((uint32_t)c9, 19u, (uint64_t)h.v[0]);
    r += (uint64_t)((uint32_t)(c9 >> 32) * 19u) << 32;
    h.v[0] = (uint32_t)r & M26;
    h.v[1] += (uint32_t)(r >> 26);
}

PV_HD void fe_mul19(uint32_t g19[10], const fe& g) {
    fe_check_g(g);
#pragma unroll
    for (int i = 0; i < 10; i++) g19[i] = 19u * g.v[i];
}

// h = f * g with g19 = 19 * g precomputed (shared operands pay the 10 v_mul_lo_u32 once).
PV_HD void fe_mul_pre(fe& hout, const fe& f, const fe& g, const uint32_t g19[10]) {
    fe_check_g(g);
    fe h;  // hout may alias f or g
    uint32_t f2[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        f2[i] = (i & 1) ? dbl32(f.v[i]) : f.v[i];
        PV_ASSERT(f.v[i] < 0x80000000u, "mul f operand");
    }
#ifdef PV_BOUNDS_CHECK
    unsigned __int128 col128[10] = {0};
#endif
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        uint32_t ca[10], cb[10];
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int j = k - i;
            uint32_t a, b;
            if (j >= 0) {
                a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
                b = g.v[j];
            } else {
                a = ((i & 1) && ((j + 10) & 1)) ? f2[i] : f.v[i];
                b = g19[j + 10];
            }
            PV_COL_TRACK(k, a, b);
            ca[i] = a;
            cb[i] = b;
        }
#if defined(__HIP_DEVICE_COMPILE__) && PV_MAD_COLASM
        if (k == 0) pv_madcol<10, true>(acc, ca, cb);
        else pv_madcol<10, false>(acc, ca, cb);
#else
#pragma unroll
        for (int i = 0; i < 10; i++) {
            acc = (k == 0 && i == 0) ? mul64(ca[i], cb[i]) : mad64(ca[i], cb[i], acc);
            if (i == 0 && k > 0) acc = pv_opaque64(acc);
        }
#endif
#ifdef PV_BOUNDS_CHECK
        if (k > 0) col128[k] += col128[k - 1] >> ((k & 1) ? 26 : 25);
        PV_ASSERT((col128[k] >> 64) == 0, "mul column overflow");
#endif
        const int sh = (k & 1) ? 25 : 26;
        h.v[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
        acc >>= sh;
    }
    fe_wrap_carry(h, acc);
    fe_check_reduced(h);
    hout = h;
}

PV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
    uint32_t g19[10];
    fe_mul19(g19, g);
    fe_mul_pre(h, f, g, g19);
    pv_sched_fence();
}

// h = f^2: 55 products, column by column (pairs i <= j with i + j = k or k + 10).
PV_HD void fe_sq(fe& hout, const fe& f) {
    fe_check_g(f);
    fe h;  // hout may alias f
    uint32_t f2[10], f4[10], f19[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        f2[i] = dbl32(f.v[i]);
        f4[i] = dbl32(f2[i]);
        f19[i] = 19u * f.v[i];
    }
#ifdef PV_BOUNDS_CHECK
    unsigned __int128 col128[10] = {0};
#endif
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        uint32_t ca[6], cb[6];
        int nt = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
#pragma unroll
            for (int wrap = 0; wrap < 2; wrap++) {
                const int j = k + 10 * wrap - i;
                if (j < i || j > 9) continue;
                // coefficient (i == j ? 1 : 2) * (i, j both odd ? 2 : 1) * (wrapped ? 19 : 1)
                const int c = (i == j ? 1 : 2) * (((i & j) & 1) ? 2 : 1);
                const uint32_t a = (c == 1) ? f.v[i] : (c == 2 ? f2[i] : f4[i]);
                const uint32_t b = wrap ? f19[j] : f.v[j];
                PV_COL_TRACK(k, a, b);
                ca[nt] = a;
                cb[nt] = b;
                nt++;
            }
        }
        // even columns have 6 terms, odd columns 5
#if defined(__HIP_DEVICE_COMPILE__) && PV_MAD_COLASM
        if (k == 0) pv_madcol<6, true>(acc, ca, cb);
        else if (k & 1) pv_madcol<5, false>(acc, ca, cb);
        else pv_madcol<6, false>(acc, ca, cb);
#else
#pragma unroll
        for (int t = 0; t < 6 - (k & 1); t++) {
            acc = (k == 0 && t == 0) ? mul64(ca[t], cb[t]) : mad64(ca[t], cb[t], acc);
            if (t == 0 && k > 0) acc = pv_opaque64(acc);
        }
#endif
#ifdef PV_BOUNDS_CHECK
        if (k > 0) col128[k] += col128[k - 1] >> ((k & 1) ? 26 : 25);
        PV_ASSERT((col128[k] >> 64) == 0, "sq column overflow");
#endif
        const int sh = (k & 1) ? 25 : 26;
        h.v[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
        acc >>= sh;
    }
    fe_wrap_carry(h, acc);
    fe_check_reduced(h);
    hout = h;
    pv_sched_fence();
}

// h = f^(2^n)
PV_HD void fe_sqn(fe& h, const fe& f, int n) {
    fe_sq(h, f);
#pragma nounroll
    for (int i = 1; i < n; i++) fe_sq(h, h);
}

// Fully reduce to the canonical representative in [0, p) and pack into 8 little-endian words.
PV_HD void fe_tobytes32(uint32_t s[8], const fe& f) {
    fe h;
    fe_carry(h, f);
    // two normalisation passes (each with the 2^255 -> 19 wrap) leave every limb strictly inside
    // its width and the value in [0, 2^255)
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = h.v[i];
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const int sh = (i & 1) ? 25 : 26;
            t[i + 1] += t[i] >> sh;
            t[i] &= (i & 1) ? M25 : M26;
        }
        t[0] += (t[9] >> 25) * 19u;
        t[9] &= M25;
    }
    // now value v in [0, 2^255); v >= p iff v + 19 >= 2^255
    uint32_t q = (t[0] + 19u) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++) q = (t[i] + q) >> ((i & 1) ? 25 : 26);
    t[0] += 19u * q;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int sh = (i & 1) ? 25 : 26;
        t[i + 1] += t[i] >> sh;
        t[i] &= (i & 1) ? M25 : M26;
    }
    t[9] &= M25;  // drops 2^255 when q = 1
    // pack: offsets 0,26,51,77,102,128,153,179,204,230
    s[0] = t[0] | (t[1] << 26);
    s[1] = (t[1] >> 6) | (t[2] << 19);
    s[2] = (t[2] >> 13) | (t[3] << 13);
    s[3] = (t[3] >> 19) | (t[4] << 6);
    s[4] = t[5] | (t[6] << 25);
    s[5] = (t[6] >> 7) | (t[7] << 19);
    s[6] = (t[7] >> 13) | (t[8] << 12);
    s[7] = (t[8] >> 20) | (t[9] << 6);
}

// Load 255 bits (bit 255 ignored) from 8 little-endian words; the value may be >= p (non-canonical),
// exactly like libsodium's fe25519_frombytes.
PV_HD void fe_frombytes32(fe& h, const uint32_t s[8]) {
    h.v[0] = s[0] & M26;
    h.v[1] = ((s[0] >> 26) | (s[1] << 6)) & M25;
    h.v[2] = ((s[1] >> 19) | (s[2] << 13)) & M26;
    h.v[3] = ((s[2] >> 13) | (s[3] << 19)) & M25;
    h.v[4] = (s[3] >> 6) & M26;
    h.v[5] = s[4] & M25;
    h.v[6] = ((s[4] >> 25) | (s[5] << 7)) & M26;
    h.v[7] = ((s[5] >> 19) | (s[6] << 13)) & M25;
    h.v[8] = ((s[6] >> 12) | (s[7] << 20)) & M26;
    h.v[9] = (s[7] >> 6) & M25;
}

PV_HD bool fe_iszero(const fe& f) {
    uint32_t s[8];
    fe_tobytes32(s, f);
    uint32_t z = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) z |= s[i];
    return z == 0;
}
PV_HD uint32_t fe_isnegative(const fe& f) {
    uint32_t s[8];
    fe_tobytes32(s, f);
    return s[0] & 1;
}

// z^(2^250 - 1) and z^11 helper shared by invert and pow22523 (standard addition chain).
PV_HD void fe_pow_2_250_1(fe& out, fe& z11, const fe& z) {
    fe t0, t1, t2;
    fe_sq(t0, z);            // z^2
    fe_sqn(t1, t0, 2);       // z^8
    fe_mul(t1, z, t1);       // z^9
    fe_mul(z11, t0, t1);     // z^11
    fe_sq(t2, z11);          // z^22
    fe_mul(t1, t1, t2);      // z^(2^5 - 1)
    fe_sqn(t2, t1, 5);
    fe_mul(t1, t2, t1);      // z^(2^10 - 1)
    fe_sqn(t2, t1, 10);
    fe_mul(t2, t2, t1);      // z^(2^20 - 1)
    fe_sqn(t0, t2, 20);
    fe_mul(t2, t0, t2);      // z^(2^40 - 1)
    fe_sqn(t2, t2, 10);
    fe_mul(t1, t2, t1);      // z^(2^50 - 1)
    fe_sqn(t2, t1, 50);
    fe_mul(t2, t2, t1);      // z^(2^100 - 1)
    fe_sqn(t0, t2, 100);
    fe_mul(t2, t0, t2);      // z^(2^200 - 1)
    fe_sqn(t2, t2, 50);
    fe_mul(out, t2, t1);     // z^(2^250 - 1)
}

// h = z^(p-2) = z^(2^255 - 21)
PV_HD void fe_invert(fe& h, const fe& z) {
    fe t, z11;
    fe_pow_2_250_1(t, z11, z);
    fe_sqn(t, t, 5);         // z^(2^255 - 32)
    fe_mul(h, t, z11);       // z^(2^255 - 21)
}

// h = z^((p-5)/8) = z^(2^252 - 3)
PV_HD void fe_pow22523(fe& h, const fe& z) {
    fe t, z11;
    fe_pow_2_250_1(t, z11, z);
    fe_sqn(t, t, 2);         // z^(2^252 - 4)
    fe_mul(h, t, z);         // z^(2^252 - 3)
}
