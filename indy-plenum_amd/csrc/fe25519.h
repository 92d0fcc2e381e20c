// GF(2^255-19) arithmetic for the gfx950 Ed25519 verification kernels.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i has weight 2^ceil(25.5 i):
// even limbs carry 26 bits, odd limbs 25 bits). Products are formed with v_mad_u64_u32
// (32x32 -> 64 multiply + 64-bit accumulate in one instruction). Measured on MI355X it issues at
// ~5.2 cycles per wave64 instruction at >= 2 waves/SIMD, the same rate as a bare v_mul_lo_u32
// (profiles/r01_isa_rates.jsonl), so one mad replaces mul_lo + mul_hi + add_co + addc. 5x51-bit
// limbs would need 64x64 -> 128 products that the VALU does not have.
//
// Bound discipline (checked by tests/test_native_host.py with the PV_BOUNDS_CHECK host build):
//   "R"   reduced:     limb < 2^width + 2^17 (width 26 even / 25 odd; output of mul/sq/carry:
//                      the carries into limbs 1 and 5 are not re-propagated)
//   mul/sq inputs:     limb < 3 * 2^width + 2^18
//                      => 19 * limb < 2^32 and every product column < 2^63 (no 64-bit overflow)
//   fe_add(R, R)  -> even < 2^27, odd < 2^26          (valid mul input)
//   fe_sub(X, R)  -> X + 2p - R: needs X in R           (valid mul input)
//   anything else  -> fe_carry first.
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

PV_HD void fe_check_mul_input(const fe& f) {
#ifdef PV_BOUNDS_CHECK
    for (int i = 0; i < 10; i++)
        PV_ASSERT(f.v[i] < ((i & 1) ? 3u * (1u << 25) : 3u * (1u << 26)) + (1u << 18), "mul input");
#else
    (void)f;
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
// h = f + 2p - g, g reduced
PV_HD void fe_sub(fe& h, const fe& f, const fe& g) {
    fe_check_reduced(g);
    h.v[0] = f.v[0] + 0x7FFFFDAu - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu) - g.v[i];
}
// h = 4p - g for g with even limbs < 2^28, odd < 2^27 (negation of a non-reduced value);
// the result is NOT a valid mul input until carried.
PV_HD void fe_sub4p(fe& h, const fe& f, const fe& g) {
    h.v[0] = f.v[0] + 0xFFFFFB4u - g.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) h.v[i] = f.v[i] + ((i & 1) ? 0x7FFFFFCu : 0xFFFFFFCu) - g.v[i];
}
// conditional negate of a reduced value: h = neg ? 2p - f : f (result < 2^27 even, valid mul input)
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

// Carry chain over 64-bit column sums (each < 2^63) -> reduced limbs.
PV_HD void fe_carry64(fe& h, uint64_t t[10]) {
    t[1] += t[0] >> 26; t[0] &= M26;
    t[5] += t[4] >> 26; t[4] &= M26;
    t[2] += t[1] >> 25; t[1] &= M25;
    t[6] += t[5] >> 25; t[5] &= M25;
    t[3] += t[2] >> 26; t[2] &= M26;
    t[7] += t[6] >> 26; t[6] &= M26;
    t[4] += t[3] >> 25; t[3] &= M25;
    t[8] += t[7] >> 25; t[7] &= M25;
    t[5] += t[4] >> 26; t[4] &= M26;
    t[9] += t[8] >> 26; t[8] &= M26;
    t[0] += (t[9] >> 25) * 19u; t[9] &= M25;
    t[1] += t[0] >> 26; t[0] &= M26;
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = (uint32_t)t[i];
    fe_check_reduced(h);
}

// Weak reduction of 32-bit limbs (each < 2^31) back to the reduced range.
PV_HD void fe_carry(fe& h, const fe& f) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = f.v[i];
    t[1] += t[0] >> 26; t[0] &= M26;
    t[5] += t[4] >> 26; t[4] &= M26;
    t[2] += t[1] >> 25; t[1] &= M25;
    t[6] += t[5] >> 25; t[5] &= M25;
    t[3] += t[2] >> 26; t[2] &= M26;
    t[7] += t[6] >> 26; t[6] &= M26;
    t[4] += t[3] >> 25; t[3] &= M25;
    t[8] += t[7] >> 25; t[7] &= M25;
    t[5] += t[4] >> 26; t[4] &= M26;
    t[9] += t[8] >> 26; t[8] &= M26;
    t[0] += (t[9] >> 25) * 19u; t[9] &= M25;
    t[1] += t[0] >> 26; t[0] &= M26;
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = t[i];
    fe_check_reduced(h);
}

PV_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// Keeps the machine scheduler from interleaving independent field multiplications: each one has
// 55-100 independent v_mad_u64_u32 (ample ILP at 2 waves/SIMD), and interleaving three or four of
// them multiplies the live accumulators past the 256-VGPR budget (measured: spills to scratch).
PV_HD void pv_sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// h = f * g
PV_HD void fe_mul(fe& h, const fe& f, const fe& g) {
    fe_check_mul_input(f);
    fe_check_mul_input(g);
    uint32_t g19[10], f2[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        g19[i] = 19u * g.v[i];
        f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
    }
    uint64_t t[10];
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = 0; j < 10; j++) {
            const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
            if (i + j < 10) t[i + j] = mad64(a, g.v[j], t[i + j]);
            else t[i + j - 10] = mad64(a, g19[j], t[i + j - 10]);
        }
    }
    fe_carry64(h, t);
    pv_sched_fence();
}

// h = f^2 (55 products)
PV_HD void fe_sq(fe& h, const fe& f) {
    fe_check_mul_input(f);
    uint32_t f2[10], f19[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        f2[i] = 2u * f.v[i];
        f19[i] = 19u * f.v[i];
    }
    uint64_t t[10];
#pragma unroll
    for (int k = 0; k < 10; k++) t[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
            // coefficient: (i == j ? 1 : 2) * ((i & j & 1) ? 2 : 1) * (i + j >= 10 ? 19 : 1)
            const int c = (i == j ? 1 : 2) * (((i & j) & 1) ? 2 : 1);  // 1, 2 or 4
            uint32_t a = (c == 1) ? f.v[i] : (c == 2 ? f2[i] : 2u * f2[i]);
            const uint32_t b = (i + j >= 10) ? f19[j] : f.v[j];
            const int k = (i + j >= 10) ? i + j - 10 : i + j;
            t[k] = mad64(a, b, t[k]);
        }
    }
    fe_carry64(h, t);
    pv_sched_fence();
}

// h = 2 f^2
PV_HD void fe_sq2(fe& h, const fe& f) {
    fe t;
    fe_sq(t, f);
    fe_add(t, t, t);
    fe_carry(h, t);
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
