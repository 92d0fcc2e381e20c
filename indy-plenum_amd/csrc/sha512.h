// SHA-512 (FIPS 180-4) for the per-request hash k = SHA-512(R || A || M) of the verify kernels.
//
// 64-bit words live in VGPR pairs: additions are single v_lshl_add_u64, every rotation is two
// v_alignbit_b32 (a funnel shift of the two halves), Ch / Maj / the three-way XORs are one
// v_bitop3_b32 per half, byte swaps to v_perm_b32. Rounds are unrolled 16 at a time with the
// message schedule in a static 16-word ring and the working variables rotated by renaming, so no
// register moves or indexed register accesses remain (~34 VALU instructions per round).
// Replaces libsodium's crypto_hash_sha512 inside crypto_sign_open (reached from the reference via
// stp_core/crypto/nacl_wrappers.py:108).
#pragma once
#include "fe25519.h"

static constexpr uint64_t PV_K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// ((hi:lo) >> s) mod 2^32 for 0 <= s < 32: one v_alignbit_b32
PV_HD uint32_t pv_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

PV_HD uint64_t pv_pack64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }

// gfx950 v_bitop3_b32: any bitwise function of three operands in one instruction (truth table
// over src0 = 0xF0, src1 = 0xCC, src2 = 0xAA): XOR3 = 0x96, Ch = 0xCA, Maj = 0xE8. The compiler
// does not form it from xor/and/or trees itself (round 2: 292 v_xor_b32 per 16 unrolled rounds).
template <int TT>
PV_HD uint32_t pv_bitop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    uint32_t r = 0;
    for (int i = 0; i < 8; i++)
        if ((TT >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
#endif
}
// the halves are joined by a bit cast of a 2-vector, not (hi << 32) | lo: LLVM turns an OR of
// disjoint halves feeding an addition into two 64-bit additions (+1 v_lshl_add_u64 and a v_mov per use)
template <int TT>
PV_HD uint64_t pv_bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 v;
    v.x = pv_bitop3<TT>((uint32_t)a, (uint32_t)b, (uint32_t)c);
    v.y = pv_bitop3<TT>((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32));
    return __builtin_bit_cast(uint64_t, v);
}

// rotate right by a compile-time n (0 < n < 64, n != 32)
template <int N>
PV_HD uint64_t pv_rotr64(uint64_t x) {
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    if (N < 32) return pv_pack64(pv_alignbit(lo, hi, N), pv_alignbit(hi, lo, N));
    return pv_pack64(pv_alignbit(hi, lo, N - 32), pv_alignbit(lo, hi, N - 32));
}
template <int N>
PV_HD uint64_t pv_shr64(uint64_t x) {
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    return pv_pack64(hi >> N, pv_alignbit(hi, lo, N));
}

PV_HD uint32_t pv_bswap32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(0u, x, 0x00010203u);
#else
    return __builtin_bswap32(x);
#endif
}
// byte-reverse a 64-bit word
PV_HD uint64_t pv_bswap64(uint64_t x) {
    return pv_pack64(pv_bswap32((uint32_t)x), pv_bswap32((uint32_t)(x >> 32)));
}

PV_HD void sha512_init(uint64_t st[8]) {
    st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL;
    st[2] = 0x3c6ef372fe94f82bULL; st[3] = 0xa54ff53a5f1d36f1ULL;
    st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
    st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// One round: the eight working variables rotate by renaming (the caller passes them shifted).
#define PV_SHA_ROUND(a, b, c, d, e, f, g, h, kw)                                                   \
    do {                                                                                          \
        const uint64_t S1 = pv_bitop3_64<0x96>(pv_rotr64<14>(e), pv_rotr64<18>(e), pv_rotr64<41>(e)); \
        const uint64_t ch = pv_bitop3_64<0xCA>(e, f, g);                                          \
        const uint64_t t1 = h + S1 + ch + (kw);                                                   \
        const uint64_t S0 = pv_bitop3_64<0x96>(pv_rotr64<28>(a), pv_rotr64<34>(a), pv_rotr64<39>(a)); \
        const uint64_t mj = pv_bitop3_64<0xE8>(a, b, c);                                          \
        d += t1;                                                                                  \
        h = t1 + S0 + mj;                                                                         \
    } while (0)

// One compression of a 128-byte block given as 16 big-endian words (already byte-swapped).
PV_HD void sha512_compress(uint64_t st[8], const uint64_t blk[16]) {
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = blk[i];
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
    for (int r = 0; r < 80; r += 16) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int i = r + j;
            if (r > 0) {
                const uint64_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
                const uint64_t s0 = pv_bitop3_64<0x96>(pv_rotr64<1>(w15), pv_rotr64<8>(w15), pv_shr64<7>(w15));
                const uint64_t s1 = pv_bitop3_64<0x96>(pv_rotr64<19>(w2), pv_rotr64<61>(w2), pv_shr64<6>(w2));
                w[i & 15] += s0 + w[(i - 7) & 15] + s1;
            }
            const uint64_t kw = PV_K512[i] + w[i & 15];
            switch (j & 7) {
                case 0: PV_SHA_ROUND(a, b, c, d, e, f, g, h, kw); break;
                case 1: PV_SHA_ROUND(h, a, b, c, d, e, f, g, kw); break;
                case 2: PV_SHA_ROUND(g, h, a, b, c, d, e, f, kw); break;
                case 3: PV_SHA_ROUND(f, g, h, a, b, c, d, e, kw); break;
                case 4: PV_SHA_ROUND(e, f, g, h, a, b, c, d, kw); break;
                case 5: PV_SHA_ROUND(d, e, f, g, h, a, b, c, kw); break;
                case 6: PV_SHA_ROUND(c, d, e, f, g, h, a, b, kw); break;
                default: PV_SHA_ROUND(b, c, d, e, f, g, h, a, kw); break;
            }
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

#undef PV_SHA_ROUND
