/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the product
 * path (indy-plenum_amd/). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may use it, and only as the checker.
 *
 * Plain-C CPU restatement of the reference's signature-verification algorithm for the Plenum
 * request-authentication path:
 *
 *   plenum/server/client_authn.py:84-118  NaclAuthNr.authenticate_multi -> DidVerifier.verify
 *   plenum/common/verifier.py:53-54       DidVerifier.verify -> stp_core Verifier.verify
 *   stp_core/crypto/nacl_wrappers.py:232-242  Verifier.verify: VerifyKey.verify(signature + msg)
 *   stp_core/crypto/nacl_wrappers.py:86-108   VerifyKey.verify -> libnacl.crypto_sign_open(sm, pk)
 *
 * The arithmetic itself lives in the third-party dependency libsodium (pinned: libsodium23 =
 * 1.0.18 on Ubuntu 20.04, dev-setup/ubuntu/ubuntu-2004/SetupVMTest.txt:17; reached through
 * libnacl 1.6.1, setup.py:107-108), which is NOT in /root/reference. This file restates its
 * published algorithm (RFC 8032 Ed25519 verification, cofactorless, with libsodium 1.0.18's
 * default-build acceptance rules):
 *   1. crypto_sign_open: smlen < 64 -> reject; sig = sm[0:64], M = sm[64:].
 *   2. S = sig[32:64] must be < L (full 256-bit compare).
 *   3. R = sig[0:32] must not be one of 7 small-order encodings (bytes 0..30 exact, byte 31
 *      with bit 7 masked).
 *   4. A must be canonical: not ((A[31]&0x7f)==0x7f && A[1..30]==0xff && A[0]>=0xed).
 *   5. A must not be in the same 7-entry blacklist.
 *   6. A must decompress (ge25519_frombytes_negate_vartime: y taken mod p, x from
 *      uv^3(uv^7)^((p-5)/8), sqrt(-1) fix-up, reject non-squares; result negated).
 *   7. k = SHA-512(R || A || M) mod L.
 *   8. accept iff encode([S]B + [k](-A)) == R bytewise.
 *
 * Parity is pinned by differential tests against the libsodium 1.0.18 binary present in the
 * image (/opt/conda/lib/libsodium.so.23) and by committed golden vectors (tests/golden/), see
 * tests/test_oracle.py. The implementation below is deliberately simple (radix 2^51, unified
 * complete addition law, plain double-and-add) so that it is obviously correct; speed is not a
 * goal here. The CPU baseline in bench.py times libsodium itself, not this file.
 */
#include <stdint.h>
#include <string.h>
#include <stddef.h>

/* ------------------------------------------------------------------ SHA-512 (FIPS 180-4) */
static const uint64_t K512[80] = {
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

#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha512_block(uint64_t st[8], const uint8_t *p) {
    uint64_t w[80];
    for (int i = 0; i < 16; i++) {
        uint64_t v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * i + j];
        w[i] = v;
    }
    for (int i = 16; i < 80; i++) {
        uint64_t s0 = ROR64(w[i - 15], 1) ^ ROR64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = ROR64(w[i - 2], 19) ^ ROR64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 80; i++) {
        uint64_t S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
        uint64_t ch = (e & f) ^ (~e & g);
        uint64_t t1 = h + S1 + ch + K512[i] + w[i];
        uint64_t S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
        uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint64_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* SHA-512 over the concatenation of up to three byte strings (R || A || M). */
void oracle_sha512_3(uint8_t out[64], const uint8_t *p0, size_t n0, const uint8_t *p1, size_t n1,
                     const uint8_t *p2, size_t n2) {
    uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                      0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                      0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint8_t buf[128];
    size_t fill = 0;
    uint64_t total = (uint64_t)n0 + n1 + n2;
    const uint8_t *parts[3] = {p0, p1, p2};
    size_t lens[3] = {n0, n1, n2};
    for (int k = 0; k < 3; k++) {
        for (size_t i = 0; i < lens[k]; i++) {
            buf[fill++] = parts[k][i];
            if (fill == 128) { sha512_block(st, buf); fill = 0; }
        }
    }
    buf[fill++] = 0x80;
    if (fill > 112) {
        while (fill < 128) buf[fill++] = 0;
        sha512_block(st, buf);
        fill = 0;
    }
    while (fill < 120) buf[fill++] = 0;
    uint64_t bits = total * 8;  /* the upper 64 bits of the 128-bit length are zero */
    for (int j = 0; j < 8; j++) buf[120 + j] = (uint8_t)(bits >> (56 - 8 * j));
    sha512_block(st, buf);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(st[i] >> (56 - 8 * j));
}

/* ------------------------------------------------------------------ GF(2^255-19), radix 2^51 */
typedef struct { uint64_t v[5]; } fe;
typedef unsigned __int128 u128;
static const uint64_t M51 = (1ULL << 51) - 1;

static void fe_carry(fe *h) {
    for (int r = 0; r < 2; r++) {
        uint64_t c;
        for (int i = 0; i < 4; i++) { c = h->v[i] >> 51; h->v[i] &= M51; h->v[i + 1] += c; }
        c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
    }
}
static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_add(fe *h, const fe *f, const fe *g) {
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
    fe_carry(h);
}
/* h = f - g + 4p (all limbs of inputs are < 2^52 after fe_carry) */
static void fe_sub(fe *h, const fe *f, const fe *g) {
    static const uint64_t P4[5] = {0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                                   0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + P4[i] - g->v[i];
    fe_carry(h);
}
static void fe_mul(fe *h, const fe *f, const fe *g) {
    /* inputs: limbs < 2^54 -> every column < 5 * 19 * 2^108 < 2^115 */
    u128 t[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 5; j++) {
            u128 p = (u128)f->v[i] * g->v[j];
            if (i + j < 5) t[i + j] += p; else t[i + j - 5] += p * 19;
        }
    for (int i = 0; i < 4; i++) { t[i + 1] += t[i] >> 51; t[i] &= M51; }
    t[0] += (t[4] >> 51) * 19;
    t[4] &= M51;
    t[1] += t[0] >> 51;
    t[0] &= M51;
    for (int i = 0; i < 5; i++) h->v[i] = (uint64_t)t[i];
    fe_carry(h);
}
static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }

static void fe_frombytes(fe *h, const uint8_t s[32]) {
    /* 255 bits, little-endian; the top bit is ignored (libsodium fe25519_frombytes). */
    uint8_t t[32];
    memcpy(t, s, 32);
    t[31] &= 0x7f;
    fe_0(h);
    for (int bit = 0; bit < 255; bit++)
        if ((t[bit >> 3] >> (bit & 7)) & 1) h->v[bit / 51] |= 1ULL << (bit % 51);
}
static void fe_tobytes(uint8_t s[32], const fe *f) {
    fe h = *f;
    /* normalise to limbs < 2^51, i.e. a value in [0, 2^255) */
    for (;;) {
        int done = 1;
        for (int i = 0; i < 4; i++) { h.v[i + 1] += h.v[i] >> 51; h.v[i] &= M51; }
        if (h.v[4] >> 51) { h.v[0] += 19 * (h.v[4] >> 51); h.v[4] &= M51; done = 0; }
        for (int i = 0; i < 5; i++) if (h.v[i] >> 51) done = 0;
        if (done) break;
    }
    /* value < 2^255 < 2p: subtract p once iff value + 19 >= 2^255 */
    uint64_t t[5], c = 19;
    for (int i = 0; i < 5; i++) { t[i] = h.v[i] + c; c = t[i] >> 51; t[i] &= M51; }
    if (c) memcpy(h.v, t, sizeof t);
    memset(s, 0, 32);
    for (int bit = 0; bit < 255; bit++)
        if ((h.v[bit / 51] >> (bit % 51)) & 1) s[bit >> 3] |= (uint8_t)(1 << (bit & 7));
}
static int fe_isnegative(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }
static int fe_iszero(const fe *f) {
    uint8_t s[32], z = 0;
    fe_tobytes(s, f);
    for (int i = 0; i < 32; i++) z |= s[i];
    return z == 0;
}
static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
/* h = f^e, e given as 32 little-endian bytes; plain MSB-first square-and-multiply. */
static void fe_pow(fe *h, const fe *f, const uint8_t e[32]) {
    fe r;
    fe_1(&r);
    for (int bit = 255; bit >= 0; bit--) {
        fe_sq(&r, &r);
        if ((e[bit >> 3] >> (bit & 7)) & 1) fe_mul(&r, &r, f);
    }
    *h = r;
}
/* exponents: p-2 and (p-5)/8 = 2^252 - 3 */
static const uint8_t EXP_PM2[32] = {0xeb, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f};
static const uint8_t EXP_P58[32] = {0xfd, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x0f};
static void fe_invert(fe *h, const fe *f) { fe_pow(h, f, EXP_PM2); }

/* curve constants (little-endian byte encodings) */
static const uint8_t D_BYTES[32] = {0xa3, 0x78, 0x59, 0x13, 0xca, 0x4d, 0xeb, 0x75, 0xab, 0xd8, 0x41,
                                    0x41, 0x4d, 0x0a, 0x70, 0x00, 0x98, 0xe8, 0x79, 0x77, 0x79, 0x40,
                                    0xc7, 0x8c, 0x73, 0xfe, 0x6f, 0x2b, 0xee, 0x6c, 0x03, 0x52};
static const uint8_t SQRTM1_BYTES[32] = {0xb0, 0xa0, 0x0e, 0x4a, 0x27, 0x1b, 0xee, 0xc4, 0x78, 0xe4, 0x2f,
                                         0xad, 0x06, 0x18, 0x43, 0x2f, 0xa7, 0xd7, 0xfb, 0x3d, 0x99, 0x00,
                                         0x4d, 0x2b, 0x0b, 0xdf, 0xc1, 0x4f, 0x80, 0x24, 0x83, 0x2b};
/* base point B: y = 4/5, x even */
static const uint8_t B_BYTES[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                    0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                    0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};

/* ------------------------------------------------------------------ points, extended coords */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_identity(ge *p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }

/* Unified addition for a = -1 twisted Edwards (add-2008-hwcd-3). Complete on the whole group
 * because -1 is a square mod p and d is a non-square, so it also serves as doubling. */
static void ge_add(ge *r, const ge *p, const ge *q) {
    fe d, d2, a, b, c, dd, e, f, g, h, t0, t1;
    fe_frombytes(&d, D_BYTES);
    fe_add(&d2, &d, &d);
    fe_sub(&t0, &p->Y, &p->X); fe_sub(&t1, &q->Y, &q->X); fe_mul(&a, &t0, &t1);
    fe_add(&t0, &p->Y, &p->X); fe_add(&t1, &q->Y, &q->X); fe_mul(&b, &t0, &t1);
    fe_mul(&c, &p->T, &q->T); fe_mul(&c, &c, &d2);
    fe_mul(&dd, &p->Z, &q->Z); fe_add(&dd, &dd, &dd);
    fe_sub(&e, &b, &a); fe_sub(&f, &dd, &c); fe_add(&g, &dd, &c); fe_add(&h, &b, &a);
    fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}
/* r = [s]p, s = 32 little-endian bytes, MSB-first double-and-add */
static void ge_scalarmult(ge *r, const uint8_t s[32], const ge *p) {
    ge acc;
    ge_identity(&acc);
    for (int bit = 255; bit >= 0; bit--) {
        ge_add(&acc, &acc, &acc);
        if ((s[bit >> 3] >> (bit & 7)) & 1) ge_add(&acc, &acc, p);
    }
    *r = acc;
}
static void ge_tobytes(uint8_t s[32], const ge *p) {
    fe zi, x, y;
    fe_invert(&zi, &p->Z);
    fe_mul(&x, &p->X, &zi);
    fe_mul(&y, &p->Y, &zi);
    fe_tobytes(s, &y);
    s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}
/* libsodium ge25519_frombytes_negate_vartime: decode s, return -P. Returns -1 if y does not
 * correspond to a curve point. y is reduced mod p (no canonicity check here); an x = 0 root with
 * the sign bit set is negated to itself (no rejection in this function). */
static int ge_frombytes_negate(ge *h, const uint8_t s[32]) {
    fe d, u, v, v3, vxx, chk, sqrtm1;
    fe_frombytes(&d, D_BYTES);
    fe_frombytes(&sqrtm1, SQRTM1_BYTES);
    fe_frombytes(&h->Y, s);
    fe_1(&h->Z);
    fe_sq(&u, &h->Y);
    fe_mul(&v, &u, &d);
    fe_sub(&u, &u, &h->Z);          /* u = y^2 - 1 */
    fe_add(&v, &v, &h->Z);          /* v = d y^2 + 1 */
    fe_sq(&v3, &v);
    fe_mul(&v3, &v3, &v);           /* v^3 */
    fe_sq(&h->X, &v3);
    fe_mul(&h->X, &h->X, &v);
    fe_mul(&h->X, &h->X, &u);       /* u v^7 */
    fe_pow(&h->X, &h->X, EXP_P58);  /* (u v^7)^((p-5)/8) */
    fe_mul(&h->X, &h->X, &v3);
    fe_mul(&h->X, &h->X, &u);       /* u v^3 (u v^7)^((p-5)/8) */
    fe_sq(&vxx, &h->X);
    fe_mul(&vxx, &vxx, &v);
    fe_sub(&chk, &vxx, &u);
    if (!fe_iszero(&chk)) {
        fe_add(&chk, &vxx, &u);
        if (!fe_iszero(&chk)) return -1;
        fe_mul(&h->X, &h->X, &sqrtm1);
    }
    if (fe_isnegative(&h->X) == (s[31] >> 7)) fe_neg(&h->X, &h->X);
    fe_mul(&h->T, &h->X, &h->Y);
    return 0;
}

/* ------------------------------------------------------------------ scalars mod L */
static const uint8_t L_BYTES[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                    0xa2, 0xde, 0xf9, 0xde, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                                    0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x10};

/* 1 iff s < L as 256-bit little-endian integers (libsodium sc25519_is_canonical) */
int oracle_sc_is_canonical(const uint8_t s[32]) {
    for (int i = 31; i >= 0; i--) {
        if (s[i] < L_BYTES[i]) return 1;
        if (s[i] > L_BYTES[i]) return 0;
    }
    return 0; /* s == L */
}

/* r = x mod L for a 512-bit little-endian x, by binary long division (obviously correct). */
void oracle_sc_reduce64(uint8_t r[32], const uint8_t x[64]) {
    uint64_t acc[5] = {0, 0, 0, 0, 0}; /* 257-bit running remainder, < 2L */
    uint64_t L[4];
    for (int i = 0; i < 4; i++) {
        uint64_t v = 0;
        for (int j = 7; j >= 0; j--) v = (v << 8) | L_BYTES[8 * i + j];
        L[i] = v;
    }
    for (int bit = 511; bit >= 0; bit--) {
        /* acc = 2*acc + bit */
        for (int i = 4; i > 0; i--) acc[i] = (acc[i] << 1) | (acc[i - 1] >> 63);
        acc[0] = (acc[0] << 1) | ((x[bit >> 3] >> (bit & 7)) & 1);
        /* if acc >= L: acc -= L */
        int ge = acc[4] != 0;
        if (!ge) {
            ge = 1;
            for (int i = 3; i >= 0; i--) {
                if (acc[i] > L[i]) { ge = 1; break; }
                if (acc[i] < L[i]) { ge = 0; break; }
            }
        }
        if (ge) {
            uint64_t borrow = 0;
            for (int i = 0; i < 4; i++) {
                u128 d = (u128)acc[i] - L[i] - borrow;
                acc[i] = (uint64_t)d;
                borrow = (uint64_t)(d >> 64) ? 1 : 0;
            }
            acc[4] -= borrow;
        }
    }
    for (int i = 0; i < 32; i++) r[i] = (uint8_t)(acc[i >> 3] >> (8 * (i & 7)));
}

/* r = (a*b + c) mod L (test-vector forging helper) */
void oracle_sc_muladd(uint8_t r[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
    uint8_t prod[64];
    uint32_t t[64];
    memset(t, 0, sizeof t);
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) t[i + j] += (uint32_t)a[i] * b[j];
    for (int i = 0; i < 32; i++) t[i] += c[i];
    uint32_t carry = 0;
    for (int i = 0; i < 64; i++) { t[i] += carry; prod[i] = (uint8_t)t[i]; carry = t[i] >> 8; }
    oracle_sc_reduce64(r, prod);
}

/* ------------------------------------------------------------------ libsodium acceptance rules */
static const uint8_t BLACKLIST[7][32] = {
    /* 0 (order 4) */
    {0},
    /* 1 (order 1) */
    {0x01},
    /* order-8 points */
    {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0, 0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
     0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39, 0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05},
    {0xc7, 0x17, 0x6a, 0x70, 0x3d, 0x4d, 0xd8, 0x4f, 0xba, 0x3c, 0x0b, 0x76, 0x0d, 0x10, 0x67, 0x0f,
     0x2a, 0x20, 0x53, 0xfa, 0x2c, 0x39, 0xcc, 0xc6, 0x4e, 0xc7, 0xfd, 0x77, 0x92, 0xac, 0x03, 0x7a},
    /* p-1 (order 2) */
    {0xec, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f},
    /* p (= 0, order 4) */
    {0xed, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f},
    /* p+1 (= 1, order 1) */
    {0xee, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f}};

int oracle_has_small_order(const uint8_t s[32]) {
    for (int k = 0; k < 7; k++) {
        int eq = 1;
        for (int j = 0; j < 31; j++) eq &= s[j] == BLACKLIST[k][j];
        eq &= (s[31] & 0x7f) == BLACKLIST[k][31];
        if (eq) return 1;
    }
    return 0;
}

int oracle_ge_is_canonical(const uint8_t s[32]) {
    if ((s[31] & 0x7f) != 0x7f) return 1;
    for (int i = 30; i > 0; i--)
        if (s[i] != 0xff) return 1;
    return s[0] < 0xed;
}

/* crypto_sign_ed25519_verify_detached (libsodium 1.0.18 default build): 0 = valid, -1 = invalid */
int oracle_verify_detached(const uint8_t sig[64], const uint8_t *m, size_t mlen, const uint8_t pk[32]) {
    ge A, sB, kA, Q, Bp;
    uint8_t h[64], k[32], rcheck[32];
    if (!oracle_sc_is_canonical(sig + 32) || oracle_has_small_order(sig)) return -1;
    if (!oracle_ge_is_canonical(pk) || oracle_has_small_order(pk)) return -1;
    if (ge_frombytes_negate(&A, pk) != 0) return -1;
    oracle_sha512_3(h, sig, 32, pk, 32, m, mlen);
    oracle_sc_reduce64(k, h);
    /* base point: decode B (negate twice) */
    ge_frombytes_negate(&Bp, B_BYTES);
    fe_neg(&Bp.X, &Bp.X);
    fe_neg(&Bp.T, &Bp.T);
    ge_scalarmult(&sB, sig + 32, &Bp);
    ge_scalarmult(&kA, k, &A); /* A already holds -A */
    ge_add(&Q, &sB, &kA);
    ge_tobytes(rcheck, &Q);
    return memcmp(rcheck, sig, 32) == 0 ? 0 : -1;
}

/* crypto_sign_open semantics on the concatenation sm = sig || msg (nacl_wrappers.py:105) */
int oracle_sign_open(const uint8_t *sm, size_t smlen, const uint8_t pk[32]) {
    if (smlen < 64) return -1;
    return oracle_verify_detached(sm, sm + 64, smlen - 64, pk);
}

/* Batch driver for tests: sm blob + n+1 prefix offsets + n 32-byte keys -> verdict bytes (1=ok).
 * Requests [lo, hi) only; tests split work over processes. */
void oracle_sign_open_batch(const uint8_t *blob, const uint64_t *off, const uint8_t *pk, uint64_t lo,
                            uint64_t hi, uint8_t *verdict) {
    for (uint64_t i = lo; i < hi; i++)
        verdict[i] = oracle_sign_open(blob + off[i], (size_t)(off[i + 1] - off[i]), pk + 32 * i) == 0;
}

/* ------------------------------------------------------------------ test-vector helpers */
/* out = encode([s]B) */
void oracle_scalarmult_base(uint8_t out[32], const uint8_t s[32]) {
    ge Bp, r;
    ge_frombytes_negate(&Bp, B_BYTES);
    fe_neg(&Bp.X, &Bp.X);
    fe_neg(&Bp.T, &Bp.T);
    ge_scalarmult(&r, s, &Bp);
    ge_tobytes(out, &r);
}
/* out = encode(P + Q) for encodings p, q (decoded with libsodium rules, no blacklist). -1 if
 * either fails to decode. */
int oracle_point_add(uint8_t out[32], const uint8_t p[32], const uint8_t q[32]) {
    ge P, Q, R;
    if (ge_frombytes_negate(&P, p) || ge_frombytes_negate(&Q, q)) return -1;
    ge_add(&R, &P, &Q); /* (-P) + (-Q) */
    fe_neg(&R.X, &R.X);
    fe_neg(&R.T, &R.T);
    ge_tobytes(out, &R);
    return 0;
}
/* Raw signing with explicit nonce r and secret scalar a against an arbitrary public encoding
 * A_enc: R = [r]B, k = H(R||A_enc||M) mod L, S = r + k a mod L. Used to forge adversarial vectors
 * (e.g. mixed-order keys with honest signatures) that libsodium's own signer cannot produce. */
void oracle_sign_raw(uint8_t sig[64], const uint8_t r[32], const uint8_t a[32], const uint8_t A_enc[32],
                     const uint8_t *m, size_t mlen) {
    uint8_t h[64], k[32];
    oracle_scalarmult_base(sig, r);
    oracle_sha512_3(h, sig, 32, A_enc, 32, m, mlen);
    oracle_sc_reduce64(k, h);
    oracle_sc_muladd(sig + 32, k, a, r);
}
