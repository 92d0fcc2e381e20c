// Edwards25519 group arithmetic (a = -1 twisted Edwards, extended coordinates) for the gfx950
// verify kernels. Formulas: Hisil-Wong-Carter-Dawson 2008 (dbl-2008-hwcd, add-2008-hwcd-3);
// the addition law is complete on the whole group (a square, d non-square), so table lookups
// never branch on exceptional inputs (identity, equal points, small-order components).
//
// Representations (x = X/Z, y = Y/Z, T = XY/Z):
//   ge_p2     (X : Y : Z)
//   ge_p3     (X : Y : Z : T)
//   ge_p1p1   completed: x = X/Z, y = Y/T
//   ge_cached (Y+X, Y-X, 2Z, 2d T)      per-verify table of multiples of -A
//   ge_niels  (y+x, y-x, 2d x y)        affine, fixed-base table of multiples of B
// Replaces libsodium's ge25519 (ge25519_frombytes_negate_vartime, ge25519_double_scalarmult_vartime,
// ge25519_tobytes), reached from stp_core/crypto/nacl_wrappers.py:108.
#pragma once
#include "fe25519.h"

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YplusX, YminusX, Z2, T2d; };
struct ge_niels { fe yplusx, yminusx, xy2d; };

// d, 2d and sqrt(-1) as reduced limbs
static constexpr uint32_t PV_D[10] = {0x35978a3u, 0x0d37284u, 0x3156ebdu, 0x06a0a0eu, 0x001c029u,
                                      0x179e898u, 0x3a03cbbu, 0x1ce7198u, 0x2e2b6ffu, 0x1480db3u};
static constexpr uint32_t PV_D2[10] = {0x2b2f159u, 0x1a6e509u, 0x22add7au, 0x0d4141du, 0x0038052u,
                                       0x0f3d130u, 0x3407977u, 0x19ce331u, 0x1c56dffu, 0x0901b67u};
// 1/d
static constexpr uint32_t PV_INVD[10] = {0x1c9f843u, 0x03c9db3u, 0x285c4bcu, 0x0c213cau, 0x02d775au,
                                         0x1b9cf66u, 0x3108a66u, 0x1c86562u, 0x1214d5cu, 0x10241fbu};
// 1/2 = (p + 1) / 2
static constexpr uint32_t PV_INV2[10] = {0x3fffff7u, 0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu,
                                         0x1ffffffu, 0x3ffffffu, 0x1ffffffu, 0x3ffffffu, 0x0ffffffu};
static constexpr uint32_t PV_SQRTM1[10] = {0x20ea0b0u, 0x186c9d2u, 0x08f189du, 0x035697fu, 0x0bd0c60u,
                                           0x1fbd7a7u, 0x2804c9eu, 0x1e16569u, 0x004fc1du, 0x0ae0c92u};

PV_HD void fe_const(fe& h, const uint32_t c[10]) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = c[i];
}

// r = 2 (X : Y : Z), X, Y, Z in R (dbl-2008-hwcd, 4S). Output p1p1, bounds chosen so that only
// ONE carry pass is needed:
//   r.X = (X+Y)^2 + 4p - (YY+XX)   uncarried, limbs < 2^28.4: only ever an f operand
//   r.Y = YY + XX                  < 2^27 + 2^18
//   r.Z = YY + 2p - XX             < 3 * 2^w + 2^17  (< PV_GMAX)
//   r.T = 2 ZZ + 4p - r.Z          carried (R)
PV_HD void ge_p2_dbl(ge_p1p1& r, const fe& X, const fe& Y, const fe& Z) {
    fe XX, YY, ZZ, S, t;
    fe_add(t, X, Y);
    fe_sq(XX, X);
    fe_sq(YY, Y);
    fe_add(r.Y, YY, XX);
    fe_sub(r.Z, YY, XX);
    fe_sq(S, t);
    fe_sub4p(r.X, S, r.Y);
    fe_sq(ZZ, Z);
    fe_add(t, ZZ, ZZ);
    fe_sub4p(t, t, r.Z);
    fe_carry(r.T, t);
}

// p1p1 -> p2 / p3. g operands (19-multiplied, shared): T and Z for p2, plus Y for p3; X is always
// the f side, so r.X may be uncarried (ge_p2_dbl) and T/Z/Y only need limbs < PV_GMAX.
PV_HD void ge_p1p1_to_p2(fe& X, fe& Y, fe& Z, const ge_p1p1& p) {
    uint32_t g19[10];
    fe_mul19(g19, p.Z);
    fe_mul_pre(Y, p.Y, p.Z, g19);
    pv_sched_fence();
    fe_mul19(g19, p.T);
    fe_mul_pre(X, p.X, p.T, g19);
    pv_sched_fence();
    fe_mul_pre(Z, p.Z, p.T, g19);
    pv_sched_fence();
}

// X3 = X T, Z3 = Z T, Y3 = Z Y, T3 = X Y: two g operands (T, Y), so 19 g is formed twice, not 3 times
// (every p1p1 limb here is < 3 * 2^26 + 2^18 < PV_GMAX, a valid g operand).
PV_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
    uint32_t g19[10];
    fe_mul19(g19, p.T);
    fe_mul_pre(r.X, p.X, p.T, g19);
    pv_sched_fence();
    fe_mul_pre(r.Z, p.Z, p.T, g19);
    pv_sched_fence();
    fe_mul19(g19, p.Y);
    fe_mul_pre(r.Y, p.Z, p.Y, g19);
    pv_sched_fence();
    fe_mul_pre(r.T, p.X, p.Y, g19);
    pv_sched_fence();
}

// r = p + q  (q cached, possibly negated by the caller; p in R). Output limbs < 3 * 2^w + 2^18.
PV_HD void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
    fe a, b, c, d, t;
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, q.YminusX);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, q.YplusX);
    fe_mul(c, p.T, q.T2d);
    fe_mul(d, p.Z, q.Z2);
    fe_sub(r.X, b, a);            // E
    fe_add(r.Y, b, a);            // H
    fe_add(r.Z, d, c);            // G
    fe_sub(r.T, d, c);            // F
}

// r = p + q  (q affine niels, Z = 1). 2Z is not carried, so F = 2Z + 2p - c has limbs up to
// 2^28: the result must go through ge_niels_p1p1_to_p2, which keeps F on the f side.
PV_HD void ge_add_niels(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
    fe a, b, c, d, t;
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, q.yminusx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, q.yplusx);
    fe_mul(c, p.T, q.xy2d);
    fe_add(d, p.Z, p.Z);          // 2 Z
    fe_sub(r.X, b, a);
    fe_add(r.Y, b, a);
    fe_add(r.Z, d, c);
    fe_sub(r.T, d, c);
}

// p1p1 -> p2 for a ge_add_niels result: X = E F, Y = H G, Z = G F with E and G as g operands.
PV_HD void ge_niels_p1p1_to_p2(fe& X, fe& Y, fe& Z, const ge_p1p1& p) {
    uint32_t g19[10];
    fe_mul19(g19, p.X);
    fe_mul_pre(X, p.T, p.X, g19);
    pv_sched_fence();
    fe_mul19(g19, p.Z);
    fe_mul_pre(Y, p.Y, p.Z, g19);
    pv_sched_fence();
    fe_mul_pre(Z, p.T, p.Z, g19);
    pv_sched_fence();
}

// p1p1 -> p3 for a ge_add_niels result (F kept on the f side): X = F E, Y = H G, Z = F G, T = H E.
PV_HD void ge_niels_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
    uint32_t g19[10];
    fe_mul19(g19, p.X);
    fe_mul_pre(r.X, p.T, p.X, g19);
    pv_sched_fence();
    fe_mul_pre(r.T, p.Y, p.X, g19);
    pv_sched_fence();
    fe_mul19(g19, p.Z);
    fe_mul_pre(r.Y, p.Y, p.Z, g19);
    pv_sched_fence();
    fe_mul_pre(r.Z, p.T, p.Z, g19);
    pv_sched_fence();
}

PV_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
    fe d2, t;
    fe_add(r.YplusX, p.Y, p.X);
    fe_sub(r.YminusX, p.Y, p.X);
    fe_add(t, p.Z, p.Z);
    fe_carry(r.Z2, t);
    fe_const(d2, PV_D2);
    fe_mul(r.T2d, p.T, d2);
}

PV_HD void ge_cached_identity(ge_cached& r) {
    fe_1(r.YplusX);
    fe_1(r.YminusX);
    fe_1(r.Z2);
    r.Z2.v[0] = 2;
    fe_0(r.T2d);
}

PV_HD void ge_p3_identity(ge_p3& r) {
    fe_0(r.X);
    fe_1(r.Y);
    fe_1(r.Z);
    fe_0(r.T);
}

// In-place conditional negation of a cached point: swap Y+X / Y-X and negate 2dT.
// Table values are carried to reduced form before storage, so fe_cneg's input bound holds.
PV_HD void ge_cached_cneg(ge_cached& q, bool neg) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t a = q.YplusX.v[i], b = q.YminusX.v[i];
        q.YplusX.v[i] = neg ? b : a;
        q.YminusX.v[i] = neg ? a : b;
    }
    fe_cneg(q.T2d, q.T2d, neg);
}

PV_HD void ge_niels_cneg(ge_niels& q, bool neg) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t a = q.yplusx.v[i], b = q.yminusx.v[i];
        q.yplusx.v[i] = neg ? b : a;
        q.yminusx.v[i] = neg ? a : b;
    }
    fe_cneg(q.xy2d, q.xy2d, neg);
}

// libsodium ge25519_frombytes_negate_vartime: decode the 32-byte encoding s (y mod p; bit 255 =
// sign of x), return -P. false if (y^2 - 1)/(d y^2 + 1) is not a square.
PV_HD bool ge_frombytes_negate(ge_p3& h, const uint32_t s[8]) {
    fe u, v, v3, vxx, chk, d, one;
    fe_frombytes32(h.Y, s);
    fe_1(h.Z);
    fe_1(one);
    fe_sq(u, h.Y);
    fe_const(d, PV_D);
    fe_mul(v, u, d);
    fe_sub(u, u, one);            // u = y^2 - 1
    fe_carry(u, u);
    fe_add(v, v, one);            // v = d y^2 + 1
    fe_carry(v, v);
    fe_sq(v3, v);
    fe_mul(v3, v3, v);            // v^3
    fe_sq(h.X, v3);
    fe_mul(h.X, h.X, v);
    fe_mul(h.X, h.X, u);          // u v^7
    fe_pow22523(h.X, h.X);        // (u v^7)^((p-5)/8)
    fe_mul(h.X, h.X, v3);
    fe_mul(h.X, h.X, u);          // u v^3 (u v^7)^((p-5)/8)
    fe_sq(vxx, h.X);
    fe_mul(vxx, vxx, v);          // v x^2
    fe_sub(chk, vxx, u);
    const bool root_ok = fe_iszero(chk);
    fe_add(chk, vxx, u);
    const bool root_neg = fe_iszero(chk);
    fe sqm1, xs;
    fe_const(sqm1, PV_SQRTM1);
    fe_mul(xs, h.X, sqm1);
    fe_cmov(h.X, xs, !root_ok);
    const uint32_t sign = s[7] >> 31;
    fe_cneg(h.X, h.X, fe_isnegative(h.X) == sign);
    fe_carry(h.X, h.X);
    fe_mul(h.T, h.X, h.Y);
    fe_carry(h.Y, h.Y);
    return root_ok || root_neg;
}

// encode (X:Y:Z) -> 8 words: y canonical, bit 255 = parity of x
PV_HD void ge_p2_tobytes(uint32_t s[8], const fe& X, const fe& Y, const fe& Z) {
    fe zi, x, y;
    fe_invert(zi, Z);
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    fe_tobytes32(s, y);
    s[7] ^= fe_isnegative(x) << 31;
}
