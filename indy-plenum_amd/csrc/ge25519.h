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
static constexpr uint32_t PV_SQRTM1[10] = {0x20ea0b0u, 0x186c9d2u, 0x08f189du, 0x035697fu, 0x0bd0c60u,
                                           0x1fbd7a7u, 0x2804c9eu, 0x1e16569u, 0x004fc1du, 0x0ae0c92u};

PV_HD void fe_const(fe& h, const uint32_t c[10]) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = c[i];
}

// r = 2 * p (p: X, Y, Z reduced). Output limbs are valid mul inputs.
PV_HD void ge_p2_dbl(ge_p1p1& r, const fe& X, const fe& Y, const fe& Z) {
    fe XX, YY, B, S, t;
    fe_sq(XX, X);
    fe_sq(YY, Y);
    fe_sq2(B, Z);
    fe_add(t, X, Y);
    fe_sq(S, t);
    fe_add(r.Y, YY, XX);          // YY + XX            (R + R)
    fe_sub(r.Z, YY, XX);          // YY - XX            (R - R)
    fe_sub4p(t, S, r.Y);          // S - YY - XX = 2XY
    fe_carry(r.X, t);
    fe_sub4p(t, B, r.Z);          // 2Z^2 - YY + XX
    fe_carry(r.T, t);
}

PV_HD void ge_p1p1_to_p2(fe& X, fe& Y, fe& Z, const ge_p1p1& p) {
    fe_mul(X, p.X, p.T);
    fe_mul(Y, p.Y, p.Z);
    fe_mul(Z, p.Z, p.T);
}

PV_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
    fe_mul(r.X, p.X, p.T);
    fe_mul(r.Y, p.Y, p.Z);
    fe_mul(r.Z, p.Z, p.T);
    fe_mul(r.T, p.X, p.Y);
}

// r = p + q  (q cached, possibly negated by the caller)
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

// r = p + q  (q affine niels, Z = 1)
PV_HD void ge_add_niels(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
    fe a, b, c, d, t;
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, q.yminusx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, q.yplusx);
    fe_mul(c, p.T, q.xy2d);
    fe_add(t, p.Z, p.Z);
    fe_carry(d, t);               // 2 Z, reduced
    fe_sub(r.X, b, a);
    fe_add(r.Y, b, a);
    fe_add(r.Z, d, c);
    fe_sub(r.T, d, c);
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
