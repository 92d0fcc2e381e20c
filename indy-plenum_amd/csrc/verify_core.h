// One Ed25519 verification per lane: libsodium 1.0.18 crypto_sign_open acceptance, bit-exact.
//
// Reference path: stp_core/crypto/nacl_wrappers.py:232-242 Verifier.verify
// -> VerifyKey.verify(signature + msg) (:86-108) -> libnacl.crypto_sign_open(sm, pk) -> libsodium
// crypto_sign_ed25519_open -> crypto_sign_ed25519_verify_detached.
//
// Pipeline per request (all integer VALU work):
//   1. checks: smlen >= 64, S < L, R and A not small-order, A canonical      (bytewise)
//   2. A' = -A by decompression (one x^((p-5)/8) chain)                       (~265 field ops)
//   3. k = SHA-512(R || A || M) mod L                                         (3 compressions @ 299 B)
//   4. Q = [S]B + [k]A' by a Straus double-scalar multiplication with regular windows: signed
//      radix-16 digits of k against a 9-entry table of [j]A' (cached form, per-lane, in HBM),
//      signed radix-256 digits of S against a 129-entry niels table of [j]B (LDS). Regular windows
//      keep all 64 lanes of a wave on one instruction stream (sliding windows would diverge).
//   5. accept iff encode(Q) == R bytewise (one inversion, canonical encoding).
// The table/B-table storage is a template parameter so the same code runs on the host in tests.
#pragma once
#include "fe25519.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

// The 7 small-order encodings libsodium 1.0.18 rejects (ge25519_has_small_order), as words.
static constexpr uint32_t PV_BLACKLIST[7][8] = {
    {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x8f95e826u, 0xb027b2c2u, 0x89f4c345u, 0xf098eff2u, 0x05acdfd5u, 0x3933c6d3u, 0x880238b1u, 0x05fc536du},
    {0x706a17c7u, 0x4fd84d3du, 0x760b3cbau, 0x0f67100du, 0xfa53202au, 0xc6cc392cu, 0x77fdc74eu, 0x7a03ac92u},
    {0xffffffecu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
    {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu},
    {0xffffffeeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu}};

PV_HD bool pv_has_small_order(const uint32_t s[8]) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < 7; k++) {
        uint32_t diff = 0;
#pragma unroll
        for (int i = 0; i < 7; i++) diff |= s[i] ^ PV_BLACKLIST[k][i];
        diff |= (s[7] & 0x7fffffffu) ^ PV_BLACKLIST[k][7];
        any |= diff == 0;
    }
    return any;
}

// libsodium ge25519_is_canonical: false iff y in [p, 2^255) (top bit ignored)
PV_HD bool pv_ge_is_canonical(const uint32_t s[8]) {
    uint32_t all = s[1] & s[2] & s[3] & s[4] & s[5] & s[6];
    const bool top = ((s[7] & 0x7fffffffu) == 0x7fffffffu) && all == 0xffffffffu;
    const bool low = s[0] >= 0xffffffedu;
    return !(top && low);
}

struct pv_sig_words {
    uint32_t R[8], S[8], A[8];
};

PV_HD void ge_cached_store_words(uint32_t w[40], const ge_cached& c) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        w[i] = c.YplusX.v[i];
        w[10 + i] = c.YminusX.v[i];
        w[20 + i] = c.Z2.v[i];
        w[30 + i] = c.T2d.v[i];
    }
}
PV_HD void ge_cached_load_words(ge_cached& c, const uint32_t w[40]) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        c.YplusX.v[i] = w[i];
        c.YminusX.v[i] = w[10 + i];
        c.Z2.v[i] = w[20 + i];
        c.T2d.v[i] = w[30 + i];
    }
}

// Build the 9-entry table of [j](-A), j = 0..8, in cached form (entry 0 = identity). PV_TABLE_DBL: the
// even entries 2, 4, 6, 8 by doubling (4 S + 4 M) entries 1, 2, 3, 4 -- read back from the table as the
// projective point (Y+X - (Y-X) : Y+X + (Y-X) : 2Z) = (2X : 2Y : 2Z) -- and the odd ones by one addition
// (8 M) of entry 1: 3 additions and 4 doublings instead of 6 and 1.
#ifndef PV_TABLE_DBL
#define PV_TABLE_DBL 0  // measured slower: table stage 1.76 vs 1.71-1.73 ms (profiles/r06/ab/ab_straus_topload_tabdbl.txt)
#endif
// (2X : 2Y : 2Z) of a stored cached entry, X and Y carried (ge_p2_dbl takes reduced limbs)
template <class ATab>
PV_HD void pv_table_entry_p2(fe& X, fe& Y, fe& Z, const ATab& tab, int j) {
    uint32_t w[40];
    tab.load(j, w);
    fe ypx, ymx, t;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = w[i];
        ymx.v[i] = w[10 + i];
        Z.v[i] = w[20 + i];
    }
    fe_sub4p(t, ypx, ymx);  // Y-X is a sum of reduced values (ge_p3_to_cached)
    fe_carry(X, t);
    fe_add(t, ypx, ymx);
    fe_carry(Y, t);
}
template <class ATab>
PV_HD void pv_build_a_table(ATab& tab, const ge_p3& negA) {
    ge_cached c, c1;
    uint32_t w[40];
    ge_cached_identity(c);
    ge_cached_store_words(w, c);
    tab.store(0, w);
    ge_p3_to_cached(c1, negA);
    ge_cached_store_words(w, c1);
    tab.store(1, w);
    ge_p1p1 t;
    ge_p3 cur;
    ge_p2_dbl(t, negA.X, negA.Y, negA.Z);
    ge_p1p1_to_p3(cur, t);
    ge_p3_to_cached(c, cur);
    ge_cached_store_words(w, c);
    tab.store(2, w);
#if PV_TABLE_DBL
#pragma nounroll
    for (int j = 3; j <= 7; j += 2) {
        ge_add_cached(t, cur, c1);            // [j] = [j - 1] + [1]
        ge_p1p1_to_p3(cur, t);
        ge_p3_to_cached(c, cur);
        ge_cached_store_words(w, c);
        tab.store(j, w);
        fe X, Y, Z;
        pv_table_entry_p2(X, Y, Z, tab, (j + 1) / 2);
        ge_p2_dbl(t, X, Y, Z);                // [j + 1] = 2 [(j + 1) / 2]
        ge_p1p1_to_p3(cur, t);
        ge_p3_to_cached(c, cur);
        ge_cached_store_words(w, c);
        tab.store(j + 1, w);
    }
#else
#pragma nounroll
    for (int j = 3; j <= 8; j++) {
        ge_add_cached(t, cur, c1);
        ge_p1p1_to_p3(cur, t);
        ge_p3_to_cached(c, cur);
        ge_cached_store_words(w, c);
        tab.store(j, w);
    }
#endif
}

// Signed digit i of the packed recodings: nibble i of ek (radix 16), byte i of fs (radix 256).
PV_HD int pv_nibble(uint32_t word, int i) { return ((int32_t)(word << (28 - 4 * (i & 7)))) >> 28; }
PV_HD int pv_byte(uint32_t word, int i) { return ((int32_t)(word << (24 - 8 * (i & 3)))) >> 24; }
PV_HD int pv_half(uint32_t word, int i) { return ((int32_t)(word << (16 - 16 * (i & 1)))) >> 16; }

// A-table lookups come in two halves so that only 20 words of the entry are live at a time:
// half 0 = (Y+X, Y-X), half 1 = (2Z, 2dT) of [|e|](-A); negative digits swap Y+X / Y-X and negate
// 2dT. r = acc + [e](-A) as a p1p1 point (ge_add_cached with the loads interleaved).
template <class ATab>
PV_HD void pv_add_a(ge_p1p1& r, const ge_p3& p, const ATab& atab, int e) {
    const int j = e < 0 ? -e : e;
    const bool neg = e < 0;
    fe ypx, ymx, t, a, b, c, d;
    uint32_t w[20];
    atab.load_half(j, 0, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = neg ? w[10 + i] : w[i];
        ymx.v[i] = neg ? w[i] : w[10 + i];
    }
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, ymx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, ypx);
    fe z2, t2d;
    atab.load_half(j, 1, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        z2.v[i] = w[i];
        t2d.v[i] = w[10 + i];
    }
    fe_cneg(t2d, t2d, neg);
    fe_mul(c, p.T, t2d);
    fe_mul(d, p.Z, z2);
    fe_sub(r.X, b, a);            // E
    fe_add(r.Y, b, a);            // H
    fe_add(r.Z, d, c);            // G
    fe_sub(r.T, d, c);            // F
}

// acc = [e](table point) straight from the cached entry (Y+X, Y-X, 2Z, 2dT): the extended point
// (2X : 2Y : 2Z : 2T) with 2T = 2dT / d -- one product, where adding the entry to the identity took an
// addition and its conversion (8). X and Y carried (X is subtracted by the next addition).
template <class ATab>
PV_HD void pv_load_a_p3(ge_p3& r, const ATab& atab, int e) {
    const int j = e < 0 ? -e : e;
    const bool neg = e < 0;
    fe ypx, ymx, t, invd;
    uint32_t w[20];
    atab.load_half(j, 0, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = neg ? w[10 + i] : w[i];
        ymx.v[i] = neg ? w[i] : w[10 + i];
    }
    fe_sub4p(t, ypx, ymx);        // the entry's Y-X is a sum of reduced values (ge_p3_to_cached)
    fe_carry(r.X, t);             // 2X
    fe_add(t, ypx, ymx);
    fe_carry(r.Y, t);             // 2Y
    atab.load_half(j, 1, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.Z.v[i] = w[i];          // 2Z
        t.v[i] = w[10 + i];
    }
    fe_cneg(t, t, neg);
    fe_const(invd, PV_INVD);
    fe_mul(r.T, t, invd);         // 2T
}

// r = acc + [f]B (B-table entry in affine niels form, loaded in two parts like pv_add_a).
template <class BTab>
PV_HD void pv_add_b(ge_p1p1& r, const ge_p3& p, const BTab& btab, int f) {
    const int j = f < 0 ? -f : f;
    const bool neg = f < 0;
    fe ypx, ymx, xy2d, t, a, b, c, d;
    uint32_t w[20];
    btab.load_part(j, 0, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = neg ? w[10 + i] : w[i];
        ymx.v[i] = neg ? w[i] : w[10 + i];
    }
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, ymx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, ypx);
    btab.load_part(j, 1, w);
#pragma unroll
    for (int i = 0; i < 10; i++) xy2d.v[i] = w[i];
    fe_cneg(xy2d, xy2d, neg);
    fe_mul(c, p.T, xy2d);
    fe_add(d, p.Z, p.Z);          // 2 Z, not carried (see ge_add_niels)
    fe_sub(r.X, b, a);
    fe_add(r.Y, b, a);
    fe_add(r.Z, d, c);
    fe_sub(r.T, d, c);
}

// Q = [S]B + [k]A' (A' = -A, tabulated) from the packed signed digits of k (radix 16) and
// S (radix 256), read from dig one 32-bit word (8 windows) at a time; returns encode(Q) in out[8].
template <class ATab, class BTab, class Dig>
PV_HD void pv_straus_xyz(fe& X, fe& Y, fe& Z, const ATab& atab, const BTab& btab, const Dig& dig) {
    ge_p3 acc;
    ge_p3_identity(acc);
    ge_p1p1 t;
    uint32_t ekw = 0, fsw = 0;
    for (int win = 63; win >= 0; win--) {
        if ((win & 7) == 7) {
            ekw = dig.ek(win >> 3);
            fsw = dig.fs(win >> 3);
        }
        const int e = pv_nibble(ekw, win);
        if (win != 63) {
            for (int j = 0; j < 3; j++) {
                ge_p2_dbl(t, X, Y, Z);
                ge_p1p1_to_p2(X, Y, Z, t);
            }
            ge_p2_dbl(t, X, Y, Z);
            ge_p1p1_to_p3(acc, t);
        }
        pv_add_a(t, acc, atab, e);
        if ((win & 1) == 0) {
            const int f = pv_byte(fsw, win >> 1);
            ge_p1p1_to_p3(acc, t);
            pv_add_b(t, acc, btab, f);
            ge_niels_p1p1_to_p2(X, Y, Z, t);
        } else {
            ge_p1p1_to_p2(X, Y, Z, t);
        }
    }
}

// Q = [k]A' + accB: the same regular-window loop over the radix-16 digits of k with the A table
// only, then ONE cached addition of accB = [S]B (extended; the wide fixed-base comb, comb.h
// pv_comb_b_acc_w). Drops the 32 interleaved B additions (32 x 7 products) for ~11 additions in
// the comb plus the final one. load_accB(p) fetches accB only after the loop (no registers held).
template <class ATab, class Dig, class AccB>
PV_HD void pv_straus_a_xyz(fe& X, fe& Y, fe& Z, const ATab& atab, const Dig& dig, const AccB& load_accB) {
    ge_p3 acc;
    ge_p3_identity(acc);
    ge_p1p1 t;
    uint32_t ekw = 0;
    for (int win = 63; win >= 0; win--) {
        if ((win & 7) == 7) ekw = dig.ek(win >> 3);
        const int e = pv_nibble(ekw, win);
        if (win != 63) {
            for (int j = 0; j < 3; j++) {
                ge_p2_dbl(t, X, Y, Z);
                ge_p1p1_to_p2(X, Y, Z, t);
            }
            ge_p2_dbl(t, X, Y, Z);
            ge_p1p1_to_p3(acc, t);
        }
        pv_add_a(t, acc, atab, e);
        if (win > 0) ge_p1p1_to_p2(X, Y, Z, t);
    }
    ge_p1p1_to_p3(acc, t);
    ge_p3 accB;
    load_accB(accB);
    ge_cached cb;
    ge_p3_to_cached(cb, accB);
    ge_add_cached(t, acc, cb);
    ge_p1p1_to_p2(X, Y, Z, t);
}

// Half-size-scalar Straus loop (sc25519.h sc_halfsize): Q' = [k1](+-A) + [k2](-R') over nw signed
// radix-16 windows of both scalars (two per-lane tables, two cached additions per window, ~33 windows
// instead of 64), then + accB = [k2 S mod L]B and + R' (the R table's entry -1). The result encodes
// to R exactly when Q' + [k2 S]B = [k2](SB - kA - R') is the identity, i.e. when libsodium's
// encode(SB - kA) == R holds (see sc_halfsize). dig.ek(q) / dig.ek2(q): packed digits of |k1| / k2;
// nw: windows (uniform across the wave on the device: the wave's maximum).
// add_b(acc): acc += [k2 S mod L]B, in place (pv_msm_kernel: the wide fixed-base comb's niels additions
// straight into the loop's point; pv_straus_ar_xyz: one cached addition of a point computed elsewhere).
#ifndef PV_STRAUS_TOP_LOAD
#define PV_STRAUS_TOP_LOAD 1  // the top window's A entry loaded as the starting point (0: added to the identity)
#endif
template <class ATab, class RTab, class Dig, class AddB>
PV_HD void pv_straus_ar_xyz_addb(fe& X, fe& Y, fe& Z, const ATab& atab, const RTab& rtab, const Dig& dig, int nw,
                                 const AddB& add_b) {
    ge_p3 acc;
    ge_p1p1 t;
    uint32_t w1 = 0, w2 = 0;
    for (int win = nw - 1; win >= 0; win--) {
        if (win == nw - 1 || (win & 7) == 7) {
            w1 = dig.ek(win >> 3);
            w2 = dig.ek2(win >> 3);
        }
        const int e1 = pv_nibble(w1, win), e2 = pv_nibble(w2, win);
        if (win != nw - 1 || !PV_STRAUS_TOP_LOAD) {
            if (win != nw - 1) {
                for (int j = 0; j < 3; j++) {
                    ge_p2_dbl(t, X, Y, Z);
                    ge_p1p1_to_p2(X, Y, Z, t);
                }
                ge_p2_dbl(t, X, Y, Z);
                ge_p1p1_to_p3(acc, t);
            } else {
                ge_p3_identity(acc);
            }
            pv_add_a(t, acc, atab, e1);
            ge_p1p1_to_p3(acc, t);
        } else {
            pv_load_a_p3(acc, atab, e1);  // the top window starts from the A entry itself
        }
        pv_add_a(t, acc, rtab, e2);
        if (win > 0) ge_p1p1_to_p2(X, Y, Z, t);
    }
    ge_p1p1_to_p3(acc, t);
    add_b(acc);
    pv_add_a(t, acc, rtab, -1);
    ge_p1p1_to_p2(X, Y, Z, t);
}
template <class ATab, class RTab, class Dig, class AccB>
PV_HD void pv_straus_ar_xyz(fe& X, fe& Y, fe& Z, const ATab& atab, const RTab& rtab, const Dig& dig, int nw,
                            const AccB& load_accB) {
    pv_straus_ar_xyz_addb(X, Y, Z, atab, rtab, dig, nw, [&](ge_p3& acc) {
        ge_p3 accB;
        load_accB(accB);
        ge_cached cb;
        ge_p3_to_cached(cb, accB);
        ge_p1p1 t;
        ge_add_cached(t, acc, cb);
        ge_p1p1_to_p3(acc, t);
    });
}

// The same loop with the table entries software-pipelined (as comb.h pv_comb_a_xyz_staged): st.stage(t,
// j) starts fetching entry j of table t (0: [j](+-A), 1: [j](-R')) into the lane's staging buffer (on
// the device LDS-DMA: no VGPRs held while in flight), st.staged(h, w) reads half h of it back. Each
// addition starts the NEXT addition's fetch once it has read its own entry: R_w's during A_w's last
// products, A_(w-1)'s during R_w's and the next window's four doublings.
template <class St>
PV_HD void pv_ar_step(ge_p1p1& r, const ge_p3& p, const St& st, int e, bool next, int nt, int ne) {
    const bool neg = e < 0;
    uint32_t w[20];
    st.staged(0, w);
    fe ypx, ymx, t, a, b, c, d, z2, t2d;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = neg ? w[10 + i] : w[i];
        ymx.v[i] = neg ? w[i] : w[10 + i];
    }
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, ymx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, ypx);
    st.staged(1, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        z2.v[i] = w[i];
        t2d.v[i] = w[10 + i];
    }
    if (next) st.stage(nt, ne < 0 ? -ne : ne);
    fe_cneg(t2d, t2d, neg);
    fe_mul(c, p.T, t2d);
    fe_mul(d, p.Z, z2);
    fe_sub(r.X, b, a);
    fe_add(r.Y, b, a);
    fe_add(r.Z, d, c);
    fe_sub(r.T, d, c);
}
template <class St, class Dig, class AccB>
PV_HD void pv_straus_ar_xyz_staged(fe& X, fe& Y, fe& Z, const St& st, const Dig& dig, int nw, const AccB& load_accB) {
    ge_p3 acc;
    ge_p3_identity(acc);
    ge_p1p1 t;
    uint32_t w1 = dig.ek((nw - 1) >> 3), w2 = dig.ek2((nw - 1) >> 3);
    int e1 = pv_nibble(w1, nw - 1), e2 = pv_nibble(w2, nw - 1);
    st.stage(0, e1 < 0 ? -e1 : e1);
    for (int win = nw - 1; win >= 0; win--) {
        if (win != nw - 1) {
            for (int j = 0; j < 3; j++) {
                ge_p2_dbl(t, X, Y, Z);
                ge_p1p1_to_p2(X, Y, Z, t);
            }
            ge_p2_dbl(t, X, Y, Z);
            ge_p1p1_to_p3(acc, t);
        }
        pv_ar_step(t, acc, st, e1, true, 1, e2);
        ge_p1p1_to_p3(acc, t);
        // the next window's digits (a new word every 8 windows), then R_w with A_(win-1)'s fetch
        int n1 = 0, n2 = 0;
        if (win > 0) {
            if ((win & 7) == 0) {
                w1 = dig.ek((win - 1) >> 3);
                w2 = dig.ek2((win - 1) >> 3);
            }
            n1 = pv_nibble(w1, win - 1);
            n2 = pv_nibble(w2, win - 1);
        }
        pv_ar_step(t, acc, st, e2, win > 0, 0, n1);
        if (win > 0) ge_p1p1_to_p2(X, Y, Z, t);
        e1 = n1;
        e2 = n2;
    }
    ge_p1p1_to_p3(acc, t);
    ge_p3 accB;
    load_accB(accB);
    ge_cached cb;
    ge_p3_to_cached(cb, accB);
    ge_add_cached(t, acc, cb);
    ge_p1p1_to_p3(acc, t);
    st.stage(1, 1);  // + R'
    pv_ar_step(t, acc, st, -1, false, 0, 0);
    ge_p1p1_to_p2(X, Y, Z, t);
}
// Staging over two plain table objects (host tests): stage() remembers the entry, staged() reads it.
template <class ATab>
struct PvTabStage2 {
    const ATab& a;
    const ATab& r;
    mutable int t, j;
    PV_HD void stage(int tab, int ent) const { t = tab; j = ent; }
    PV_HD void staged(int h, uint32_t w[20]) const { (t ? r : a).load_half(j, h, w); }
};

template <class ATab, class BTab, class Dig>
PV_HD void pv_straus(uint32_t out[8], const ATab& atab, const BTab& btab, const Dig& dig) {
    fe X, Y, Z;
    pv_straus_xyz(X, Y, Z, atab, btab, dig);
    ge_p2_tobytes(out, X, Y, Z);
}

// Encodings of PV_ENC_BATCH projective points with ONE field inversion (Montgomery's trick):
// c_t = z_0 ... z_t, inv = c_last^-1, then z_t^-1 = inv * c_{t-1} and inv *= z_t going down.
// A point whose use flag is clear (failed pre-checks, or Z = 0 on garbage input) contributes
// z = 1 so it cannot poison the shared inverse; its encoding is then meaningless and the caller
// masks its verdict. `src` streams the points: src.z(t, Z) and src.xy(t, X, Y) may be called more
// than once for the same t (the device reloads instead of holding the points in registers), and
// sink(t, enc, use) receives each encoding once (in descending t within a group of 8). With 16 points
// per lane the two groups of 8 share the inversion (pv_encode_batch_stream).
#ifndef PV_ENC_BATCH_N
#define PV_ENC_BATCH_N 8
#endif
static constexpr int PV_ENC_BATCH = PV_ENC_BATCH_N;
// One group of H points t0 .. t0 + H - 1 whose prefix products c[0..H-1] (of the masked z) are in c and
// whose product's inverse is inv: the encodings, in descending t. Each point's loads are issued one
// point ahead (the next point's z, x, y land while this one's four products run: the encode runs at one
// or two waves per SIMD, where nothing else would cover them).
template <int H, class Src, class Sink>
PV_HD void pv_encode_group(const Src& src, const bool* use, const Sink& sink, const fe* c, fe inv, int t0) {
    fe Zn, Xn, Yn;
    src.z(t0 + H - 1, Zn);
    src.xy(t0 + H - 1, Xn, Yn);
#pragma unroll
    for (int t = H - 1; t >= 0; t--) {
        const fe Z = Zn, X = Xn, Y = Yn;
        if (t > 0) {
            src.z(t0 + t - 1, Zn);
            src.xy(t0 + t - 1, Xn, Yn);
        }
        fe zi;
        if (t > 0) {
            fe z;
            fe_1(z);
            fe_cmov(z, Z, use[t0 + t]);
            fe_mul(zi, inv, c[t - 1]);
            fe_mul(inv, inv, z);
        } else {
            fe_copy(zi, inv);
        }
        fe x, y;
        fe_mul(x, X, zi);
        fe_mul(y, Y, zi);
        uint32_t enc[8];
        fe_tobytes32(enc, y);
        enc[7] ^= fe_isnegative(x) << 31;
        sink(t0 + t, enc, use[t0 + t]);
    }
}
// Prefix products c[t] = z_t0 ... z_(t0+t) of a group's masked z; sets use[] false where Z = 0. The
// group's z are all loaded before the products.
template <int H, class Src>
PV_HD void pv_encode_prefix(const Src& src, bool* use, fe* c, int t0) {
    fe Zs[H];
#pragma unroll
    for (int t = 0; t < H; t++) src.z(t0 + t, Zs[t]);
#pragma unroll
    for (int t = 0; t < H; t++) {
        fe z;
        use[t0 + t] = use[t0 + t] && !fe_iszero(Zs[t]);
        fe_1(z);
        fe_cmov(z, Zs[t], use[t0 + t]);
        if (t == 0) fe_copy(c[0], z);
        else fe_mul(c[t], c[t - 1], z);
    }
}
// The batch's one inversion: each lane inverts its own product (fe_invert), unless the caller passes a
// wave-wide inverter (pv_engine.hip PvWaveInvert: every lane of the wave at once, limb-parallel).
struct PvFeInvert {
    PV_HD void operator()(fe& x) const { fe_invert(x, x); }
};
template <int B, class Src, class Sink, class Inv = PvFeInvert>
PV_HD void pv_encode_batch_stream_b(const Src& src, bool use[B], const Sink& sink, const Inv& invert = Inv()) {
    static_assert(B == 16 || B <= 12, "pv_encode_batch_stream_b: 16, or one group of at most 12");
    if constexpr (B == 16) {
        // two groups of 8 under ONE inversion, holding one group's prefix products at a time: group 1's
        // product first (its prefixes are rebuilt later: 7 products), then group 0's prefixes; inv of
        // the whole product, each group's inverse by one product with the other group's product
        constexpr int H = 8;
        fe c[H];
        pv_encode_prefix<H>(src, use, c, H);
        fe p1;
        fe_copy(p1, c[H - 1]);
        pv_encode_prefix<H>(src, use, c, 0);
        fe inv, inv0, inv1;
        fe_mul(inv, c[H - 1], p1);
        invert(inv);
        fe_mul(inv0, inv, p1);
        fe_mul(inv1, inv, c[H - 1]);
        pv_encode_group<H>(src, use, sink, c, inv0, 0);
        pv_encode_prefix<H>(src, use, c, H);  // the same z (use[] already final): the same prefixes
        pv_encode_group<H>(src, use, sink, c, inv1, H);
    } else {
        fe c[B];
        pv_encode_prefix<B>(src, use, c, 0);
        fe inv;
        fe_copy(inv, c[B - 1]);
        invert(inv);
        pv_encode_group<B>(src, use, sink, c, inv, 0);
    }
}
template <class Src, class Sink>
PV_HD void pv_encode_batch_stream(const Src& src, bool use[PV_ENC_BATCH], const Sink& sink) {
    pv_encode_batch_stream_b<PV_ENC_BATCH>(src, use, sink);
}

// Array form (host tests).
struct pv_enc_arrays {
    const fe *X, *Y, *Z;
    PV_HD void z(int t, fe& o) const { o = Z[t]; }
    PV_HD void xy(int t, fe& x, fe& y) const { x = X[t]; y = Y[t]; }
};
struct pv_enc_out {
    uint32_t (*out)[8];
    PV_HD void operator()(int t, const uint32_t enc[8], bool) const {
        for (int q = 0; q < 8; q++) out[t][q] = enc[q];
    }
};
PV_HD void pv_encode_batch(uint32_t out[PV_ENC_BATCH][8], const fe X[PV_ENC_BATCH], const fe Y[PV_ENC_BATCH],
                           const fe Z[PV_ENC_BATCH], bool use[PV_ENC_BATCH]) {
    pv_encode_batch_stream(pv_enc_arrays{X, Y, Z}, use, pv_enc_out{out});
}

// Digit words held in registers (host tests and small callers).
struct pv_dig_regs {
    uint32_t e[8], f[8];
    PV_HD uint32_t ek(int q) const { return e[q]; }
    PV_HD uint32_t fs(int q) const { return f[q]; }
};

template <class ATab, class BTab>
PV_HD void pv_double_scalarmult(uint32_t out[8], const ATab& atab, const BTab& btab, const uint32_t k[8],
                                const uint32_t S[8]) {
    pv_dig_regs dig;
    sc_recode16(dig.e, k);
    sc_recode256(dig.f, S);
    pv_straus(out, atab, btab, dig);
}

// libsodium's checks on the signature half of a request: smlen >= 64, S < L, R not small-order.
PV_HD bool pv_sig_ok(const pv_sig_words& in, uint64_t smlen) {
    bool ok = smlen >= 64;
    ok &= sc_is_canonical(in.S);
    ok &= !pv_has_small_order(in.R);
    return ok;
}

// libsodium's checks on the key, then -A by decompression: canonical, not small-order, on the curve.
PV_HD bool pv_key_ok_negate(ge_p3& negA, const uint32_t A[8]) {
    bool ok = pv_ge_is_canonical(A);
    ok &= !pv_has_small_order(A);
    ok &= ge_frombytes_negate(negA, A);
    return ok;
}

// k = SHA-512(R || A || M) mod L. The hash input is sm with bytes 32..63 (S) replaced by A, so
// input word q >= 8 is sm word q; T = smlen bytes in total. Block assembly is branch-free: every
// word is loaded (msgword may read up to 152 bytes past the record: PV_BLOB_SLACK covers it), then
// masked / padded arithmetically, so lanes with different lengths never diverge inside a block.
template <class MsgWord>
PV_HD void pv_hash_k(uint32_t k[8], const pv_sig_words& in, uint64_t smlen, const MsgWord& msgword) {
    const uint32_t T = (uint32_t)smlen;
    uint64_t st[8];
    sha512_init(st);
    const uint32_t nblocks = (T + 17 + 127) / 128;
    for (uint32_t b = 0; b < nblocks; b++) {
        uint64_t blk[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t q = 16 * b + j;
            uint64_t raw = msgword(q);  // little-endian bytes 8q..8q+7 of sm
            if (j < 8) {                // block 0 only: R || A
                const uint64_t ra = j < 4 ? pv_pack64(in.R[2 * j + 1], in.R[2 * j])
                                          : pv_pack64(in.A[2 * (j - 4) + 1], in.A[2 * (j - 4)]);
                raw = (b == 0) ? ra : raw;
            }
            // bytes at or beyond T: 0x80, then zeros
            const int32_t rem = (int32_t)T - (int32_t)(8 * q);
            const uint32_t nb = rem < 0 ? 0u : (rem > 8 ? 8u : (uint32_t)rem);
            const uint64_t mask = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
            const uint64_t pad = (rem >= 0 && rem < 8) ? (0x80ull << (8 * rem)) : 0ull;
            raw = (raw & mask) | pad;
            uint64_t be = pv_bswap64(raw);
            if (j == 15 && b == nblocks - 1) be = (uint64_t)T * 8;  // bit length (upper 64 bits zero)
            blk[j] = be;
        }
        sha512_compress(st, blk);
    }
    uint32_t h[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t le = pv_bswap64(st[i]);
        h[2 * i] = (uint32_t)le;
        h[2 * i + 1] = (uint32_t)(le >> 32);
    }
    sc_reduce64(k, h);
}

// Stage 1 of a verification: the checks, A decompression and k. Returns false if any libsodium
// pre-check rejects (the caller still runs the arithmetic on harmless data and masks the verdict).
template <class MsgWord>
PV_HD bool pv_prepare(ge_p3& negA, uint32_t k[8], const pv_sig_words& in, uint64_t smlen,
                      const MsgWord& msgword) {
    bool ok = pv_sig_ok(in, smlen);
    ok &= pv_key_ok_negate(negA, in.A);
    pv_hash_k(k, in, smlen, msgword);
    return ok;
}

// R as a point for the half-size check: libsodium accepts only when encode(Q) == R bytewise, and an
// R' with encode(R') == R exists iff R is canonical (y < p), decodes, and is not x = 0 with the sign
// bit set. Returns -R' and whether such an R' exists (if not, the verdict is a reject).
PV_HD bool pv_r_decode_negate(ge_p3& negR, const uint32_t R[8]) {
    bool ok = pv_ge_is_canonical(R);
    ok &= ge_frombytes_negate(negR, R);
    ok &= !(fe_iszero(negR.X) && (R[7] >> 31));
    return ok;
}

// p = neg ? -p : p, X and T carried back to reduced limbs (p reduced on entry)
PV_HD void ge_p3_cneg(ge_p3& p, bool neg) {
    fe_cneg(p.X, p.X, neg);
    fe_carry(p.X, p.X);
    fe_cneg(p.T, p.T, neg);
    fe_carry(p.T, p.T);
}

// Stage 1 of a half-size verification: every check, PA = [sign k1](-A) (-A, or A when k1 < 0),
// -R', the split of k (sc_halfsize) and s2 = k2 S mod L. false if any check rejects.
template <class MsgWord>
PV_HD bool pv_prepare_half(ge_p3& PA, ge_p3& negR, pv_halfk& hk, uint32_t s2[8], const pv_sig_words& in,
                           uint64_t smlen, const MsgWord& msgword) {
    bool ok = pv_sig_ok(in, smlen);
    ok &= pv_key_ok_negate(PA, in.A);
    ok &= pv_r_decode_negate(negR, in.R);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, msgword);
    sc_halfsize(hk, k);
    sc_mul<5>(s2, hk.k2, in.S);
    ge_p3_cneg(PA, hk.neg);
    return ok;
}

PV_HD bool pv_words_equal(const uint32_t a[8], const uint32_t b[8]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a[i] ^ b[i];
    return d == 0;
}
