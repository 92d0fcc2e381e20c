// Keyed fixed-base comb verification: the second arithmetic path of the engine.
//
// Plenum verifies many requests per verification key (one client DID signs many requests; the
// BASELINE workload draws 1M requests from 1,024 signers). When a batch repeats keys, each DISTINCT
// key is decompressed once and expanded into a radix-256 comb table
//     T_A[key][i][d] = [d * 256^i](-A),   i = 0..31, d = 0..128   (cached form, 160 B per entry)
// and the fixed base with a wider radix, since its table is built once (at pv_init, affine niels
// form, 67 MB, Infinity-Cache resident)
//     T_B[j][d]      = [d * 65536^j] B,   j = 0..15, d = 0..32768.
// With k recoded to 32 signed radix-256 digits and S to 16 signed radix-65536 digits, a
// verification is then
//     Q = sum_i T_A[i][e_i] + sum_j T_B[j][f_j]  = [S]B - [k]A
// i.e. 48 point additions and NO doublings (the Straus path needs 252 doublings + 96 additions).
// The encoding / comparison with R is unchanged (pv_encode_batch), so the verdict is the same
// function of (R, S, A, M) as libsodium's crypto_sign_open (stp_core/crypto/nacl_wrappers.py:108).
// Per-key work: one decompression, 254 doublings (the chain of bases [256^i](-A)), ~4,130 additions.
#pragma once
#include "btable.h"
#include "verify_core.h"

static constexpr int PV_COMB_POS = 32;        // radix-256 digit positions
static constexpr int PV_COMB_ENT = 129;       // entries per position (|digit| = 0..128)
static constexpr int PV_COMB_BLOCKS = 8;      // fill work items per (key, position): 16 entries each
static constexpr int PV_BCOMB_STRIDE = 32;    // words per fixed-base entry (30 used)
static constexpr int PV_BCOMB_POS = 16;       // radix-65536 digit positions of S
static constexpr int PV_BCOMB_ENT = 32769;    // entries per position (|digit| = 0..32768)

// ---------------------------------------------------------------- per-key expansion
// Points kept per position i (P_i = [256^i](-A)) for the table fill: slot 0 = P_i, slots 1..3 =
// [16] P_i, [32] P_i, [64] P_i -- the chain passes through them on its way to P_{i+1}.
static constexpr int PV_COMB_PTS = 4;

// out.store(i, m, p): slot m of position i. 31 x 8 doublings (the last position only 6, to reach
// [64] P_31); a doubling whose result is stored or continues the chain as P_{i+1} also forms T.
template <class Bases>
PV_HD void pv_comb_chain(const Bases& out, const ge_p3& negA) {
    ge_p3 cur = negA;
    for (int i = 0; i < PV_COMB_POS; i++) {
        out.store(i, 0, cur);
        fe X = cur.X, Y = cur.Y, Z = cur.Z;
        const int nd = i + 1 < PV_COMB_POS ? 8 : 6;
        for (int j = 0; j < nd; j++) {
            ge_p1p1 t;
            ge_p2_dbl(t, X, Y, Z);
            if ((j >= 3 && j <= 5) || j == 7) {
                ge_p3 q;
                ge_p1p1_to_p3(q, t);
                if (j <= 5) out.store(i, j - 2, q);
                else cur = q;
                X = q.X;
                Y = q.Y;
                Z = q.Z;
            } else {
                ge_p1p1_to_p2(X, Y, Z, t);
            }
        }
    }
}

// Entries d = 16 b + 1 .. 16 b + 16 of one position (block b = 0..7; block 0 also writes the
// identity at d = 0). pts.load(m, p) gives slot m of the position (see pv_comb_chain). The start
// point [16 b] P is a sum of the chain's [16] P, [32] P, [64] P (at most two additions), then 16
// additions of P.
template <class Table, class Pts>
PV_HD void pv_comb_fill_block(const Table& tab, const Pts& pts, int b) {
    ge_p3 P;
    pts.load(0, P);
    ge_cached cP;
    ge_p3_to_cached(cP, P);
    ge_p3 cur;
    ge_p1p1 t;
    if (b == 0) {
        ge_cached id;
        ge_cached_identity(id);
        tab.store(0, id);
        ge_p3_identity(cur);
    } else {
        const int top = b >= 4 ? 2 : (b >= 2 ? 1 : 0);
        pts.load(1 + top, cur);
        for (int bit = top - 1; bit >= 0; bit--) {
            if ((b >> bit) & 1) {
                ge_p3 m;
                pts.load(1 + bit, m);
                ge_cached cm;
                ge_p3_to_cached(cm, m);
                ge_add_cached(t, cur, cm);
                ge_p1p1_to_p3(cur, t);
            }
        }
    }
    for (int d = 16 * b + 1; d <= 16 * b + 16; d++) {
        ge_add_cached(t, cur, cP);
        ge_p1p1_to_p3(cur, t);
        ge_cached c;
        ge_p3_to_cached(c, cur);
        tab.store(d, c);
    }
}

// Sparse fill of one position's row for a small chunk (a few requests per key, AUTO all-comb): only
// the entries the chunk's digits use are built. Always: T[0..16] (the identity and [r] P, r < 16, by
// P-steps) and T[16 q], q = 1..8 (from the chain's [16], [32], [64] P: 5 additions); then every other
// needed entry d = 16 q + r as ONE addition T[16 q] + T[r] (T[16 q] back to extended from its cached
// words: X = (y+x) - (y-x), Y = (y+x) + (y-x), Z = 2Z, T = 2dT / d, i.e. the point times 2). About 20 +
// (needed) additions per position instead of 129. need.word(w) = bits 32 w .. 32 w + 31 of the
// position's needed |digit| set; row.load(d, c) reads back a stored entry.
static constexpr uint32_t PV_SPARSE_PRE[5] = {0x0001FFFFu, 0x00010001u, 0x00010001u, 0x00010001u, 0x1u};
template <class Row, class Pts, class Need>
PV_HD void pv_comb_fill_sparse(const Row& row, const Pts& pts, const Need& need) {
    ge_p3 P, cur;
    pts.load(0, P);
    ge_cached cP, c;
    ge_p3_to_cached(cP, P);
    ge_p1p1 t;
    ge_cached_identity(c);
    row.store(0, c);
    row.store(1, cP);
    cur = P;
    for (int r = 2; r <= 16; r++) {  // [r] P; [16] P again as a check-free by-product (r = 16)
        ge_add_cached(t, cur, cP);
        ge_p1p1_to_p3(cur, t);
        ge_p3_to_cached(c, cur);
        row.store(r, c);
    }
    ge_p3 m16, m32, m64, s;
    pts.load(1, m16);
    pts.load(2, m32);
    pts.load(3, m64);
    ge_cached c16, c32, c64;
    ge_p3_to_cached(c16, m16);
    ge_p3_to_cached(c32, m32);
    ge_p3_to_cached(c64, m64);
    row.store(32, c32);
    row.store(64, c64);
    ge_add_cached(t, m32, c16);  // 48
    ge_p1p1_to_p3(s, t);
    ge_p3_to_cached(c, s);
    row.store(48, c);
    ge_add_cached(t, m64, c16);  // 80
    ge_p1p1_to_p3(s, t);
    ge_p3_to_cached(c, s);
    row.store(80, c);
    ge_add_cached(t, m64, c32);  // 96
    ge_p1p1_to_p3(s, t);
    ge_p3_to_cached(c, s);
    row.store(96, c);
    ge_add_cached(t, s, c16);    // 112
    ge_p1p1_to_p3(s, t);
    ge_p3_to_cached(c, s);
    row.store(112, c);
    ge_add_cached(t, m64, c64);  // 128
    ge_p1p1_to_p3(s, t);
    ge_p3_to_cached(c, s);
    row.store(128, c);
    fe invd;
    fe_const(invd, PV_INVD);
    uint32_t m[5];
#pragma unroll
    for (int w = 0; w < 5; w++) m[w] = need.word(w) & ~PV_SPARSE_PRE[w];
    for (;;) {
        int d = -1;
#pragma unroll
        for (int w = 4; w >= 0; w--)
            if (m[w]) d = 32 * w + __builtin_ctz(m[w]);
        if (d < 0) break;
        m[d >> 5] &= ~(1u << (d & 31));
        ge_cached cq, cr;
        row.load(d & ~15, cq);
        row.load(d & 15, cr);
        ge_p3 q;  // 2 x T[16 q] in extended coordinates
        fe_sub4p(q.X, cq.YplusX, cq.YminusX);
        fe_carry(q.X, q.X);
        fe_add(q.Y, cq.YplusX, cq.YminusX);
        fe_carry(q.Y, q.Y);
        fe_copy(q.Z, cq.Z2);
        fe_mul(q.T, cq.T2d, invd);
        ge_add_cached(t, q, cr);
        ge_p1p1_to_p3(s, t);
        ge_p3_to_cached(c, s);
        row.store(d, c);
    }
}

// ---------------------------------------------------------------- per-request accumulation
// (Y+X, Y-X) of a table entry's first 20 words for a digit of sign `neg` (negation swaps them)
PV_HD void pv_sel_pm(fe& ypx, fe& ymx, const uint32_t w[20], bool neg) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        ypx.v[i] = neg ? w[10 + i] : w[i];
        ymx.v[i] = neg ? w[i] : w[10 + i];
    }
}

// acc + sign(e) T[|e|] for a cached-form table entry (pv_add_a's arithmetic, entry via `load`).
template <class Entry>
PV_HD void pv_comb_add_cached(ge_p1p1& r, const ge_p3& p, const Entry& ent, int e) {
    const int j = e < 0 ? -e : e;
    const bool neg = e < 0;
    fe ypx, ymx, t, a, b, c, d;
    uint32_t w[20];
    ent.load_half(j, 0, w);
    pv_sel_pm(ypx, ymx, w, neg);
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, ymx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, ypx);
    fe z2, t2d;
    ent.load_half(j, 1, w);
#pragma unroll
    for (int i = 0; i < 10; i++) {
        z2.v[i] = w[i];
        t2d.v[i] = w[10 + i];
    }
    fe_cneg(t2d, t2d, neg);
    fe_mul(c, p.T, t2d);
    fe_mul(d, p.Z, z2);
    fe_sub(r.X, b, a);
    fe_add(r.Y, b, a);
    fe_add(r.Z, d, c);
    fe_sub(r.T, d, c);
}

// The two halves of a comb verification, split so that [S]B (which needs only the fixed-base table)
// can run while the per-key tables are still being built:
//   pv_comb_b_acc:  acc = [S]B = sum_j T_B[j][f_j]          16 niels additions, extended result
//   pv_comb_a_xyz:  Q = acc + sum_i T_A[i][e_i]              32 cached additions, projective result
// arows.row(i) / brows.row(j) give the A row of radix-256 position i and the B row of radix-65536
// position j (objects with load_half / load_part); dig holds the packed digits (ek: 4 signed bytes
// of k per word, fs: 2 signed halfwords of S per word).

// Software-pipelined variant (PV_COMB_PIPELINE): a table entry is a dependent load (digit ->
// address) from L2 / Infinity Cache / HBM, so each addition starts the fetch of the NEXT addition's
// entry as soon as it has read its own: `st.stage(row, d)` starts fetching entry d of a row into the
// lane's staging buffer (on the device: LDS-DMA, no VGPRs held while in flight), `st.staged(part, w)`
// reads part of the staged entry back (A: halves of 20 words; B: 20 words, then 10). The fetch of
// entry i - 1 is in flight during the last two multiplications of addition i and its p1p1 -> p3.
#ifndef PV_COMB_PIPELINE
#define PV_COMB_PIPELINE 1
#endif
template <class BStage, class Dig>
PV_HD void pv_comb_b_acc_staged(ge_p3& acc, const BStage& st, const Dig& dig) {
    ge_p3_identity(acc);
    ge_p1p1 t;
    uint32_t fw = dig.fs(7);
    int f = pv_half(fw, PV_BCOMB_POS - 1);
    st.stage(PV_BCOMB_POS - 1, f < 0 ? -f : f);
    for (int j = PV_BCOMB_POS - 1; j >= 0; j--) {
        const bool neg = f < 0;
        uint32_t w[20];
        st.staged(0, w);
        fe ypx, ymx, xy2d, tt, a, b, c, d;
        pv_sel_pm(ypx, ymx, w, neg);
        if (j > 0 && (j & 1) == 0) fw = dig.fs((j - 1) >> 1);  // lands during the two products
        fe_sub(tt, acc.Y, acc.X);
        fe_mul(a, tt, ymx);
        fe_add(tt, acc.Y, acc.X);
        fe_mul(b, tt, ypx);
        st.staged(1, w);
#pragma unroll
        for (int i = 0; i < 10; i++) xy2d.v[i] = w[i];
        if (j > 0) {
            f = pv_half(fw, j - 1);
            st.stage(j - 1, f < 0 ? -f : f);
        }
        fe_cneg(xy2d, xy2d, neg);
        fe_mul(c, acc.T, xy2d);
        fe_add(d, acc.Z, acc.Z);  // 2 Z, not carried (see ge_add_niels)
        fe_sub(t.X, b, a);
        fe_add(t.Y, b, a);
        fe_add(t.Z, d, c);
        fe_sub(t.T, d, c);
        ge_niels_p1p1_to_p3(acc, t);
    }
}

// One cached addition of the staged entry (sign `neg`) to acc; unless LAST, starts the fetch of
// position i - 1's entry (digit from ew, reloaded every 4 positions) between the products.
template <bool LAST, class AStage, class Dig>
PV_HD void pv_comb_a_step(ge_p1p1& t, const ge_p3& acc, const AStage& st, const Dig& dig, int i, uint32_t& ew,
                          int& e) {
    const bool neg = e < 0;
    uint32_t w[20];
    st.staged(0, w);
    fe ypx, ymx, tt, a, b, c, d, z2, t2d;
    pv_sel_pm(ypx, ymx, w, neg);
    if (!LAST && (i & 3) == 0) ew = dig.ek((i - 1) >> 2);  // lands during the two products
    fe_sub(tt, acc.Y, acc.X);
    fe_mul(a, tt, ymx);
    fe_add(tt, acc.Y, acc.X);
    fe_mul(b, tt, ypx);
    const bool aff = st.affine();  // an affine entry (pv_comb_row_to_affine): Z2 = 2, words 20..27 not fetched
    st.staged(1, w);
#pragma unroll
    for (int q = 0; q < 10; q++) {
        z2.v[q] = w[q];
        t2d.v[q] = w[10 + q];
    }
    if (!LAST) {
        e = pv_byte(ew, i - 1);
        st.stage(i - 1, e < 0 ? -e : e);
    }
    fe_cneg(t2d, t2d, neg);
    fe_mul(c, acc.T, t2d);
    if (aff) {
        fe_add(d, acc.Z, acc.Z);
        fe_carry(d, d);
    } else {
        fe_mul(d, acc.Z, z2);
    }
    fe_sub(t.X, b, a);
    fe_add(t.Y, b, a);
    fe_add(t.Z, d, c);
    fe_sub(t.T, d, c);
}

// Positions 31..1 in the loop (extended result, next fetch always started), position 0 peeled: the
// loop body then has no p3/p2 merge (whose phi copies cost ~30 v_mov per addition) and no
// last-iteration branches.
template <class AStage, class Dig>
PV_HD void pv_comb_a_xyz_staged(fe& X, fe& Y, fe& Z, const ge_p3& accB, const AStage& st, const Dig& dig) {
    ge_p3 acc = accB;
    ge_p1p1 t;
    uint32_t ew = dig.ek(7);
    int e = pv_byte(ew, PV_COMB_POS - 1);
    st.stage(PV_COMB_POS - 1, e < 0 ? -e : e);
    for (int i = PV_COMB_POS - 1; i >= 1; i--) {
        pv_comb_a_step<false>(t, acc, st, dig, i, ew, e);
        ge_p1p1_to_p3(acc, t);
    }
    pv_comb_a_step<true>(t, acc, st, dig, 0, ew, e);
    ge_p1p1_to_p2(X, Y, Z, t);
}

// ---------------------------------------------------------------- affine per-key rows
// The node-side key cache also keeps each cached key's rows with every entry divided by its Z: in
// the cached-form layout (40 words: Y+X, Y-X, Z2, 2dT), entry = (y+x, y-x, -, 2dxy). An addition from
// such an entry needs no Z1 Z2 product (Z2 = 2: D = 2 Z1 is an addition) and does not fetch words
// 20..27 (pv_comb_a_step with st.affine()): 7 multiplications and 128 B instead of 8 and 160 B.
// pv_comb_row_to_affine converts one 129-entry cached-form row (src.load(d, c)) with ONE inversion
// (Montgomery's trick): the running products of the Z2 are parked in words 20..29 of output entry d
// (dst.e(d): 40 words) until the backward pass has used them. Cached Z2 = 2 Z, so 1/Z = 2 / Z2.
template <class Src, class Dst>
PV_HD void pv_comb_row_to_affine(const Src& src, const Dst& dst) {
    fe prod;
    fe_1(prod);
    for (int d = 0; d < PV_COMB_ENT; d++) {
        ge_cached c;
        src.load(d, c);
        fe_mul(prod, prod, c.Z2);
        uint32_t* e = dst.e(d);
#pragma unroll
        for (int q = 0; q < 10; q++) e[20 + q] = prod.v[q];
    }
    fe inv;
    fe_invert(inv, prod);
    for (int d = PV_COMB_ENT - 1; d >= 0; d--) {
        ge_cached c;
        src.load(d, c);
        fe zi, zi2, t, ypx, ymx, xy2d;
        if (d > 0) {
            const uint32_t* p = dst.e(d - 1);
            fe prev;
#pragma unroll
            for (int q = 0; q < 10; q++) prev.v[q] = p[20 + q];
            fe_mul(zi, inv, prev);  // 1 / Z2_d
        } else {
            fe_copy(zi, inv);
        }
        fe_mul(inv, inv, c.Z2);
        fe_add(t, zi, zi);  // 1 / Z_d
        fe_carry(zi2, t);
        fe_mul(t, c.YplusX, zi2);
        fe_canonical(ypx, t);
        fe_mul(t, c.YminusX, zi2);
        fe_canonical(ymx, t);
        fe_mul(t, c.T2d, zi2);
        fe_canonical(xy2d, t);
        uint32_t* e = dst.e(d);
#pragma unroll
        for (int q = 0; q < 10; q++) {
            e[q] = ypx.v[q];
            e[10 + q] = ymx.v[q];
            e[20 + q] = 0;
            e[30 + q] = xy2d.v[q];
        }
    }
}

// Staging over plain Rows objects (host tests): stage() remembers the entry, staged() reads it.
template <class ARows>
struct PvRowsStageA {
    const ARows& rows;
    mutable int row_i, ent;
    bool aff = false;  // rows from pv_comb_row_to_affine
    PV_HD void stage(int i, int d) const { row_i = i; ent = d; }
    PV_HD void staged(int h, uint32_t w[20]) const { rows.row(row_i).load_half(ent, h, w); }
    PV_HD bool affine() const { return aff; }
};
template <class BRows>
struct PvRowsStageB {
    const BRows& rows;
    mutable int row_i, ent;
    PV_HD void stage(int i, int d) const { row_i = i; ent = d; }
    PV_HD void staged(int part, uint32_t w[20]) const { rows.row(row_i).load_part(ent, part, w); }
};

template <class BRows, class Dig>
PV_HD void pv_comb_b_acc(ge_p3& acc, const BRows& brows, const Dig& dig) {
    ge_p3_identity(acc);
    ge_p1p1 t;
    uint32_t fw = 0;
    for (int j = PV_BCOMB_POS - 1; j >= 0; j--) {
        if ((j & 1) == 1) fw = dig.fs(j >> 1);
        pv_add_b(t, acc, brows.row(j), pv_half(fw, j));
        ge_niels_p1p1_to_p3(acc, t);
    }
}

template <class ARows, class Dig>
PV_HD void pv_comb_a_xyz(fe& X, fe& Y, fe& Z, const ge_p3& accB, const ARows& arows, const Dig& dig) {
    ge_p3 acc = accB;
    ge_p1p1 t;
    uint32_t ew = 0;
    for (int i = PV_COMB_POS - 1; i >= 0; i--) {
        if ((i & 3) == 3) ew = dig.ek(i >> 2);
        pv_comb_add_cached(t, acc, arows.row(i), pv_byte(ew, i));
        if (i > 0) {
            ge_p1p1_to_p3(acc, t);
        } else {
            ge_p1p1_to_p2(X, Y, Z, t);
        }
    }
}

// Q = [S]B + [k](-A) from the comb tables (both halves in one call: host tests).
template <class ARows, class BRows, class Dig>
PV_HD void pv_comb_xyz(fe& X, fe& Y, fe& Z, const ARows& arows, const BRows& brows, const Dig& dig) {
    ge_p3 acc;
#if PV_COMB_PIPELINE
    pv_comb_b_acc_staged(acc, PvRowsStageB<BRows>{brows, 0, 0}, dig);
    pv_comb_a_xyz_staged(X, Y, Z, acc, PvRowsStageA<ARows>{arows, 0, 0}, dig);
#else
    pv_comb_b_acc(acc, brows, dig);
    pv_comb_a_xyz(X, Y, Z, acc, arows, dig);
#endif
}

// ---------------------------------------------------------------- wide fixed-base comb
// [S]B from a radix-2^W comb held in HBM (288 GB per MI355X: the table is sized for it, not for the
// 256 MB Infinity Cache):  T_B2[j][d] = [d 2^(W j)] B,  j = 0..P-1,  d = 0..2^(W-1) (the top row
// 0..2^TOP), affine niels form, 128 B per entry. W = 24: P = 11 additions per request instead of
// the radix-65536 comb's 16, a 10.7 GB table built on the device at pv_init
// (pv_bc2_build_kernel). Digits: sc_recode_w<W, P>. W = 16 reproduces the radix-65536 comb's
// digits and table (host tests run this code over it).
#ifndef PV_BCOMB_W
#define PV_BCOMB_W 24
#endif
static constexpr int PV_BC2_W = PV_BCOMB_W;
static constexpr int PV_BC2_POS = (253 + PV_BC2_W - 1) / PV_BC2_W;
static constexpr int PV_BC2_TOPBITS = 253 - PV_BC2_W * (PV_BC2_POS - 1);
static constexpr uint32_t PV_BC2_ENT = (1u << (PV_BC2_W - 1)) + 1u;        // rows 0 .. P-2
static constexpr uint32_t PV_BC2_TOP_ENT = (1u << PV_BC2_TOPBITS) + 1u;     // row P-1
static_assert(PV_BC2_TOP_ENT <= PV_BC2_ENT, "top row larger than a full row");

// acc = [S]B = sum_j T[j][e_j] for P positions, digit(j) = e_j (signed). The top position's entry
// is converted to an extended point instead of being added to the identity (X = y+x - (y-x),
// Y = y+x + y-x, Z = 2, T = X Y / 2: two products instead of an addition's seven); then P - 1 niels
// additions, each staging the next position's entry while it multiplies (st.stage / st.staged as in
// pv_comb_b_acc_staged).
//
// total > P (per lane): positions total - 1 .. 0 with the stage / digit objects mapping the extra
// positions to other niels rows -- a cached key's radix-65536 rows (pv_kc_wide: [k](-A) as 16 more
// niels additions in the same loop).
// Niels additions of positions jtop .. 0 into acc; f = the digit of position jtop, whose entry is
// already staging (st.stage(jtop, |f|)).
template <class BStage, class Digit>
PV_HD void pv_comb_b_steps_w(ge_p3& acc, const BStage& st, const Digit& digit, int f, int jtop) {
    ge_p1p1 t;
    for (int j = jtop; j >= 0; j--) {
        const bool neg = f < 0;
        uint32_t w[20];
        st.staged(0, w);
        fe ypx, ymx, xy2d, tt, a, b, c, d;
        pv_sel_pm(ypx, ymx, w, neg);
        const int fn = j > 0 ? digit(j - 1) : 0;  // lands during the two products
        fe_sub(tt, acc.Y, acc.X);
        fe_mul(a, tt, ymx);
        fe_add(tt, acc.Y, acc.X);
        fe_mul(b, tt, ypx);
        st.staged(1, w);
#pragma unroll
        for (int i = 0; i < 10; i++) xy2d.v[i] = w[i];
        if (j > 0) {
            f = fn;
            st.stage(j - 1, f < 0 ? -f : f);
        }
        fe_cneg(xy2d, xy2d, neg);
        fe_mul(c, acc.T, xy2d);
        fe_add(d, acc.Z, acc.Z);  // 2 Z, not carried (see ge_add_niels)
        fe_sub(t.X, b, a);
        fe_add(t.Y, b, a);
        fe_add(t.Z, d, c);
        fe_sub(t.T, d, c);
        ge_niels_p1p1_to_p3(acc, t);
    }
}

template <int P, class BStage, class Digit>
PV_HD void pv_comb_b_acc_w(ge_p3& acc, const BStage& st, const Digit& digit, int total = P) {
    int f = digit(total - 1);
    st.stage(total - 1, f < 0 ? -f : f);
    {
        uint32_t w[20];
        st.staged(0, w);
        fe ypx, ymx, h;
        pv_sel_pm(ypx, ymx, w, f < 0);
        f = digit(total - 2);
        st.stage(total - 2, f < 0 ? -f : f);
        fe_sub(acc.X, ypx, ymx);
        fe_carry(acc.X, acc.X);
        fe_add(acc.Y, ypx, ymx);
        fe_carry(acc.Y, acc.Y);
        fe_0(acc.Z);
        acc.Z.v[0] = 2;
        fe_const(h, PV_INV2);
        fe_mul(acc.T, acc.X, acc.Y);
        fe_mul(acc.T, acc.T, h);
    }
    pv_comb_b_steps_w(acc, st, digit, f, total - 2);
}

// acc += sum_j T[j][digit(j)], j = P-1 .. 0: the fixed-base part added into a point the caller already
// holds (the Straus loop's epilogue adds [k2 S]B this way, pv_msm_kernel).
template <int P, class BStage, class Digit>
PV_HD void pv_comb_b_add_w(ge_p3& acc, const BStage& st, const Digit& digit) {
    const int f = digit(P - 1);
    st.stage(P - 1, f < 0 ? -f : f);
    pv_comb_b_steps_w(acc, st, digit, f, P - 1);
}

// ---------------------------------------------------------------- wide per-key rows (key cache)
// A cached key may also hold radix-65536 rows W_A[q][d] = [d 65536^q](-A), q = 0..15, d = 0..32896,
// affine niels (pv_bc2_build_run's format, 128 B per entry, 67 MB per key): [k](-A) is then 16 niels
// additions (7 multiplications each) instead of 32 cached ones (8 each, 7 from the affine rows). The
// digit of position q is built from the radix-256 digits the request already has:
// d_q = e_{2q} + 256 e_{2q+1}, |d_q| <= 128 + 256 x 128 = 32896 -- no second recoding.
static constexpr int PV_KW_POS = 16;
static constexpr uint32_t PV_KW_ENT = 32897;
PV_HD int pv_kw_digit(uint32_t ek_word, int q) {  // ek_word = radix-256 digit word q >> 1
    return pv_byte(ek_word, 2 * q) + 256 * pv_byte(ek_word, 2 * q + 1);
}

// Wide fixed-base comb build, one run of cnt consecutive entries d0 .. d0 + cnt - 1 of the row of
// base point P (pv_bc2_build_kernel: one run per thread): the start [d0] P by double-and-add, then
// P-steps, each projective point parked in its own entry (row.e(d): 32 words) with the running
// product of the Z's in scr; ONE inversion per run (Montgomery's trick) then gives every entry's
// affine niels form (y+x, y-x, 2dxy) in canonical limbs -- the same entries as
// pv_bcomb_build_position for W = 16 (host test).
template <class Row, class Scr>
PV_HD void pv_bc2_build_run(const Row& row, const Scr& scr, const ge_p3& P, uint32_t d0, uint32_t cnt) {
    ge_cached cP;
    ge_p3_to_cached(cP, P);
    ge_p3 cur;
    ge_p3_identity(cur);
    ge_p1p1 t;
    for (int b = 31; b >= 0; b--) {
        if (d0 >> (b + 1)) {
            ge_p2_dbl(t, cur.X, cur.Y, cur.Z);
            ge_p1p1_to_p3(cur, t);
        }
        if ((d0 >> b) & 1u) {
            ge_add_cached(t, cur, cP);
            ge_p1p1_to_p3(cur, t);
        }
    }
    fe prod;
    fe_1(prod);
    for (uint32_t k = 0; k < cnt; k++) {
        uint32_t* e = row.e(d0 + k);
        fe_mul(prod, prod, cur.Z);
#pragma unroll
        for (int q = 0; q < 10; q++) {
            e[q] = cur.X.v[q];
            e[10 + q] = cur.Y.v[q];
            e[20 + q] = cur.Z.v[q];
        }
        scr.store(d0 + k, prod);
        ge_add_cached(t, cur, cP);
        ge_p1p1_to_p3(cur, t);
    }
    fe inv, d2;
    fe_invert(inv, prod);
    fe_const(d2, PV_D2);
    for (int k = (int)cnt - 1; k >= 0; k--) {
        uint32_t* e = row.e(d0 + (uint32_t)k);
        fe X, Y, Z, zi, x, y, tt, ypx, ymx, xy2d;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            X.v[q] = e[q];
            Y.v[q] = e[10 + q];
            Z.v[q] = e[20 + q];
        }
        if (k > 0) {
            fe prev;
            scr.load(d0 + (uint32_t)k - 1, prev);
            fe_mul(zi, inv, prev);
        } else {
            fe_copy(zi, inv);
        }
        fe_mul(inv, inv, Z);
        fe_mul(x, X, zi);
        fe_mul(y, Y, zi);
        fe_add(tt, y, x);
        fe_canonical(ypx, tt);
        fe_sub(tt, y, x);
        fe_canonical(ymx, tt);
        fe_mul(tt, x, y);
        fe_mul(tt, tt, d2);
        fe_canonical(xy2d, tt);
#pragma unroll
        for (int q = 0; q < 10; q++) {
            e[q] = ypx.v[q];
            e[10 + q] = ymx.v[q];
            e[20 + q] = xy2d.v[q];
        }
        e[30] = 0;
        e[31] = 0;
    }
}

// ---------------------------------------------------------------- fixed-base comb (host, init)
// T_B[j][d] = [d 65536^j] B in affine niels form (y+x, y-x, 2dxy), canonical limbs, PV_BCOMB_STRIDE
// words per entry. Built on the host: one thread per position (16), each with one batched
// inversion (Montgomery's trick) over its 32,769 entries.
inline void pv_bcomb_build_position(uint32_t* out, const ge_p3& P) {
    const int N = PV_BCOMB_ENT;
    ge_p3* pts = new ge_p3[N];
    fe* pre = new fe[N];
    ge_cached cP;
    ge_p3_to_cached(cP, P);
    ge_p3 cur;
    ge_p3_identity(cur);
    fe acc;
    fe_1(acc);
    for (int d = 0; d < N; d++) {
        pts[d] = cur;
        pre[d] = acc;
        fe_mul(acc, acc, cur.Z);
        ge_p1p1 t;
        ge_add_cached(t, cur, cP);
        ge_p1p1_to_p3(cur, t);
    }
    fe inv;
    fe_invert(inv, acc);
    fe d2;
    fe_const(d2, PV_D2);
    for (int d = N - 1; d >= 0; d--) {
        fe zi, x, y, t, ypx, ymx, xy2d;
        fe_mul(zi, inv, pre[d]);
        fe_mul(inv, inv, pts[d].Z);
        fe_mul(x, pts[d].X, zi);
        fe_mul(y, pts[d].Y, zi);
        fe_add(t, y, x);
        fe_canonical(ypx, t);
        fe_sub(t, y, x);
        fe_canonical(ymx, t);
        fe_mul(t, x, y);
        fe_mul(t, t, d2);
        fe_canonical(xy2d, t);
        uint32_t* e = out + (uint64_t)d * PV_BCOMB_STRIDE;
        for (int q = 0; q < 10; q++) {
            e[q] = ypx.v[q];
            e[10 + q] = ymx.v[q];
            e[20 + q] = xy2d.v[q];
        }
        e[30] = 0;
        e[31] = 0;
    }
    delete[] pre;
    delete[] pts;
}

// the 16 position bases [65536^j] B, extended
inline void pv_bcomb_bases(ge_p3 base[PV_BCOMB_POS]) {
    ge_p3 negB, P;
    ge_frombytes_negate(negB, PV_B_ENC);
    P = negB;
    fe z;
    fe_0(z);
    fe_sub(P.X, z, negB.X);
    fe_carry(P.X, P.X);
    fe_sub(P.T, z, negB.T);
    fe_carry(P.T, P.T);
    for (int j = 0; j < PV_BCOMB_POS; j++) {
        base[j] = P;
        for (int r = 0; r < 16; r++) {
            ge_p1p1 t;
            ge_p2_dbl(t, P.X, P.Y, P.Z);
            ge_p1p1_to_p3(P, t);
        }
    }
}
