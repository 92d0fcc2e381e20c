// Limb-parallel ("lp") GF(2^255-19) and Edwards25519 arithmetic for the low-latency path.
//
// The throughput kernels keep one verification per lane, so one verification is a long serial
// instruction stream: at Plenum's real batch sizes (a ZStack quota is 100 client / 1,000 node
// messages, stp_core/config.py:32-33) the GPU is nearly idle and that stream's length IS the
// latency. Here ONE wave works on ONE verification and spreads every field element over the lanes:
//
//   a field element lives in one 16-lane DPP row, lane k (k = 0..9) holding limb k of the radix-2^25.5
//   representation of fe25519.h (lanes 10..15 are scratch); the wave's four rows hold four elements,
//   e.g. the four coordinates of a point, or the four products of one group operation.
//
// A product h = f g is computed by every lane for its own column k, row by row in parallel:
//   h_k = sum_i  f_i * g_{(k - i) mod 10} * (19 if k < i) * (2 if i and k - i are odd)
// with f_i broadcast inside the row (DPP row_newbcast:i) and g rotated (DPP row_ror:i) from an
// "extended" copy whose scratch lanes 10..15 already hold 19 g_4 .. 19 g_9 (so most wrapped terms
// need no select); the column sums are then carried across lanes with two DPP shift passes.
// Rows are exchanged with gfx950's v_permlane16_swap / v_permlane32_swap (three instructions give
// every row all four rows). One lp multiplication is ~70 wave instructions (10 v_mad_u64_u32)
// instead of ~160 (100 mads) for a per-lane fe_mul, and four of them run at once, so a point
// doubling takes two multiplication latencies.
//
// The same source compiles for the host with lu/lu64/lm = 64-lane arrays and the cross-lane
// operations simulated exactly (tests/native/hostcheck.hip, tests/test_native_host.py), with the
// limb bounds asserted under PV_BOUNDS_CHECK. Bound names: "LR" = limb < 2^w + 2^22.6 (w = 26 even,
// 25 odd), the output of lp_mul; lp_mul needs g's even limbs < 2^27.75 (19 g < 2^32) and odd limbs
// < 2^27.07 (38 g < 2^32), and every column < 2^64 (checked on the host).
#pragma once
#include "fe25519.h"
#include "ge25519.h"
#include "comb.h"
#include "sc25519.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define LP_DEVICE 1
#else
#define LP_DEVICE 0
#endif

// ------------------------------------------------------------------ lane vectors
#if LP_DEVICE
typedef uint32_t lu;    // this lane's 32-bit value
typedef uint64_t lu64;  // this lane's 64-bit value
typedef bool lm;        // this lane's predicate
#define LP_FN __device__ __forceinline__

LP_FN lu lp_lane() { return __lane_id(); }
LP_FN lu lp_sel(lm c, lu a, lu b) { return c ? a : b; }
LP_FN lu64 lp_sel64(lm c, lu64 a, lu64 b) { return c ? a : b; }
LP_FN lm lp_and(lm a, lm b) { return a && b; }
LP_FN lm lp_lt(lu a, uint32_t b) { return a < b; }
LP_FN lm lp_le(lu a, uint32_t b) { return a <= b; }
LP_FN lm lp_ge(lu a, uint32_t b) { return a >= b; }
LP_FN lm lp_eq(lu a, uint32_t b) { return a == b; }
LP_FN lu lp_lo(lu64 x) { return (uint32_t)x; }
LP_FN lu lp_hi(lu64 x) { return (uint32_t)(x >> 32); }
LP_FN lu64 lp_wide(lu x) { return (uint64_t)x; }
LP_FN lu64 lp_join(lu hi, lu lo) { return ((uint64_t)hi << 32) | lo; }
LP_FN lu64 lp_shr64(lu64 x, lu s) { return x >> s; }
LP_FN lu lp_shrv(lu x, lu s) { return x >> s; }
// 64-bit multiply-accumulate: one v_mad_u64_u32
LP_FN lu64 lp_mad(lu a, lu b, lu64 c) { return (uint64_t)a * b + c; }
// DPP row operations (row = 16 lanes): lanes whose source is outside the row read 0
template <int CTRL>
LP_FN lu lp_dpp(lu x) { return (lu)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true); }
template <int I> LP_FN lu lp_bcast(lu x) { return lp_dpp<0x150 + I>(x); }  // row_newbcast:I
template <int I> LP_FN lu lp_ror(lu x) { return I == 0 ? x : lp_dpp<0x120 + I>(x); }  // row_ror:I
template <int I> LP_FN lu lp_shr(lu x) { return lp_dpp<0x110 + I>(x); }  // row_shr:I (lane k <- k - I)
template <int I> LP_FN lu lp_shl(lu x) { return lp_dpp<0x100 + I>(x); }  // row_shl:I (lane k <- k + I)
// gfx950 row exchange: (a, b) -> a with its odd rows replaced by b's even rows, b with its even rows
// replaced by a's odd rows (permlane16); the same on 32-lane halves (permlane32)
LP_FN void lp_swap16(lu& a, lu& b) {
    auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
LP_FN void lp_swap32(lu& a, lu& b) {
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
LP_FN uint32_t lp_readlane(lu x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
LP_FN lu lp_gather(const uint32_t* base, lu idx) { return base[idx]; }
LP_FN uint64_t lp_ballot(lm c) { return __ballot(c); }
LP_FN lm lp_ne(lu a, uint32_t b) { return a != b; }
LP_FN lm lp_ltv(lu a, lu b) { return a < b; }
LP_FN lm lp_or(lm a, lm b) { return a || b; }
LP_FN lu64 lp_sext64(lu x) { return (uint64_t)(int64_t)(int32_t)x; }
LP_FN lu64 lp_neg64(lu64 x) { return ~x + 1u; }
LP_FN lu lp_sar31(lu x) { return (uint32_t)((int32_t)x >> 31); }
#define LP_CHECK(cond, msg) do { } while (0)

#else  // ---------------------------------------------------------- host simulation (64 lanes)
#include <stdio.h>
#include <stdlib.h>
#define LP_FN inline
struct lu {
    uint32_t v[64];
    lu() {}
    lu(uint32_t c) { for (int l = 0; l < 64; l++) v[l] = c; }
};
struct lu64 {
    uint64_t v[64];
    lu64() {}
    lu64(uint64_t c) { for (int l = 0; l < 64; l++) v[l] = c; }
};
struct lm {
    bool v[64];
};
#define LP_MAP(T, expr) T r; for (int l = 0; l < 64; l++) r.v[l] = (expr); return r
LP_FN lu operator+(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] + b.v[l]); }
LP_FN lu operator-(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] - b.v[l]); }
LP_FN lu operator*(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] * b.v[l]); }
LP_FN lu operator&(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] & b.v[l]); }
LP_FN lu operator|(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] | b.v[l]); }
LP_FN lu operator^(const lu& a, const lu& b) { LP_MAP(lu, a.v[l] ^ b.v[l]); }
LP_FN lu operator>>(const lu& a, int s) { LP_MAP(lu, a.v[l] >> s); }
LP_FN lu operator<<(const lu& a, int s) { LP_MAP(lu, a.v[l] << s); }
LP_FN lu64 operator+(const lu64& a, const lu64& b) { LP_MAP(lu64, a.v[l] + b.v[l]); }
LP_FN lu64 operator>>(const lu64& a, int s) { LP_MAP(lu64, a.v[l] >> s); }
LP_FN lu64 operator<<(const lu64& a, int s) { LP_MAP(lu64, a.v[l] << s); }
LP_FN lu lp_lane() { LP_MAP(lu, (uint32_t)l); }
LP_FN lu lp_sel(const lm& c, const lu& a, const lu& b) { LP_MAP(lu, c.v[l] ? a.v[l] : b.v[l]); }
LP_FN lu64 lp_sel64(const lm& c, const lu64& a, const lu64& b) { LP_MAP(lu64, c.v[l] ? a.v[l] : b.v[l]); }
LP_FN lm lp_and(const lm& a, const lm& b) { LP_MAP(lm, a.v[l] && b.v[l]); }
LP_FN lm lp_lt(const lu& a, uint32_t b) { LP_MAP(lm, a.v[l] < b); }
LP_FN lm lp_le(const lu& a, uint32_t b) { LP_MAP(lm, a.v[l] <= b); }
LP_FN lm lp_ge(const lu& a, uint32_t b) { LP_MAP(lm, a.v[l] >= b); }
LP_FN lm lp_eq(const lu& a, uint32_t b) { LP_MAP(lm, a.v[l] == b); }
LP_FN lu lp_lo(const lu64& x) { LP_MAP(lu, (uint32_t)x.v[l]); }
LP_FN lu lp_hi(const lu64& x) { LP_MAP(lu, (uint32_t)(x.v[l] >> 32)); }
LP_FN lu64 lp_wide(const lu& x) { LP_MAP(lu64, (uint64_t)x.v[l]); }
LP_FN lu64 lp_join(const lu& hi, const lu& lo) { LP_MAP(lu64, ((uint64_t)hi.v[l] << 32) | lo.v[l]); }
LP_FN lu64 lp_shr64(const lu64& x, const lu& s) { LP_MAP(lu64, x.v[l] >> s.v[l]); }
LP_FN lu lp_shrv(const lu& x, const lu& s) { LP_MAP(lu, x.v[l] >> s.v[l]); }
LP_FN lu64 lp_mad(const lu& a, const lu& b, const lu64& c) {
    LP_MAP(lu64, (uint64_t)a.v[l] * b.v[l] + c.v[l]);
}
template <int I> LP_FN lu lp_bcast(const lu& x) { LP_MAP(lu, x.v[(l & ~15) + I]); }
template <int I> LP_FN lu lp_ror(const lu& x) { LP_MAP(lu, x.v[(l & ~15) + (((l & 15) - I) & 15)]); }
template <int I> LP_FN lu lp_shr(const lu& x) { LP_MAP(lu, (l & 15) >= I ? x.v[l - I] : 0u); }
template <int I> LP_FN lu lp_shl(const lu& x) { LP_MAP(lu, (l & 15) + I < 16 ? x.v[l + I] : 0u); }
LP_FN void lp_swap16(lu& a, lu& b) {
    lu na = a, nb = b;
    for (int l = 0; l < 64; l++) {
        const int row = l >> 4;
        if (row & 1) na.v[l] = b.v[l - 16];   // a's odd rows <- b's even rows
        else nb.v[l] = a.v[l + 16];           // b's even rows <- a's odd rows
    }
    a = na;
    b = nb;
}
LP_FN void lp_swap32(lu& a, lu& b) {
    lu na = a, nb = b;
    for (int l = 0; l < 32; l++) {
        na.v[l + 32] = b.v[l];  // a's upper half <- b's lower half
        nb.v[l] = a.v[l + 32];  // b's lower half <- a's upper half
    }
    a = na;
    b = nb;
}
LP_FN uint32_t lp_readlane(const lu& x, int l) { return x.v[l]; }
LP_FN lu lp_gather(const uint32_t* base, const lu& idx) { LP_MAP(lu, base[idx.v[l]]); }
LP_FN uint64_t lp_ballot(const lm& c) {
    uint64_t m = 0;
    for (int l = 0; l < 64; l++) m |= (uint64_t)c.v[l] << l;
    return m;
}
LP_FN lm lp_ne(const lu& a, uint32_t b) { LP_MAP(lm, a.v[l] != b); }
LP_FN lm lp_ltv(const lu& a, const lu& b) { LP_MAP(lm, a.v[l] < b.v[l]); }
LP_FN lm lp_or(const lm& a, const lm& b) { LP_MAP(lm, a.v[l] || b.v[l]); }
LP_FN lu64 lp_sext64(const lu& x) { LP_MAP(lu64, (uint64_t)(int64_t)(int32_t)x.v[l]); }
LP_FN lu64 lp_neg64(const lu64& x) { LP_MAP(lu64, ~x.v[l] + 1u); }
LP_FN lu lp_sar31(const lu& x) { LP_MAP(lu, (uint32_t)((int32_t)x.v[l] >> 31)); }
#undef LP_MAP
#ifdef PV_BOUNDS_CHECK
#define LP_CHECK(cond, msg) do { if (!(cond)) { fprintf(stderr, "lp bound violated: %s\n", msg); abort(); } } while (0)
#else
#define LP_CHECK(cond, msg) do { } while (0)
#endif
#endif  // LP_DEVICE

#if !LP_DEVICE
// host bound checks on the limb lanes (k < 10) only
inline void lp_check_limbs(const lu& x, uint32_t bound, const char* msg) {
#ifdef PV_BOUNDS_CHECK
    for (int l = 0; l < 64; l++)
        if ((l & 15) < 10) LP_CHECK(x.v[l] < bound, msg);
#else
    (void)x; (void)bound; (void)msg;
#endif
}
#define LP_BOUND(x, b, msg) lp_check_limbs(x, b, msg)
#else
#define LP_BOUND(x, b, msg) do { } while (0)
#endif

// ------------------------------------------------------------------ per-lane constants
struct LpLane {
    lu k;        // limb index within the row (lane & 15)
    lu row;      // row index (lane >> 4)
    lu w;        // limb width: 26 (even k) / 25 (odd k)
    lu mask;     // 2^w - 1
    lu two_p;    // limb k of 2p (fe_sub's offset)
    lu four_p;   // limb k of 4p
    lm k0;       // k == 0
    lm kge10;    // scratch lane
    lm keven;
    lm row0, row1, row2, row3;
    LP_FN static LpLane make() {
        LpLane c;
        const lu lane = lp_lane();
        c.k = lane & 15u;
        c.row = lane >> 4;
        const lm odd = lp_eq(c.k & 1u, 1u);
        c.w = lp_sel(odd, 25u, 26u);
        c.mask = lp_sel(odd, (uint32_t)M25, (uint32_t)M26);
        c.k0 = lp_eq(c.k, 0u);
        c.two_p = lp_sel(c.k0, 0x7FFFFDAu, lp_sel(odd, 0x3FFFFFEu, 0x7FFFFFEu));
        c.four_p = lp_sel(c.k0, 0xFFFFFB4u, lp_sel(odd, 0x7FFFFFCu, 0xFFFFFFCu));
        c.kge10 = lp_ge(c.k, 10u);
        c.keven = lp_eq(c.k & 1u, 0u);
        c.row0 = lp_eq(c.row, 0u);
        c.row1 = lp_eq(c.row, 1u);
        c.row2 = lp_eq(c.row, 2u);
        c.row3 = lp_eq(c.row, 3u);
        return c;
    }
    // limb k of a constant fe (same value in every row)
    LP_FN lu limb(const uint32_t c[10]) const {
        lu r = 0u;
#pragma unroll
        for (int i = 0; i < 10; i++) r = lp_sel(lp_eq(k, (uint32_t)i), c[i], r);
        return r;
    }
    // row r of the result from a, b, c, d
    LP_FN lu rows(const lu& a, const lu& b, const lu& c, const lu& d) const {
        return lp_sel(row0, a, lp_sel(row1, b, lp_sel(row2, c, d)));
    }
};

// ------------------------------------------------------------------ field operations
LP_FN lu lp_add(const lu& a, const lu& b) { return a + b; }
// a + 2p - b (b limbs <= 2p limbs, e.g. LR)
LP_FN lu lp_sub(const LpLane& c, const lu& a, const lu& b) { return a + c.two_p - b; }
LP_FN lu lp_sub4p(const LpLane& c, const lu& a, const lu& b) { return a + c.four_p - b; }

// One 32-bit carry pass: limbs < 2^32 - 2^13 -> limb < 2^w + 19 * 2^7 (the wrap goes to limb 0).
LP_FN lu lp_carry1(const LpLane& c, const lu& x) {
    const lu cy = lp_shrv(x, c.w);
    const lu l = x & c.mask;
    const lu in = lp_sel(c.k0, lp_shl<9>(cy) * 19u, lp_shr<1>(cy));
    return l + in;
}

// h = f g (row by row). g: even limbs < 2^27.75 (19 g < 2^32), odd limbs < 2^27.07 (38 g < 2^32);
// f: any 32-bit limbs within the column bound (every column < 2^64, checked on the host). Output LR.
// Odd limbs are only 25 bits wide, so every g operand the group formulas form (reduced values,
// sums of two, differences with 2p) meets the odd-limb bound, and the factor 2 of the odd x odd
// terms is applied once to the rotated operand's odd source lanes instead of per term.
LP_FN lu lp_mul(const LpLane& c, const lu& f, const lu& g) {
#if !LP_DEVICE
    for (int l = 0; l < 64; l++) {
        if ((l & 15) >= 10) continue;
        LP_CHECK(g.v[l] < ((l & 1) ? 0x8600000u : 0xD790000u), "lp_mul g operand");
    }
#endif
    // g extended: lanes m >= 6 of Y hold 19 g_{m-6}; X = g on lanes 0..9, Y on scratch lanes 10..15;
    // X2 / Y2: the same with odd lanes doubled (the limb index m or m - 6 has the lane's parity)
    const lu Y = lp_shr<6>(g) * 19u;
    const lu X = lp_sel(c.kge10, Y, g);
    const lu X2 = lp_sel(c.keven, X, X + X);
    const lu Y2 = lp_sel(c.keven, Y, Y + Y);
    lu64 acc = lp_mad(lp_bcast<0>(f), X, lu64(0ull));
#define LP_TERM(I)                                                                        \
    {                                                                                     \
        const lu& src = (I & 1) ? X2 : X;                                                 \
        lu gi = lp_ror<I>(src);                                                           \
        if (I >= 7) gi = lp_sel(lp_le(c.k, (uint32_t)(I - 7)), lp_ror<I>((I & 1) ? Y2 : Y), gi); \
        acc = lp_mad(lp_bcast<I>(f), gi, acc);                                            \
    }
    LP_TERM(1) LP_TERM(2) LP_TERM(3) LP_TERM(4) LP_TERM(5) LP_TERM(6) LP_TERM(7) LP_TERM(8) LP_TERM(9)
#undef LP_TERM
#if !LP_DEVICE && defined(PV_BOUNDS_CHECK)
    {   // exact column bound: recompute each lane's column in 128 bits
        for (int l = 0; l < 64; l++) {
            const int k = l & 15, base = l & ~15;
            if (k >= 10) continue;
            unsigned __int128 s = 0;
            for (int i = 0; i < 10; i++) {
                const int j = ((k - i) % 10 + 10) % 10;
                unsigned __int128 t = (unsigned __int128)f.v[base + i] * g.v[base + j];
                if (k < i) t *= 19;
                if ((i & 1) && (j & 1)) t *= 2;
                s += t;
            }
            LP_CHECK((s >> 64) == 0, "lp_mul column overflow");
            LP_CHECK((uint64_t)s == acc.v[l], "lp_mul column mismatch");
        }
    }
#endif
    // carry pass 1 (64-bit): column k -> limb k + carry from k - 1 (19 * carry of 9 into limb 0)
    const lu64 cy = lp_shr64(acc, c.w);
    const lu lo = lp_lo(acc) & c.mask;
    const lu clo = lp_lo(cy), chi = lp_hi(cy);  // cy < 2^39
    const lu wlo = lp_shl<9>(clo), whi = lp_shl<9>(chi);
    const lu64 w19 = lp_mad(wlo, 19u, lp_join(whi * 19u, 0u));
    const lu64 in = lp_sel64(c.k0, w19, lp_join(lp_shr<1>(chi), lp_shr<1>(clo)));
    const lu64 t = in + lp_wide(lo);  // < 2^26 + 2^43.3
    // carry pass 2 (32-bit)
    const lu cy2 = lp_lo(lp_shr64(t, c.w));  // < 2^18.3
    const lu l2 = lp_lo(t) & c.mask;
    const lu h = l2 + lp_sel(c.k0, lp_shl<9>(cy2) * 19u, lp_shr<1>(cy2));
    LP_BOUND(h, (1u << 26) + (1u << 23), "lp_mul output");
    return h;
}
LP_FN lu lp_sq(const LpLane& c, const lu& f) { return lp_mul(c, f, f); }

// lp_mul for operands whose rows 2, 3 repeat rows 0, 1 (two elements, each held twice, as in the
// decompression chain): rows 0, 1 sum the column terms i = 0..4 and rows 2, 3 the terms i = 5..9 (f
// and the extended g pre-rotated by five limbs there), the halves are added across with one
// v_permlane32_swap per word, and every row carries the full product: 5 term products per lane
// instead of 10. Same bounds and output as lp_mul.
LP_FN lu lp_mul_dual(const LpLane& c, const lu& f, const lu& g) {
#if !LP_DEVICE
    for (int l = 0; l < 32; l++) {
        if ((l & 15) >= 10) continue;  // scratch lanes are never read
        LP_CHECK(f.v[l] == f.v[l + 32] && g.v[l] == g.v[l + 32], "lp_mul_dual rows 2, 3 repeat rows 0, 1");
        LP_CHECK(g.v[l] < ((l & 1) ? 0x8600000u : 0xD790000u), "lp_mul g operand");
    }
#endif
    const lm hi = lp_ge(c.row, 2u);
    // rows 0, 1 (as lp_mul): lanes 0..9 g, lanes m >= 10 19 g_{m-6}
    const lu Y = lp_shr<6>(g) * 19u;
    const lu X = lp_sel(c.kge10, Y, g);
    // rows 2, 3: lane j < 5 19 g_{j+5}, 5 <= j < 10 g_{j-5}, m >= 12 19 g_{m-11}: row_ror:i (i <= 4) of
    // it gives lane k the factor g_{(k-i-5) mod 10} (19 when wrapped) of term i + 5
    const lu Xr = lp_sel(lp_lt(c.k, 5u), lp_shl<5>(g) * 19u, lp_sel(c.kge10, lp_shr<11>(g) * 19u, lp_shr<5>(g)));
    // odd x odd terms doubled on the rotated operand: rows 0, 1 hold limb index = lane parity, rows
    // 2, 3 the opposite; term i + 5 has f index parity opposite to i
    const lu Xo = lp_sel(hi, Xr, X);                       // the operand undoubled ...
    const lu Xd = Xo + Xo;                                 // ... and doubled
    const lm odd_limb = lp_eq((c.k ^ lp_sel(hi, 1u, 0u)) & 1u, 1u);
    const lu D = lp_sel(odd_limb, Xd, Xo);                 // odd limbs doubled
    const lu Ev = lp_sel(hi, D, Xo);                        // even i (rows 2, 3: odd f index i + 5)
    const lu Od = lp_sel(hi, Xo, D);                        // odd i (rows 2, 3: even f index)
    const lu fr = lp_sel(hi, lp_shl<5>(f), f);             // row_newbcast:i gives f_i / f_{i+5}
    lu64 acc = lp_mad(lp_bcast<0>(fr), Ev, lu64(0ull));
    acc = lp_mad(lp_bcast<1>(fr), lp_ror<1>(Od), acc);
    acc = lp_mad(lp_bcast<2>(fr), lp_ror<2>(Ev), acc);
    acc = lp_mad(lp_bcast<3>(fr), lp_ror<3>(Od), acc);
    acc = lp_mad(lp_bcast<4>(fr), lp_ror<4>(Ev), acc);
    // + the other half's partial column (rows r and r ^ 2)
    lu plo = lp_lo(acc), qlo = plo, phi = lp_hi(acc), qhi = phi;
    lp_swap32(plo, qlo);
    lp_swap32(phi, qhi);
    acc = lp_join(phi, plo) + lp_join(qhi, qlo);
    // carries as lp_mul
    const lu64 cy = lp_shr64(acc, c.w);
    const lu lo = lp_lo(acc) & c.mask;
    const lu clo = lp_lo(cy), chi = lp_hi(cy);
    const lu wlo = lp_shl<9>(clo), whi = lp_shl<9>(chi);
    const lu64 w19 = lp_mad(wlo, 19u, lp_join(whi * 19u, 0u));
    const lu64 in = lp_sel64(c.k0, w19, lp_join(lp_shr<1>(chi), lp_shr<1>(clo)));
    const lu64 t = in + lp_wide(lo);
    const lu cy2 = lp_lo(lp_shr64(t, c.w));
    const lu l2 = lp_lo(t) & c.mask;
    const lu h = l2 + lp_sel(c.k0, lp_shl<9>(cy2) * 19u, lp_shr<1>(cy2));
    LP_BOUND(h, (1u << 26) + (1u << 23), "lp_mul_dual output");
    return h;
}

// every row gets row r of x: o0 = row 0 in all rows, ... (3 permlane instructions)
LP_FN void lp_allrows(const lu& x, lu& o0, lu& o1, lu& o2, lu& o3) {
    lu p = x, q = x;
    lp_swap16(p, q);  // p = [x0 x0 x2 x2], q = [x1 x1 x3 x3]
    o0 = p;
    o2 = p;
    lp_swap32(o0, o2);  // o0 = [x0 x0 x0 x0], o2 = [x2 x2 x2 x2]
    o1 = q;
    o3 = q;
    lp_swap32(o1, o3);
}

// DUAL: the operands' rows 2, 3 repeat rows 0, 1 (lp_mul_dual)
template <bool DUAL>
LP_FN lu lp_mulx(const LpLane& c, const lu& f, const lu& g) {
    if constexpr (DUAL) return lp_mul_dual(c, f, g);
    else return lp_mul(c, f, g);
}
template <bool DUAL = false>
LP_FN lu lp_sqn(const LpLane& c, lu x, int n) {
    for (int i = 0; i < n; i++) x = lp_mulx<DUAL>(c, x, x);
    return x;
}
// z^(2^252 - 3) in every row at once (libsodium's chain, as fe_pow22523)
template <bool DUAL = false>
LP_FN lu lp_pow22523(const LpLane& c, const lu& z) {
    lu t0 = lp_mulx<DUAL>(c, z, z);              // z^2
    lu t1 = lp_sqn<DUAL>(c, t0, 2);              // z^8
    t1 = lp_mulx<DUAL>(c, z, t1);                // z^9
    t0 = lp_mulx<DUAL>(c, t0, t1);               // z^11
    lu t2 = lp_mulx<DUAL>(c, t0, t0);            // z^22
    t1 = lp_mulx<DUAL>(c, t1, t2);               // z^(2^5 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 5);
    t1 = lp_mulx<DUAL>(c, t2, t1);               // z^(2^10 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 10);
    t2 = lp_mulx<DUAL>(c, t2, t1);               // z^(2^20 - 1)
    lu t3 = lp_sqn<DUAL>(c, t2, 20);
    t2 = lp_mulx<DUAL>(c, t3, t2);               // z^(2^40 - 1)
    t2 = lp_sqn<DUAL>(c, t2, 10);
    t1 = lp_mulx<DUAL>(c, t2, t1);               // z^(2^50 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 50);
    t2 = lp_mulx<DUAL>(c, t2, t1);               // z^(2^100 - 1)
    t3 = lp_sqn<DUAL>(c, t2, 100);
    t2 = lp_mulx<DUAL>(c, t3, t2);               // z^(2^200 - 1)
    t2 = lp_sqn<DUAL>(c, t2, 50);
    t1 = lp_mulx<DUAL>(c, t2, t1);               // z^(2^250 - 1)
    t1 = lp_sqn<DUAL>(c, t1, 2);                 // z^(2^252 - 4)
    return lp_mulx<DUAL>(c, t1, z);              // z^(2^252 - 3)
}

// z^(p - 2) = 1 / z in every row at once (fe_invert's chain: z^(2^250 - 1), five squarings, times
// z^11). The encode kernel inverts the wave's cross-lane products with it (pv_engine.hip PvWaveInvert):
// a chain of limb-parallel products, ~300 cycles each (fewer with DUAL: two values, five column terms
// per lane), instead of each lane's own chain of 101-instruction squarings.
template <bool DUAL = false>
LP_FN lu lp_invert(const LpLane& c, const lu& z) {
    lu t0 = lp_mulx<DUAL>(c, z, z);               // z^2
    lu t1 = lp_sqn<DUAL>(c, t0, 2);               // z^8
    t1 = lp_mulx<DUAL>(c, z, t1);                 // z^9
    t0 = lp_mulx<DUAL>(c, t0, t1);                // z^11
    lu t2 = lp_mulx<DUAL>(c, t0, t0);             // z^22
    t1 = lp_mulx<DUAL>(c, t1, t2);                // z^(2^5 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 5);
    t1 = lp_mulx<DUAL>(c, t2, t1);                // z^(2^10 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 10);
    t2 = lp_mulx<DUAL>(c, t2, t1);                // z^(2^20 - 1)
    lu t3 = lp_sqn<DUAL>(c, t2, 20);
    t2 = lp_mulx<DUAL>(c, t3, t2);                // z^(2^40 - 1)
    t2 = lp_sqn<DUAL>(c, t2, 10);
    t1 = lp_mulx<DUAL>(c, t2, t1);                // z^(2^50 - 1)
    t2 = lp_sqn<DUAL>(c, t1, 50);
    t2 = lp_mulx<DUAL>(c, t2, t1);                // z^(2^100 - 1)
    t3 = lp_sqn<DUAL>(c, t2, 100);
    t2 = lp_mulx<DUAL>(c, t3, t2);                // z^(2^200 - 1)
    t2 = lp_sqn<DUAL>(c, t2, 50);
    t1 = lp_mulx<DUAL>(c, t2, t1);                // z^(2^250 - 1)
    t1 = lp_sqn<DUAL>(c, t1, 5);                  // z^(2^255 - 32)
    return lp_mulx<DUAL>(c, t1, t0);              // z^(2^255 - 21)
}

// The 10 limbs of row r as a scalar fe (uniform values: v_readlane).
LP_FN fe lp_row_fe(const lu& x, int r) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = lp_readlane(x, 16 * r + i);
    return h;
}

// Lane k of the row gets limb k of the 255-bit little-endian value s[8] (bit 255 ignored), as
// fe_frombytes32. s may differ per row (each lane passes its own row's words).
LP_FN lu lp_from_words(const LpLane& c, const lu s[8]) {
    // limb k = bits [o_k, o_k + w_k) with o = 0, 26, 51, 77, 102, 128, 153, 179, 204, 230
    lu r = 0u;
#define LP_LIMB(K, EXPR) r = lp_sel(lp_eq(c.k, (uint32_t)(K)), (EXPR), r)
    LP_LIMB(0, s[0] & M26);
    LP_LIMB(1, ((s[0] >> 26) | (s[1] << 6)) & M25);
    LP_LIMB(2, ((s[1] >> 19) | (s[2] << 13)) & M26);
    LP_LIMB(3, ((s[2] >> 13) | (s[3] << 19)) & M25);
    LP_LIMB(4, (s[3] >> 6) & M26);
    LP_LIMB(5, s[4] & M25);
    LP_LIMB(6, ((s[4] >> 25) | (s[5] << 7)) & M26);
    LP_LIMB(7, ((s[5] >> 19) | (s[6] << 13)) & M25);
    LP_LIMB(8, ((s[6] >> 12) | (s[7] << 20)) & M26);
    LP_LIMB(9, (s[7] >> 6) & M25);
#undef LP_LIMB
    return r;
}

// ------------------------------------------------------------------ group operations
// Layouts (one lu, rows 0..3):
//   ext      [X, Y, Z, T]          extended coordinates (p3), every limb LR
//   cached   [Y-X, Y+X, 2dT, 2Z]   addend; an affine niels entry [y-x, y+x, 2dxy, 2] has the same form
// Addition / doubling end with a p1p1 -> p3 multiplication, so every result is a full ext point.

// r = p + q (q cached or niels, possibly negated by the caller)
LP_FN lu lp_add_cached(const LpLane& c, const lu& p, const lu& q) {
    // one row exchange gives a = [X X Z Z], b = [Y Y T T]: the operand rows (Y-X, Y+X, T, Z)
    lu a = p, b = p;
    lp_swap16(a, b);
    const lu f = c.rows(lp_sub(c, b, a), b + a, b, a);  // < 2^27.6
    const lu abcd = lp_mul(c, f, q);                     // [A, B, C, D]
    lu A, B, C, D;
    lp_allrows(abcd, A, B, C, D);
    const lu E = lp_sub(c, B, A), H = B + A, G = D + C, F = lp_sub(c, D, C);
    // X3 = E F, Y3 = G H, Z3 = F G, T3 = E H
    return lp_mul(c, c.rows(E, G, F, E), c.rows(F, H, G, H));
}

// r = 2 p (dbl-2008-hwcd with 2XY = 2TZ: rows square X, Y, Z and multiply T Z at once, so the input
// needs no row exchange; p must carry a consistent T, which every lp operation produces)
LP_FN lu lp_dbl(const LpLane& c, const lu& p) {
    lu a = p, b = p;
    lp_swap16(a, b);                                       // a = [X X Z Z]: row 3 gets Z
    const lu sq = lp_mul(c, p, lp_sel(c.row3, a, p));      // [XX, YY, ZZ, TZ]
    lu XX, YY, ZZ, TZ;
    lp_allrows(sq, XX, YY, ZZ, TZ);
    const lu rY = YY + XX;                                 // H
    const lu rZ = lp_sub(c, YY, XX);                       // G
    const lu rX = TZ + TZ;                                 // E = 2XY
    const lu rT = lp_carry1(c, lp_sub4p(c, ZZ + ZZ, rZ));  // F (carried: a g operand)
    // X3 = E F, Y3 = H G, Z3 = G F, T3 = E H
    return lp_mul(c, c.rows(rX, rY, rZ, rX), c.rows(rT, rZ, rT, rY));
}

// ext -> cached [Y-X, Y+X, 2dT, 2Z] (one multiplication: every component reduced)
LP_FN lu lp_to_cached(const LpLane& c, const lu& p, const lu& d2) {
    lu X, Y, Z, T;
    lp_allrows(p, X, Y, Z, T);
    const lu one = lp_sel(c.k0, 1u, 0u), two = lp_sel(c.k0, 2u, 0u);
    return lp_mul(c, c.rows(lp_sub(c, Y, X), Y + X, T, Z), c.rows(one, one, d2, two));
}

// -q for a cached / niels addend: swap rows 0 and 1, negate row 2
LP_FN lu lp_neg_cached(const LpLane& c, const lu& q) {
    lu p = q, s = q;
    lp_swap16(p, s);  // p = [q0 q0 q2 q2], s = [q1 q1 q3 q3]
    return c.rows(s, p, lp_sub(c, 0u, q), q);
}

LP_FN lu lp_identity_ext(const LpLane& c) {
    const lu one = lp_sel(c.k0, 1u, 0u);
    return c.rows(0u, one, one, 0u);
}

// ------------------------------------------------------------------ verification pieces
// Constants every lp routine needs, one VGPR each (limb k of the row).
struct LpConsts {
    lu d, d2, sqrtm1, one;
    LP_FN static LpConsts make(const LpLane& c) {
        LpConsts k;
        k.d = c.limb(PV_D);
        k.d2 = c.limb(PV_D2);
        k.sqrtm1 = c.limb(PV_SQRTM1);
        k.one = lp_sel(c.k0, 1u, 0u);
        return k;
    }
};

// Canonical-zero / parity tests of one row (uniform: the row's limbs are read into scalars).
LP_FN bool lp_row_iszero(const lu& x, int r) { return fe_iszero(lp_row_fe(x, r)); }
LP_FN uint32_t lp_row_isnegative(const lu& x, int r) { return fe_isnegative(lp_row_fe(x, r)); }

// Decompression of the key A (row 0, returned negated: -A, as ge_frombytes_negate) and of the
// signature's R (row 1, NOT negated: x with parity = R's bit 255), both in one pass of the
// x^((p-5)/8) chain. s[8] = this lane's row's encoding (A's words in row 0, R's in row 1; rows 2-3
// repeat them). Outputs: X, Y with the x / y of row 0 (-A) and row 1 (R); ok_a / ok_r = the point
// decompresses ((y^2-1)/(dy^2+1) is a square); x_r_zero = R's x is 0.
struct LpDecomp {
    lu X, Y;
    bool ok_a, ok_r, x_r_zero;
};
LP_FN LpDecomp lp_decompress_ar(const LpLane& c, const LpConsts& K, const lu s[8]) {
    LpDecomp o;
    const lu y = lp_from_words(c, s);
    lu u = lp_mul_dual(c, y, y);
    lu v = lp_mul_dual(c, u, K.d);
    u = lp_carry1(c, lp_sub(c, u, K.one));  // u = y^2 - 1
    v = lp_carry1(c, v + K.one);              // v = d y^2 + 1
    lu v3 = lp_mul_dual(c, lp_mul_dual(c, v, v), v);        // v^3
    lu x = lp_mul_dual(c, lp_mul_dual(c, lp_mul_dual(c, v3, v3), v), u);  // u v^7
    x = lp_pow22523<true>(c, x);
    x = lp_mul_dual(c, lp_mul_dual(c, x, v3), u);       // u v^3 (u v^7)^((p-5)/8)
    const lu vxx = lp_mul_dual(c, lp_mul_dual(c, x, x), v);
    const lu chk_m = lp_sub(c, vxx, u), chk_p = vxx + u;
    const bool ok0 = lp_row_iszero(chk_m, 0), ok1 = lp_row_iszero(chk_m, 1);
    o.ok_a = ok0 || lp_row_iszero(chk_p, 0);
    o.ok_r = ok1 || lp_row_iszero(chk_p, 1);
    const lu xs = lp_mul(c, x, K.sqrtm1);
    // per row: x or x sqrt(-1)
    const lm use_s = lp_and(lp_lt(c.row, 2u), lp_eq(lp_sel(c.row0, ok0 ? 0u : 1u, ok1 ? 0u : 1u), 1u));
    x = lp_sel(use_s, xs, x);
    // sign: row 0 (A) negated iff parity == sign bit (ge_frombytes_negate); row 1 (R) iff parity != sign
    const uint32_t sa = lp_readlane(s[7], 0) >> 31, sr = lp_readlane(s[7], 16) >> 31;
    const uint32_t pa = lp_row_isnegative(x, 0), pr = lp_row_isnegative(x, 1);
    o.x_r_zero = lp_row_iszero(x, 1);
    const uint32_t neg0 = pa == sa ? 1u : 0u, neg1 = pr != sr ? 1u : 0u;
    const lm neg = lp_eq(lp_sel(c.row0, neg0, lp_sel(c.row1, neg1, 0u)), 1u);
    o.X = lp_sel(neg, lp_carry1(c, lp_sub(c, 0u, x)), x);
    o.Y = y;
    return o;
}

// ext point from row `r` of X and Y (Z = 1, T = X Y): the decompressed key as [X, Y, Z, T]
LP_FN lu lp_ext_from_xy(const LpLane& c, const LpConsts& K, const lu& X, const lu& Y, int r) {
    lu xr[4], yr[4];
    lp_allrows(X, xr[0], xr[1], xr[2], xr[3]);
    lp_allrows(Y, yr[0], yr[1], yr[2], yr[3]);
    const lu x = r == 0 ? xr[0] : xr[1], y = r == 0 ? yr[0] : yr[1];
    // rows [X, Y, 1, X Y]: one multiplication forms T (rows 0-2 multiply by 1)
    return lp_mul(c, c.rows(x, y, K.one, x), c.rows(K.one, K.one, K.one, y));
}

// The comb key chain (comb.h pv_comb_chain) over positions [lo, hi): P = P_lo = [256^lo](-A) on
// entry; store(i, m, P) receives slot m of position i (P_i, then its [16], [32], [64] multiples);
// returns P_hi for the next part (hi < 32). pv_key_chain_lp_kernel runs the 32 positions in parts so
// that the table fill of a part overlaps the chain of the next.
template <class Store>
LP_FN lu lp_comb_chain_part(const LpLane& c, lu P, int lo, int hi, const Store& store) {
    for (int i = lo; i < hi; i++) {
        store(i, 0, P);
        const int nd = i + 1 < 32 ? 8 : 6;
        for (int j = 0; j < nd; j++) {
            P = lp_dbl(c, P);
            if (j >= 3 && j <= 5) store(i, j - 2, P);
        }
    }
    return P;
}
// An extended point back from its 40 stored words (X, Y, Z, T, 10 carried limbs each): lane
// 16 r + k <- word 10 r + k, the scratch lanes 10..15 of a row 0. A stored point is a valid lp
// operand (carried limbs, consistent T), so a chain part resumes from the previous part's P_hi.
LP_FN lu lp_load_ext40(const LpLane& c, const uint32_t* w) {
    return lp_sel(c.kge10, 0u, lp_gather(w, lp_sel(c.kge10, 0u, c.row * 10u + c.k)));
}

// The table of [j](-A), j = -8..8, cached form, for the signed radix-16 digits of k. store(j, q).
template <class Store>
LP_FN void lp_build_a_table(const LpLane& c, const LpConsts& K, const lu& negA, const Store& store) {
    const lu one = K.one, two = lp_sel(c.k0, 2u, 0u);
    store(0, c.rows(one, one, 0u, two));  // identity
    const lu c1 = lp_to_cached(c, negA, K.d2);
    store(1, c1);
    store(-1, lp_neg_cached(c, c1));
    lu cur = lp_dbl(c, negA);
    for (int j = 2; j <= 8; j++) {
        if (j > 2) cur = lp_add_cached(c, cur, c1);
        const lu cj = lp_to_cached(c, cur, K.d2);
        store(j, cj);
        store(-j, lp_neg_cached(c, cj));
    }
}

// Parts of that table for waves building it at once: part 0 the entries 0, +-1..+-4 (one doubling,
// two additions), part 1 +-5, +-6 from [4]P = 2(2P) (two doublings, two additions), part 2 +-7, +-8
// from [8]P = 2(2(2P)) and [7]P = [8]P - P (three doublings, one addition). Same points as
// lp_build_a_table (any projective representative serves a lookup).
template <class Store>
LP_FN void lp_build_a_table_part(const LpLane& c, const LpConsts& K, const lu& P, int part, const Store& store) {
    const lu c1 = lp_to_cached(c, P, K.d2);
    auto put = [&](int j, const lu& pt) {
        const lu cj = lp_to_cached(c, pt, K.d2);
        store(j, cj);
        store(-j, lp_neg_cached(c, cj));
    };
    if (part == 0) {
        const lu one = K.one, two = lp_sel(c.k0, 2u, 0u);
        store(0, c.rows(one, one, 0u, two));
        store(1, c1);
        store(-1, lp_neg_cached(c, c1));
        lu cur = lp_dbl(c, P);
        put(2, cur);
        cur = lp_add_cached(c, cur, c1);
        put(3, cur);
        put(4, lp_add_cached(c, cur, c1));
    } else if (part == 1) {
        lu cur = lp_add_cached(c, lp_dbl(c, lp_dbl(c, P)), c1);  // [5]P
        put(5, cur);
        put(6, lp_add_cached(c, cur, c1));
    } else {
        const lu p8 = lp_dbl(c, lp_dbl(c, lp_dbl(c, P)));
        put(8, p8);
        put(7, lp_add_cached(c, p8, lp_neg_cached(c, c1)));
    }
}

// [2^n] P without P's x: on -x^2 + y^2 = 1 + d x^2 y^2, x^2 = (y^2 - 1) / (d y^2 + 1) is a function of
// y, so doubling maps y to a function of y alone, and x to x times a function of y:
//   y' = (d a^2 + 2ab - b^2) / (-d a^2 + 2d ab + b^2),  x' / x = 2YZ (d a + b) / (d a^2 + b^2)
// for y = Y / Z, a = Y^2, b = Z^2 (both denominators are nonzero for every y: -1/d is not a fourth power
// and the doubling is complete). The chain can therefore start from the encoding's y at once,
// while x is still being decompressed, and x enters once at the end (lp_ydbl_finish): three
// multiplications a doubling (rows [a, b, YZ, U num], [a^2, b^2, ab, d a], [d a^2, d ab, YZ (d a + b),
// W den]) against two for lp_dbl, off the critical path. State rows [Y, Z, U, W] with x_n = x_0 U / W
// (the last step's num / den still pending in num_den rows 0 / 1).
struct LpYChain {
    lu st;       // [Y, Z, U, W]
    lu num_den;  // [num, den, -, -] of the last doubling (applied by the next one / the finish)
};
LP_FN LpYChain lp_ydbl_chain(const LpLane& c, const LpConsts& K, const lu& y0, int n) {
    const lu one = K.one;
    lu Y = y0, Z = one, U = one, W = one, num = one, den = one;
    for (int i = 0; i < n; i++) {
        const lu m1 = lp_mul(c, c.rows(Y, Z, Y, U), c.rows(Y, Z, Z, num));  // [a, b, YZ, U num]
        lu a, b, yz, u1;
        lp_allrows(m1, a, b, yz, u1);
        const lu m2 = lp_mul(c, c.rows(a, b, a, K.d), c.rows(a, b, b, a));  // [a^2, b^2, ab, d a]
        lu a2, b2, ab, da;
        lp_allrows(m2, a2, b2, ab, da);
        const lu m3 = lp_mul(c, c.rows(da, da, yz, W), c.rows(a, b, da + b, den));  // [d a^2, d ab, YZ (d a + b), W den]
        lu da2, dab, nm, w1;
        lp_allrows(m3, da2, dab, nm, w1);
        Y = lp_carry1(c, lp_sub(c, da2 + ab + ab, b2));
        Z = lp_carry1(c, lp_sub(c, dab + dab + b2, da2));
        U = u1;
        W = w1;
        num = nm + nm;
        den = da2 + b2;
    }
    LpYChain o;
    o.st = c.rows(Y, Z, U, W);
    o.num_den = c.rows(num, den, 0u, 0u);
    return o;
}
// The ext point [2^n] P of the chain once P's x is known: x0 = P's affine x in every row.
// (x0 U Z : Y W : Z W : x0 U Y), U and W with the pending num / den applied.
LP_FN lu lp_ydbl_finish(const LpLane& c, const LpConsts& K, const LpYChain& ch, const lu& x0) {
    lu Y, Z, U, W, num, den, t0, t1;
    lp_allrows(ch.st, Y, Z, U, W);
    lp_allrows(ch.num_den, num, den, t0, t1);
    const lu uw = lp_mul(c, c.rows(U, W, U, W), c.rows(num, den, num, den));  // [Uf, Wf, Uf, Wf]
    lu Uf, Wf;
    lp_allrows(uw, Uf, Wf, t0, t1);
    const lu g = lp_mul(c, c.rows(Uf, Y, Z, Uf), c.rows(x0, Wf, Wf, x0));  // [G = x0 Uf, Y Wf, Z Wf, G]
    lu G, YW, ZW, t2;
    lp_allrows(g, G, YW, ZW, t2);
    return lp_mul(c, c.rows(G, YW, ZW, G), c.rows(Z, K.one, K.one, Y));
}

// [k](-A) by regular signed radix-16 windows: 63 x 4 doublings + 64 table additions. digit(i) =
// the i-th signed digit (wave-uniform), load(e) = the table entry for digit e.
template <class Digit, class Load>
LP_FN lu lp_straus_a(const LpLane& c, const Digit& digit, const Load& load) {
    lu acc = lp_add_cached(c, lp_identity_ext(c), load(digit(63)));
    for (int win = 62; win >= 0; win--) {
        acc = lp_dbl(c, lp_dbl(c, lp_dbl(c, lp_dbl(c, acc))));
        acc = lp_add_cached(c, acc, load(digit(win)));
    }
    return acc;
}

// [e](P) over the first nw signed radix-16 windows (nw wave-uniform: the half-size split's window
// count, sc25519.h sc_halfsize; 64 for a full scalar): (nw - 1) x 4 doublings + nw table additions.
template <class Digit, class Load>
LP_FN lu lp_straus_nw(const LpLane& c, int nw, const Digit& digit, const Load& load) {
    lu acc = lp_add_cached(c, lp_identity_ext(c), load(digit(nw - 1)));
    for (int win = nw - 2; win >= 0; win--) {
        acc = lp_dbl(c, lp_dbl(c, lp_dbl(c, lp_dbl(c, acc))));
        acc = lp_add_cached(c, acc, load(digit(win)));
    }
    return acc;
}

// The windows [lo, hi) of a signed radix-16 scalar against the table of P (window i weighs 16^(i-lo):
// the caller's table is of [16^lo] P): (hi - lo - 1) x 4 doublings + (hi - lo) additions; the identity
// when hi <= lo (uniform bounds).
template <class Digit, class Load>
LP_FN lu lp_straus_range(const LpLane& c, int lo, int hi, const Digit& digit, const Load& load) {
    if (hi <= lo) return lp_identity_ext(c);
    lu acc = lp_add_cached(c, lp_identity_ext(c), load(digit(hi - 1)));
    for (int win = hi - 2; win >= lo; win--) {
        acc = lp_dbl(c, lp_dbl(c, lp_dbl(c, lp_dbl(c, acc))));
        acc = lp_add_cached(c, acc, load(digit(win)));
    }
    return acc;
}

// Entry d = |f| of position j of the fixed-base comb T_B (comb.h: affine niels, words y+x at 0..9,
// y-x at 10..19, 2dxy at 20..29 of a PV_BCOMB_STRIDE-word entry) in lp cached layout
// [y-x, y+x, 2dxy, 2], negated for f < 0 (y+x <-> y-x, -2dxy).
LP_FN lu lp_bcomb_entry(const LpLane& c, const uint32_t* bcomb, int j, int f) {
    const bool neg = f < 0;
    const uint32_t d = (uint32_t)(neg ? -f : f);
    const uint32_t* e = bcomb + ((uint64_t)j * PV_BCOMB_ENT + d) * PV_BCOMB_STRIDE;
    const lu kk = lp_sel(c.kge10, 9u, c.k);
    const lu w = lp_sel(c.row0, neg ? kk : kk + 10u, lp_sel(c.row1, neg ? kk + 10u : kk, kk + 20u));
    return lp_gather(e, w);
}
// The same for entry |f| of row q of a cached key's radix-65536 rows (comb.h PV_KW_*: niels entries
// in T_B's format, rows of PV_KW_ENT entries).
LP_FN lu lp_kw_entry(const LpLane& c, const uint32_t* wrows, int q, int f) {
    const bool neg = f < 0;
    const uint32_t d = (uint32_t)(neg ? -f : f);
    const uint32_t* e = wrows + ((uint64_t)q * PV_KW_ENT + d) * PV_BCOMB_STRIDE;
    const lu kk = lp_sel(c.kge10, 9u, c.k);
    const lu w = lp_sel(c.row0, neg ? kk : kk + 10u, lp_sel(c.row1, neg ? kk + 10u : kk, kk + 20u));
    return lp_gather(e, w);
}
LP_FN lu lp_bcomb_fix(const LpLane& c, const lu& raw, int f) {
    lu v = raw;
    if (f < 0) v = lp_sel(c.row2, lp_sub(c, 0u, v), v);
    return lp_sel(c.row3, lp_sel(c.k0, 2u, 0u), v);
}

// [S]B from the fixed-base comb T_B[j][|f_j|] (comb.h: 16 signed radix-65536 digits of S). entry(j)
// returns the niels entry of position j for its digit, already in lp cached form (negated for a
// negative digit): [y-x, y+x, 2dxy, 2].
template <class Entry>
LP_FN lu lp_comb_b(const LpLane& c, const Entry& entry) {
    lu acc = lp_identity_ext(c);
    for (int j = 15; j >= 0; j--) acc = lp_add_cached(c, acc, entry(j));
    return acc;
}

// Entry |e| of position i of a key's radix-256 comb table (comb.h: [32][129] cached points, words
// Y+X at 0..9, Y-X at 10..19, 2Z at 20..29, 2dT at 30..39) in lp cached layout [Y-X, Y+X, 2dT, 2Z]
// (rows 0 / 1 swapped for e < 0; lp_ctab_fix then negates 2dT). Split from the fix-up so all 32
// loads of a verification can be issued before the first addition.
LP_FN lu lp_ctab_load(const LpLane& c, const uint32_t* tab, int i, int e) {
    const bool neg = e < 0;
    const uint32_t d = (uint32_t)(neg ? -e : e);
    const uint32_t* p = tab + ((uint32_t)i * PV_COMB_ENT + d) * 40u;
    const lu kk = lp_sel(c.kge10, 9u, c.k);
    return lp_gather(p, c.rows(neg ? kk : kk + 10u, neg ? kk + 10u : kk, kk + 30u, kk + 20u));
}
LP_FN lu lp_ctab_fix(const LpLane& c, const lu& raw, int e) {
    return e < 0 ? lp_sel(c.row2, lp_sub(c, 0u, raw), raw) : raw;
}

// [k](-A) from a cached key table: 32 additions of T_A[i][e_i] (signed radix-256 digits e_i of k),
// no doublings. entry(i) = the fixed-up entry of position i.
template <class Entry>
LP_FN lu lp_comb_a(const LpLane& c, const Entry& entry) {
    lu acc = lp_identity_ext(c);
    for (int i = PV_COMB_POS - 1; i >= 0; i--) acc = lp_add_cached(c, acc, entry(i));
    return acc;
}

// The final check: Q = QA + SB (SB as ext), then libsodium's encode(Q) == R rewritten without an
// inversion: R canonical (checked by the caller), R decompressed (X row 1 = x_R with R's sign,
// Y row 1 = y_R), and x_R != 0 or sign 0; accept iff X_Q = x_R Z_Q and Y_Q = y_R Z_Q. Given y_Q =
// y_R, the two roots x, -x have opposite parity (p odd) unless x = 0, so parity(x_Q) = sign(R)
// exactly when x_Q is the root decompression picked; y_Q = y_R < p is the canonical-y condition.
// sb: the second summand already in cached form (the four-wave kernel's waves convert their parts
// before the last barrier, off wave 0's chain).
LP_FN bool lp_final_check_cached(const LpLane& c, const lu& QA, const lu& sb, const lu& X, const lu& Y) {
    const lu Q = lp_add_cached(c, QA, sb);
    lu QX, QY, QZ, QT;
    lp_allrows(Q, QX, QY, QZ, QT);
    lu xr[4], yr[4];
    lp_allrows(X, xr[0], xr[1], xr[2], xr[3]);
    lp_allrows(Y, yr[0], yr[1], yr[2], yr[3]);
    // row 0: x_R Z_Q, row 1: y_R Z_Q
    const lu prod = lp_mul(c, c.rows(xr[1], yr[1], 0u, 0u), QZ);
    const lu diff = lp_sub(c, c.rows(QX, QY, 0u, 0u), prod);
    return lp_row_iszero(diff, 0) && lp_row_iszero(diff, 1);
}
LP_FN bool lp_final_check(const LpLane& c, const LpConsts& K, const lu& QA, const lu& SB, const lu& X, const lu& Y) {
    return lp_final_check_cached(c, QA, lp_to_cached(c, SB, K.d2), X, Y);
}

// ------------------------------------------------------------------ the half-size split, limb-parallel
// sc25519.h sc_halfsize for ONE wave whose lanes all hold the same k (the latency path): the same
// Lehmer blocks and exact steps, with the multiword state spread over the lanes -- lane 16 r + i holds
// word i of row r: r0, r1 (9 words, two's complement) and t0, t1 (8 words, mod 2^256) -- so a block's
// matrix update is two products per lane and a carry pass across the row (DPP row_shr) instead of
// ~600 dependent scalar instructions. The leading digits and every test are read back with readlane /
// ballot (uniform control). Same quotients, invariant and fallback as sc_halfsize, so the same split.

// Words of the signed sum P_i 2^(32 i) of per-lane 64-bit partials, per row modulo 2^(32 n) (r rows:
// n = 9, t rows: n = 8; lanes past the row's words stay 0).
LP_FN lu lp_mp_norm(const LpLane& c, const lu64& P) {
    const lm keep = lp_ltv(c.k, lp_sel(lp_lt(c.row, 2u), 9u, 8u));
    lu64 s = lp_wide(lp_lo(P)) + lp_sext64(lp_shr<1>(lp_hi(P)));
    lu w = lp_sel(keep, lp_lo(s), 0u);
    lu cr = lp_sel(keep, lp_hi(s), 0u);
    for (int it = 0; it < 10; it++) {  // carries of -1 / 0 / +1 ripple one word per pass
        const lu cin = lp_shr<1>(cr);
        if (lp_ballot(lp_ne(cin, 0u)) == 0) break;
        s = lp_wide(w) + lp_sext64(cin);
        w = lp_sel(keep, lp_lo(s), 0u);
        cr = lp_sel(keep, lp_hi(s), 0u);
    }
    return w;
}
// (r0, r1, t0, t1) <- (A r0 + B r1, C r0 + D r1, A t0 + B t1, C t0 + D t1), |A|, |B|, |C|, |D| < 2^31
LP_FN lu lp_mat_update(const LpLane& c, const lu& st, int64_t A, int64_t B, int64_t C, int64_t D) {
    lu a = st, b = st;
    lp_swap16(a, b);  // a = [r0 r0 t0 t0], b = [r1 r1 t1 t1]
    const lm odd = lp_eq(c.row & 1u, 1u);
    const int64_t cs[4] = {A, B, C, D};
    const uint32_t ma[2] = {(uint32_t)(A < 0 ? -A : A), (uint32_t)(C < 0 ? -C : C)};
    const uint32_t mb[2] = {(uint32_t)(B < 0 ? -B : B), (uint32_t)(D < 0 ? -D : D)};
    const lu64 pa = lp_mad(a, lp_sel(odd, ma[1], ma[0]), lu64(0u));
    const lu64 pb = lp_mad(b, lp_sel(odd, mb[1], mb[0]), lu64(0u));
    const lm na = lp_eq(lp_sel(odd, cs[2] < 0 ? 1u : 0u, cs[0] < 0 ? 1u : 0u), 1u);
    const lm nb = lp_eq(lp_sel(odd, cs[3] < 0 ? 1u : 0u, cs[1] < 0 ? 1u : 0u), 1u);
    return lp_mp_norm(c, lp_sel64(na, lp_neg64(pa), pa) + lp_sel64(nb, lp_neg64(pb), pb));
}
// 0 <= r1 < r0 (both rows read as 9-word two's complement)
LP_FN bool lp_pair_ordered(const LpLane& c, const lu& st) {
    if ((int32_t)lp_readlane(st, 8) < 0 || (int32_t)lp_readlane(st, 24) < 0) return false;
    lu a = st, b = st;
    lp_swap16(a, b);
    const uint64_t gt = lp_ballot(lp_and(lp_eq(c.row, 1u), lp_ltv(a, b)));  // r1 word > r0 word
    const uint64_t lt = lp_ballot(lp_and(lp_eq(c.row, 1u), lp_ltv(b, a)));
    if (lt == 0) return false;
    return gt == 0 || (63 - __builtin_clzll(lt)) > (63 - __builtin_clzll(gt));
}
// |t0|, |t1| < 2^168: bits 168..255 of each t row equal its sign
LP_FN bool lp_t_small(const LpLane& c, const lu& st) {
    const lu sg = lp_sar31(lp_bcast<7>(st));
    const lm hi67 = lp_and(lp_ge(c.k, 6u), lp_le(c.k, 7u));
    const lm bad = lp_and(lp_ge(c.row, 2u),
                          lp_or(lp_and(hi67, lp_ne(st ^ sg, 0u)), lp_and(lp_eq(c.k, 5u), lp_ne((st ^ sg) >> 8, 0u))));
    return lp_ballot(bad) == 0;
}

// PV_LP_SPLIT_53 = 1: a Lehmer block reads 53 leading bits (exact doubles), takes one division per
// quotient and accepts it under Jebelean's conditions (~25 bits per block: ~5 blocks); 0: sc_halfsize's
// 31-bit blocks with Knuth's two-division test (~9 blocks). Both settle only true quotients, so both
// give sc_halfsize's split.
#ifndef PV_LP_SPLIT_53
#define PV_LP_SPLIT_53 1
#endif
// 1 / x to 1 ulp (v_rcp_f32 on the device)
LP_FN float lp_rcpf(float x) {
#if LP_DEVICE
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
#ifndef LP_SPLIT_MARK  // phase timer hook of microbench/lp_split_lat.hip (no-op otherwise)
#define LP_SPLIT_MARK(i)
#endif
// stats (measurement only, nullptr otherwise): as sc_halfsize's
LP_FN void lp_halfsize(const LpLane& c, pv_halfk& h, const uint32_t k[8], uint32_t* stats = nullptr) {
    lu st = 0u;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        st = lp_sel(lp_eq(lp_lane(), (uint32_t)i), i < 8 ? SC_8L[i] : 0u, st);
        st = lp_sel(lp_eq(lp_lane(), (uint32_t)(16 + i)), i < 8 ? k[i] : 0u, st);
    }
    st = lp_sel(lp_eq(lp_lane(), 48u), 1u, st);  // t1 = 1
    bool bad = false;
    // ---- Lehmer blocks while r1 >= 2^131
    for (int blk = 0; blk < PV_HALF_BLOCKS && !bad; blk++) {
        const uint64_t nz = lp_ballot(lp_ne(st, 0u));
        const uint32_t r1nz = (uint32_t)(nz >> 16) & 0x1FFu;
        if ((r1nz >> 5) == 0 && (lp_readlane(st, 20) >> 3) == 0) break;
        if (stats) stats[0]++;
        LP_SPLIT_MARK(0);
        const int w = 31 - __builtin_clz((uint32_t)nz & 0x1FFu);  // >= 4 (r0 > r1 >= 2^131)
#if PV_LP_SPLIT_53
        // 53 leading bits of r0 (2^52 <= xh < 2^53) and r1 at the same shift e, exact in doubles
        const uint32_t a1 = lp_readlane(st, w), a0 = lp_readlane(st, w - 1), a2 = lp_readlane(st, w - 2);
        const uint32_t b1 = lp_readlane(st, 16 + w), b0 = lp_readlane(st, 15 + w), b2 = lp_readlane(st, 14 + w);
        const int s = 43 - (int)__builtin_clz(a1);  // bits of (a1:a0:a2) = 96 - clz(a1); keep 53 (s = 12..43)
        const uint64_t ah = ((uint64_t)a1 << 32) | a0, bh = ((uint64_t)b1 << 32) | b0;
        const uint64_t xi = s <= 32 ? (ah << (32 - s)) | ((uint64_t)a2 >> s) : ah >> (s - 32);
        const uint64_t yi = s <= 32 ? (bh << (32 - s)) | ((uint64_t)b2 >> s) : bh >> (s - 32);
        const int e = 32 * (w - 2) + s;  // >= 79 here (r0 >= 2^132)
        const double ythr = e >= 130 ? 1.0 : (double)(1ull << (130 - e));  // stop the block above 2^130
        // Euclid on the digits, (x, y) = (r_n, r_{n+1}) estimates, with the cosequence rows as sign-free
        // magnitudes: row j is (+P, -N) for even j, (-N, +P) for odd j, and P_j = P_{j-2} + q N_{j-1},
        // N_j = N_{j-2} + q P_{j-1}. The true r_j = x_j 2^e + delta_j with -N_j 2^e < delta_j < P_j 2^e,
        // so the digit quotient is the true one when the new remainder is >= N_j and the old one
        // exceeds it by >= N_{j-1} + P_j (Jebelean's conditions); the two slots alternate roles.
        double x = (double)xi, y = (double)yi, Px = 1.0, Nx = 0.0, Py = 1.0, Ny = 0.0;
        int n = 0;
#define LP_QSTEP(U, V, PU, NU, PV, NV)                                                                       \
    {                                                                                                        \
        /* |estimate - quotient| <= 1 for quotients < 2^21 (f32 operands, 1-ulp reciprocal) */              \
        double q = (double)__builtin_floorf((float)U * lp_rcpf((float)V));                     \
        double nr = __builtin_fma(-q, V, U);                                                                 \
        /* branch-free fix-up (uniform values: selects, not jumps) */                                       \
        const bool lo_ = nr < 0.0;                                                                           \
        q = lo_ ? q - 1.0 : q;                                                                               \
        nr = lo_ ? nr + V : nr;                                                                              \
        const bool hi_ = nr >= V;                                                                            \
        q = hi_ ? q + 1.0 : q;                                                                               \
        nr = hi_ ? nr - V : nr;                                                                              \
        const double nP = __builtin_fma(q, NV, PU), nN = __builtin_fma(q, PV, NU);                           \
        const bool ok_ = (q < 2097152.0) & (nr >= ythr) & (nr >= nN) & (V - nr >= NV + nP) &                 \
                         (nP + nN < 2147483648.0);                                                           \
        LP_QCOMMIT(U, PU, NU)                                                                                \
    }
#define LP_QCOMMIT(U, PU, NU)                                                                                \
        if (!ok_) break;                                                                                     \
        U = nr;                                                                                              \
        PU = nP;                                                                                             \
        NU = nN;                                                                                             \
        n++;                                                                                                 \
        if (stats) stats[1]++;
        for (int it = 0; it < 48; it++) {
            LP_QSTEP(x, y, Px, Nx, Py, Ny)
            LP_QSTEP(y, x, Py, Ny, Px, Nx)
        }
#undef LP_QSTEP
#undef LP_QCOMMIT
        // rows n (A, B) and n + 1 (C, D): slot x always holds the even row, slot y the odd one
        const double Pe = Px, Ne = Nx, Po = Py, No = Ny;
        // even row (P, -N), odd row (-N, P); n even: (A, B) even, (C, D) odd; n odd: the reverse
        const double A = (n & 1) ? -No : Pe, B = (n & 1) ? Po : -Ne;
        const double C = (n & 1) ? Pe : -No, D = (n & 1) ? -Ne : Po;
#else
        const uint32_t a1 = lp_readlane(st, w), a0 = lp_readlane(st, w - 1);
        const uint32_t b1 = lp_readlane(st, 16 + w), b0 = lp_readlane(st, 15 + w);
        const int sh = 33 - (int)__builtin_clz(a1);
        const int s = sh > 0 ? sh : 0;
        int32_t xh = (int32_t)((((uint64_t)a1 << 32) | a0) >> s);
        int32_t yh = (int32_t)((((uint64_t)b1 << 32) | b0) >> s);
        const int e = 32 * (w - 1) + s;
        const int32_t ythr = e >= 130 ? 1 : (int32_t)(1u << (130 - e));
        int32_t A = 1, B = 0, C = 0, D = 1;
        for (int it = 0; it < 24; it++) {
            const int32_t n1 = xh + A, d1 = yh + C, n2 = xh + B, d2 = yh + D;
            bool ok1, ok2;
            const uint32_t q = pv_qdiv31(n1, d1, ok1);
            const uint32_t q2 = pv_qdiv31(n2, d2, ok2);
            if (!ok1 || !ok2 || q != q2) break;
            const int64_t ny = (int64_t)xh - (int64_t)q * yh;
            const int64_t nC = (int64_t)A - (int64_t)q * C, nD = (int64_t)B - (int64_t)q * D;
            if (ny < ythr || nC >= 32768 || nC <= -32768 || nD >= 32768 || nD <= -32768) break;
            A = C;
            C = (int32_t)nC;
            B = D;
            D = (int32_t)nD;
            xh = yh;
            yh = (int32_t)ny;
            if (stats) stats[1]++;
        }
#endif
        LP_SPLIT_MARK(1);
        if (B == 0) {
            // one exact step: q from the top three words, then fixed by whole additions of r0
            const uint32_t ta1 = lp_readlane(st, w), ta0 = lp_readlane(st, w - 1), ta2 = lp_readlane(st, w - 2);
            const uint32_t tb1 = lp_readlane(st, 16 + w), tb0 = lp_readlane(st, 15 + w), tb2 = lp_readlane(st, 14 + w);
            const double qd = ((double)ta1 * 4294967296.0 + (double)ta0 + (double)ta2 / 4294967296.0) /
                              ((double)tb1 * 4294967296.0 + (double)tb0 + (double)tb2 / 4294967296.0);
            if (!(qd < 2147483647.0)) {
                bad = true;
                break;
            }
            const int64_t q = (int64_t)qd;
            st = lp_mat_update(c, st, 0, 1, 1, -q);
            if ((int32_t)lp_readlane(st, 24) < 0) st = lp_mat_update(c, st, 1, 0, 1, 1);
            else if (!lp_pair_ordered(c, st)) st = lp_mat_update(c, st, 1, 0, -1, 1);
        } else {
            st = lp_mat_update(c, st, (int64_t)A, (int64_t)B, (int64_t)C, (int64_t)D);
        }
        LP_SPLIT_MARK(2);
        bad |= !lp_pair_ordered(c, st) || !lp_t_small(c, st);
        LP_SPLIT_MARK(3);
    }
    // ---- exact single steps until r1 < 2^128 with t1 odd
    for (int it = 0; it < PV_HALF_MAXIT && !bad; it++) {
        const uint64_t nz = lp_ballot(lp_ne(st, 0u));
        if ((((uint32_t)(nz >> 16) & 0x1FFu) >> 4) == 0 && (lp_readlane(st, 48) & 1u)) break;
        if (stats) stats[2]++;
        const int w = 31 - __builtin_clz(((uint32_t)nz & 0x1FFu) | 1u);
        if (w < 2 || ((nz >> 16) & 0x1FFu) == 0) {
            bad = true;
            break;
        }
        const uint32_t a1 = lp_readlane(st, w), a0 = lp_readlane(st, w - 1), a2 = lp_readlane(st, w - 2);
        const uint32_t b1 = lp_readlane(st, 16 + w), b0 = lp_readlane(st, 15 + w), b2 = lp_readlane(st, 14 + w);
        const double qd = ((double)a1 * 4294967296.0 + (double)a0 + (double)a2 / 4294967296.0) /
                          ((double)b1 * 4294967296.0 + (double)b0 + (double)b2 / 4294967296.0);
        if (!(qd < 2147483647.0)) {
            bad = true;
            break;
        }
        const int64_t q = (int64_t)qd;
        st = lp_mat_update(c, st, 0, 1, 1, -q);
        if ((int32_t)lp_readlane(st, 24) < 0) st = lp_mat_update(c, st, 1, 0, 1, 1);
        else if (!lp_pair_ordered(c, st)) st = lp_mat_update(c, st, 1, 0, -1, 1);
        bad |= !lp_pair_ordered(c, st) || !lp_t_small(c, st);
    }
    const uint64_t nz = lp_ballot(lp_ne(st, 0u));
    const bool done = !bad && (((uint32_t)(nz >> 16) & 0x1FFu) >> 4) == 0 && (lp_readlane(st, 48) & 1u);
    // k2 = |t1|, k1 = r1 with t1's sign moved onto it
    uint32_t t1[8], ta[8];
#pragma unroll
    for (int i = 0; i < 8; i++) t1[i] = lp_readlane(st, 48 + i);
    const bool tneg = (int32_t)t1[7] < 0;
    uint64_t cy = tneg ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)(tneg ? ~t1[i] : t1[i]) + cy;
        ta[i] = (uint32_t)t;
        cy = t >> 32;
    }
    const bool ok = done && (ta[5] | ta[6] | ta[7]) == 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        h.k1[i] = ok ? lp_readlane(st, 16 + i) : k[i];
        h.k2[i] = ok ? ta[i] : (i == 0 ? 1u : 0u);
    }
    h.neg = ok && tneg;
    h.fallback = !ok;
}
