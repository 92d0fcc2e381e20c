// Fixed-base table for the Straus loop: [j]B for j = 0..128 in affine niels form
// (y+x, y-x, 2d x y), canonical limbs. Computed once on the host at library init with the same
// field code the kernels use, then copied to the device; each workgroup stages it into LDS.
#pragma once
#include "ge25519.h"

static constexpr int PV_BTAB_ENTRIES = 129;
static constexpr int PV_BTAB_STRIDE = 32;  // words per entry (30 used, padded for 16-B LDS reads)

// Base point encoding: y = 4/5, x even.
static constexpr uint32_t PV_B_ENC[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                                         0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};

// canonical reduced limbs of f
PV_HD void fe_canonical(fe& h, const fe& f) {
    uint32_t s[8];
    fe_tobytes32(s, f);
    fe_frombytes32(h, s);
}

inline void pv_build_b_table(uint32_t* out /* PV_BTAB_ENTRIES * PV_BTAB_STRIDE */) {
    ge_p3 negB, B, cur;
    ge_frombytes_negate(negB, PV_B_ENC);
    B = negB;
    fe z;
    fe_0(z);
    fe_sub(B.X, z, negB.X);
    fe_carry(B.X, B.X);
    fe_sub(B.T, z, negB.T);
    fe_carry(B.T, B.T);
    ge_cached cB;
    ge_p3_to_cached(cB, B);
    ge_p3_identity(cur);
    fe d2;
    fe_const(d2, PV_D2);
    for (int j = 0; j < PV_BTAB_ENTRIES; j++) {
        fe zi, x, y, t, ypx, ymx, xy2d;
        fe_invert(zi, cur.Z);
        fe_mul(x, cur.X, zi);
        fe_mul(y, cur.Y, zi);
        fe_add(t, y, x);
        fe_canonical(ypx, t);
        fe_sub(t, y, x);
        fe_canonical(ymx, t);
        fe_mul(t, x, y);
        fe_mul(t, t, d2);
        fe_canonical(xy2d, t);
        uint32_t* e = out + j * PV_BTAB_STRIDE;
        for (int i = 0; i < 10; i++) {
            e[i] = ypx.v[i];
            e[10 + i] = ymx.v[i];
            e[20 + i] = xy2d.v[i];
        }
        e[30] = 0;
        e[31] = 0;
        ge_p1p1 r;
        ge_add_cached(r, cur, cB);
        ge_p1p1_to_p3(cur, r);
    }
}

// Host/LDS-agnostic reader of the flat table.
struct pv_btab_flat {
    const uint32_t* base;
    // part 0: words 0..19 (y+x, y-x); part 1: words 20..29 (2d x y) into w[0..9]
    PV_HD void load_part(int j, int part, uint32_t w[20]) const {
        const uint32_t* e = base + j * PV_BTAB_STRIDE + 20 * part;
        for (int i = 0; i < (part ? 10 : 20); i++) w[i] = e[i];
    }
    PV_HD void load(int j, ge_niels& q) const {
        const uint32_t* e = base + j * PV_BTAB_STRIDE;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            q.yplusx.v[i] = e[i];
            q.yminusx.v[i] = e[10 + i];
            q.xy2d.v[i] = e[20 + i];
        }
    }
};
