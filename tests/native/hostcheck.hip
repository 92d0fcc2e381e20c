// TEST INFRASTRUCTURE: host-compiled build of the device arithmetic headers
// (indy-plenum_amd/csrc/*.h) with PV_BOUNDS_CHECK, so tests can drive the exact kernel code on the
// CPU against Python big integers, the C oracle and libsodium. Not part of the product library.
#define PV_BOUNDS_CHECK 1
#include "verify_core.h"
#include "btable.h"
#include "comb.h"
#include <map>
#include "lp25519.h"
#include <string.h>
#include <algorithm>
#include <vector>
#include <thread>

extern "C" {

static void load_words(uint32_t w[8], const uint8_t* b) { memcpy(w, b, 32); }

// raw limb ops (limbs supplied by the caller, so bound assertions are exercised)
void hc_fe_mul(uint32_t* h, const uint32_t* f, const uint32_t* g) {
    fe a, b, c; memcpy(a.v, f, 40); memcpy(b.v, g, 40); fe_mul(c, a, b); memcpy(h, c.v, 40);
}
void hc_fe_sq(uint32_t* h, const uint32_t* f) {
    fe a, c; memcpy(a.v, f, 40); fe_sq(c, a); memcpy(h, c.v, 40);
}
void hc_fe_carry(uint32_t* h, const uint32_t* f) {
    fe a, c; memcpy(a.v, f, 40); fe_carry(c, a); memcpy(h, c.v, 40);
}
void hc_fe_tobytes(uint8_t* s, const uint32_t* f) {
    fe a; memcpy(a.v, f, 40); uint32_t w[8]; fe_tobytes32(w, a); memcpy(s, w, 32);
}
void hc_fe_frombytes(uint32_t* h, const uint8_t* s) {
    uint32_t w[8]; load_words(w, s); fe a; fe_frombytes32(a, w); memcpy(h, a.v, 40);
}
void hc_fe_invert(uint32_t* h, const uint32_t* f) {
    fe a, c; memcpy(a.v, f, 40); fe_invert(c, a); memcpy(h, c.v, 40);
}
void hc_fe_pow22523(uint32_t* h, const uint32_t* f) {
    fe a, c; memcpy(a.v, f, 40); fe_pow22523(c, a); memcpy(h, c.v, 40);
}
void hc_sc_reduce64(uint8_t* r, const uint8_t* x) {
    uint32_t xw[16], rw[8]; memcpy(xw, x, 64); sc_reduce64(rw, xw); memcpy(r, rw, 32);
}
int hc_sc_is_canonical(const uint8_t* s) { uint32_t w[8]; load_words(w, s); return sc_is_canonical(w); }
void hc_sc_recode16(uint8_t* out, const uint8_t* a) { uint32_t w[8], o[8]; load_words(w, a); sc_recode16(o, w); memcpy(out, o, 32); }
void hc_sc_recode256(uint8_t* out, const uint8_t* a) { uint32_t w[8], o[8]; load_words(w, a); sc_recode256(o, w); memcpy(out, o, 32); }
void hc_sc_recode65536(uint8_t* out, const uint8_t* a) { uint32_t w[8], o[8]; load_words(w, a); sc_recode65536(o, w); memcpy(out, o, 32); }
int hc_has_small_order(const uint8_t* s) { uint32_t w[8]; load_words(w, s); return pv_has_small_order(w); }
int hc_ge_is_canonical(const uint8_t* s) { uint32_t w[8]; load_words(w, s); return pv_ge_is_canonical(w); }

void hc_build_b_table(uint32_t* out) { pv_build_b_table(out); }

struct HostATab {
    uint32_t e[9][40];
    void store(int j, const uint32_t w[40]) { memcpy(e[j], w, 160); }
    void load(int j, uint32_t w[40]) const { memcpy(w, e[j], 160); }
    void load_half(int j, int h, uint32_t w[20]) const { memcpy(w, e[j] + 20 * h, 80); }
};

struct HostMsg {
    const uint8_t* sm;
    uint64_t operator()(uint64_t q) const { uint64_t v; memcpy(&v, sm + 8 * q, 8); return v; }
};

// Full pipeline on the host: crypto_sign_open(sm, smlen, pk) == 0 ? 1 : 0.
// sm is copied into a buffer with PV_BLOB_SLACK bytes of zero slack (the kernel contract).
int hc_sign_open(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    static std::vector<uint32_t> btab;
    if (btab.empty()) { btab.resize(PV_BTAB_ENTRIES * PV_BTAB_STRIDE); pv_build_b_table(btab.data()); }
    std::vector<uint8_t> buf(smlen + 256, 0);  // PV_BLOB_SLACK
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    ge_p3 negA; uint32_t k[8];
    HostMsg mw{buf.data()};
    bool ok = pv_prepare(negA, k, in, smlen, mw);
    HostATab at;
    pv_build_a_table(at, negA);
    pv_btab_flat bt{btab.data()};
    uint32_t enc[8];
    pv_double_scalarmult(enc, at, bt, k, in.S);
    return ok && pv_words_equal(enc, in.R);
}

// Batched encoding (one shared inversion) of PV_ENC_BATCH projective points given as 30 limbs
// each (X, Y, Z); use[t] in/out. Writes 32-byte encodings.
void hc_encode_batch(uint8_t* out, const uint32_t* xyz, int* use) {
    fe X[PV_ENC_BATCH], Y[PV_ENC_BATCH], Z[PV_ENC_BATCH];
    bool u[PV_ENC_BATCH];
    for (int t = 0; t < PV_ENC_BATCH; t++) {
        memcpy(X[t].v, xyz + 30 * t, 40); memcpy(Y[t].v, xyz + 30 * t + 10, 40); memcpy(Z[t].v, xyz + 30 * t + 20, 40);
        u[t] = use[t] != 0;
    }
    uint32_t enc[PV_ENC_BATCH][8];
    pv_encode_batch(enc, X, Y, Z, u);
    for (int t = 0; t < PV_ENC_BATCH; t++) { memcpy(out + 32 * t, enc[t], 32); use[t] = u[t]; }
}
int hc_enc_batch_size(void) { return PV_ENC_BATCH; }
// The same with 16 points in two groups of 8 under one inversion (pv_encode_batch_stream_b<16>: the
// device's encode for chunks of >= 1M requests).
void hc_encode_batch16(uint8_t* out, const uint32_t* xyz, int* use) {
    fe X[16], Y[16], Z[16];
    bool u[16];
    for (int t = 0; t < 16; t++) {
        memcpy(X[t].v, xyz + 30 * t, 40); memcpy(Y[t].v, xyz + 30 * t + 10, 40); memcpy(Z[t].v, xyz + 30 * t + 20, 40);
        u[t] = use[t] != 0;
    }
    uint32_t enc[16][8];
    pv_encode_batch_stream_b<16>(pv_enc_arrays{X, Y, Z}, u, pv_enc_out{enc});
    for (int t = 0; t < 16; t++) { memcpy(out + 32 * t, enc[t], 32); use[t] = u[t]; }
}

// ---- keyed comb path on the host (comb.h): same code the comb kernels run
struct HostBases {
    ge_p3* b;  // [32][PV_COMB_PTS]
    void store(int i, int m, const ge_p3& p) const { b[i * PV_COMB_PTS + m] = p; }
};
struct HostBasePts {
    const ge_p3* b;  // the position's PV_COMB_PTS points
    void load(int m, ge_p3& p) const { p = b[m]; }
};
struct HostCombRow {
    uint32_t* r;  // [129][40]
    void store(int d, const ge_cached& c) const { ge_cached_store_words(r + 40 * d, c); }
    void load(int d, ge_cached& c) const { ge_cached_load_words(c, r + 40 * d); }
    void load_half(int d, int h, uint32_t w[20]) const { memcpy(w, r + 40 * d + 20 * h, 80); }
};
struct HostCombRows {
    uint32_t* base;
    HostCombRow row(int i) const { return HostCombRow{base + (size_t)i * PV_COMB_ENT * 40}; }
};
struct HostBRow {
    const uint32_t* r;
    void load_part(int d, int part, uint32_t w[20]) const {
        memcpy(w, r + d * PV_BCOMB_STRIDE + 20 * part, part ? 40 : 80);
    }
};
struct HostBRows {
    const uint32_t* base;
    HostBRow row(int i) const { return HostBRow{base + (size_t)i * PV_BCOMB_ENT * PV_BCOMB_STRIDE}; }
};

// crypto_sign_open through the comb path: key expansion (chain + all fill blocks), radix-256
// digits, 64 additions, batched encoding.
static const std::vector<uint32_t>& host_bcomb() {
    static std::vector<uint32_t> bcomb;
    if (bcomb.empty()) {
        bcomb.resize((size_t)PV_BCOMB_POS * PV_BCOMB_ENT * PV_BCOMB_STRIDE);
        ge_p3 base[PV_BCOMB_POS];
        pv_bcomb_bases(base);
        std::vector<std::thread> th;
        for (int j = 0; j < PV_BCOMB_POS; j++)
            th.emplace_back(pv_bcomb_build_position, bcomb.data() + (size_t)j * PV_BCOMB_ENT * PV_BCOMB_STRIDE,
                            std::cref(base[j]));
        for (auto& t : th) t.join();
    }
    return bcomb;
}

int hc_sign_open_comb(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);  // PV_BLOB_SLACK
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    bool ok = pv_sig_ok(in, smlen);
    ge_p3 negA;
    ok &= pv_key_ok_negate(negA, in.A);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    std::vector<ge_p3> bases(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{bases.data()}, negA);
    std::vector<uint32_t> ctab((size_t)PV_COMB_POS * PV_COMB_ENT * 40);
    for (int pos = 0; pos < PV_COMB_POS; pos++)
        for (int b = 0; b < PV_COMB_BLOCKS; b++)
            pv_comb_fill_block(HostCombRow{ctab.data() + (size_t)pos * PV_COMB_ENT * 40},
                               HostBasePts{bases.data() + pos * PV_COMB_PTS}, b);
    pv_dig_regs dig;
    sc_recode256(dig.e, k);
    sc_recode65536(dig.f, in.S);
    fe X[PV_ENC_BATCH], Y[PV_ENC_BATCH], Z[PV_ENC_BATCH];
    bool use[PV_ENC_BATCH];
    pv_comb_xyz(X[0], Y[0], Z[0], HostCombRows{ctab.data()}, HostBRows{bcomb.data()}, dig);
    use[0] = ok;
    for (int t = 1; t < PV_ENC_BATCH; t++) { X[t] = X[0]; Y[t] = Y[0]; Z[t] = Z[0]; use[t] = false; }
    uint32_t enc[PV_ENC_BATCH][8];
    pv_encode_batch(enc, X, Y, Z, use);
    return use[0] && pv_words_equal(enc[0], in.R);
}

// Wide fixed-base comb (comb.h PV_BC2_*): signed radix-2^W digits of a 32-byte scalar; returns P.
int hc_sc_recode_w(int w, int32_t* out, const uint8_t* a) {
    uint32_t x[8];
    load_words(x, a);
    switch (w) {
        case 16: sc_recode_w<16, 16>(out, x); return 16;
        case 20: sc_recode_w<20, 13>(out, x); return 13;
        case 22: sc_recode_w<22, 12>(out, x); return 12;
        case 24: sc_recode_w<24, 11>(out, x); return 11;
        default: return 0;
    }
}

// pv_bc2_build_run over entries [d0, d0 + cnt) of the radix-65536 row with base [65536^j] B
// (out: cnt x 32 words), for comparison with pv_bcomb_build_position's table (W = 16).
struct HostBc2Row {
    uint32_t* r;
    uint32_t d0;
    uint32_t* e(uint32_t d) const { return r + (size_t)(d - d0) * PV_BCOMB_STRIDE; }
};
struct HostBc2Scratch {
    fe* z;
    uint32_t d0;
    void store(uint32_t d, const fe& f) const { z[d - d0] = f; }
    void load(uint32_t d, fe& f) const { f = z[d - d0]; }
};
void hc_bc2_build_run16(uint32_t* out, int j, uint32_t d0, uint32_t cnt) {
    ge_p3 base[PV_BCOMB_POS];
    pv_bcomb_bases(base);
    std::vector<fe> z(cnt);
    pv_bc2_build_run(HostBc2Row{out, d0}, HostBc2Scratch{z.data(), d0}, base[j], d0, cnt);
}
const uint32_t* hc_bcomb_table(void) { return host_bcomb().data(); }

// crypto_sign_open through the comb path with [S]B from pv_comb_b_acc_w<16> (the wide comb's code,
// W = 16) over the radix-65536 host table, [k](-A) from the staged per-key comb.
struct HostAffineRowDst {
    uint32_t* r;  // [129][40]
    uint32_t* e(int d) const { return r + 40 * d; }
};
static int sign_open_comb_wide16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk, bool affine);
int hc_sign_open_comb_wide16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    return sign_open_comb_wide16(sm, smlen, pk, false);
}
// The same with the per-key rows converted by pv_comb_row_to_affine (the key cache's affine rows) and
// [k](-A) from pv_comb_a_xyz_staged in its affine mode (the device comb kernels on a cached key).
int hc_sign_open_comb_affine16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    return sign_open_comb_wide16(sm, smlen, pk, true);
}
static int sign_open_comb_wide16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk, bool affine) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    bool ok = pv_sig_ok(in, smlen);
    ge_p3 negA;
    ok &= pv_key_ok_negate(negA, in.A);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    std::vector<ge_p3> bases(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{bases.data()}, negA);
    std::vector<uint32_t> ctab((size_t)PV_COMB_POS * PV_COMB_ENT * 40);
    for (int pos = 0; pos < PV_COMB_POS; pos++)
        for (int b = 0; b < PV_COMB_BLOCKS; b++)
            pv_comb_fill_block(HostCombRow{ctab.data() + (size_t)pos * PV_COMB_ENT * 40},
                               HostBasePts{bases.data() + pos * PV_COMB_PTS}, b);
    pv_dig_regs dig;
    sc_recode256(dig.e, k);
    int32_t fb[16];
    sc_recode_w<16, 16>(fb, in.S);
    HostBRows brows{bcomb.data()};
    ge_p3 acc;
    pv_comb_b_acc_w<16>(acc, PvRowsStageB<HostBRows>{brows, 0, 0}, [&](int j) { return fb[j]; });
    std::vector<uint32_t> atab;
    if (affine) {
        atab.resize(ctab.size());
        for (int pos = 0; pos < PV_COMB_POS; pos++)
            pv_comb_row_to_affine(HostCombRow{ctab.data() + (size_t)pos * PV_COMB_ENT * 40},
                                  HostAffineRowDst{atab.data() + (size_t)pos * PV_COMB_ENT * 40});
    }
    HostCombRows arows{affine ? atab.data() : ctab.data()};
    fe X[PV_ENC_BATCH], Y[PV_ENC_BATCH], Z[PV_ENC_BATCH];
    bool use[PV_ENC_BATCH];
    pv_comb_a_xyz_staged(X[0], Y[0], Z[0], acc, PvRowsStageA<HostCombRows>{arows, 0, 0, affine}, dig);
    use[0] = ok;
    for (int t = 1; t < PV_ENC_BATCH; t++) { X[t] = X[0]; Y[t] = Y[0]; Z[t] = Z[0]; use[t] = false; }
    uint32_t enc[PV_ENC_BATCH][8];
    pv_encode_batch(enc, X, Y, Z, use);
    return use[0] && pv_words_equal(enc[0], in.R);
}

// crypto_sign_open through the comb path with a key's wide cached rows (comb.h PV_KW_*): the key's
// radix-65536 rows [d 65536^q](-A), d = 0..32896, built by pv_bc2_build_run from the chain's P_{2q},
// and ONE niels loop over the 16 fixed-base positions (W = 16 host table) and the key's 16 positions
// with digits d_q = e_{2q} + 256 e_{2q+1} (pv_comb_b_acc_w with total = 32) -- the device's
// pv_comb_bw_acc. Wide rows are cached per key (a few seconds to build on the host).
struct HostBWStage {
    const HostBRows& brows;
    const uint32_t* wrows;  // [16][PV_KW_ENT][32]
    mutable int row_i, ent;
    void stage(int i, int d) const { row_i = i; ent = d; }
    void staged(int part, uint32_t w[20]) const {
        const uint32_t* e = row_i < PV_KW_POS ? wrows + ((size_t)row_i * PV_KW_ENT + ent) * PV_BCOMB_STRIDE
                                              : brows.base + ((size_t)(row_i - PV_KW_POS) * PV_BCOMB_ENT + ent) * PV_BCOMB_STRIDE;
        memcpy(w, e + 20 * part, part ? 40 : 80);
    }
};
int hc_sign_open_comb_kw16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    static std::map<std::string, std::vector<uint32_t>> wide;  // key -> rows
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    bool ok = pv_sig_ok(in, smlen);
    ge_p3 negA;
    ok &= pv_key_ok_negate(negA, in.A);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    std::string key(reinterpret_cast<const char*>(pk), 32);
    auto it = wide.find(key);
    if (it == wide.end()) {
        std::vector<ge_p3> bases(PV_COMB_POS * PV_COMB_PTS);
        pv_comb_chain(HostBases{bases.data()}, negA);
        std::vector<uint32_t> rows((size_t)PV_KW_POS * PV_KW_ENT * PV_BCOMB_STRIDE);
        std::vector<std::thread> th;
        for (int q = 0; q < PV_KW_POS; q++)
            th.emplace_back([&, q] {
                std::vector<fe> z(PV_KW_ENT);
                uint32_t* r = rows.data() + (size_t)q * PV_KW_ENT * PV_BCOMB_STRIDE;
                for (uint32_t d0 = 0; d0 < PV_KW_ENT; d0 += 64)
                    pv_bc2_build_run(HostBc2Row{r, 0}, HostBc2Scratch{z.data(), 0}, bases[2 * q * PV_COMB_PTS], d0,
                                     std::min<uint32_t>(64, PV_KW_ENT - d0));
            });
        for (auto& t : th) t.join();
        it = wide.emplace(key, std::move(rows)).first;
    }
    pv_dig_regs dig;
    sc_recode256(dig.e, k);
    int32_t fb[16];
    sc_recode_w<16, 16>(fb, in.S);
    HostBRows brows{bcomb.data()};
    ge_p3 acc;
    pv_comb_b_acc_w<16>(acc, HostBWStage{brows, it->second.data(), 0, 0},
                        [&](int j) {
                            if (j < PV_KW_POS) return pv_kw_digit(dig.e[j >> 1], j);
                            return (int)fb[j - PV_KW_POS];
                        },
                        16 + PV_KW_POS);
    fe X[PV_ENC_BATCH], Y[PV_ENC_BATCH], Z[PV_ENC_BATCH];
    bool use[PV_ENC_BATCH];
    X[0] = acc.X;
    Y[0] = acc.Y;
    Z[0] = acc.Z;
    use[0] = ok;
    for (int t = 1; t < PV_ENC_BATCH; t++) { X[t] = X[0]; Y[t] = Y[0]; Z[t] = Z[0]; use[t] = false; }
    uint32_t enc[PV_ENC_BATCH][8];
    pv_encode_batch(enc, X, Y, Z, use);
    return use[0] && pv_words_equal(enc[0], in.R);
}

// The Straus path with [S]B from the wide comb (PV_STRAUS_WIDE_B): checks, -A, k, the [j](-A)
// table, pv_comb_b_acc_w<16> over the radix-65536 host table, pv_straus_a_xyz (loop over k only,
// then one addition of [S]B), encoding.
int hc_sign_open_straus_wide16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    ge_p3 negA;
    uint32_t k[8];
    HostMsg mw{buf.data()};
    bool ok = pv_prepare(negA, k, in, smlen, mw);
    HostATab at;
    pv_build_a_table(at, negA);
    pv_dig_regs dig;
    sc_recode16(dig.e, k);
    int32_t fb[16];
    sc_recode_w<16, 16>(fb, in.S);
    HostBRows brows{bcomb.data()};
    ge_p3 accB;
    pv_comb_b_acc_w<16>(accB, PvRowsStageB<HostBRows>{brows, 0, 0}, [&](int j) { return fb[j]; });
    fe X, Y, Z;
    pv_straus_a_xyz(X, Y, Z, at, dig, [&](ge_p3& p) { p = accB; });
    uint32_t enc[8];
    ge_p2_tobytes(enc, X, Y, Z);
    return ok && pv_words_equal(enc, in.R);
}

// sc_halfsize on a 32-byte scalar: |k1| and k2 (32 bytes each), *neg = k1 < 0; returns 1 if the
// (k, 1) fallback was taken.
int hc_sc_halfsize(const uint8_t* k, uint8_t* k1, uint8_t* k2, int* neg) {
    uint32_t kw[8];
    load_words(kw, k);
    pv_halfk h;
    sc_halfsize(h, kw);
    memcpy(k1, h.k1, 32);
    memcpy(k2, h.k2, 32);
    *neg = h.neg;
    return h.fallback;
}
void hc_sc_mul(uint8_t* r, const uint8_t* a, const uint8_t* b) {
    uint32_t aw[8], bw[8], rw[8];
    load_words(aw, a);
    load_words(bw, b);
    sc_mul(rw, aw, bw);
    memcpy(r, rw, 32);
}
int hc_sc_nwin16(const uint8_t* a) {
    uint32_t w[8], e[8];
    load_words(w, a);
    sc_recode16(e, w);
    return sc_nwin16(e);
}

// lp_halfsize (the latency path's limb-parallel split) on a 32-byte scalar, same outputs as
// hc_sc_halfsize
int hc_lp_halfsize(const uint8_t* k, uint8_t* k1, uint8_t* k2, int* neg) {
    uint32_t kw[8];
    load_words(kw, k);
    const LpLane c = LpLane::make();
    pv_halfk h;
    lp_halfsize(c, h, kw);
    memcpy(k1, h.k1, 32);
    memcpy(k2, h.k2, 32);
    *neg = h.neg;
    return h.fallback;
}
// lp_ydbl_chain + lp_ydbl_finish (the four-wave latency kernel's y-only [2^n] chains) against n
// lp_dbl steps of the decompressed point, for -A (row 0) and R (row 1) of lp_decompress_ar: bit r of
// the result is set when row r's two points are equal projectively; -1 if either does not decompress.
int hc_lp_ydbl_check(const uint8_t* a_enc, const uint8_t* r_enc, int n) {
    uint32_t wa[8], wr[8];
    load_words(wa, a_enc);
    load_words(wr, r_enc);
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    lu sw[8];
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(lp_eq(c.row & 1u, 1u), wr[q], wa[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    if (!dec.ok_a || !dec.ok_r) return -1;
    int mask = 0;
    for (int which = 0; which < 2; which++) {
        const lu P = lp_ext_from_xy(c, K, dec.X, dec.Y, which);
        lu Q = P;
        for (int i = 0; i < n; i++) Q = lp_dbl(c, Q);
        lu yw[8];
        for (int q = 0; q < 8; q++) yw[q] = which ? wr[q] : wa[q];
        const LpYChain ch = lp_ydbl_chain(c, K, lp_from_words(c, yw), n);
        lu x0, t1, t2, t3;
        lp_allrows(P, x0, t1, t2, t3);
        const lu R = lp_ydbl_finish(c, K, ch, x0);
        bool same = true;
        for (int r = 0; r < 4; r += (r == 1 ? 2 : 1)) {  // X, Y and T against Z
            fe a, b, d;
            fe_mul(a, lp_row_fe(Q, r), lp_row_fe(R, 2));
            fe_mul(b, lp_row_fe(R, r), lp_row_fe(Q, 2));
            fe_sub(d, a, b);
            same &= fe_iszero(d);
        }
        mask |= same ? 1 << which : 0;
    }
    return mask;
}
// lp_build_a_table_part (the four-wave kernel's R' table built by three waves): 1 if parts 0, 1, 2
// together give the points of lp_build_a_table at every entry j = -8..8, 0 if not, -1 if the
// encoding does not decompress.
int hc_lp_table_parts_check(const uint8_t* enc) {
    uint32_t wa[8];
    load_words(wa, enc);
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    lu sw[8];
    for (int q = 0; q < 8; q++) sw[q] = wa[q];
    const LpDecomp d = lp_decompress_ar(c, K, sw);
    if (!d.ok_a) return -1;
    const lu P = lp_ext_from_xy(c, K, d.X, d.Y, 0);
    lu full[17], part[17];
    lp_build_a_table(c, K, P, [&](int j, const lu& q) { full[j + 8] = q; });
    for (int pt = 0; pt < 3; pt++) lp_build_a_table_part(c, K, P, pt, [&](int j, const lu& q) { part[j + 8] = q; });
    for (int e = 0; e < 17; e++)
        for (int r = 0; r < 3; r++) {  // cached rows [Y-X, Y+X, 2dT] against 2Z (row 3)
            fe a, b, dd;
            fe_mul(a, lp_row_fe(full[e], r), lp_row_fe(part[e], 3));
            fe_mul(b, lp_row_fe(part[e], r), lp_row_fe(full[e], 3));
            fe_sub(dd, a, b);
            if (!fe_iszero(dd)) return 0;
        }
    return 1;
}
// lp_halfsize's counts for one scalar: [0] Lehmer blocks, [1] quotients settled inside them, [2] exact steps
void hc_lp_halfsize_stats(const uint8_t* k, uint32_t* stats) {
    uint32_t kw[8];
    load_words(kw, k);
    const LpLane c = LpLane::make();
    pv_halfk h;
    stats[0] = stats[1] = stats[2] = 0;
    lp_halfsize(c, h, kw, stats);
}

// The half-size Straus path as the device runs it: pv_prepare_half (checks, +-A, -R', split of k,
// k2 S mod L), the [j]PA and [j](-R') tables, [k2 S]B from pv_comb_b_acc_w<16> over the radix-65536
// host table, pv_straus_ar_xyz (and the fused epilogue's form), encoding compared with R. force_fallback: use (k, 1) as the split (the
// lane fallback). extra_windows: run that many leading all-zero windows (a wave whose maximum exceeds
// this lane's need).
struct HostDig2 {
    uint32_t e[8], e2[8];
    uint32_t ek(int q) const { return e[q]; }
    uint32_t ek2(int q) const { return e2[q]; }
};
int hc_sign_open_straus_half16(const uint8_t* sm, uint64_t smlen, const uint8_t* pk, int force_fallback,
                               int extra_windows) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    ge_p3 PA, negR;
    pv_halfk hk;
    uint32_t s2[8];
    bool ok = pv_prepare_half(PA, negR, hk, s2, in, smlen, mw);
    if (force_fallback) {
        // redo the split as the fallback lane would have it
        ge_p3_cneg(PA, hk.neg);  // back to -A
        uint32_t k[8];
        pv_hash_k(k, in, smlen, mw);
        for (int i = 0; i < 8; i++) {
            hk.k1[i] = k[i];
            hk.k2[i] = i == 0 ? 1u : 0u;
        }
        hk.neg = false;
        sc_mul<5>(s2, hk.k2, in.S);
    }
    HostATab at, rt;
    pv_build_a_table(at, PA);
    pv_build_a_table(rt, negR);
    HostDig2 dig;
    sc_recode16(dig.e, hk.k1);
    sc_recode16(dig.e2, hk.k2);
    int nw = sc_nwin16(dig.e);
    const int nw2 = sc_nwin16(dig.e2);
    nw = nw > nw2 ? nw : nw2;
    nw += extra_windows;
    if (nw > 64) nw = 64;
    int32_t fb[16];
    sc_recode_w<16, 16>(fb, s2);
    HostBRows brows{bcomb.data()};
    ge_p3 accB;
    pv_comb_b_acc_w<16>(accB, PvRowsStageB<HostBRows>{brows, 0, 0}, [&](int j) { return fb[j]; });
    fe X, Y, Z, X2, Y2, Z2;
    pv_straus_ar_xyz(X, Y, Z, at, rt, dig, nw, [&](ge_p3& p) { p = accB; });
    // the LDS-staged loop the device runs (pv_straus_ar_xyz_staged) gives the same point
    pv_straus_ar_xyz_staged(X2, Y2, Z2, PvTabStage2<HostATab>{at, rt, 0, 0}, dig, nw, [&](ge_p3& p) { p = accB; });
    // the device's fused epilogue (pv_msm_kernel, PV_MSM_FUSED_B): [k2 S]B's niels additions straight
    // into the loop's point (pv_comb_b_add_w) instead of one cached addition of accB
    fe X3, Y3, Z3;
    pv_straus_ar_xyz_addb(X3, Y3, Z3, at, rt, dig, nw, [&](ge_p3& acc) {
        pv_comb_b_add_w<16>(acc, PvRowsStageB<HostBRows>{brows, 0, 0}, [&](int j) { return fb[j]; });
    });
    uint32_t enc[8], enc2[8], enc3[8];
    ge_p2_tobytes(enc, X, Y, Z);
    ge_p2_tobytes(enc2, X2, Y2, Z2);
    ge_p2_tobytes(enc3, X3, Y3, Z3);
    // the fused form adds in another order: the same point whenever every operand is a curve point (the
    // addition law is complete); a request whose R or A failed its checks is rejected either way
    if (!pv_words_equal(enc, enc2) || (ok && !pv_words_equal(enc, enc3))) return -1;
    return ok && pv_words_equal(enc, in.R);
}

// pv_comb_fill_sparse (the small-chunk table fill) against pv_comb_fill_block (the full fill) for one
// key: every position, a pseudo-random need set of about `density` x 129 entries (seeded); returns the
// number of needed or always-built entries whose point differs from the full table's.
struct HostNeed {
    const uint32_t* p;
    uint32_t word(int w) const { return p[w]; }
};
int hc_comb_fill_sparse_check(const uint8_t* pk, uint32_t seed, double density) {
    uint32_t A[8];
    memcpy(A, pk, 32);
    ge_p3 negA;
    if (!pv_key_ok_negate(negA, A)) return -1;
    std::vector<ge_p3> bases(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{bases.data()}, negA);
    std::vector<uint32_t> full((size_t)PV_COMB_POS * PV_COMB_ENT * 40), sparse(full.size(), 0);
    int bad = 0;
    uint64_t st = seed * 6364136223846793005ull + 1442695040888963407ull;
    for (int pos = 0; pos < PV_COMB_POS; pos++) {
        for (int b = 0; b < PV_COMB_BLOCKS; b++)
            pv_comb_fill_block(HostCombRow{full.data() + (size_t)pos * PV_COMB_ENT * 40},
                               HostBasePts{bases.data() + pos * PV_COMB_PTS}, b);
        uint32_t need[5] = {0, 0, 0, 0, 0};
        for (int d = 0; d < PV_COMB_ENT; d++) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            if ((double)(st >> 11) / 9007199254740992.0 < density) need[d >> 5] |= 1u << (d & 31);
        }
        pv_comb_fill_sparse(HostCombRow{sparse.data() + (size_t)pos * PV_COMB_ENT * 40},
                            HostBasePts{bases.data() + pos * PV_COMB_PTS}, HostNeed{need});
        for (int d = 0; d < PV_COMB_ENT; d++) {
            const bool built = ((need[d >> 5] | PV_SPARSE_PRE[d >> 5]) >> (d & 31)) & 1;
            if (!built) continue;
            ge_cached a, c;
            ge_cached_load_words(a, full.data() + ((size_t)pos * PV_COMB_ENT + d) * 40);
            ge_cached_load_words(c, sparse.data() + ((size_t)pos * PV_COMB_ENT + d) * 40);
            const fe* fa[3] = {&a.YplusX, &a.YminusX, &a.T2d};
            const fe* fc[3] = {&c.YplusX, &c.YminusX, &c.T2d};
            for (int k = 0; k < 3; k++) {
                fe x, y;
                fe_mul(x, *fa[k], c.Z2);
                fe_mul(y, *fc[k], a.Z2);
                uint32_t u[8], v[8];
                fe_tobytes32(u, x);
                fe_tobytes32(v, y);
                if (memcmp(u, v, sizeof u)) bad++;
            }
        }
    }
    return bad;
}

// k = SHA-512(R||A||M) mod L through pv_prepare (exposes the hashing + reduction)
void hc_prepare_k(uint8_t* kout, const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    std::vector<uint8_t> buf(smlen + 256, 0);  // PV_BLOB_SLACK
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in; memcpy(in.R, buf.data(), 32); memcpy(in.S, buf.data() + 32, 32); memcpy(in.A, pk, 32);
    ge_p3 negA; uint32_t k[8]; HostMsg mw{buf.data()};
    pv_prepare(negA, k, in, smlen, mw);
    memcpy(kout, k, 32);
}

// ---- latency path (lp25519.h) on the host: the 64 lanes of a wave simulated exactly
static lu hc_rows_in(const uint32_t* x /* 4 x 10 limbs */) {
    lu v;
    for (int l = 0; l < 64; l++) v.v[l] = (l & 15) < 10 ? x[10 * (l >> 4) + (l & 15)] : 0x1234567u + l;
    return v;
}
static void hc_rows_out(uint32_t* x, const lu& v) {
    for (int r = 0; r < 4; r++)
        for (int k = 0; k < 10; k++) x[10 * r + k] = v.v[16 * r + k];
}
void hc_lp_mul(uint32_t* h, const uint32_t* f, const uint32_t* g) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_mul(c, hc_rows_in(f), hc_rows_in(g)));
}
void hc_lp_pow22523(uint32_t* h, const uint32_t* f) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_pow22523(c, hc_rows_in(f)));
}
void hc_lp_invert(uint32_t* h, const uint32_t* f) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_invert(c, hc_rows_in(f)));
}
// lp_mul_dual / lp_pow22523<true>: rows 2, 3 of the inputs must repeat rows 0, 1
void hc_lp_mul_dual(uint32_t* h, const uint32_t* f, const uint32_t* g) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_mul_dual(c, hc_rows_in(f), hc_rows_in(g)));
}
void hc_lp_invert_dual(uint32_t* h, const uint32_t* f) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_invert<true>(c, hc_rows_in(f)));
}
void hc_lp_pow22523_dual(uint32_t* h, const uint32_t* f) {
    const LpLane c = LpLane::make();
    hc_rows_out(h, lp_pow22523<true>(c, hc_rows_in(f)));
}
// group ops on an ext point given as 4 rows [X, Y, Z, T]
void hc_lp_dbl(uint32_t* out, const uint32_t* p) {
    const LpLane c = LpLane::make();
    hc_rows_out(out, lp_dbl(c, hc_rows_in(p)));
}
void hc_lp_add(uint32_t* out, const uint32_t* p, const uint32_t* q) {
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    hc_rows_out(out, lp_add_cached(c, hc_rows_in(p), lp_to_cached(c, hc_rows_in(q), K.d2)));
}
void hc_lp_sub(uint32_t* out, const uint32_t* p, const uint32_t* q) {
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    hc_rows_out(out, lp_add_cached(c, hc_rows_in(p), lp_neg_cached(c, lp_to_cached(c, hc_rows_in(q), K.d2))));
}

// crypto_sign_open through the latency path: the kernel's two waves, one after the other (wave 1
// up to its barrier, wave 0 up to its barrier, wave 1's loop, wave 0's loop and the final check)
int hc_lp_sign_open(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);  // PV_BLOB_SLACK
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    // wave 1: checks, k, the half-size split, s2 = k2 S mod L and its comb entries
    const bool sig_ok = pv_sig_ok(in, smlen);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    pv_halfk hk;
    lp_halfsize(c, hk, k);
    uint32_t s2[8], fs[8], e1[8], e2[8];
    sc_mul<5>(s2, hk.k2, in.S);
    sc_recode65536(fs, s2);
    lu ent[PV_BCOMB_POS];
    for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb.data(), j, pv_half(fs[j >> 1], j));
    sc_recode16(e1, hk.k1);
    sc_recode16(e2, hk.k2);
    const int nw = std::max(sc_nwin16(e1), sc_nwin16(e2));
    // wave 0: decompression of A and R, key checks, both tables
    lu sw[8];
    const lm odd_row = lp_eq(c.row & 1u, 1u);
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    const bool key_ok = pv_ge_is_canonical(in.A) && !pv_has_small_order(in.A) && dec.ok_a;
    const bool r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
    std::vector<lu> tab(17), rtab(17);
    lp_build_a_table(c, K, lp_ext_from_xy(c, K, dec.X, dec.Y, 0), [&](int j, const lu& q) { tab[j + 8] = q; });
    lp_build_a_table(c, K, lp_ext_from_xy(c, K, dec.X, dec.Y, 1), [&](int j, const lu& q) { rtab[j + 8] = q; });
    // wave 1 after barrier 1: [k2](-R') + [s2]B
    lu SB = lp_straus_nw(c, nw, [&](int i) { return pv_nibble(e2[i >> 3], i); },
                         [&](int e) { return rtab[8 - e]; });
    for (int j = PV_BCOMB_POS - 1; j >= 0; j--) SB = lp_add_cached(c, SB, lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)));
    // wave 0 after barrier 1: [k1](-A) (signed) + R'
    const int sgn = hk.neg ? -1 : 1;
    const lu QA = lp_add_cached(c, lp_straus_nw(c, nw, [&](int i) { return sgn * pv_nibble(e1[i >> 3], i); },
                                                [&](int e) { return tab[e + 8]; }),
                                rtab[9]);
    const bool eq = lp_final_check(c, K, QA, SB, dec.X, dec.Y);
    return eq && key_ok && r_ok && sig_ok;
}

// The four-wave form (pv_lat4_kernel): [k1](+-A) and [k2](-R') each split at window `split`, the high
// parts on tables of [2^(4 split)](-A) and [2^(4 split)]R' (4 split doublings each), summed as wave 0
// sums them, then lp_final_check against R'.
int hc_lp4_sign_open(const uint8_t* sm, uint64_t smlen, const uint8_t* pk, int split) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    const bool sig_ok = pv_sig_ok(in, smlen);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    pv_halfk hk;
    lp_halfsize(c, hk, k);
    uint32_t s2[8], fs[8], e1[8], e2[8];
    sc_mul<5>(s2, hk.k2, in.S);
    sc_recode65536(fs, s2);
    sc_recode16(e1, hk.k1);
    sc_recode16(e2, hk.k2);
    const int nw = std::max(sc_nwin16(e1), sc_nwin16(e2));
    lu sw[8];
    const lm odd_row = lp_eq(c.row & 1u, 1u);
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    const bool key_ok = pv_ge_is_canonical(in.A) && !pv_has_small_order(in.A) && dec.ok_a;
    const bool r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
    const lu negA = lp_ext_from_xy(c, K, dec.X, dec.Y, 0), Rp = lp_ext_from_xy(c, K, dec.X, dec.Y, 1);
    std::vector<lu> tab[4];
    lu base[4] = {negA, Rp, negA, Rp};
    for (int w = 2; w < 4; w++)
        for (int j = 0; j < 4 * split; j++) base[w] = lp_dbl(c, base[w]);
    for (int w = 0; w < 4; w++) {
        tab[w].resize(17);
        lp_build_a_table(c, K, base[w], [&](int j, const lu& q) { tab[w][j + 8] = q; });
    }
    const int sgn = hk.neg ? -1 : 1;
    const int hi = std::min(nw, split);
    auto d1 = [&](int i) { return sgn * pv_nibble(e1[i >> 3], i); };
    auto d2 = [&](int i) { return -pv_nibble(e2[i >> 3], i); };
    lu SB = lp_straus_range(c, 0, hi, d2, [&](int e) { return tab[1][e + 8]; });
    for (int j = PV_BCOMB_POS - 1; j >= 0; j--)
        SB = lp_add_cached(c, SB, lp_bcomb_fix(c, lp_bcomb_entry(c, bcomb.data(), j, pv_half(fs[j >> 1], j)), pv_half(fs[j >> 1], j)));
    const lu p2 = lp_straus_range(c, split, nw, d1, [&](int e) { return tab[2][e + 8]; });
    const lu p3 = lp_straus_range(c, split, nw, d2, [&](int e) { return tab[3][e + 8]; });
    lu QA = lp_straus_range(c, 0, hi, d1, [&](int e) { return tab[0][e + 8]; });
    QA = lp_add_cached(c, QA, tab[1][9]);
    QA = lp_add_cached(c, QA, lp_to_cached(c, p2, K.d2));
    QA = lp_add_cached(c, QA, lp_to_cached(c, p3, K.d2));
    const bool eq = lp_final_check(c, K, QA, SB, dec.X, dec.Y);
    return eq && key_ok && r_ok && sig_ok;
}

// the cache-hit branch: [k](-A) as 32 additions from the key's comb table (built on the host with
// the same chain / fill code the engine's key kernels run)
int hc_lp_sign_open_cached(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    const std::vector<uint32_t>& bcomb = host_bcomb();
    std::vector<uint8_t> buf(smlen + 256, 0);
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in;
    memcpy(in.R, buf.data(), 32);
    memcpy(in.S, buf.data() + 32, 32);
    memcpy(in.A, pk, 32);
    HostMsg mw{buf.data()};
    // the cache build: key checks + table (pv_key_chain_quad_kernel / pv_key_fill_kernel)
    ge_p3 negA;
    const bool key_ok = pv_key_ok_negate(negA, in.A);
    std::vector<ge_p3> bases(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{bases.data()}, negA);
    std::vector<uint32_t> ctab((size_t)PV_COMB_POS * PV_COMB_ENT * 40);
    for (int pos = 0; pos < PV_COMB_POS; pos++)
        for (int b = 0; b < PV_COMB_BLOCKS; b++)
            pv_comb_fill_block(HostCombRow{ctab.data() + (size_t)pos * PV_COMB_ENT * 40},
                               HostBasePts{bases.data() + pos * PV_COMB_PTS}, b);
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    uint32_t fs[8];
    sc_recode65536(fs, in.S);
    lu ent[PV_BCOMB_POS];
    for (int j = 0; j < PV_BCOMB_POS; j++) ent[j] = lp_bcomb_entry(c, bcomb.data(), j, pv_half(fs[j >> 1], j));
    const bool sig_ok = pv_sig_ok(in, smlen);
    uint32_t k[8], e256[8];
    pv_hash_k(k, in, smlen, mw);
    sc_recode256(e256, k);
    const lu SB = lp_comb_b(c, [&](int j) { return lp_bcomb_fix(c, ent[j], pv_half(fs[j >> 1], j)); });
    lu sw[8];
    const lm odd_row = lp_eq(c.row & 1u, 1u);
    for (int q = 0; q < 8; q++) sw[q] = lp_sel(odd_row, in.R[q], in.A[q]);
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    const bool r_ok = pv_ge_is_canonical(in.R) && dec.ok_r && !(dec.x_r_zero && (in.R[7] >> 31));
    lu ta[PV_COMB_POS];
    for (int i = 0; i < PV_COMB_POS; i++) ta[i] = lp_ctab_load(c, ctab.data(), i, pv_byte(e256[i >> 2], i));
    const lu QA = lp_comb_a(c, [&](int i) { return lp_ctab_fix(c, ta[i], pv_byte(e256[i >> 2], i)); });
    const bool eq = lp_final_check(c, K, QA, SB, dec.X, dec.Y);
    return eq && key_ok && r_ok && sig_ok;
}

// pv_key_chain_lp_kernel's chain on the host vs pv_comb_chain (the quad / per-lane chain): every
// stored base equal as a point (affine x, y canonical) and every limb reduced. Returns the number of
// mismatching bases (0 = identical), or -1 if the key does not decompress.
int hc_lp_chain_check(const uint8_t* pk) {
    uint32_t A[8];
    memcpy(A, pk, 32);
    ge_p3 negA;
    if (!pv_key_ok_negate(negA, A)) return -1;
    std::vector<ge_p3> ref(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{ref.data()}, negA);
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    lu sw[8];
    for (int q = 0; q < 8; q++) sw[q] = A[q];
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    auto affine = [](const fe& X, const fe& Y, const fe& Z, uint32_t out[16]) {
        fe zi, x, y;
        fe_invert(zi, Z);
        fe_mul(x, X, zi);
        fe_mul(y, Y, zi);
        fe_tobytes32(out, x);
        fe_tobytes32(out + 8, y);
    };
    int bad = 0;
    auto cmp = [&](int i, int m, const lu& P) {
        const lu R = lp_carry1(c, P);
        fe X = lp_row_fe(R, 0), Y = lp_row_fe(R, 1), Z = lp_row_fe(R, 2), T = lp_row_fe(R, 3);
        for (const fe* f : {&X, &Y, &Z, &T}) fe_check_reduced(*f);
        uint32_t a[16], b[16];
        affine(X, Y, Z, a);
        const ge_p3& r = ref[i * PV_COMB_PTS + m];
        affine(r.X, r.Y, r.Z, b);
        if (memcmp(a, b, sizeof a)) bad++;
        // T consistent: X Y == T Z
        fe xy, tz;
        fe_mul(xy, X, Y);
        fe_mul(tz, T, Z);
        uint32_t u[8], v[8];
        fe_tobytes32(u, xy);
        fe_tobytes32(v, tz);
        if (memcmp(u, v, sizeof u)) bad++;
    };
    lu P = lp_ext_from_xy(c, K, dec.X, dec.Y, 0);
    for (int i = 0; i < PV_COMB_POS; i++) {
        cmp(i, 0, P);
        const int nd = i + 1 < PV_COMB_POS ? 8 : 6;
        for (int j = 0; j < nd; j++) {
            P = lp_dbl(c, P);
            if (j >= 3 && j <= 5) cmp(i, j - 2, P);
        }
    }
    return bad;
}

// The chain as pv_key_chain_lp_kernel runs it with PV_CHAIN_PARTS = parts: lp_comb_chain_part per
// part, every point stored as its 40 carried words, and each later part resuming from the stored
// P_lo (lp_load_ext40). Returns the number of stored points that differ from pv_comb_chain's (as
// affine points) or whose T is inconsistent.
int hc_lp_chain_parts_check(const uint8_t* pk, int parts) {
    uint32_t A[8];
    memcpy(A, pk, 32);
    ge_p3 negA;
    if (!pv_key_ok_negate(negA, A)) return -1;
    std::vector<ge_p3> ref(PV_COMB_POS * PV_COMB_PTS);
    pv_comb_chain(HostBases{ref.data()}, negA);
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    lu sw[8];
    for (int q = 0; q < 8; q++) sw[q] = A[q];
    const LpDecomp dec = lp_decompress_ar(c, K, sw);
    std::vector<uint32_t> b(PV_COMB_POS * PV_COMB_PTS * 40, 0xDEADBEEFu);
    auto store = [&](int i, int m, const lu& P) {
        const lu R = lp_carry1(c, P);
        for (int l = 0; l < 64; l++)
            if ((l & 15) < 10) b[(i * PV_COMB_PTS + m) * 40 + 10 * (l >> 4) + (l & 15)] = R.v[l];
    };
    for (int part = 0; part < parts; part++) {
        const int lo = part * PV_COMB_POS / parts, hi = (part + 1) * PV_COMB_POS / parts;
        lu P = lo == 0 ? lp_ext_from_xy(c, K, dec.X, dec.Y, 0) : lp_load_ext40(c, b.data() + lo * PV_COMB_PTS * 40);
        P = lp_comb_chain_part(c, P, lo, hi, store);
        if (hi < PV_COMB_POS) store(hi, 0, P);
    }
    int bad = 0;
    for (int i = 0; i < PV_COMB_POS; i++)
        for (int m = 0; m < PV_COMB_PTS; m++) {
            fe X, Y, Z, T;
            memcpy(X.v, &b[(i * PV_COMB_PTS + m) * 40], 40);
            memcpy(Y.v, &b[(i * PV_COMB_PTS + m) * 40 + 10], 40);
            memcpy(Z.v, &b[(i * PV_COMB_PTS + m) * 40 + 20], 40);
            memcpy(T.v, &b[(i * PV_COMB_PTS + m) * 40 + 30], 40);
            for (const fe* f : {&X, &Y, &Z, &T}) fe_check_reduced(*f);
            const ge_p3& r = ref[i * PV_COMB_PTS + m];
            fe a1, a2, zi, t;
            uint32_t u[8], v[8];
            // X / Z == r.X / r.Z and Y / Z == r.Y / r.Z, cross-multiplied
            fe_mul(a1, X, r.Z); fe_mul(a2, r.X, Z); fe_tobytes32(u, a1); fe_tobytes32(v, a2);
            if (memcmp(u, v, sizeof u)) bad++;
            fe_mul(a1, Y, r.Z); fe_mul(a2, r.Y, Z); fe_tobytes32(u, a1); fe_tobytes32(v, a2);
            if (memcmp(u, v, sizeof u)) bad++;
            fe_mul(a1, X, Y); fe_mul(a2, T, Z); fe_tobytes32(u, a1); fe_tobytes32(v, a2);
            if (memcmp(u, v, sizeof u)) bad++;
            (void)zi; (void)t;
        }
    return bad;
}

}  // extern "C"
