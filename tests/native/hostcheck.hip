// TEST INFRASTRUCTURE: host-compiled build of the device arithmetic headers
// (indy-plenum_amd/csrc/*.h) with PV_BOUNDS_CHECK, so tests can drive the exact kernel code on the
// CPU against Python big integers, the C oracle and libsodium. Not part of the product library.
#define PV_BOUNDS_CHECK 1
#include "verify_core.h"
#include "btable.h"
#include "comb.h"
#include <string.h>
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
int hc_sign_open_comb(const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
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

// k = SHA-512(R||A||M) mod L through pv_prepare (exposes the hashing + reduction)
void hc_prepare_k(uint8_t* kout, const uint8_t* sm, uint64_t smlen, const uint8_t* pk) {
    std::vector<uint8_t> buf(smlen + 256, 0);  // PV_BLOB_SLACK
    memcpy(buf.data(), sm, smlen);
    pv_sig_words in; memcpy(in.R, buf.data(), 32); memcpy(in.S, buf.data() + 32, 32); memcpy(in.A, pk, 32);
    ge_p3 negA; uint32_t k[8]; HostMsg mw{buf.data()};
    pv_prepare(negA, k, in, smlen, mw);
    memcpy(kout, k, 32);
}
}
