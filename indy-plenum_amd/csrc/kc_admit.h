// Automatic key-cache admission bookkeeping (host only; pv_key_cache_auto in include/plenum_verify.h).
//
// Every signature a node checks is untrusted input (plenum/server/client_authn.py:84-118 verifies
// whatever a client sent; plenum/server/req_authenticator.py:23-51 runs it for every request), so
// the counter that decides which keys earn a 660 KB + 67 MB cached table must not be steerable by a
// sender that holds no valid signature, nor floodable on the node's Looper thread:
//   * only appearances of keys whose request VERIFIED are counted (the caller filters by the
//     verdicts before calling count());
//   * the table's hash is keyed by a per-process random secret (NH, an almost-universal hash, then
//     multiply-shift), so colliding keys cannot be chosen offline;
//   * a probe sequence is capped at MAX_PROBE entries: an appearance that would probe further is
//     dropped (counted in dropped()), so one call's counting time is bounded whatever the keys;
//   * an evicted key (or one whose admission failed) is forgotten: its count restarts and it is
//     re-admitted on its next min_seen verified appearances, instead of staying marked admitted
//     until the counting window turns over.
// Counting window: the table holds up to WINDOW distinct keys, then starts over (a key needs its
// min_seen verified appearances within the last ~WINDOW distinct keys).
#pragma once
#include <stdint.h>
#include <string.h>

#include <random>
#include <vector>

namespace pvhost {

// NH (Black, Halevi, Krawczyk, Krovetz, Rogaway: "UMAC: fast and secure message authentication",
// CRYPTO 1999) of a 32-byte key, eight 32-bit words m_j, under eight random 32-bit secrets a_j:
// sum over pairs of (m_2i + a_2i mod 2^32) * (m_2i+1 + a_2i+1 mod 2^32) mod 2^64. Two distinct keys
// collide with probability <= 2^-32 over the secret. The bucket is the top bits of that sum times a
// random odd multiplier (Dietzfelbinger's multiply-shift). Four multiplications: ~2 ns.
inline uint64_t nh32(const uint32_t m[8], const uint32_t a[8]) {
    uint64_t h = 0;
    for (int i = 0; i < 8; i += 2) h += (uint64_t)(uint32_t)(m[i] + a[i]) * (uint32_t)(m[i + 1] + a[i + 1]);
    return h;
}

template <int LOG2_H>
class AdmitTableT {
   public:
    static constexpr uint32_t H = 1u << LOG2_H;   // entries
    static constexpr uint32_t WINDOW = H / 4;     // distinct keys per counting window (load <= 1/4)
    static constexpr uint32_t MAX_PROBE = 64;     // longest probe sequence counted
    static constexpr uint8_t ADMITTED = 255;
    enum Outcome : int { COUNTED = 0, ADMIT = 1, ALREADY = 2, DROPPED = 3 };

    // seed 0: a random secret from std::random_device (tests pass fixed seeds)
    explicit AdmitTableT(uint64_t seed = 0) {
        std::random_device rd;
        std::mt19937_64 fixed(seed);
        auto draw = [&] { return seed ? (uint32_t)fixed() : (uint32_t)rd(); };
        for (auto& x : a_) x = draw();
        mult_ = ((uint64_t)draw() << 32 | draw()) | 1u;
    }

    // A new counting window: every count restarts.
    void reset() {
        if (!e_.empty()) memset(e_.data(), 0, e_.size() * sizeof(Entry));
        used_ = 0;
        gen_++;
    }

    // Read-only lookup (the engine runs it while the batch's kernels run, before the verdicts are
    // known): the key's entry index, or -1 if it is not in the table. Nothing is inserted, so keys of
    // requests that turn out not to verify never occupy the window.
    int32_t find(const uint8_t key[32]) const {
        if (e_.empty()) return -1;
        uint64_t w[4];
        memcpy(w, key, 32);
        uint32_t h = slot_of(w);
        for (uint32_t p = 0; p < MAX_PROBE; p++, h = (h + 1) & (H - 1)) {
            const Entry& e = e_[h];
            if (!e.used) return -1;
            if (e.w[0] == w[0] && e.w[1] == w[1] && e.w[2] == w[2] && e.w[3] == w[3]) return (int32_t)h;
        }
        return -1;
    }
    // One verified appearance of the key find() located at `idx` (valid while generation() is
    // unchanged): the same outcome count() would give.
    Outcome bump_at(int32_t idx, uint32_t min_seen) {
        probes_++;
        return bump(e_[(uint32_t)idx], min_seen);
    }
    uint64_t generation() const { return gen_; }

    // One verified appearance of `key`. ADMIT: it has reached min_seen in this window now (it is
    // marked admitted); ALREADY: it was admitted before; COUNTED: below min_seen; DROPPED: its probe
    // sequence is longer than MAX_PROBE (not counted).
    Outcome count(const uint8_t key[32], uint32_t min_seen) {
        if (e_.empty()) e_.assign(H, Entry{});
        if (used_ >= WINDOW) reset();
        uint64_t w[4];
        memcpy(w, key, 32);
        uint32_t h = slot_of(w);
        for (uint32_t p = 0; p < MAX_PROBE; p++, h = (h + 1) & (H - 1)) {
            Entry& e = e_[h];
            probes_++;
            if (!e.used) {
                memcpy(e.w, w, 32);
                e.used = 1;
                e.cnt = 0;
                used_++;
                return bump(e, min_seen);
            }
            if (e.w[0] == w[0] && e.w[1] == w[1] && e.w[2] == w[2] && e.w[3] == w[3]) return bump(e, min_seen);
        }
        dropped_++;
        return DROPPED;
    }

    // The key left the cache (evicted, or its admission failed): its count restarts at zero.
    bool forget(const uint8_t key[32]) {
        if (e_.empty()) return false;
        uint64_t w[4];
        memcpy(w, key, 32);
        uint32_t h = slot_of(w);
        for (uint32_t p = 0; p < MAX_PROBE; p++, h = (h + 1) & (H - 1)) {
            Entry& e = e_[h];
            if (!e.used) return false;
            if (e.w[0] == w[0] && e.w[1] == w[1] && e.w[2] == w[2] && e.w[3] == w[3]) {
                e.cnt = 0;
                return true;
            }
        }
        return false;
    }

    uint32_t used() const { return used_; }
    const uint32_t* secret() const { return a_; }
    uint64_t multiplier() const { return mult_; }
    uint64_t probes() const { return probes_; }
    uint64_t dropped() const { return dropped_; }
    uint32_t slot_of(const uint64_t w[4]) const {
        uint32_t m[8];
        memcpy(m, w, 32);
        return (uint32_t)((nh32(m, a_) * mult_) >> (64 - LOG2_H));
    }

   private:
    struct Entry {
        uint64_t w[4];
        uint8_t used, cnt;
    };
    Outcome bump(Entry& e, uint32_t min_seen) {
        if (e.cnt == ADMITTED) return ALREADY;
        if (++e.cnt >= min_seen || e.cnt >= ADMITTED) {
            e.cnt = ADMITTED;
            return ADMIT;
        }
        return COUNTED;
    }
    uint32_t a_[8];
    uint64_t mult_;
    std::vector<Entry> e_;
    uint32_t used_ = 0;
    uint64_t probes_ = 0, dropped_ = 0, gen_ = 0;
};

// 2^17 entries (5.2 MB, allocated on first use): windows of 32,768 distinct keys
using AdmitTable = AdmitTableT<17>;

}  // namespace pvhost
