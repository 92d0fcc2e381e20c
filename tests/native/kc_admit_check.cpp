// CPU check of the automatic key-cache admission table (csrc/kc_admit.h, the header the library
// compiles): prints one JSON object for tests/test_kc_admit.py.
//   nh           buckets of fixed keys under seeded secrets (checked against a Python restatement)
//   old_collide  32,000 keys that all fall in ONE bucket of the round-5 table's unseeded hash
//                ((w0 ^ w3) * 0x9E3779B97F4A7C15 >> 48): counted twice at min_seen 2 under the keyed
//                table -- probes, drops, admissions and wall time
//   flood        200 keys brute-forced into one slot of a 1,024-entry table whose secret is known:
//                every count stops after MAX_PROBE probes (dropped), so the time stays bounded
//   forget       admit, ALREADY, forget (eviction), re-admission after min_seen new appearances
//   window       WINDOW distinct keys fill a counting window; the next count starts a new one
//   ns_per_count mean cost of one count() of a fresh random key
#include <chrono>
#include <cstdio>
#include <random>
#include <set>
#include <vector>

#include "../../indy-plenum_amd/csrc/kc_admit.h"

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

static void key_of(std::mt19937_64& r, uint8_t k[32]) {
    for (int i = 0; i < 4; i++) {
        const uint64_t w = r();
        memcpy(k + 8 * i, &w, 8);
    }
}

int main() {
    std::printf("{");
    // bucket of fixed keys under two seeded secrets
    {
        std::printf("\"nh\": [");
        std::mt19937_64 r(1);
        for (int t = 0; t < 2; t++) {
            pvhost::AdmitTable tab(100 + t);
            std::printf("%s{\"a\": [", t ? ", " : "");
            for (int i = 0; i < 8; i++) std::printf("%s%u", i ? ", " : "", tab.secret()[i]);
            std::printf("], \"mult\": \"%016llx\", \"keys\": [", (unsigned long long)tab.multiplier());
            for (int k = 0; k < 6; k++) {
                uint64_t w[4];
                for (auto& x : w) x = k == 0 ? ~0ull : r();  // key 0: all ones (every NH term wraps)
                std::printf("%s[\"%016llx\", \"%016llx\", \"%016llx\", \"%016llx\", %u]", k ? ", " : "",
                            (unsigned long long)w[0], (unsigned long long)w[1], (unsigned long long)w[2],
                            (unsigned long long)w[3], tab.slot_of(w));
            }
            std::printf("]}");
        }
        std::printf("], ");
    }
    // 32,000 keys in one bucket of the old hash
    {
        const int n = 32000;
        std::mt19937_64 r(2);
        std::vector<uint8_t> keys(32ull * n);
        std::set<uint32_t> old_buckets;
        for (int i = 0; i < n; i++) {
            uint64_t w[4] = {r(), r(), r(), 0};
            w[3] = w[0] ^ 0x0123456789abcdefull;  // w0 ^ w3 fixed
            memcpy(&keys[32ull * i], w, 32);
            old_buckets.insert((uint32_t)(((w[0] ^ w[3]) * 0x9E3779B97F4A7C15ull) >> 48) & 0xFFFFu);
        }
        pvhost::AdmitTable t;
        const auto t0 = clk::now();
        int counted = 0, admitted = 0;
        for (int pass = 0; pass < 2; pass++)
            for (int i = 0; i < n; i++) {
                const auto o = t.count(&keys[32ull * i], 2);
                counted += o == pvhost::AdmitTable::COUNTED;
                admitted += o == pvhost::AdmitTable::ADMIT;
            }
        const double ms = ms_since(t0);
        std::printf("\"old_collide\": {\"keys\": %d, \"old_buckets\": %zu, \"counted\": %d, \"admitted\": %d, "
                    "\"dropped\": %llu, \"probes\": %llu, \"ms\": %.3f, \"window\": %u}, ",
                    n, old_buckets.size(), counted, admitted, (unsigned long long)t.dropped(),
                    (unsigned long long)t.probes(), ms, pvhost::AdmitTable::WINDOW);
    }
    // a flood of keys colliding under a KNOWN secret (what an attacker would need the secret for)
    {
        using Small = pvhost::AdmitTableT<10>;
        Small t(11);
        std::mt19937_64 r(3);
        std::vector<uint8_t> keys;
        uint8_t k[32];
        while (keys.size() < 32ull * 200) {  // 200 keys in slot 0 (the window is 256 keys)
            key_of(r, k);
            uint64_t w[4];
            memcpy(w, k, 32);
            if (t.slot_of(w) == 0) keys.insert(keys.end(), k, k + 32);
        }
        const int n = (int)(keys.size() / 32);
        const auto t0 = clk::now();
        int drops = 0;
        for (int pass = 0; pass < 3; pass++)
            for (int i = 0; i < n; i++) drops += t.count(&keys[32ull * i], 2) == Small::DROPPED;
        std::printf("\"flood\": {\"keys\": %d, \"max_probe\": %u, \"probes\": %llu, \"dropped\": %d, \"ms\": %.3f}, ", n,
                    Small::MAX_PROBE, (unsigned long long)t.probes(), drops, ms_since(t0));
    }
    // forget / re-admission
    {
        pvhost::AdmitTable t;
        std::mt19937_64 r(4);
        uint8_t a[32], b[32];
        key_of(r, a);
        key_of(r, b);
        std::vector<int> seq;
        seq.push_back(t.count(a, 2));   // COUNTED
        seq.push_back(t.count(a, 2));   // ADMIT
        seq.push_back(t.count(a, 2));   // ALREADY
        seq.push_back(t.forget(a));     // 1
        seq.push_back(t.forget(b));     // 0: never seen
        seq.push_back(t.count(a, 2));   // COUNTED
        seq.push_back(t.count(a, 2));   // ADMIT
        seq.push_back(t.count(b, 1));   // ADMIT at once
        std::printf("\"forget\": [");
        for (size_t i = 0; i < seq.size(); i++) std::printf("%s%d", i ? ", " : "", seq[i]);
        std::printf("], ");
    }
    // find / bump_at (the engine's lookups while the kernels run) give what count gives
    {
        pvhost::AdmitTable a, b;
        std::mt19937_64 r(7);
        std::vector<uint8_t> keys(32ull * 64);
        for (auto& x : keys) x = (uint8_t)r();
        int same = 1, absent_first = 1;
        for (int pass = 0; pass < 4; pass++)
            for (int j = 0; j < 64; j++) {
                const uint8_t* k = &keys[32ull * ((j * 7 + pass) % 64)];
                const int32_t at = b.find(k);
                if (pass == 0 && j < 8 && at != -1) absent_first = 0;  // never inserted by find
                const auto gen = b.generation();
                const int ob = at >= 0 && b.generation() == gen ? b.bump_at(at, 3) : b.count(k, 3);
                same &= ob == a.count(k, 3);
            }
        std::printf("\"find_bump\": {\"same_as_count\": %d, \"find_inserts_nothing\": %d, \"used\": %u}, ", same,
                    absent_first, b.used());
    }
    // window turnover
    {
        using Small = pvhost::AdmitTableT<10>;
        Small t;
        std::mt19937_64 r(5);
        uint8_t first[32], k[32];
        key_of(r, first);
        t.count(first, 2);  // one appearance of `first`
        for (uint32_t i = 1; i < Small::WINDOW; i++) {
            key_of(r, k);
            t.count(k, 2);
        }
        const uint32_t full = t.used();
        const int again = t.count(first, 2);  // a new window: `first` counts from zero
        std::printf("\"window\": {\"window\": %u, \"used_full\": %u, \"first_again\": %d, \"used_after\": %u}, ",
                    Small::WINDOW, full, again, t.used());
    }
    // cost per count: 24,576 distinct random keys, one verified appearance each (a table of 2^17
    // entries is 5.2 MB: most probes miss the core's L1 and L2)
    {
        pvhost::AdmitTable t;
        std::mt19937_64 r(6);
        const int n = 24576;
        std::vector<uint8_t> keys(32ull * n);
        for (auto& x : keys) x = (uint8_t)r();
        t.count(&keys[0], 2);  // allocates the table
        int sink = 0;
        const auto t0 = clk::now();
        for (int i = 1; i < n; i++) sink += t.count(&keys[32ull * i], 2);
        std::printf("\"ns_per_count\": %.2f, \"sink\": %d", ms_since(t0) * 1e6 / (n - 1), sink & 1);
    }
    std::printf("}\n");
    return 0;
}
