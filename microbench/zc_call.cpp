// Host-buffer latency of pv_verify_batch for 1 / 100 requests from C (no Python), on the bench's NYM
// records written by tools/lat_parts.py (development tool). Prints the median of 300 calls per size.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../include/plenum_verify.h"

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    uint64_t n, blen;
    if (fread(&n, 8, 1, f) != 1 || fread(&blen, 8, 1, f) != 1) return 1;
    std::vector<uint64_t> off(n + 1);
    std::vector<uint8_t> blob(blen), pk(32 * n);
    if (fread(off.data(), 8, n + 1, f) != n + 1 || fread(blob.data(), 1, blen, f) != blen ||
        fread(pk.data(), 1, 32 * n, f) != 32 * n) return 1;
    fclose(f);
    if (pv_init(0) != PV_OK) return 2;
    for (uint64_t k : {1ull, 100ull}) {
        if (k > n) break;
        std::vector<uint8_t> bits((k + 7) / 8);
        std::vector<double> ts;
        for (int i = 0; i < 320; i++) {
            const auto t0 = std::chrono::steady_clock::now();
            const int rc = pv_verify_batch(blob.data(), off.data(), k, pk.data(), bits.data());
            const auto t1 = std::chrono::steady_clock::now();
            if (rc != PV_OK) return 3;
            if (i >= 20) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"requests\": %llu, \"median_us\": %.1f, \"first_bits\": %u}\n", (unsigned long long)k, ts[ts.size() / 2], bits[0]);
    }
    return 0;
}
