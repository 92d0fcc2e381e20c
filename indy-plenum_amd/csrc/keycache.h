// Node-side cache of per-key comb tables, persistent across calls (pv_key_cache_* in
// include/plenum_verify.h).
//
// A Plenum node verifies requests from a fairly stable set of signers whose verkeys it already holds
// (the domain ledger's NYM records, plenum/server/request_handlers/utils.py:30-39). For a cached key
// the latency path replaces the 252 doublings + 64 additions of [k](-A) by 32 table additions from
// the key's radix-256 comb T_A[i][d] = [d 256^i](-A) (comb.h, built by the engine's own key-chain and
// fill kernels when the key is put into the cache). The verdict is the same function of (R, S, A, M):
// the table holds exact multiples of -A and the libsodium key checks ran when it was built.
//
// Device layout: keys [cap][8] u32 (the 32-byte encodings), flags [cap] u32 (1 = libsodium's key
// checks passed), tab [cap][32][129][10] uint4 (cached form, 660 KB per key), and an open-addressing
// hash table htab [hmask + 1] u32 of slot indices (PV_KC_EMPTY = free) maintained by the host.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

static constexpr uint32_t PV_KC_EMPTY = 0xFFFFFFFFu;

struct PvKeyCacheView {
    const uint32_t* htab;
    const uint32_t* keys;
    const uint32_t* flags;
    const uint4* tab;
    uint32_t hmask;   // 0 when the cache is disabled (htab may then be null)
    uint32_t seed;
    const uint4* wtab = nullptr;  // radix-65536 niels rows of slots < wcap (comb.h PV_KW_*), or null
    uint32_t wcap = 0;
    uint32_t* stamp = nullptr;    // per-slot epoch of the last launch that read the slot (LRU refresh), or null
    uint32_t epoch = 0;
};

__host__ __device__ __forceinline__ uint32_t pv_kc_hash(const uint32_t A[8], uint32_t seed) {
    uint32_t h = seed;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        h = (h ^ A[q]) * 0x9E3779B1u;
        h ^= h >> 15;
    }
    return h;
}

// Slot of key A, or PV_KC_EMPTY. Every lane computes the same (wave-uniform) result. A hit stamps the
// slot with the launch's epoch (a plain vector store; every lane of a wave stores the same word).
__device__ __forceinline__ uint32_t pv_kc_lookup(const PvKeyCacheView& kc, const uint32_t A[8]) {
    if (kc.hmask == 0) return PV_KC_EMPTY;
    uint32_t h = pv_kc_hash(A, kc.seed) & kc.hmask;
    for (uint32_t probe = 0; probe <= kc.hmask; probe++) {
        const uint32_t s = kc.htab[h];
        if (s == PV_KC_EMPTY) return PV_KC_EMPTY;
        uint32_t d = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) d |= kc.keys[8 * s + q] ^ A[q];
        if (d == 0) {
            if (kc.stamp) kc.stamp[s] = kc.epoch;
            return s;
        }
        h = (h + 1) & kc.hmask;
    }
    return PV_KC_EMPTY;
}
