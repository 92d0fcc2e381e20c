// libplenum_verify: MI355X batch Ed25519 verification engine (kernels + device-side C ABI).
//
// One lane per request, 256-thread workgroups, two workgroups per CU (2 waves/SIMD: measured
// v_mad_u64_u32 throughput saturates at >= 2 waves/SIMD, profiles/r01_isa_rates.jsonl). The grid is
// a fixed number of workgroups that stride over the batch, so the per-lane HBM table of [j](-A)
// (9 cached points x 160 B) is sized by resident lanes, not by the batch.
//
// Replaces (per request) stp_core/crypto/nacl_wrappers.py:108 libnacl.crypto_sign_open(sm, pk);
// see include/plenum_verify.h for the ABI contract and verify_core.h for the arithmetic.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <list>
#include <unordered_map>
#include <mutex>
#include <chrono>
#include <atomic>
#include <random>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <thread>
#include <string>
#include <vector>

#include "btable.h"
#include "copy_pool.h"
#include "kc_admit.h"
#include "comb.h"
#include "keycache.h"
#include "lp25519.h"
#include "verify_core.h"
#include "pv_internal.h"
#include "../../include/plenum_verify.h"
#include "../../include/plenum_verify_test.h"

static constexpr int PV_BLOCK = 256;
#ifndef PV_CHAIN_MODE
// per-key chain kernel: 2 = limb-parallel, one wave per key (pv_key_chain_lp_kernel); 1 = four lanes
// per key (pv_key_chain_quad_kernel, round 1); 0 = one lane per key (pv_key_chain_kernel)
#define PV_CHAIN_MODE 2
#endif
// an integer from the environment (A/B knobs read once at first use), or dflt
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

#ifndef PV_COMB_A_MINBLOCKS
#define PV_COMB_A_MINBLOCKS 3
#endif
#ifndef PV_FILL_MINBLOCKS
#define PV_FILL_MINBLOCKS 2
#endif
// [S]B of a keyed chunk per request from the chunk's start, beside the dedup (A/B knob, off): the
// dedup's atomics slow 2-4x under it and the headline gains nothing measurable; config 3 loses
// 0.1 ms (profiles/r03/half/ab_comb_b_early)
#ifndef PV_ZERO_COPY  // small latency-path host-buffer calls read the pinned staging buffer in place
#define PV_ZERO_COPY 1
#endif
#ifndef PV_ZC_SPIN  // ... and the host spins on their verdict bytes instead of a stream sync
#define PV_ZC_SPIN 1
#endif
#ifndef PV_COMB_B_EARLY
#define PV_COMB_B_EARLY 0
#endif
#ifndef PV_ATAB_NT  // per-request Straus tables read with the streaming (evict-first) cache policy
#define PV_ATAB_NT 0
#endif
#ifndef PV_SIDE_PRIO
#define PV_SIDE_PRIO 0
#endif
#ifndef PV_MSM_MINBLOCKS
// workgroups per CU the msm kernel's register budget is sized for (3: <= 168 VGPRs, 3 waves/SIMD; the
// full-length loop fits that at 2 as well)
#define PV_MSM_MINBLOCKS 3
#endif
#ifndef PV_PREP_MINBLOCKS
#define PV_PREP_MINBLOCKS 2  // Straus prep (decompression + SHA-512 + recoding)
#endif
// Dynamic LDS requested by every pv_comb_prep_kernel workgroup, unused: it caps the kernel's residency
// so that the key chain, launched beside it on the key stream, finds a wave slot on every SIMD at
// once instead of waiting for prep workgroups to retire (env PV_PREP_LDS_PAD overrides at pv_init).
// 41,984 B: 3 workgroups per CU (126 KB of the 160 KB), 3 prep waves per SIMD leave the chain's wave a
// slot from the start -- A/B (profiles/r04/ab_pad.txt): chain 0.40 -> 0.31 ms in-step, comb kernel
// starts 0.83 -> 0.79 ms, step -2 %; 54 KB (2 per CU) slows the prep more than it helps
#ifndef PV_PREP_LDS_PAD
#define PV_PREP_LDS_PAD 41984
#endif
static constexpr uint64_t PV_CHUNK = 1ull << 20;  // requests per launch sequence (workspace ~1.8 GB)
static constexpr uint32_t PV_KEY_CAP = 16384;     // distinct keys the comb tables hold (10.8 GB)
// AUTO: chunks above the latency path's range go keyed (dedup, then comb keys / Straus side). At
// medium sizes (4k-256k requests) the Straus side's one-lane latency (~0.9 ms) is paid by the whole
// launch as soon as it has any request, so a chunk with few distinct keys makes EVERY key a comb
// key (PV_ALLCOMB_*): tools/latency_probe.py on MI355X, 1,024 signers, device time per call --
// 10k requests 0.77 ms all-comb vs 0.91 Straus, 32k 0.76 vs 0.95 (and 1.02 split at >= 48 requests
// per key); bounded so the fill never exceeds 2,048 keys' tables (~0.5 ms).
static constexpr uint64_t PV_KEYED_MIN = 4097;
static constexpr uint32_t PV_ALLCOMB_KEYS = 2048;
static constexpr uint32_t PV_ALLCOMB_CHUNK = 262144;
static constexpr uint32_t PV_XT_KEYS = 2048;      // tables shared by a pipelined call's sub-batches (1.35 GB)
static constexpr uint32_t PV_XT_HASH = 4096;      // their hash table (>= 2 x keys)
// An all-comb chunk of at most PV_SPARSE_CHUNK requests and at most PV_SPARSE_PER_KEY requests per key
// on average builds only the table entries its digits use (comb.h pv_comb_fill_sparse; the need
// masks are set by pv_comb_prep_kernel). A/B on MI355X (1,024 signers, device time,
// profiles/r02/ab_sparse_fill.txt): 6k requests 0.71 -> 0.54 ms, 10k 0.70 -> 0.56; at 32 requests
// per key the per-position thread's serial additions outlast the parallel full fill (32k 0.69 ->
// 0.72, 64k 0.74 -> 0.89), hence the per-key bound.
#ifndef PV_SPARSE_CHUNK
#define PV_SPARSE_CHUNK 65536
#endif
#ifndef PV_SPARSE_PER_KEY
#define PV_SPARSE_PER_KEY 16
#endif
// Key chain launches per keyed chunk (the table fill of part p overlaps the chain of part p + 1).
// A/B on MI355X (profiles/r02/ab_chain_parts.txt, interleaved): 1 part is best -- 10k requests
// 0.70 ms device vs 0.74 (4 parts) / 0.92 (8), 1M 3.02 ms/step vs 3.04-3.11 / 3.15: the fill of a
// part competes with the next chain part for the SIMDs and each part is a launch of its own.
#ifndef PV_CHAIN_PARTS
#define PV_CHAIN_PARTS 1
#endif
#ifndef PV_DIRECT_FILL  // large chunks: fill on the key stream right behind the chain (no fstream hop)
#define PV_DIRECT_FILL 1
#endif
static_assert(32 % PV_CHAIN_PARTS == 0, "PV_CHAIN_PARTS must divide the 32 comb positions");
#ifndef PV_LP_CHAIN_BLOCKS
#define PV_LP_CHAIN_BLOCKS 2048  // waves of the limb-parallel key chain (one key each at a time)
#endif
// Dedup contention (1,024 signers x ~1,000 requests each per 1M chunk). Kernel times on MI355X
// (rocprofv3, profiles/r02/ab_dedup_seed.txt): insert + assign 143 us with one atomic counter per
// key and an atomic first read; 95 us with the seed pre-pass; 92 with a plain first read; 85 us
// (+ 8 us seed) with the counters split 8 ways (16: 86, 32: 87 -- the assign kernel's sums grow).
#ifndef PV_KEY_SEED
#define PV_KEY_SEED 4096  // requests of a keyed chunk whose keys are inserted first (pv_key_seed_kernel)
#endif
#ifndef PV_INSERT_PLAIN_LOAD
#define PV_INSERT_PLAIN_LOAD 1  // the insert's first slot read is a plain load (0: an atomic load)
#endif
// Per-key request counters of the dedup are split PV_RANK_SUB ways (sub-table = the request's
// workgroup index mod PV_RANK_SUB), so the ~1,000 requests of a hot key queue on PV_RANK_SUB
// device-scope atomics instead of one; the assign kernel turns the sub-counts into offsets.
#ifndef PV_RANK_SUB
#define PV_RANK_SUB 8
#endif
static_assert((PV_RANK_SUB & (PV_RANK_SUB - 1)) == 0, "PV_RANK_SUB must be a power of two");
#ifndef PV_LATENCY_MAX
#define PV_LATENCY_MAX 4096  // AUTO: batches up to this size take the latency path (pv_latency.hip)
#endif
// AUTO picks latency vs keyed by key repeats from this size up to PV_LATENCY_MAX (pv_keyed_hint on
// the host, the dedup's lat_choice on the device)
#ifndef PV_KEYED_HINT_MIN
#define PV_KEYED_HINT_MIN 2049
#endif

// ---------------------------------------------------------------------------------------- device

// Row r of a [rows][S] structure-of-arrays buffer: a wave-uniform pointer (SGPRs), so each access
// is one global_load/store with a 32-bit per-lane offset instead of a live 64-bit address per row.
template <class T>
__device__ __forceinline__ T* pv_row(T* base, uint32_t r, uint32_t S) {
    return base + (size_t)r * S;
}

// [rows][S] u32 structure-of-arrays buffer through a buffer resource: every access is one
// buffer_load/store_dword with the lane's 32-bit byte offset in a VGPR and the row offset in an
// SGPR (soffset), so rows cost no per-lane address registers (global_load addressing kept 40 live
// 64-bit addresses for a 40-row point).
struct Soa {
    __amdgpu_buffer_rsrc_t r;
    uint32_t S4;  // row stride in bytes
    __device__ __forceinline__ Soa(uint32_t* base, uint64_t rows, uint64_t S)
        : r(__builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)(rows * S * 4 < 0x7fffffffull ? rows * S * 4 : 0x7fffffffull),
                                              0x00020000)),
          S4((uint32_t)(S * 4)) {}
    __device__ __forceinline__ uint32_t ld(uint32_t row, uint32_t i) const {
        return __builtin_amdgcn_raw_buffer_load_b32(r, i * 4, row * S4, 0);
    }
    __device__ __forceinline__ void st(uint32_t row, uint32_t i, uint32_t v) const {
        __builtin_amdgcn_raw_buffer_store_b32(v, r, i * 4, row * S4, 0);
    }
};

// Per-lane cached table of [j](-A) in HBM. Indices are 32-bit (chunk <= 2^20 slots, 90 quads per
// slot < 2^32) so each access is a uniform 64-bit base plus one per-lane 32-bit offset instead of ten
// live 64-bit addresses. Layout PV_ATAB_AOS = 1: [slot][entry][quad] uint4 -- the lanes of a wave pick
// different entries (their own digits), so each lane reads its own contiguous 160 B entry (two
// 128 B lines) instead of a 16 B piece of a line shared with lanes that want other entries
// ([entry][quad][slot], PV_ATAB_AOS = 0: coalesced only when every lane has the same digit).
#ifndef PV_ATAB_AOS
#define PV_ATAB_AOS 1
#endif
// Half-size Straus path (sc25519.h sc_halfsize, verify_core.h pv_straus_ar_xyz): k = k1 / k2 (mod 8L)
// with |k1|, k2 ~ 2^128, so the per-request loop runs ~33 windows of both scalars against two tables
// ([j](+-A) and [j](-R')) instead of 64 windows of k against one. 0: the full-length loop over k.
#ifndef PV_STRAUS_HALF
#define PV_STRAUS_HALF 1
#endif
static constexpr uint32_t PV_ATAB_ENT = PV_STRAUS_HALF ? 18u : 9u;  // table entries per slot
// half-size msm: table entries fetched one addition ahead into LDS (pv_straus_ar_xyz_staged)
#ifndef PV_MSM_STAGED
#define PV_MSM_STAGED 0
#endif
struct DevATab {
    uint4* base;
    uint32_t nslots;
    uint32_t slot;
    uint32_t t0 = 0;  // first entry of this table in the slot (the R table starts at 9)
    __device__ __forceinline__ uint4& at(int j, int q) const {
#if PV_ATAB_AOS
        // [slot / 64][entry][slot % 64][quad]: a lane's entry is 160 contiguous bytes, and one wave's
        // ten stores of an entry cover 10 KB contiguously (full lines reach HBM)
        return base[(((slot >> 6) * PV_ATAB_ENT + t0 + (uint32_t)j) * 64u + (slot & 63u)) * 10u + (uint32_t)q];
#else
        return base[(uint32_t)((t0 + j) * 10 + q) * nslots + slot];
#endif
    }
    __device__ __forceinline__ void store(int j, const uint32_t w[40]) const {
#pragma unroll
        for (int q = 0; q < 10; q++) at(j, q) = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    __device__ __forceinline__ void store_p3(int j, const ge_p3& p) const {
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            w[q] = p.X.v[q];
            w[10 + q] = p.Y.v[q];
            w[20 + q] = p.Z.v[q];
            w[30 + q] = p.T.v[q];
        }
        store(j, w);
    }
    __device__ __forceinline__ void load_p3(int j, ge_p3& p) const {
        uint32_t w[40];
        load(j, w);
#pragma unroll
        for (int q = 0; q < 10; q++) {
            p.X.v[q] = w[q];
            p.Y.v[q] = w[10 + q];
            p.Z.v[q] = w[20 + q];
            p.T.v[q] = w[30 + q];
        }
    }
    __device__ __forceinline__ void load_half(int j, int h, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < 5; q++) {
#if PV_ATAB_NT
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(&at(j, 5 * h + q)));
            const uint4 v = make_uint4(t.x, t.y, t.z, t.w);
#else
            const uint4 v = at(j, 5 * h + q);
#endif
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    }
    __device__ __forceinline__ void load(int j, uint32_t w[40]) const {
        load_half(j, 0, w);
        load_half(j, 1, w + 20);
    }
};

struct LdsBTab {
    const uint32_t* base;  // LDS
    __device__ __forceinline__ void load_part(int j, int part, uint32_t w[20]) const {
        const uint4* e = reinterpret_cast<const uint4*>(base + j * PV_BTAB_STRIDE + 20 * part);
#pragma unroll
        for (int i = 0; i < (part ? 3 : 5); i++) {
            const uint4 v = e[i];
            if (4 * i < (part ? 10 : 20)) w[4 * i] = v.x;
            if (4 * i + 1 < (part ? 10 : 20)) w[4 * i + 1] = v.y;
            if (4 * i + 2 < (part ? 10 : 20)) w[4 * i + 2] = v.z;
            if (4 * i + 3 < (part ? 10 : 20)) w[4 * i + 3] = v.w;
        }
    }
    __device__ __forceinline__ void load(int j, ge_niels& q) const {
        const uint4* e = reinterpret_cast<const uint4*>(base + j * PV_BTAB_STRIDE);
        uint32_t w[32];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint4 v = e[i];
            w[4 * i] = v.x;
            w[4 * i + 1] = v.y;
            w[4 * i + 2] = v.z;
            w[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 10; i++) {
            q.yplusx.v[i] = w[i];
            q.yminusx.v[i] = w[10 + i];
            q.xy2d.v[i] = w[20 + i];
        }
    }
};

// Digit words of k (radix 16, rows 0..7) and S (radix 256, rows 8..15), one coalesced load each time
// the Straus loop enters a new group of 8 windows.
// digits rows: 0..7 k (both paths), 8.. S: 8 packed words (Straus, radix 256) or PV_BC2_POS signed
// radix-2^W digits (comb path, wide fixed-base comb)
// Radix of the wide fixed-base comb chosen at pv_init: PV_BC2_W (24: 10.7 GB of HBM) or, when that
// allocation fails (or PV_FORCE_BCOMB16 is set), W = 16 over the radix-65536 comb T_B the latency
// path already holds (the same layout and digits: comb.h). Kernels that recode or read S's digits
// are instantiated for both.
template <int W>
struct Bc2 {
    static constexpr int POS = (253 + W - 1) / W;
    static constexpr uint32_t ENT = (1u << (W - 1)) + 1u;
};
static_assert(Bc2<16>::ENT == PV_BCOMB_ENT && Bc2<16>::POS == PV_BCOMB_POS, "W = 16 is the radix-65536 comb");
// half-size Straus path: rows PV_K2_ROW.. hold k2's radix-16 digits, row PV_NW_ROW the lane's window count
static constexpr int PV_K2_ROW = 8 + (Bc2<16>::POS > PV_BC2_POS ? Bc2<16>::POS : PV_BC2_POS);
static constexpr int PV_NW_ROW = PV_K2_ROW + 8;
static constexpr int PV_DIGIT_ROWS = PV_STRAUS_HALF ? PV_NW_ROW + 1 : PV_K2_ROW;
struct DevDigits {
    Soa d;
    uint32_t slot;
    __device__ __forceinline__ DevDigits(uint32_t* base, uint32_t stride, uint32_t slot_)
        : d(base, PV_DIGIT_ROWS, stride), slot(slot_) {}
    __device__ __forceinline__ uint32_t ek(int q) const { return d.ld(q, slot); }
    __device__ __forceinline__ uint32_t ek2(int q) const { return d.ld(PV_K2_ROW + q, slot); }
    __device__ __forceinline__ uint32_t nw() const { return d.ld(PV_NW_ROW, slot); }
    __device__ __forceinline__ uint32_t fs(int q) const { return d.ld(8 + q, slot); }
    __device__ __forceinline__ int fb(int j) const { return (int)d.ld(8 + j, slot); }
};

// Request bytes at an arbitrary byte offset: aligned dword loads + v_alignbyte_b32 funnel shifts.
struct DevMsg {
    const uint32_t* ap;  // rec rounded down to 4 bytes
    uint32_t sh;         // rec & 3
    __device__ __forceinline__ uint32_t dw(uint64_t i) const {
        return __builtin_amdgcn_alignbyte(ap[i + 1], ap[i], sh);
    }
    // little-endian bytes [8q, 8q + 8) of the record
    __device__ __forceinline__ uint64_t operator()(uint64_t q) const {
        return ((uint64_t)dw(2 * q + 1) << 32) | dw(2 * q);
    }
};

// Per-request intermediate state between the two kernels (SoA, coalesced per wave):
//   atab  [9 entries][10 quads][n] uint4   cached [j](-A), j = 0..8
//   digits[PV_DIGIT_ROWS][n] uint32          radix-16 digits of k (8 words), radix-256 of S (8 words);
//                                           comb path: radix-256 k, radix-2^W S (PV_BC2_POS words)
//   flags [n] uint32                        1 = every libsodium pre-check passed
//   q     [40][n] uint32                    projective Q = (X, Y, Z) from the msm kernel (rows 0..29);
//                                           the comb path's [S]B half parks an extended point here
struct Work {
    uint4* atab;
    uint32_t* digits;
    uint32_t* flags;
    uint32_t* q;
    uint4* qb;        // [S]B per REQUEST of a keyed chunk, 160 B each (pv_comb_b_req_kernel)
    uint64_t stride;  // chunk capacity (requests)
    uint4* aos;       // per REQUEST comb-prep results, PrepAos<W>::Q uint4 each (pv_comb_prep_req_kernel)
};

// How a chunk's requests are split between the two arithmetic paths, decided ON THE DEVICE by the
// dedup/sort kernels (no host round trip). split == nullptr: the Straus path was forced (or the
// chunk is too small for dedup to pay) -- no key kernels ran and slot == request. Otherwise the
// requests are in key-sorted slot order, the first split[PV_SPLIT_SLOTS] slots belong to keys
// that take the comb path and the remaining slots take the Straus path (request = slot_req[slot]).
static constexpr int PV_SPLIT_KEYS = 0;        // distinct keys in the chunk
static constexpr int PV_SPLIT_COMB_KEYS = 1;   // keys given a comb table
static constexpr int PV_SPLIT_SLOTS = 2;       // requests (slots) of those keys
static constexpr int PV_SPLIT_SPARSE = 3;      // 1: the comb tables are filled sparsely (small chunk)
static constexpr int PV_SPLIT_LAT = 4;         // 1: the dedup chose the latency path for this chunk
static constexpr uint32_t PV_SPLIT_WORDS = 8;  // counters cleared per keyed chunk
static constexpr uint32_t PV_NSEG = 8;         // key-id segments (pv_key_assign_kernel)
// segment g's id counter: word PV_SEG_BASE + g * PV_SEG_STRIDE of the split buffer, one counter per
// 1 KB so that the segments' atomics land on different memory channels (same-line counters
// serialise like one)
#ifndef PV_SEG_STRIDE
#define PV_SEG_STRIDE 256
#endif
static constexpr uint32_t PV_SEG_BASE = 256;
static constexpr uint32_t PV_SPLIT_ALLOC_WORDS = PV_SEG_BASE + PV_NSEG * PV_SEG_STRIDE;
struct Gate {
    const uint32_t* split;
    const uint32_t* slot_req;
    __device__ __forceinline__ bool keyed() const { return split != nullptr; }
    // the dedup handed this chunk to the latency path (pv_key_scan_kernel, lat_choice): every
    // kernel of the throughput paths exits at once, the unpermute kernel only cleans up
    __device__ __forceinline__ bool off() const { return split != nullptr && split[PV_SPLIT_LAT] != 0u; }
    // Straus-path kernels loop over 256-slot tiles t = blockIdx.x, blockIdx.x + gridDim.x, ...;
    // split, the tiles are taken from the END of the slot range (where the Straus slots are) and a
    // small grid strides over them, so the first tile with no Straus slot ends the loop and no
    // flood of empty workgroups competes with the comb kernels for CUs.
    __device__ __forceinline__ uint32_t stile(uint32_t t, uint32_t ntiles) const { return split ? ntiles - 1 - t : t; }
    __device__ __forceinline__ uint32_t ncomb() const { return split ? split[PV_SPLIT_SLOTS] : 0u; }
    // request of a Straus-path slot
    __device__ __forceinline__ uint32_t req(uint32_t i) const { return split ? slot_req[i] : i; }
};

// Keyed workspace (comb.h). The hash table maps a 32-byte key to the index of the first request
// that carried it; slot_id gives the dense key id of an owned slot (ids < chunk size).
//   slot     [H] u32   owner request index, PV_EMPTY = free
//   slot_id  [H] u32   dense key id of an owned slot
//   slot_cnt [PV_RANK_SUB][H]  requests carrying the key per sub-table (request workgroup mod
//            PV_RANK_SUB); the assign kernel replaces each nonzero count by its offset in the key
//   req_key  [stride]  the request's hash slot;         req_rank [stride] its rank in its sub-table
//   nkeys    [3]       PV_SPLIT_* counters (see Gate)
//   key_owner[stride]  a request carrying key id
//   key_cid  [stride]  comb index of key id (PV_EMPTY: its requests take the Straus path)
//   comb_key [kcap]    key id of comb index j;  key_flag [kcap]  libsodium key checks passed
//   bases    [kcap][32][4][10] uint4 [256^i](-A) and its [16], [32], [64] multiples, extended
//   ctab     [kcap][32][129][10] uint4  T_A, cached form
//   key_cslot [stride] / comb_cslot [kcap]  node-side key cache slot of a key id / comb index: a key
//            in the cache is a comb key whatever its request count, its T_A is the cache's table
//            and the key stream (chain, fill) skips it
// A key takes the comb path when it carries >= min_req requests of the chunk (the per-key table
// costs about as much as ~50 requests save; 1 when the comb path is forced) and fewer than kcap
// keys came before it; the rest -- singletons such as the adversarial keys of config 3 -- take the
// Straus path in the same launch.
// Key-sorted processing order ("slots"): after dedup the requests of each key occupy a contiguous
// range of slots, comb keys first, so consecutive lanes and waves read the same key's table rows
// (L2-resident) instead of 1,024 keys' tables at random:
//   key_count[stride], key_cursor[stride]  requests per key id, then the key's first slot
//   slot_req [stride]                   slot -> request index;  req_pos [stride] request -> slot
//   skey     [stride]                   slot -> comb index;     sverdict [stride / 64] slot verdicts
struct KeyWork {
    uint32_t* slot;
    uint32_t* slot_id;
    uint32_t* slot_cnt;
    uint32_t* req_key;
    uint32_t* req_rank;
    uint32_t* nkeys;
    uint32_t* key_owner;
    uint32_t* key_cid;
    uint32_t* comb_key;
    uint32_t* key_flag;
    uint4* bases;
    uint4* ctab;
    uint32_t* key_count;
    uint32_t* key_cursor;
    uint32_t* slot_req;
    uint32_t* req_pos;
    uint32_t* skey;
    uint64_t* sverdict;
    uint32_t* key_cslot;   // [stride] node-side key cache slot of key id (PV_EMPTY: not cached)
    uint32_t* comb_cslot;  // [kcap] the same per comb index: its table is read from the cache
    uint32_t* need;        // [PV_ALLCOMB_KEYS][32][5] needed |digit| bits per (comb index, position)
    const uint4* kc_tab;   // the cache's tables [cap][32][129][10] (keycache.h)
    const uint4* kc_ntab;  // the same divided by Z [cap][32][129][10] (comb.h pv_comb_row_to_affine), or null
    const uint4* kc_wtab;  // radix-65536 rows of slots < kc_wcap [kc_wcap][16][32897][8] (comb.h PV_KW_*), or null
    uint32_t kc_wcap;
    // a later sub-batch of a pipelined host call with a non-empty node cache: the keys the node cache
    // misses are looked up in the call's shared store too; a hit there is slot | PV_CSLOT_XT
    const uint32_t* xt_flags;
    const uint4* xt_tab;
    uint32_t hmask;
    uint32_t kcap;
    uint32_t seed;
    uint32_t min_req;
    uint32_t kc_on;    // this launch consults the key cache (pv_key_cache_probe_kernel ran)
    uint32_t chunk_n;  // requests in this chunk
    uint32_t lat_choice;  // the scan picks latency vs keyed for this chunk (AUTO, device-buffer call)
    uint32_t seg_cap;     // key ids of segment s are s * seg_cap + [0, its counter)
    uint32_t dense_only;  // never fill sparsely (the tables outlive the chunk: pv_xtab_publish_kernel)
};
static constexpr uint32_t PV_EMPTY = 0xFFFFFFFFu;
static constexpr uint32_t PV_CSLOT_XT = 0x40000000u;  // cache slot in the call's shared store (KeyWork::xt_*)
#ifndef PV_COMB_MIN_REQ
#define PV_COMB_MIN_REQ 48
#endif

// LDS-DMA staging of one table entry per lane (comb.h, PV_COMB_PIPELINE). An entry of Q uint4 is
// fetched by Q global_load_lds_dwordx4, each writing 1 KiB = 16 B x 64 lanes of the wave's staging
// area, laid out [q][lane] so that reading it back is one conflict-free ds_read_b128 per q.
__device__ __forceinline__ void pv_glds16(const uint4* g, uint4* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
// Q pieces of 16 B from g[0..Q) to l[q * 64 + lane] (a wave's [q][lane] staging area). The
// instruction's immediate offset (16 q) applies to BOTH the global and the LDS address, so the LDS
// base of piece q is moved back by the same 16 q bytes (M0 is set per instruction anyway): all Q
// loads then share ONE 64-bit global address instead of Q 64-bit adds per staged entry.
template <int Q, int q = 0>
__device__ __forceinline__ void pv_glds16_row(const uint4* g, uint4* l) {
    if constexpr (q < Q) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(l + q * 64 - q), 16, 16 * q, 0);
        pv_glds16_row<Q, q + 1>(g, l);
    }
}
// A 10-piece entry whose pieces 5 and 6 (words 20..27) are skipped on lanes with `skip` (affine comb rows:
// their Z2 words are not read). Lanes that skip leave those pieces of their staging column stale.
__device__ __forceinline__ void pv_glds16_row10_skip56(const uint4* g, uint4* l, bool skip) {
    pv_glds16_row<5>(g, l);
    if (!skip) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(l + 5 * 64 - 5), 16, 16 * 5, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(l + 6 * 64 - 6), 16, 16 * 6, 0);
    }
    pv_glds16_row<10, 7>(g, l);
}
// the LDS reads of the previous staged entry must be complete before its buffer is refilled
__device__ __forceinline__ void pv_lds_reads_done() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Wide fixed-base comb rows (comb.h PV_BC2_*): row j = entries 0..PV_BC2_ENT-1 of [d 2^(W j)] B,
// 8 uint4 each, LDS-staged like DevBStage; 64-bit entry index (the table is ~10.7 GB at W = 24).
template <uint32_t ENT>
struct DevB2Stage {
    const uint4* base;
    uint4* lds;
    uint32_t lane;
    __device__ __forceinline__ void stage(int j, int d) const {
        const uint4* e = base + ((uint64_t)j * ENT + (uint32_t)d) * (PV_BCOMB_STRIDE / 4);
        pv_lds_reads_done();
        pv_glds16_row<PV_BCOMB_STRIDE / 4>(e, lds);
    }
    __device__ __forceinline__ void staged(int part, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < (part ? 3 : 5); q++) {
            const uint4 v = lds[(5 * part + q) * 64 + lane];
            const int lim = part ? 10 : 20;
            if (4 * q < lim) w[4 * q] = v.x;
            if (4 * q + 1 < lim) w[4 * q + 1] = v.y;
            if (4 * q + 2 < lim) w[4 * q + 2] = v.z;
            if (4 * q + 3 < lim) w[4 * q + 3] = v.w;
        }
    }
};

#if PV_STRAUS_HALF
// The half-size msm's per-lane tables (DevATab layout, tile-major): entry j of table t of slot i staged
// into the wave's [10][64] area (pv_straus_ar_xyz_staged)
struct DevATabStage {
    uint4* base;
    uint32_t slot;
    uint4* lds;
    uint32_t lane;
    __device__ __forceinline__ void stage(int t, int j) const {
        const uint4* e = &DevATab{base, 0u, slot, t ? 9u : 0u}.at(j, 0);
        pv_lds_reads_done();
        pv_glds16_row<10>(e, lds);
    }
    __device__ __forceinline__ void staged(int h, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint4 v = lds[(5 * h + q) * 64 + lane];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    }
};
#endif
// Straus path: [S]B from the wide fixed-base comb (pv_straus_b_kernel) and a Straus loop over k only
// (pv_straus_a_xyz), instead of 32 B additions interleaved in the loop (LDS table of [j]B).
#ifndef PV_STRAUS_WIDE_B
#define PV_STRAUS_WIDE_B 1
#endif
static_assert(!PV_STRAUS_HALF || PV_STRAUS_WIDE_B, "the half-size path takes [k2 S]B from pv_straus_b_kernel");

__device__ __forceinline__ void pv_load_pk(uint32_t A[8], const uint8_t* pk, uint32_t i) {
    const uint4* p4 = reinterpret_cast<const uint4*>(pk + 32 * (uint64_t)i);
    const uint4 a0 = p4[0], a1 = p4[1];
    A[0] = a0.x; A[1] = a0.y; A[2] = a0.z; A[3] = a0.w;
    A[4] = a1.x; A[5] = a1.y; A[6] = a1.z; A[7] = a1.w;
}

// Straus path, per slot i (request r): checks, decompression of A, k = SHA-512(R||A||M) mod L,
// recoding; -A for the table kernel.
template <int W>
__device__ __forceinline__ void pv_prep_slot(const uint8_t* __restrict__ sm, const uint64_t* __restrict__ off,
                                             const uint8_t* __restrict__ pk, const Work& wk, uint32_t i, uint32_t r) {
    const uint64_t o0 = off[r], o1 = off[r + 1];
    const uint64_t smlen = o1 - o0;
    const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
    const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
    pv_sig_words in;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    const uint4* pk4 = reinterpret_cast<const uint4*>(pk + 32 * (uint64_t)r);
    const uint4 a0 = pk4[0], a1 = pk4[1];
    in.A[0] = a0.x; in.A[1] = a0.y; in.A[2] = a0.z; in.A[3] = a0.w;
    in.A[4] = a1.x; in.A[5] = a1.y; in.A[6] = a1.z; in.A[7] = a1.w;
#if PV_STRAUS_HALF
    {
        // pv_prepare_half over three kernels: here the signature checks, k (to rows 0..7 for
        // pv_split_kernel), A's checks and -A (table entry 1); the split of k and the digits in
        // pv_split_kernel; the sign of k1 on -A, R's checks, -R' and both tables in pv_table_kernel
        bool ok = pv_sig_ok(in, smlen);
        const Soa ds(wk.digits, PV_DIGIT_ROWS, wk.stride);
        {
            uint32_t k[8];
            pv_hash_k(k, in, smlen, mw);
#pragma unroll
            for (int q = 0; q < 8; q++) ds.st(q, (uint32_t)i, k[q]);
        }
        {
            ge_p3 negA;
            ok &= pv_key_ok_negate(negA, in.A);
            const DevATab at{wk.atab, (uint32_t)wk.stride, (uint32_t)i};
            at.store_p3(1, negA);
        }
        wk.flags[i] = ok ? 1u : 0u;
        return;
    }
#endif

    ge_p3 negA;
    uint32_t k[8];
    const bool ok = pv_prepare(negA, k, in, smlen, mw);
    // -A goes to table slot 1 as an extended point; pv_table_kernel expands it to [j](-A)
    uint32_t w[40];
#pragma unroll
    for (int q = 0; q < 10; q++) {
        w[q] = negA.X.v[q];
        w[10 + q] = negA.Y.v[q];
        w[20 + q] = negA.Z.v[q];
        w[30 + q] = negA.T.v[q];
    }
    const DevATab at{wk.atab, (uint32_t)wk.stride, (uint32_t)i};
    at.store(1, w);
    uint32_t ek[8];
    sc_recode16(ek, k);
    const Soa ds(wk.digits, PV_DIGIT_ROWS, wk.stride);
#pragma unroll
    for (int q = 0; q < 8; q++) ds.st(q, (uint32_t)i, ek[q]);
#if PV_STRAUS_WIDE_B
    int32_t fb[Bc2<W>::POS];  // [S]B from the wide fixed-base comb (pv_straus_b_kernel)
    sc_recode_w<W, Bc2<W>::POS>(fb, in.S);
#pragma unroll
    for (int j = 0; j < Bc2<W>::POS; j++) ds.st(8 + j, (uint32_t)i, (uint32_t)fb[j]);
#else
    uint32_t fs[8];
    sc_recode256(fs, in.S);
#pragma unroll
    for (int q = 0; q < 8; q++) ds.st(8 + q, (uint32_t)i, fs[q]);
#endif
    wk.flags[i] = ok ? 1u : 0u;
}

// Optional wave priority (s_setprio) for the Straus-path kernels, which in a split chunk run on
// their own stream beside the comb kernels. A/B on config 3 (tools/ab_config3.sh,
// profiles/r02/ab_straus_prio.txt): priority 3 shortens the wait for the Straus side (msm stage
// 1.55 -> 1.45 ms) but slows the key stream's table fill more (0.92 -> 1.07 ms): off by default.
#ifndef PV_STRAUS_PRIO
#define PV_STRAUS_PRIO 0
#endif
__device__ __forceinline__ void pv_straus_prio() {
#if PV_STRAUS_PRIO > 0
    __builtin_amdgcn_s_setprio(PV_STRAUS_PRIO);
#endif
}

// Kernel 1 (Straus path): pv_prep_slot over the Straus slots.
template <int W>
__global__ __launch_bounds__(PV_BLOCK, PV_PREP_MINBLOCKS) void pv_prep_kernel(const uint8_t* __restrict__ sm,
                                                               const uint64_t* __restrict__ off, uint64_t n,
                                                               const uint8_t* __restrict__ pk, Work wk, Gate gate) {
    if (gate.off()) return;
    pv_straus_prio();
    const uint32_t nc = gate.ncomb(), ntiles = (uint32_t)((n + PV_BLOCK - 1) / PV_BLOCK);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sb = gate.stile(t, ntiles);
        if ((sb + 1) * PV_BLOCK <= nc) break;  // this and every later tile: comb-path slots
        const uint32_t i = sb * PV_BLOCK + threadIdx.x;  // slot
        if (i < n && i >= nc) pv_prep_slot<W>(sm, off, pk, wk, i, gate.req(i));
    }
}

#if PV_STRAUS_HALF
// Kernel 1a (half-size path): the split k = k1 / k2 (mod 8L) of each Straus slot's k (rows 0..7, from
// pv_prep_kernel), s2 = k2 S mod L; writes the digits of |k1| (rows 0..7), k2 (PV_K2_ROW..), the window
// count and k1's sign (row PV_NW_ROW: nw | neg << 8) and the wide-comb digits of s2 (rows 8..). Its own
// kernel: few registers, so the latency of the Euclid steps is hidden by occupancy.
template <int W>
__global__ __launch_bounds__(PV_BLOCK) void pv_split_kernel(const uint8_t* __restrict__ sm,
                                                            const uint64_t* __restrict__ off, uint64_t n, Work wk,
                                                            Gate gate) {
    if (gate.off()) return;
    pv_straus_prio();
    const uint32_t nc = gate.ncomb(), ntiles = (uint32_t)((n + PV_BLOCK - 1) / PV_BLOCK);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sb = gate.stile(t, ntiles);
        if ((sb + 1) * PV_BLOCK <= nc) break;
        const uint32_t i = sb * PV_BLOCK + threadIdx.x;  // slot
        if (i >= n || i < nc) continue;
        const Soa ds(wk.digits, PV_DIGIT_ROWS, wk.stride);
        uint32_t k[8], S[8];
#pragma unroll
        for (int q = 0; q < 8; q++) k[q] = ds.ld(q, i);
        {
            const uint64_t raddr = reinterpret_cast<uint64_t>(sm + off[gate.req(i)]);
            const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
#pragma unroll
            for (int q = 0; q < 8; q++) S[q] = mw.dw(8 + q);
        }
        pv_halfk hk;
        sc_halfsize(hk, k);
        uint32_t s2[8];
        sc_mul<5>(s2, hk.k2, S);
        int32_t fb[Bc2<W>::POS];
        sc_recode_w<W, Bc2<W>::POS>(fb, s2);
#pragma unroll
        for (int j = 0; j < Bc2<W>::POS; j++) ds.st(8 + j, i, (uint32_t)fb[j]);
        uint32_t e1[8], e2[8];
        sc_recode16(e1, hk.k1);
        sc_recode16(e2, hk.k2);
        const int nw1 = sc_nwin16(e1), nw2 = sc_nwin16(e2);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            ds.st(q, i, e1[q]);
            ds.st(PV_K2_ROW + q, i, e2[q]);
        }
        ds.st(PV_NW_ROW, i, (uint32_t)(nw1 > nw2 ? nw1 : nw2) | (hk.neg ? 0x100u : 0u));
    }
}
#endif

// Kernel 1b: the cached table [j](-A), j = 0..8 (full-length path: -A from entry 1); half-size path:
// decompression and checks of A and R, tables [j](+-A) (entries 0..8) and [j](-R') (entries 9..17).
#ifndef PV_TABLE_MINBLOCKS
#define PV_TABLE_MINBLOCKS 2  // waves per SIMD (256 VGPRs; 3 spills 264 B)
#endif
__global__ __launch_bounds__(PV_BLOCK, PV_TABLE_MINBLOCKS) void pv_table_kernel(const uint8_t* __restrict__ sm,
                                                                const uint64_t* __restrict__ off, uint64_t n,
                                                                const uint8_t* __restrict__ pk, Work wk, Gate gate) {
    if (gate.off()) return;
    pv_straus_prio();
    const uint32_t nc = gate.ncomb(), ntiles = (uint32_t)((n + PV_BLOCK - 1) / PV_BLOCK);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sb = gate.stile(t, ntiles);
        if ((sb + 1) * PV_BLOCK <= nc) break;
        const uint32_t i = sb * PV_BLOCK + threadIdx.x;  // slot
        if (i >= n || i < nc) continue;
#if PV_STRAUS_HALF
        // [j](+-A) from -A (entry 1, pv_prep_kernel) and k1's sign (pv_split_kernel), then R's
        // canonical-decoding rule and [j](-R')
        const uint32_t r = gate.req(i);
        const uint64_t raddr = reinterpret_cast<uint64_t>(sm + off[r]);
        const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
        {
            DevATab at{wk.atab, (uint32_t)wk.stride, i};
            ge_p3 PA;
            at.load_p3(1, PA);
            ge_p3_cneg(PA, (Soa(wk.digits, PV_DIGIT_ROWS, wk.stride).ld(PV_NW_ROW, i) & 0x100u) != 0);  // +-A
            pv_build_a_table(at, PA);
        }
        bool ok;
        {
            uint32_t R[8];
#pragma unroll
            for (int q = 0; q < 8; q++) R[q] = mw.dw(q);
            ge_p3 negR;
            ok = pv_r_decode_negate(negR, R);
            DevATab rt{wk.atab, (uint32_t)wk.stride, i, 9u};
            pv_build_a_table(rt, negR);
        }
        if (!ok) wk.flags[i] = 0u;
#else
        const DevATab at{wk.atab, (uint32_t)wk.stride, i};
        uint32_t w[40];
        at.load(1, w);
        ge_p3 negA;
#pragma unroll
        for (int q = 0; q < 10; q++) {
            negA.X.v[q] = w[q];
            negA.Y.v[q] = w[10 + q];
            negA.Z.v[q] = w[20 + q];
            negA.T.v[q] = w[30 + q];
        }
        pv_build_a_table(at, negA);
#endif
    }
}

// Kernel 2: Q = [S]B + [k](-A) by the regular-window Straus loop, encode, compare with R, ballot.
// PV_MSM_FUSED_B: [k2 S]B is added inside the loop's epilogue (the wide comb's niels additions straight
// into the loop's point, entries LDS-staged one addition ahead) instead of pv_straus_b_kernel writing it
// to q for the epilogue to read
#ifndef PV_MSM_FUSED_B
#define PV_MSM_FUSED_B 1
#endif
// PV_MSM_SORT: the msm kernel regroups each 256-slot tile's lanes by window count (below)
#ifndef PV_MSM_SORT
#define PV_MSM_SORT 1
#endif
static constexpr int PV_MSM_SORT_CLS = 8;
template <int W>
__global__ __launch_bounds__(PV_BLOCK, PV_MSM_MINBLOCKS) void pv_msm_kernel(const uint8_t* __restrict__ sm,
                                                              const uint64_t* __restrict__ off, uint64_t n,
                                                              const uint32_t* __restrict__ btab_g, Work wk,
                                                              const uint4* __restrict__ bcomb, Gate gate) {
    if (gate.off()) return;
    const uint32_t nc = gate.ncomb(), ntiles = (uint32_t)((n + PV_BLOCK - 1) / PV_BLOCK);
    // nothing for this block (or no Straus slot at all): leave before the LDS fill
    if (blockIdx.x >= ntiles || nc >= n || (gate.stile(blockIdx.x, ntiles) + 1) * PV_BLOCK <= nc) return;
    pv_straus_prio();
#if PV_STRAUS_HALF && PV_MSM_STAGED
    __shared__ uint4 stg[PV_BLOCK / 64][10][64];
    uint4* stg_wave = &stg[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0][0];
#endif
#if PV_STRAUS_HALF && PV_MSM_SORT
    __shared__ uint32_t s_wcnt[PV_BLOCK / 64][PV_MSM_SORT_CLS];
    __shared__ uint16_t s_perm[PV_BLOCK];
#endif
#if PV_STRAUS_HALF && PV_MSM_FUSED_B && !PV_MSM_STAGED
    __shared__ uint4 stgb[PV_BLOCK / 64][PV_BCOMB_STRIDE / 4][64];
    uint4* stgb_wave = &stgb[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0][0];
#else
    (void)bcomb;
#endif
#if !PV_STRAUS_WIDE_B
    __shared__ __attribute__((aligned(16))) uint32_t sbt[PV_BTAB_ENTRIES * PV_BTAB_STRIDE];
    for (int t = threadIdx.x; t < PV_BTAB_ENTRIES * PV_BTAB_STRIDE / 4; t += PV_BLOCK)
        reinterpret_cast<uint4*>(sbt)[t] = reinterpret_cast<const uint4*>(btab_g)[t];
    __syncthreads();
    const LdsBTab bt{sbt};
#endif
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sb = gate.stile(t, ntiles);
        if ((sb + 1) * PV_BLOCK <= nc) break;
        const uint32_t i0 = sb * PV_BLOCK + threadIdx.x;  // slot
#if PV_STRAUS_HALF && PV_MSM_SORT
        // the tile's lanes regrouped by their window count (a stable counting sort: lanes with no Straus
        // slot first, then counts <= 30, 31, ..., >= 36), so a wave runs the largest count of lanes that
        // need about as many: 33.1 windows per wave on average at random scalars instead of 33.9
        // (lane mean 32.7). Block-uniform: every thread of the block takes the same tiles.
        uint32_t src = threadIdx.x;
        {
            int cls = 0;
            if (i0 < n && i0 >= nc) {
                const int w = (int)(DevDigits{wk.digits, (uint32_t)wk.stride, i0}.nw() & 0xFFu);
                cls = 1 + min(max(w - 30, 0), PV_MSM_SORT_CLS - 2);
            }
            const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
            const uint64_t below = (1ull << ln) - 1ull;
            uint32_t rank = 0;
            for (int c = 0; c < PV_MSM_SORT_CLS; c++) {
                const uint64_t m = __ballot(cls == c);
                if (c == cls) rank = (uint32_t)__popcll(m & below);
                if (ln == 0) s_wcnt[wv][c] = (uint32_t)__popcll(m);
            }
            __syncthreads();
            uint32_t base = 0;
            for (int c = 0; c < PV_MSM_SORT_CLS; c++)
                for (int w2 = 0; w2 < PV_BLOCK / 64; w2++)
                    if (c < cls || (c == cls && w2 < (int)wv)) base += s_wcnt[w2][c];
            s_perm[base + rank] = (uint16_t)threadIdx.x;
            __syncthreads();
            src = s_perm[threadIdx.x];
            __syncthreads();  // the next tile rewrites s_wcnt and s_perm
        }
        const uint32_t is = sb * PV_BLOCK + src;
#else
        const uint32_t is = i0;
#endif
        const bool active = is < n && is >= nc;
        const uint32_t i = active ? is : (uint32_t)n - 1;  // n - 1 >= nc here: a Straus slot
#if !(PV_STRAUS_HALF && PV_MSM_STAGED)
        const DevATab at{wk.atab, (uint32_t)wk.stride, i};
#endif
        const DevDigits dig{wk.digits, (uint32_t)wk.stride, i};
        const Soa qs(wk.q, 40, wk.stride);
        fe X, Y, Z;
#if PV_STRAUS_HALF
        // the wave's window count: its lanes' maximum (a lane's digits above its own count are 0)
        int nw = (int)(dig.nw() & 0xFFu);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) nw = max(nw, __shfl_xor(nw, m));
        nw = __builtin_amdgcn_readfirstlane(nw);
#if PV_MSM_STAGED
        pv_straus_ar_xyz_staged(X, Y, Z, DevATabStage{wk.atab, i, stg_wave, threadIdx.x & 63u}, dig, nw,
                                [&](ge_p3& accB) {  // [k2 S]B (pv_straus_b_kernel)
#pragma unroll
                                    for (int q = 0; q < 10; q++) {
                                        accB.X.v[q] = qs.ld(q, i);
                                        accB.Y.v[q] = qs.ld(10 + q, i);
                                        accB.Z.v[q] = qs.ld(20 + q, i);
                                        accB.T.v[q] = qs.ld(30 + q, i);
                                    }
                                });
#else
        const DevATab rt{wk.atab, (uint32_t)wk.stride, i, 9u};
#if PV_MSM_FUSED_B
        pv_straus_ar_xyz_addb(X, Y, Z, at, rt, dig, nw, [&](ge_p3& acc) {  // + [k2 S]B from the wide comb
            pv_comb_b_add_w<Bc2<W>::POS>(acc, DevB2Stage<Bc2<W>::ENT>{bcomb, stgb_wave, threadIdx.x & 63u},
                                         [&](int j) { return dig.fb(j); });
        });
#else
        pv_straus_ar_xyz(X, Y, Z, at, rt, dig, nw, [&](ge_p3& accB) {  // [k2 S]B (pv_straus_b_kernel)
#pragma unroll
            for (int q = 0; q < 10; q++) {
                accB.X.v[q] = qs.ld(q, i);
                accB.Y.v[q] = qs.ld(10 + q, i);
                accB.Z.v[q] = qs.ld(20 + q, i);
                accB.T.v[q] = qs.ld(30 + q, i);
            }
        });
#endif
#endif
#elif PV_STRAUS_WIDE_B
        pv_straus_a_xyz(X, Y, Z, at, dig, [&](ge_p3& accB) {  // [S]B, written by pv_straus_b_kernel
#pragma unroll
            for (int q = 0; q < 10; q++) {
                accB.X.v[q] = qs.ld(q, i);
                accB.Y.v[q] = qs.ld(10 + q, i);
                accB.Z.v[q] = qs.ld(20 + q, i);
                accB.T.v[q] = qs.ld(30 + q, i);
            }
        });
#else
        pv_straus_xyz(X, Y, Z, at, bt, dig);
#endif
        if (active) {
#pragma unroll
            for (int q = 0; q < 10; q++) {
                qs.st(q, i, X.v[q]);
                qs.st(10 + q, i, Y.v[q]);
                qs.st(20 + q, i, Z.v[q]);
            }
        }
    }
}

// ------------------------------------------------------------------ keyed comb path (comb.h)


__device__ __forceinline__ uint32_t pv_key_hash(const uint32_t A[8], uint32_t seed) {
    uint32_t h = seed;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        h = (h ^ A[q]) * 0x9E3779B1u;
        h ^= h >> 15;
    }
    return h;
}

// Sub-table of request i's per-key counter: its workgroup of the insert / scatter / unpermute grids
// (all PV_BLOCK requests per workgroup, request i in workgroup i / PV_BLOCK).
// PV_INSERT_LDS: the insert kernel's workgroup takes PV_INS_REQS consecutive requests, counts their
// keys in an LDS table and makes ONE device atomic per (key, workgroup) for the whole group's ranks
// (the per-request atomics on the keys' counters were ~56 of the kernel's ~74 us at 1M requests);
// the sub-table is then the request's insert-workgroup index mod PV_RANK_SUB.
#ifndef PV_INSERT_LDS
#define PV_INSERT_LDS 1
#endif
static constexpr uint32_t PV_INS_THREADS = 1024, PV_INS_PER_THREAD = 4;
static constexpr uint32_t PV_INS_REQS = PV_INS_THREADS * PV_INS_PER_THREAD;
static constexpr uint32_t PV_INS_LT = 4096;  // LDS table entries (more distinct keys: direct atomics)
__device__ __forceinline__ uint32_t pv_rank_sub(uint32_t i) {
#if PV_INSERT_LDS
    return (i / PV_INS_REQS) & (PV_RANK_SUB - 1u);
#else
    return (i / PV_BLOCK) & (PV_RANK_SUB - 1u);
#endif
}

// Dedup 1/2: open-addressing insert of every request's key; req_key[i] = the key's slot.
__global__ __launch_bounds__(PV_BLOCK) void pv_key_insert_kernel(const uint8_t* __restrict__ pk, uint64_t n,
                                                                  KeyWork kw) {
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;
    // the chunk's split counters start at 0 (the assign kernel, next on the stream, counts keys into
    // them); done here instead of a separate hipMemsetAsync (~11 us of dispatch + gap per chunk)
    if (i < PV_SPLIT_WORDS) kw.nkeys[i] = 0u;
    if (i < PV_NSEG) kw.nkeys[PV_SEG_BASE + i * PV_SEG_STRIDE] = 0u;
    if (i >= n) return;
    uint32_t A[8];
    pv_load_pk(A, pk, i);
    uint32_t h = pv_key_hash(A, kw.seed) & kw.hmask;
    for (uint32_t probe = 0; probe <= kw.hmask; probe++) {  // the table is >= 2x the chunk: never full
        // a plain read first: once a key is in, its other requests find it without an atomic (the
        // atomics of one key's requests all queue on one slot)
#if PV_INSERT_PLAIN_LOAD
        // a plain (L2-cached) read: a stale PV_EMPTY only sends the request to the CAS, which returns
        // the slot's current value; a slot never changes once set within the kernel
        uint32_t cur = kw.slot[h];
#else
        uint32_t cur = __hip_atomic_load(&kw.slot[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (cur == PV_EMPTY) cur = atomicCAS(&kw.slot[h], PV_EMPTY, i);
        if (cur == PV_EMPTY) break;
        uint32_t B[8];
        pv_load_pk(B, pk, cur);
        if (pv_words_equal(A, B)) break;
        h = (h + 1) & kw.hmask;
    }
    kw.req_key[i] = h;
    // the request's rank among its key's requests, and (final after this kernel) the key's count;
    // the 1,024-odd counters of a batch sit on distinct hash slots, i.e. mostly distinct L2 lines
#ifdef PV_AB_NO_RANK_ATOMIC  // measurement-only: wrong slot order
    kw.req_rank[i] = 0u;
    kw.slot_cnt[pv_rank_sub(i) * (kw.hmask + 1ull) + h] = 1u;
#else
    kw.req_rank[i] = atomicAdd(&kw.slot_cnt[pv_rank_sub(i) * (kw.hmask + 1ull) + h], 1u);
#endif
}

// The key's slot of request i (open addressing; the key is inserted if new), as pv_key_insert_kernel.
__device__ __forceinline__ uint32_t pv_key_slot(const uint8_t* __restrict__ pk, const KeyWork& kw, uint32_t i) {
    uint32_t A[8];
    pv_load_pk(A, pk, i);
    uint32_t h = pv_key_hash(A, kw.seed) & kw.hmask;
    for (uint32_t probe = 0; probe <= kw.hmask; probe++) {  // the table is >= 2x the chunk: never full
#if PV_INSERT_PLAIN_LOAD
        uint32_t cur = kw.slot[h];
#else
        uint32_t cur = __hip_atomic_load(&kw.slot[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (cur == PV_EMPTY) cur = atomicCAS(&kw.slot[h], PV_EMPTY, i);
        if (cur == PV_EMPTY) break;
        uint32_t B[8];
        pv_load_pk(B, pk, cur);
        if (pv_words_equal(A, B)) break;
        h = (h + 1) & kw.hmask;
    }
    return h;
}

// Dedup 1/2, LDS-aggregated form (PV_INSERT_LDS): every request's key slot as above, then its rank
// among the key's requests = the workgroup's base for the key (one device atomic per distinct key of
// the workgroup) + its rank inside the workgroup (an LDS atomic).
__global__ __launch_bounds__(PV_INS_THREADS) void pv_key_insert_lds_kernel(const uint8_t* __restrict__ pk, uint64_t n,
                                                                          KeyWork kw) {
    __shared__ uint32_t lkey[PV_INS_LT], lcnt[PV_INS_LT];
    const uint32_t t = threadIdx.x;
    const uint32_t g = blockIdx.x * PV_INS_THREADS + t;
    if (g < PV_SPLIT_WORDS) kw.nkeys[g] = 0u;  // the chunk's split counters (see pv_key_insert_kernel)
    if (g < PV_NSEG) kw.nkeys[PV_SEG_BASE + g * PV_SEG_STRIDE] = 0u;
    for (uint32_t e = t; e < PV_INS_LT; e += PV_INS_THREADS) {
        lkey[e] = PV_EMPTY;
        lcnt[e] = 0u;
    }
    __syncthreads();
    const uint32_t i0 = blockIdx.x * PV_INS_REQS;
    uint32_t* cnt = kw.slot_cnt + (uint64_t)((blockIdx.x & (PV_RANK_SUB - 1u))) * (kw.hmask + 1ull);
    uint32_t es[PV_INS_PER_THREAD], lr[PV_INS_PER_THREAD];
#pragma unroll
    for (uint32_t u = 0; u < PV_INS_PER_THREAD; u++) {
        const uint32_t i = i0 + u * PV_INS_THREADS + t;
        es[u] = PV_EMPTY;
        if (i >= n) continue;
        const uint32_t h = pv_key_slot(pk, kw, i);
        kw.req_key[i] = h;
        uint32_t e = (h * 2654435761u) >> (32 - 12);  // log2(PV_INS_LT)
        for (int probe = 0; probe < 64; probe++) {
            const uint32_t cur = atomicCAS(&lkey[e], PV_EMPTY, h);
            if (cur == PV_EMPTY || cur == h) {
                es[u] = e;
                break;
            }
            e = (e + 1) & (PV_INS_LT - 1u);
        }
        if (es[u] != PV_EMPTY) lr[u] = atomicAdd(&lcnt[e], 1u);
        else lr[u] = atomicAdd(&cnt[h], 1u);  // LDS table crowded: this request counts itself
    }
    __syncthreads();
    for (uint32_t e = t; e < PV_INS_LT; e += PV_INS_THREADS) {
        const uint32_t h = lkey[e];
        if (h != PV_EMPTY) lcnt[e] = atomicAdd(&cnt[h], lcnt[e]);  // count -> the workgroup's base
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < PV_INS_PER_THREAD; u++) {
        const uint32_t i = i0 + u * PV_INS_THREADS + t;
        if (i >= n) continue;
        kw.req_rank[i] = es[u] != PV_EMPTY ? lcnt[es[u]] + lr[u] : lr[u];
    }
}

// Dedup 0/2: the first requests of the chunk claim their keys' slots before the full insert, so a
// frequent key is already in the table when its other requests arrive: the full insert then finds
// it with a plain read instead of hundreds of its requests racing a compare-and-swap on one slot.
__global__ __launch_bounds__(PV_BLOCK) void pv_key_seed_kernel(const uint8_t* __restrict__ pk, uint64_t n,
                                                                KeyWork kw) {
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t A[8];
    pv_load_pk(A, pk, i);
    uint32_t h = pv_key_hash(A, kw.seed) & kw.hmask;
    for (uint32_t probe = 0; probe <= kw.hmask; probe++) {
        uint32_t cur = __hip_atomic_load(&kw.slot[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == PV_EMPTY) cur = atomicCAS(&kw.slot[h], PV_EMPTY, i);
        if (cur == PV_EMPTY) return;
        uint32_t B[8];
        pv_load_pk(B, pk, cur);
        if (pv_words_equal(A, B)) return;
        h = (h + 1) & kw.hmask;
    }
}

// Dedup 2/2: the owner request of each occupied slot takes a key id and records its key's request
// count. One atomic per wave that owns keys, on one of PV_NSEG counters (the wave's index mod
// PV_NSEG): same-address atomics serialise (~7 ns each), and with one counter a chunk of 7k distinct
// keys spent ~50 us in them (config 3), against ~11 us at 1,024 keys. Ids are segment-major
// (s * seg_cap + rank in segment s: a segment holds at most seg_cap requests, so it never
// overflows); the scan kernel walks the segments in order.
__global__ __launch_bounds__(PV_BLOCK) void pv_key_assign_kernel(uint64_t n, KeyWork kw) {
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;
    const uint32_t s = i < n ? kw.req_key[i] : 0u;
    const bool own = i < n && kw.slot[s] == i;
    const uint64_t owners = __ballot(own);
    if (owners == 0) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t seg = (i >> 6) & (PV_NSEG - 1u);
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)owners) - 1u;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&kw.nkeys[PV_SEG_BASE + seg * PV_SEG_STRIDE], (uint32_t)__popcll(owners));
    base = __shfl(base, (int)leader);
    if (!own) return;
    const uint32_t id = seg * kw.seg_cap + base + (uint32_t)__popcll(owners & ((1ull << lane) - 1ull));
    kw.slot_id[s] = id;
    kw.key_owner[id] = i;
    // sub-counts -> offsets (zero counts stay zero: no request reads them); all loads before the stores
    uint32_t v[PV_RANK_SUB];
    const uint64_t H = kw.hmask + 1ull;
#pragma unroll
    for (int u = 0; u < PV_RANK_SUB; u++) v[u] = kw.slot_cnt[u * H + s];
    uint32_t total = 0;
#pragma unroll
    for (int u = 0; u < PV_RANK_SUB; u++) {
        if (v[u]) kw.slot_cnt[u * H + s] = total;
        total += v[u];
    }
    kw.key_count[id] = total;
}

// Dedup 2b (only when the node-side key cache holds keys): every distinct key id looks its key up
// in the cache (keycache.h); key_cslot[id] = its cache slot or PV_EMPTY. xt (hmask != 0 only for a
// later sub-batch of a pipelined host call): a key the cache misses is looked up in the call's shared
// table store next, a hit there giving its slot | PV_CSLOT_XT.
__global__ __launch_bounds__(PV_BLOCK) void pv_key_cache_probe_kernel(const uint8_t* __restrict__ pk, KeyWork kw,
                                                                       PvKeyCacheView kc, PvKeyCacheView xt) {
    const uint32_t id = blockIdx.x * PV_BLOCK + threadIdx.x;  // grid: PV_NSEG * seg_cap ids
    const uint32_t seg = id / kw.seg_cap;
    if (seg >= PV_NSEG || id - seg * kw.seg_cap >= kw.nkeys[PV_SEG_BASE + seg * PV_SEG_STRIDE]) return;
    uint32_t A[8];
    pv_load_pk(A, pk, kw.key_owner[id]);
    uint32_t s = pv_kc_lookup(kc, A);
    if (s == PV_KC_EMPTY && xt.hmask) {
        const uint32_t x = pv_kc_lookup(xt, A);
        if (x != PV_KC_EMPTY) s = x | PV_CSLOT_XT;
    }
    kw.key_cslot[id] = s;
}

// Tables shared by the sub-batches of one pipelined host call (stage_and_launch): sub-batch 0 builds
// its comb keys' tables straight into the call's table store (kw.ctab points there), then this kernel
// publishes them as a key-cache view -- comb index j = slot j: its key's bytes and libsodium flag, and j
// inserted into the view's open-addressing hash table (cleared before the call) -- so the later
// sub-batches find those keys with the cache probe and read the tables instead of rebuilding them.
__global__ __launch_bounds__(PV_BLOCK) void pv_xtab_publish_kernel(const uint8_t* __restrict__ pk, KeyWork kw,
                                                                    uint32_t* __restrict__ htab, uint32_t hmask,
                                                                    uint32_t seed, uint32_t* __restrict__ keys,
                                                                    uint32_t* __restrict__ flags) {
    const uint32_t j = blockIdx.x * PV_BLOCK + threadIdx.x;
    if (j >= kw.nkeys[PV_SPLIT_COMB_KEYS] || kw.comb_cslot[j] != PV_EMPTY) return;
    uint32_t A[8];
    pv_load_pk(A, pk, kw.key_owner[kw.comb_key[j]]);
#pragma unroll
    for (int q = 0; q < 8; q++) keys[8 * j + q] = A[q];
    flags[j] = kw.key_flag[j];
    __threadfence();  // the key bytes before the hash entry that names them
    uint32_t h = pv_kc_hash(A, seed) & hmask;
    for (uint32_t probe = 0; probe <= hmask; probe++) {  // distinct keys, hmask + 1 >= 2 x entries
        if (atomicCAS(&htab[h], PV_KC_EMPTY, j) == PV_KC_EMPTY) return;
        h = (h + 1) & hmask;
    }
}

// Exclusive prefix sum of one value per thread over a 1024-thread workgroup; *total = the sum.
#ifndef PV_SCAN_WAVE
#define PV_SCAN_WAVE 1
#endif
static constexpr uint32_t PV_SCAN_THREADS = 1024;  // pv_key_scan_kernel's block
#if PV_SCAN_WAVE
// Wave scans by shuffles, then the 16 wave totals (two barriers instead of Hillis-Steele's twenty).
// Written for 64-lane waves and exactly 16 of them (the 1,024-thread pv_key_scan_kernel).
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "pv_block_scan assumes wave64 (gfx950)"
#endif
__device__ uint32_t pv_block_scan(uint32_t v, uint32_t* part, uint32_t* total) {
    static_assert(PV_SCAN_THREADS == 16 * 64, "16 wave64 totals");
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    __syncthreads();  // every thread is done with the previous scan's results
    if (lane == 63) part[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t u = 0; u < 16; u++) {
        const uint32_t pw = part[u];
        before += u < w ? pw : 0u;
        all += pw;
    }
    *total = all;
    return before + x - v;
}
#else
__device__ uint32_t pv_block_scan(uint32_t v, uint32_t* part, uint32_t* total) {
    const uint32_t t = threadIdx.x;
    __syncthreads();  // every thread is done with the previous scan's results
    part[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    *total = part[1023];
    return t ? part[t - 1] : 0u;
}
#endif

// Sort 2/3 (one workgroup): split the keys between the paths and give each key its slot range.
// Comb keys (>= min_req requests, the first kcap of them in id order) take slots [0, CS) in id
// order, every other key's requests the slots [CS, n). Threads own contiguous id ranges; three
// passes over key_count: comb index, slot totals, cursors.
static constexpr uint32_t PV_SCAN_REG = 16;  // key counts a scan thread keeps in registers
// launched with exactly PV_SCAN_THREADS threads (pv_block_scan's 16 wave totals)
__global__ __launch_bounds__(1024) void pv_key_scan_kernel(KeyWork kw, const uint32_t* __restrict__ kc_flags) {
    __shared__ uint32_t part[1024];
    // the key ids are segment-major (pv_key_assign_kernel): v-th key in segment order = id vid(v)
    uint32_t pre[PV_NSEG + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t g = 0; g < PV_NSEG; g++) pre[g + 1] = pre[g] + kw.nkeys[PV_SEG_BASE + g * PV_SEG_STRIDE];
    const uint32_t nk = pre[PV_NSEG];
    auto vid = [&](uint32_t v) -> uint32_t {
        uint32_t id = v;
#pragma unroll
        for (uint32_t g = 1; g < PV_NSEG; g++)
            if (v >= pre[g]) id = v - pre[g] + g * kw.seg_cap;
        return id;
    };
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nk + 1023) / 1024;
    const uint32_t lo = min(t * per, nk), hi = min(lo + per, nk);
    // a key in the node-side cache costs no table build: it is a comb candidate at any count; a
    // medium chunk with few distinct keys makes every key a comb key (PV_ALLCOMB_*)
    const bool all_comb = nk <= PV_ALLCOMB_KEYS && kw.chunk_n <= PV_ALLCOMB_CHUNK;
    auto is_cand = [&](uint32_t id, uint32_t c) {
        return all_comb || c >= kw.min_req || (kw.kc_on && kw.key_cslot[id] != PV_EMPTY);
    };
    // up to 16k keys every count is loaded once, all loads in flight together (three dependent
    // passes of L2 reads took ~18 us at 7k keys); above that the passes re-read
    const bool reg = per <= PV_SCAN_REG;
    uint32_t cr[PV_SCAN_REG];
#pragma unroll
    for (uint32_t u = 0; u < PV_SCAN_REG; u++) cr[u] = reg && lo + u < hi ? kw.key_count[vid(lo + u)] : 0u;
    auto count = [&](uint32_t v, uint32_t id) -> uint32_t {
        if (!reg) return kw.key_count[id];
        uint32_t c = 0;
#pragma unroll
        for (uint32_t u = 0; u < PV_SCAN_REG; u++) c = v - lo == u ? cr[u] : c;
        return c;
    };
    uint32_t cand = 0;
    for (uint32_t v = lo; v < hi; v++) {
        const uint32_t id = vid(v);
        cand += is_cand(id, count(v, id)) ? 1u : 0u;
    }
    uint32_t ncand;
    const uint32_t jbase = pv_block_scan(cand, part, &ncand);
    uint32_t cs = 0, ss = 0;
    for (uint32_t v = lo, j = jbase; v < hi; v++) {
        const uint32_t id = vid(v);
        const uint32_t c = count(v, id);
        if (is_cand(id, c) && j++ < kw.kcap) cs += c;
        else ss += c;
    }
    uint32_t ctotal, stotal;
    uint32_t cc = pv_block_scan(cs, part, &ctotal);
    uint32_t sc = ctotal + pv_block_scan(ss, part, &stotal);
    for (uint32_t v = lo, j = jbase; v < hi; v++) {
        const uint32_t id = vid(v);
        const uint32_t c = count(v, id);
        const bool cand_id = is_cand(id, c);
        if (cand_id && j < kw.kcap) {
            const uint32_t cslot = kw.kc_on ? kw.key_cslot[id] : PV_EMPTY;
            kw.key_cid[id] = j;
            kw.comb_key[j] = id;
            kw.comb_cslot[j] = cslot;
            // a cached key's libsodium checks ran when its table was built (the chain skips it)
            if (cslot != PV_EMPTY)
                kw.key_flag[j] = (cslot & PV_CSLOT_XT) ? kw.xt_flags[cslot & ~PV_CSLOT_XT] : kc_flags[cslot];
            kw.key_cursor[id] = cc;
            cc += c;
        } else {
            kw.key_cid[id] = PV_EMPTY;
            kw.key_cursor[id] = sc;
            sc += c;
        }
        if (cand_id) j++;
    }
    if (t == 0) {
        kw.nkeys[PV_SPLIT_KEYS] = nk;  // distinct keys (pv_last_path)
        // AUTO's device-side choice for a 2,049..4,096-request batch of pv_verify_batch_device: the
        // rule pv_keyed_hint applies on the host (>= 3 requests per key, every key a comb key) now
        // that the dedup has counted the keys; otherwise the latency kernel runs after this chunk
        kw.nkeys[PV_SPLIT_LAT] = kw.lat_choice && !(nk <= PV_ALLCOMB_KEYS && 3u * nk <= kw.chunk_n) ? 1u : 0u;
        kw.nkeys[PV_SPLIT_COMB_KEYS] = min(ncand, kw.kcap);
        kw.nkeys[PV_SPLIT_SLOTS] = ctotal;
        kw.nkeys[PV_SPLIT_SPARSE] =
            !kw.dense_only && all_comb && kw.chunk_n <= PV_SPARSE_CHUNK && kw.chunk_n <= PV_SPARSE_PER_KEY * nk ? 1u : 0u;
    }
}

// Sort 3/3: each request takes its key's first slot + its rank among the key's requests.
__global__ __launch_bounds__(PV_BLOCK) void pv_key_scatter_kernel(uint64_t n, KeyWork kw) {
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = kw.req_key[i];
    const uint32_t id = kw.slot_id[h];
    const uint32_t sub_off = kw.slot_cnt[pv_rank_sub(i) * (kw.hmask + 1ull) + h];
    const uint32_t pos = kw.key_cursor[id] + sub_off + kw.req_rank[i];
    kw.slot_req[pos] = i;
    kw.req_pos[i] = pos;
    kw.skey[pos] = kw.key_cid[id];
}

// Slot verdict bits back to request order: one ballot per 64 requests.
__global__ __launch_bounds__(PV_BLOCK) void pv_unpermute_kernel(uint64_t n, KeyWork kw, uint64_t* __restrict__ verdict,
                                                                 Gate gate) {
    if (!gate.keyed()) return;
    const bool lat = gate.off();  // handed to the latency path: zero words for its OR, clean up
    const uint32_t r = blockIdx.x * PV_BLOCK + threadIdx.x;
    bool ok = false;
    if (r < n) {
        const uint32_t s = kw.req_pos[r];
        ok = !lat && ((kw.sverdict[s >> 6] >> (s & 63)) & 1);
        // leave the key hash table empty for the next keyed chunk (instead of a 16 MB memset there):
        // every occupied slot is some request's slot
        const uint32_t h = kw.req_key[r];
        kw.slot[h] = PV_EMPTY;
        kw.slot_cnt[pv_rank_sub(r) * (kw.hmask + 1ull) + h] = 0u;
    }
    const uint64_t bits = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && r < n) verdict[r >> 6] = bits;
}

struct DevBases {
    uint4* b;  // [32][PV_COMB_PTS][10]: per position P_i, [16] P_i, [32] P_i, [64] P_i (extended)
    __device__ __forceinline__ void store(int i, int m, const ge_p3& p) const {
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            w[q] = p.X.v[q];
            w[10 + q] = p.Y.v[q];
            w[20 + q] = p.Z.v[q];
            w[30 + q] = p.T.v[q];
        }
        uint4* e = b + (i * PV_COMB_PTS + m) * 10;
#pragma unroll
        for (int q = 0; q < 10; q++) e[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    __device__ __forceinline__ void load(int i, int m, ge_p3& p) const {
        const uint4* e = b + (i * PV_COMB_PTS + m) * 10;
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            const uint4 v = e[q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int q = 0; q < 10; q++) {
            p.X.v[q] = w[q];
            p.Y.v[q] = w[10 + q];
            p.Z.v[q] = w[20 + q];
            p.T.v[q] = w[30 + q];
        }
    }
};
struct DevBasePts {  // the points of one position, for pv_comb_fill_block
    DevBases bs;
    int i;
    __device__ __forceinline__ void load(int m, ge_p3& p) const { bs.load(i, m, p); }
};

// One position's row of a key's comb table: entries d = 0..128, 10 uint4 (160 B) each.
struct DevCombRow {
    uint4* r;
    __device__ __forceinline__ void store(int d, const ge_cached& c) const {
        uint32_t w[40];
        ge_cached_store_words(w, c);
#pragma unroll
        for (int q = 0; q < 10; q++) r[d * 10 + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    __device__ __forceinline__ void load(int d, ge_cached& c) const {
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            const uint4 v = r[d * 10 + q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
        ge_cached_load_words(c, w);
    }
    __device__ __forceinline__ void load_half(int d, int h, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint4 v = r[d * 10 + 5 * h + q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    }
};
struct DevCombRows {
    uint4* base;  // key's table [32][129][10]
    __device__ __forceinline__ DevCombRow row(int i) const { return DevCombRow{base + (uint32_t)i * PV_COMB_ENT * 10}; }
};

// One position's row of the fixed-base comb: entries d = 0..32768, PV_BCOMB_STRIDE words each.
struct DevBRow {
    const uint4* r;
    __device__ __forceinline__ void load_part(int d, int part, uint32_t w[20]) const {
        const uint4* e = r + d * (PV_BCOMB_STRIDE / 4) + 5 * part;
#pragma unroll
        for (int q = 0; q < (part ? 3 : 5); q++) {
            const uint4 v = e[q];
            const int lim = part ? 10 : 20;
            if (4 * q < lim) w[4 * q] = v.x;
            if (4 * q + 1 < lim) w[4 * q + 1] = v.y;
            if (4 * q + 2 < lim) w[4 * q + 2] = v.z;
            if (4 * q + 3 < lim) w[4 * q + 3] = v.w;
        }
    }
};
struct DevBRows {
    const uint4* base;
    __device__ __forceinline__ DevBRow row(int i) const {
        return DevBRow{base + (uint32_t)i * PV_BCOMB_ENT * (PV_BCOMB_STRIDE / 4)};
    }
};

struct DevCombStage {  // per-key comb table rows, entries of 10 uint4
    const uint4* key;  // the key's table [32][129][10]
    uint4* lds;        // this wave's [10][64] staging area
    uint32_t lane;
    bool aff;          // affine rows (the key cache's pv_comb_row_to_affine form): rows 5, 6 not fetched
    __device__ __forceinline__ void stage(int i, int d) const {
        const uint4* e = key + ((uint32_t)i * PV_COMB_ENT + (uint32_t)d) * 10;
        pv_lds_reads_done();
        pv_glds16_row10_skip56(e, lds, aff);
    }
    __device__ __forceinline__ bool affine() const { return aff; }
    __device__ __forceinline__ void staged(int h, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint4 v = lds[(5 * h + q) * 64 + lane];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    }
};
struct DevBStage {  // fixed-base comb rows, entries of PV_BCOMB_STRIDE words (8 uint4, 30 words used)
    const uint4* base;  // T_B [16][32769][8]
    uint4* lds;         // this wave's [8][64] staging area
    uint32_t lane;
    __device__ __forceinline__ void stage(int j, int d) const {
        const uint4* e = base + ((uint32_t)j * PV_BCOMB_ENT + (uint32_t)d) * (PV_BCOMB_STRIDE / 4);
        pv_lds_reads_done();
        pv_glds16_row<PV_BCOMB_STRIDE / 4>(e, lds);
    }
    __device__ __forceinline__ void staged(int part, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < (part ? 3 : 5); q++) {
            const uint4 v = lds[(5 * part + q) * 64 + lane];
            const int lim = part ? 10 : 20;
            if (4 * q < lim) w[4 * q] = v.x;
            if (4 * q + 1 < lim) w[4 * q + 1] = v.y;
            if (4 * q + 2 < lim) w[4 * q + 2] = v.z;
            if (4 * q + 3 < lim) w[4 * q + 3] = v.w;
        }
    }
};

// The key chain is the keyed path's long serial dependency and shares SIMDs with the per-request
// prep kernel: its waves take issue priority (PV_CHAIN_PRIO, s_setprio).
#ifndef PV_CHAIN_PRIO
#define PV_CHAIN_PRIO 3
#endif
__device__ __forceinline__ void pv_chain_prio() {
#if PV_CHAIN_PRIO > 0
    __builtin_amdgcn_s_setprio(PV_CHAIN_PRIO);
#endif
}

// Per distinct key: libsodium's key checks, -A, and the chain of bases [256^i](-A).
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_key_chain_kernel(const uint8_t* __restrict__ pk, KeyWork kw,
                                                                    Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    pv_chain_prio();
    const uint32_t id = blockIdx.x * PV_BLOCK + threadIdx.x;  // comb index
    if (id >= kw.nkeys[PV_SPLIT_COMB_KEYS] || kw.comb_cslot[id] != PV_EMPTY) return;
    uint32_t A[8];
    pv_load_pk(A, pk, kw.key_owner[kw.comb_key[id]]);
    ge_p3 negA;
    const bool ok = pv_key_ok_negate(negA, A);
    kw.key_flag[id] = ok ? 1u : 0u;
    pv_comb_chain(DevBases{kw.bases + (uint64_t)id * PV_COMB_POS * PV_COMB_PTS * 10}, negA);
}

// ---- quad-cooperative key chain: four lanes per key shorten the per-key critical path ~2x.
// The chain of 248 doublings is the only long dependency of the comb path and it runs on very few
// lanes (one per distinct key), so its LATENCY, not its work, is what the batch waits for. Each
// doubling's four squarings (X^2, Y^2, Z^2, (X+Y)^2) run on the four lanes of a quad at once and
// so do its three (or four) products; quad_perm DPP broadcasts exchange the results.
__device__ __forceinline__ uint32_t pv_quad_bcast(uint32_t v, int r) {
    switch (r) {
        case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false);
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, false);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, false);
        default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xF, 0xF, false);
    }
}
__device__ __forceinline__ void pv_fe_bcast(fe& h, const fe& f, int r) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = pv_quad_bcast(f.v[i], r);
}
// h = (role == 0) ? a : (role == 1) ? b : (role == 2) ? c : d, branch-free: the role masks are
// opaque to the compiler (see pv_key_chain_quad_kernel), so it selects per lane with v_cndmask
// instead of specialising the field arithmetic per role into divergent copies.
struct QuadRole {
    uint32_t m0, m1, m2;  // all-ones iff role == 0 / 1 / 2
};
__device__ __forceinline__ void pv_fe_sel4(fe& h, const fe& a, const fe& b, const fe& c, const fe& d,
                                           const QuadRole& q) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t cd = q.m2 ? c.v[i] : d.v[i];
        const uint32_t bcd = q.m1 ? b.v[i] : cd;
        h.v[i] = q.m0 ? a.v[i] : bcd;
    }
}

// One doubling of (X : Y : Z) (ge_p2_dbl + ge_p1p1_to_p2/p3), quad-parallel; T is produced when
// want_t (it is the fourth lane's product).
__device__ __forceinline__ void pv_quad_dbl(fe& X, fe& Y, fe& Z, fe& T, const QuadRole& role, bool want_t) {
    fe in, s, XX, YY, ZZ, S, t;
    fe_add(t, X, Y);
    pv_fe_sel4(in, X, Y, Z, t, role);
    fe_sq(s, in);
    pv_fe_bcast(XX, s, 0);
    pv_fe_bcast(YY, s, 1);
    pv_fe_bcast(ZZ, s, 2);
    pv_fe_bcast(S, s, 3);
    ge_p1p1 r;
    fe_add(r.Y, YY, XX);
    fe_sub(r.Z, YY, XX);
    fe_sub4p(r.X, S, r.Y);
    fe_add(t, ZZ, ZZ);
    fe_sub4p(t, t, r.Z);
    fe_carry(r.T, t);
    // lane 0: X = rX rT, 1: Y = rY rZ, 2: Z = rZ rT, 3: T = rX rY (f side may be uncarried rX)
    fe f, g, o;
    pv_fe_sel4(f, r.X, r.Y, r.Z, r.X, role);
    pv_fe_sel4(g, r.T, r.Z, r.T, r.Y, role);
    fe_mul(o, f, g);
    pv_fe_bcast(X, o, 0);
    pv_fe_bcast(Y, o, 1);
    pv_fe_bcast(Z, o, 2);
    if (want_t) pv_fe_bcast(T, o, 3);
}

// Per distinct key, four lanes: libsodium's key checks, -A, and the bases [256^i](-A), i = 0..31.
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_key_chain_quad_kernel(const uint8_t* __restrict__ pk, KeyWork kw,
                                                                         Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    // the chain is the batch's critical path and shares SIMDs with the per-request prep kernel:
    // take issue priority over it
    pv_chain_prio();
    const uint32_t g = blockIdx.x * PV_BLOCK + threadIdx.x;
    const uint32_t nk = kw.nkeys[PV_SPLIT_COMB_KEYS];
    const uint32_t id = g >> 2;  // comb index
    uint32_t rl = g & 3;
    asm volatile("" : "+v"(rl));  // opaque: keep the per-role selects branch-free
    const QuadRole role{rl == 0 ? ~0u : 0u, rl == 1 ? ~0u : 0u, rl == 2 ? ~0u : 0u};
    // whole quads exit together (nk is uniform), so the DPP partners of a live lane are live
    if (id >= nk || kw.comb_cslot[id] != PV_EMPTY) return;  // uniform per quad
    uint32_t A[8];
    pv_load_pk(A, pk, kw.key_owner[kw.comb_key[id]]);
    ge_p3 cur;
    const bool ok = pv_key_ok_negate(cur, A);
    if (rl == 0) kw.key_flag[id] = ok ? 1u : 0u;
    uint32_t* b = reinterpret_cast<uint32_t*>(kw.bases + (uint64_t)id * PV_COMB_POS * PV_COMB_PTS * 10);
    fe X = cur.X, Y = cur.Y, Z = cur.Z, T = cur.T;
    // lane r stores component r (X, Y, Z, T) of a point: words 10 r .. 10 r + 9 of its 40
    auto store = [&](int i, int m) {
        fe mine;
        pv_fe_sel4(mine, X, Y, Z, T, role);
#pragma unroll
        for (int q = 0; q < 10; q++) b[(i * PV_COMB_PTS + m) * 40 + 10 * rl + q] = mine.v[q];
    };
    for (int i = 0; i < PV_COMB_POS; i++) {
        store(i, 0);
        // [2] .. [256] P_i; [16], [32], [64] P_i are kept for the table fill (pv_comb_chain)
        const int nd = i + 1 < PV_COMB_POS ? 8 : 6;
        for (int j = 0; j < nd; j++) {
            pv_quad_dbl(X, Y, Z, T, role, (j >= 3 && j <= 5) || j == 7);
            if (j >= 3 && j <= 5) store(i, j - 2);
        }
    }
}

#if LP_DEVICE
// Positions [lo, hi) of one key's chain. Part 0 decompresses -A and writes the key flag; a later part
// resumes from P_lo, which the previous part stored as slot 0 of position lo.
__device__ __forceinline__ void pv_key_chain_lp(const uint8_t* __restrict__ pk, const KeyWork& kw, uint32_t id,
                                                const LpLane& c, const LpConsts& K, int lo, int hi) {
    uint32_t* b = reinterpret_cast<uint32_t*>(kw.bases + (uint64_t)id * PV_COMB_POS * PV_COMB_PTS * 10);
    const uint32_t w = 10u * (threadIdx.x >> 4) + (threadIdx.x & 15u);  // word of [X, Y, Z, T] x 10 limbs
    const bool limb = (threadIdx.x & 15u) < 10u;
    auto store = [&](int i, int m, const lu& P) {
        const lu R = lp_carry1(c, P);  // LR -> limb < 2^w + 19: the per-lane code's reduced bound
        if (limb) b[(i * PV_COMB_PTS + m) * 40 + w] = R;
    };
    lu P;
    if (lo == 0) {
        uint32_t A[8];
        pv_load_pk(A, pk, kw.key_owner[kw.comb_key[id]]);
        lu sw[8];
#pragma unroll
        for (int q = 0; q < 8; q++) sw[q] = A[q];
        const LpDecomp dec = lp_decompress_ar(c, K, sw);
        const bool ok = pv_ge_is_canonical(A) && !pv_has_small_order(A) && dec.ok_a;
        if (threadIdx.x == 0) kw.key_flag[id] = ok ? 1u : 0u;
        P = lp_ext_from_xy(c, K, dec.X, dec.Y, 0);
    } else {
        P = lp_load_ext40(c, b + lo * PV_COMB_PTS * 40);
    }
    P = lp_comb_chain_part(c, P, lo, hi, store);
    if (hi < PV_COMB_POS) store(hi, 0, P);  // P_hi: where the next part resumes
}
#endif

// Limb-parallel key chain (lp25519.h): ONE wave per key, every field element over a 16-lane row and
// the four squarings / products of a doubling in the four rows at once, so the 254 dependent
// doublings take ~4x less time than on a quad of lanes. Blocks stride over the keys (a batch with
// more keys than blocks runs them in turn), so the launch needs no host-side key count and no gated
// companion kernel: a gated launch is not free on a saturated chip, its blocks wait ~0.2 ms for
// dispatch slots (rocprofv3, profiles/r02/prof_a). Same outputs as pv_key_chain_quad_kernel: key_flag
// and the bases [256^i](-A) with their [16], [32], [64] multiples, carried to reduced limbs.
__global__ __launch_bounds__(64) void pv_key_chain_lp_kernel(const uint8_t* __restrict__ pk, KeyWork kw, Gate gate,
                                                              int lo, int hi) {
#if LP_DEVICE
    if (!gate.keyed() || gate.off()) return;
    const uint32_t nk = kw.nkeys[PV_SPLIT_COMB_KEYS];
    if (blockIdx.x >= nk) return;
    pv_chain_prio();
    const LpLane c = LpLane::make();
    const LpConsts K = LpConsts::make(c);
    for (uint32_t id = blockIdx.x; id < nk; id += gridDim.x)
        if (kw.comb_cslot[id] == PV_EMPTY) pv_key_chain_lp(pk, kw, id, c, K, lo, hi);  // cached: table ready
#endif
}

// Per (key, position in [lo, hi), block of 16 entries): the comb table rows. Grid-stride over
// nkeys * (hi - lo) * 8 items.
// Optional wave priority for the fill (A/B knob): it runs beside the request-order prep and is the
// later of the two inputs of the comb kernel.
#ifndef PV_FILL_PRIO
#define PV_FILL_PRIO 0
#endif
__global__ __launch_bounds__(PV_BLOCK, PV_FILL_MINBLOCKS) void pv_key_fill_kernel(KeyWork kw, Gate gate, int lo,
                                                                                  int hi) {
    if (!gate.keyed() || gate.off() || kw.nkeys[PV_SPLIT_SPARSE]) return;
#if PV_FILL_PRIO > 0
    __builtin_amdgcn_s_setprio(PV_FILL_PRIO);
#endif
    const uint32_t np = (uint32_t)(hi - lo);
    const uint32_t items = kw.nkeys[PV_SPLIT_COMB_KEYS] * np * PV_COMB_BLOCKS;
    for (uint32_t it = blockIdx.x * PV_BLOCK + threadIdx.x; it < items; it += gridDim.x * PV_BLOCK) {
        const uint32_t id = it / (np * PV_COMB_BLOCKS);
        if (kw.comb_cslot[id] != PV_EMPTY) continue;  // the key's table is in the node-side cache
        const int pos = lo + (int)((it / PV_COMB_BLOCKS) % np);
        const int b = it % PV_COMB_BLOCKS;
        const DevBasePts pts{DevBases{kw.bases + (uint64_t)id * PV_COMB_POS * PV_COMB_PTS * 10}, pos};
        pv_comb_fill_block(DevCombRow{kw.ctab + ((uint64_t)id * PV_COMB_POS + pos) * PV_COMB_ENT * 10}, pts, b);
    }
}

// Sparse variant for small chunks (PV_SPLIT_SPARSE): one thread per (comb key, position), only the
// entries the chunk's digits use (pv_comb_fill_sparse). Runs on the main stream after
// pv_comb_prep_kernel (need masks) and the key chain (bases). Sparse chunks have <= PV_ALLCOMB_KEYS
// comb keys: the grid covers that many.
struct DevNeed {
    const uint32_t* p;  // the position's 5 mask words (registers of the caller)
    __device__ __forceinline__ uint32_t word(int w) const { return p[w]; }
};
__global__ __launch_bounds__(PV_BLOCK) void pv_key_fill_sparse_kernel(KeyWork kw, Gate gate) {
    if (!gate.keyed() || gate.off() || !kw.nkeys[PV_SPLIT_SPARSE]) return;
    const uint32_t it = blockIdx.x * PV_BLOCK + threadIdx.x;
    const uint32_t id = it / PV_COMB_POS;
    const int pos = (int)(it % PV_COMB_POS);
    if (id >= kw.nkeys[PV_SPLIT_COMB_KEYS]) return;
    uint32_t* nd = kw.need + ((uint64_t)id * PV_COMB_POS + pos) * 5;
    uint32_t m[5];
#pragma unroll
    for (int w = 0; w < 5; w++) {  // read and clear: the masks start empty for the next sparse chunk
        m[w] = nd[w];
        nd[w] = 0u;
    }
    if (kw.comb_cslot[id] != PV_EMPTY) return;
    const DevBasePts pts{DevBases{kw.bases + (uint64_t)id * PV_COMB_POS * PV_COMB_PTS * 10}, pos};
    pv_comb_fill_sparse(DevCombRow{kw.ctab + ((uint64_t)id * PV_COMB_POS + pos) * PV_COMB_ENT * 10}, pts,
                        DevNeed{m});
}

// Key cache fill: comb index j of a put batch (tables built in the workspace by the chain / fill
// kernels) -> cache slot slots[j]: its 660 KB table, its key words and its libsodium key-check flag.
__global__ __launch_bounds__(PV_BLOCK) void pv_kc_scatter_kernel(const uint4* __restrict__ ctab,
                                                                  const uint32_t* __restrict__ key_flag,
                                                                  const uint8_t* __restrict__ pk,
                                                                  const uint32_t* __restrict__ slots, uint32_t m,
                                                                  uint4* __restrict__ tab, uint32_t* __restrict__ flags,
                                                                  uint32_t* __restrict__ keys) {
    constexpr uint32_t per = PV_COMB_POS * PV_COMB_ENT * 10;  // uint4 per key table
    const uint32_t j = blockIdx.y;
    if (j >= m) return;
    const uint64_t dst = (uint64_t)slots[j] * per, src = (uint64_t)j * per;
    for (uint32_t t = blockIdx.x * PV_BLOCK + threadIdx.x; t < per; t += gridDim.x * PV_BLOCK)
        tab[dst + t] = ctab[src + t];
    if (blockIdx.x == 0 && threadIdx.x < 8) {
        keys[8 * slots[j] + threadIdx.x] = reinterpret_cast<const uint32_t*>(pk)[8 * j + threadIdx.x];
        if (threadIdx.x == 0) flags[slots[j]] = key_flag[j];
    }
}

// Key cache fill, second part: the affine rows of every slot just filled (one thread per (slot, position):
// pv_comb_row_to_affine over the 129 cached-form entries, one inversion).
struct DevCachedRowSrc {
    const uint4* r;  // [129][10]
    __device__ __forceinline__ void load(int d, ge_cached& c) const {
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            const uint4 v = r[d * 10 + q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
        ge_cached_load_words(c, w);
    }
};
struct DevAffineRowDst {
    uint4* r;  // [129][10]
    __device__ __forceinline__ uint32_t* e(int d) const { return reinterpret_cast<uint32_t*>(r + d * 10); }
};
__global__ __launch_bounds__(64) void pv_kc_affine_kernel(const uint4* __restrict__ tab,
                                                          const uint32_t* __restrict__ slots, uint32_t m,
                                                          uint4* __restrict__ atab) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    if (t >= m * PV_COMB_POS) return;
    const uint64_t slot = slots[t / PV_COMB_POS], pos = t % PV_COMB_POS;
    pv_comb_row_to_affine(DevCachedRowSrc{tab + (slot * PV_COMB_POS + pos) * PV_COMB_ENT * 10},
                          DevAffineRowDst{atab + (slot * PV_COMB_POS + pos) * PV_COMB_ENT * 10});
}

// Key cache put: the workspace set up for m keys given in order (d_put_pk[j] is comb index j's key):
// identity key ids, no cached table, split counters {m keys, m comb keys, everything else 0}.
__global__ __launch_bounds__(PV_BLOCK) void pv_kc_put_prep_kernel(KeyWork kw, uint32_t m) {
    const uint32_t j = blockIdx.x * PV_BLOCK + threadIdx.x;
    if (j < PV_SPLIT_WORDS) kw.nkeys[j] = (j == PV_SPLIT_KEYS || j == PV_SPLIT_COMB_KEYS) ? m : 0u;
    if (j < m) {
        kw.comb_key[j] = j;
        kw.key_owner[j] = j;
        kw.comb_cslot[j] = PV_EMPTY;
    }
}

// Per request on the comb path: signature checks, k, key id and validity, radix-256 digits of k, S.
template <int W>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_comb_prep_kernel(const uint8_t* __restrict__ sm,
                                                                    const uint64_t* __restrict__ off, uint64_t n,
                                                                    const uint8_t* __restrict__ pk, Work wk,
                                                                    KeyWork kw, Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;  // slot
    if (i >= gate.ncomb()) return;
    const uint32_t r = kw.slot_req[i];                         // request
    const uint64_t o0 = off[r], o1 = off[r + 1];
    const uint64_t smlen = o1 - o0;
    const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
    const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
    pv_sig_words in;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    pv_load_pk(in.A, pk, r);
    bool ok = pv_sig_ok(in, smlen);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    // the key's own checks (key_flag) are written by the chain kernel on the key stream, which
    // runs concurrently with this kernel: pv_comb_a_kernel folds them into flags[slot]
    uint32_t ek[8];
    int32_t fb[Bc2<W>::POS];
    sc_recode256(ek, k);
    sc_recode_w<W, Bc2<W>::POS>(fb, in.S);
    const Soa ds(wk.digits, PV_DIGIT_ROWS, wk.stride);
#pragma unroll
    for (int q = 0; q < 8; q++) ds.st(q, i, ek[q]);
#pragma unroll
    for (int j = 0; j < Bc2<W>::POS; j++) ds.st(8 + j, i, (uint32_t)fb[j]);
    wk.flags[i] = ok ? 1u : 0u;
    if (kw.nkeys[PV_SPLIT_SPARSE]) {  // small chunk: record which entries of each row this request uses
        uint32_t* nd = kw.need + (uint64_t)kw.skey[i] * PV_COMB_POS * 5;
#pragma unroll
        for (int pos = 0; pos < PV_COMB_POS; pos++) {
            const int e = pv_byte(ek[pos >> 2], pos);
            const uint32_t d = (uint32_t)(e < 0 ? -e : e);
            atomicOr(nd + pos * 5 + (d >> 5), 1u << (d & 31));
        }
    }
}

// Request-order form of the comb prep (PV_PREP_REQ_ORDER). Slot order gives every lane a record at a
// random place in the blob, and a record's 128-byte SHA-512 blocks straddle cache lines that the next
// block re-reads long after they left L2 (round 3 PMC: 1.06 GB fetched per 1M launch for ~0.42 GB of
// records and keys). In request order the 64 lanes of a wave read 64 CONSECUTIVE records, ~23 KB of
// contiguous blob, so the lines that straddle two lanes' records or two blocks of one record are
// reused within the wave's own burst. The per-request results (radix-256 digits of k, radix-2^W digits
// of S, the signature-check flag) go to a per-request AoS record, written coalesced;
// pv_comb_digits_kernel then gathers them into the slot-ordered rows the comb kernel reads.
#ifndef PV_PREP_REQ_ORDER
#define PV_PREP_REQ_ORDER 1
#endif
template <int W>
struct PrepAos {  // uint4 per request: ek[8], fb[POS], flag, padding
    static constexpr int WORDS = 8 + Bc2<W>::POS + 1;
    static constexpr int Q = (WORDS + 3) / 4;
};
static constexpr int PV_PREP_AOS_QMAX = 7;  // the largest PrepAos<W>::Q (W = 16: 25 words)
static_assert(PrepAos<16>::Q <= PV_PREP_AOS_QMAX && PrepAos<PV_BC2_W>::Q <= PV_PREP_AOS_QMAX, "AoS record size");
template <int W>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_comb_prep_req_kernel(const uint8_t* __restrict__ sm,
                                                                        const uint64_t* __restrict__ off, uint64_t n,
                                                                        const uint8_t* __restrict__ pk, Work wk,
                                                                        KeyWork kw, Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t r = blockIdx.x * PV_BLOCK + threadIdx.x;  // request
    if (r >= n) return;
    const uint32_t i = kw.req_pos[r];  // its slot
    if (i >= gate.ncomb()) return;     // a Straus-path request (its prep runs on the side stream)
    const uint64_t o0 = off[r], o1 = off[r + 1];
    const uint64_t smlen = o1 - o0;
    const uint64_t raddr = reinterpret_cast<uint64_t>(sm + o0);
    const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
    pv_sig_words in;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        in.R[q] = mw.dw(q);
        in.S[q] = mw.dw(8 + q);
    }
    pv_load_pk(in.A, pk, r);
    const bool ok = pv_sig_ok(in, smlen);
    uint32_t k[8];
    pv_hash_k(k, in, smlen, mw);
    constexpr int P = Bc2<W>::POS;
    uint32_t w[4 * PrepAos<W>::Q];
    sc_recode256(w, k);
    int32_t fb[P];
    sc_recode_w<W, P>(fb, in.S);
#pragma unroll
    for (int j = 0; j < P; j++) w[8 + j] = (uint32_t)fb[j];
    w[8 + P] = ok ? 1u : 0u;
#pragma unroll
    for (int j = 9 + P; j < 4 * PrepAos<W>::Q; j++) w[j] = 0u;
    uint4* o = wk.aos + (uint64_t)r * PrepAos<W>::Q;
#pragma unroll
    for (int q = 0; q < PrepAos<W>::Q; q++) o[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    if (kw.nkeys[PV_SPLIT_SPARSE]) {  // small chunk: record which entries of each row this request uses
        uint32_t* nd = kw.need + (uint64_t)kw.skey[i] * PV_COMB_POS * 5;
#pragma unroll
        for (int pos = 0; pos < PV_COMB_POS; pos++) {
            const int e = pv_byte(w[pos >> 2], pos);
            const uint32_t d = (uint32_t)(e < 0 ? -e : e);
            atomicOr(nd + pos * 5 + (d >> 5), 1u << (d & 31));
        }
    }
}

// Slot order: every comb slot's digit rows and flag from its request's AoS record (80-112 contiguous
// bytes per lane), written as the coalesced rows pv_comb_ab_kernel / pv_comb_a_kernel and the encode read.
template <int W>
__global__ __launch_bounds__(PV_BLOCK) void pv_comb_digits_kernel(Work wk, KeyWork kw, Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;  // slot
    if (i >= gate.ncomb()) return;
    const uint4* a = wk.aos + (uint64_t)kw.slot_req[i] * PrepAos<W>::Q;
    uint32_t w[4 * PrepAos<W>::Q];
#pragma unroll
    for (int q = 0; q < PrepAos<W>::Q; q++) {
        const uint4 v = a[q];
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
    const Soa ds(wk.digits, PV_DIGIT_ROWS, wk.stride);
#pragma unroll
    for (int q = 0; q < 8 + Bc2<W>::POS; q++) ds.st(q, i, w[q]);
    wk.flags[i] = w[8 + Bc2<W>::POS];
}

// The niels loop of a comb slot over the wide fixed-base rows and, when the slot's key has wide cached
// rows (wkey != null), over those too: positions 16.. are the fixed base's (row j - 16), 0..15 the
// key's radix-65536 rows (comb.h PV_KW_*). Same entry format, same LDS staging as DevB2Stage.
template <uint32_t ENT>
struct DevBWStage {
    const uint4* base;  // T_B2
    const uint4* wkey;  // the key's wide rows [16][PV_KW_ENT][8], or null
    uint4* lds;
    uint32_t lane;
    __device__ __forceinline__ void stage(int j, int d) const {
        const uint4* e = wkey && j < PV_KW_POS
                             ? wkey + ((uint64_t)j * PV_KW_ENT + (uint32_t)d) * (PV_BCOMB_STRIDE / 4)
                             : base + ((uint64_t)(wkey ? j - PV_KW_POS : j) * ENT + (uint32_t)d) * (PV_BCOMB_STRIDE / 4);
        pv_lds_reads_done();
        pv_glds16_row<PV_BCOMB_STRIDE / 4>(e, lds);
    }
    __device__ __forceinline__ void staged(int part, uint32_t w[20]) const {
#pragma unroll
        for (int q = 0; q < (part ? 3 : 5); q++) {
            const uint4 v = lds[(5 * part + q) * 64 + lane];
            const int lim = part ? 10 : 20;
            if (4 * q < lim) w[4 * q] = v.x;
            if (4 * q + 1 < lim) w[4 * q + 1] = v.y;
            if (4 * q + 2 < lim) w[4 * q + 2] = v.z;
            if (4 * q + 3 < lim) w[4 * q + 3] = v.w;
        }
    }
};
// The wide rows of slot i's key (null unless the key is cached with wide rows).
__device__ __forceinline__ const uint4* pv_kw_rows(const KeyWork& kw, uint32_t i) {
    if (!kw.kc_wtab) return nullptr;
    const uint32_t cslot = kw.comb_cslot[kw.skey[i]];
    return cslot < kw.kc_wcap ? kw.kc_wtab + (uint64_t)cslot * PV_KW_POS * PV_KW_ENT * (PV_BCOMB_STRIDE / 4)
                              : nullptr;
}
// [S]B, plus [k](-A) when wkey: the niels loop over 11 (+ 16) positions (comb.h pv_comb_b_acc_w).
template <int W>
__device__ __forceinline__ void pv_comb_bw_acc(ge_p3& acc, const uint4* bcomb, const uint4* wkey, const DevDigits& dig,
                                               uint4* stg_wave) {
    constexpr int P = Bc2<W>::POS;
    pv_comb_b_acc_w<P>(
        acc, DevBWStage<Bc2<W>::ENT>{bcomb, wkey, stg_wave, threadIdx.x & 63u},
        [&](int j) {
            if (wkey && j < PV_KW_POS) return pv_kw_digit(dig.ek(j >> 1), j);
            return dig.fb(wkey ? j - PV_KW_POS : j);
        },
        wkey ? P + PV_KW_POS : P);
}
// A slot whose [k](-A) was added in the niels loop: projective Q to q rows 0..29 and the key's flag.
__device__ __forceinline__ void pv_comb_store_q(const Work& wk, const KeyWork& kw, uint32_t i, const ge_p3& acc) {
    if (kw.key_flag[kw.skey[i]] == 0) wk.flags[i] = 0;
    const Soa qs(wk.q, 40, wk.stride);
#pragma unroll
    for (int q = 0; q < 10; q++) {
        qs.st(q, i, acc.X.v[q]);
        qs.st(10 + q, i, acc.Y.v[q]);
        qs.st(20 + q, i, acc.Z.v[q]);
    }
}


// Per request on the comb path, first half: acc = [S]B from the wide fixed-base comb (PV_BC2_POS
// positions: one entry conversion + PV_BC2_POS - 1 additions). Needs no per-key data, so it runs on
// the main stream while the key stream builds the tables. acc (extended, 40 words) goes to q rows
// 0..39.
// A slot whose key has wide cached rows gets [k](-A) here too (16 more niels additions): pv_comb_a_kernel
// then only copies its flag.
template <int W>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_comb_b_kernel(uint64_t n, Work wk, KeyWork kw,
                                                                 const uint4* __restrict__ bcomb, Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t i = blockIdx.x * PV_BLOCK + threadIdx.x;  // slot
    if (i >= gate.ncomb()) return;
    const DevDigits dig{wk.digits, (uint32_t)wk.stride, i};
    ge_p3 acc;
    __shared__ uint4 stg[PV_BLOCK / 64][PV_BCOMB_STRIDE / 4][64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    pv_comb_bw_acc<W>(acc, bcomb, pv_kw_rows(kw, i), dig, &stg[wv][0][0]);
    const Soa qs(wk.q, 40, wk.stride);
#pragma unroll
    for (int q = 0; q < 10; q++) {
        qs.st(q, i, acc.X.v[q]);
        qs.st(10 + q, i, acc.Y.v[q]);
        qs.st(20 + q, i, acc.Z.v[q]);
        qs.st(30 + q, i, acc.T.v[q]);
    }
}

// Keyed chunk, [S]B per REQUEST (not slot): needs only S, so it starts with the chunk on its own
// stream and runs beside the dedup kernels (atomics and scattered stores that leave the ALUs idle for
// ~0.14 ms) instead of after the key sort. acc (extended, 40 words) to qb[r], 160 contiguous bytes,
// which pv_comb_a_kernel gathers by slot_req. Requests of Straus keys get a value nobody reads.
template <int W>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_comb_b_req_kernel(const uint8_t* __restrict__ sm,
                                                                     const uint64_t* __restrict__ off, uint64_t n,
                                                                     Work wk, const uint4* __restrict__ bcomb) {
    const uint32_t r0 = blockIdx.x * PV_BLOCK + threadIdx.x;  // request
    if (blockIdx.x * PV_BLOCK >= n) return;
    const uint32_t r = r0 < n ? r0 : (uint32_t)n - 1;  // whole waves stay in step for the staging
    uint32_t S[8];
    {
        const uint64_t raddr = reinterpret_cast<uint64_t>(sm + off[r]);
        const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
#pragma unroll
        for (int q = 0; q < 8; q++) S[q] = mw.dw(8 + q);
    }
    constexpr int P = Bc2<W>::POS;
    int32_t fb[P];
    sc_recode_w<W, P>(fb, S);  // any S (an S >= L is rejected by the prep's check)
    __shared__ uint4 stg[PV_BLOCK / 64][PV_BCOMB_STRIDE / 4][64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    ge_p3 acc;
    pv_comb_b_acc_w<P>(acc, DevB2Stage<Bc2<W>::ENT>{bcomb, &stg[wv][0][0], threadIdx.x & 63u}, [&](int j) {
        int32_t d = 0;
#pragma unroll
        for (int u = 0; u < P; u++) d = j == u ? fb[u] : d;
        return (int)d;
    });
    if (r0 >= n) return;
    uint4* o = wk.qb + (uint64_t)r * 10u;
    uint32_t w[40];
#pragma unroll
    for (int q = 0; q < 10; q++) {
        w[q] = acc.X.v[q];
        w[10 + q] = acc.Y.v[q];
        w[20 + q] = acc.Z.v[q];
        w[30 + q] = acc.T.v[q];
    }
#pragma unroll
    for (int q = 0; q < 10; q++) o[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Straus path, [S]B of every Straus slot from the wide fixed-base comb (tiles from the end of the
// slot range, like the other Straus kernels), extended, to q rows 0..39 for pv_msm_kernel.
template <int W>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_straus_b_kernel(uint64_t n, Work wk, const uint4* __restrict__ bcomb,
                                                                   Gate gate) {
    if (gate.off()) return;
    const uint32_t nc = gate.ncomb(), ntiles = (uint32_t)((n + PV_BLOCK - 1) / PV_BLOCK);
    if (blockIdx.x >= ntiles || nc >= n || (gate.stile(blockIdx.x, ntiles) + 1) * PV_BLOCK <= nc) return;
    pv_straus_prio();
    __shared__ uint4 stg[PV_BLOCK / 64][PV_BCOMB_STRIDE / 4][64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Soa qs(wk.q, 40, wk.stride);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t sb = gate.stile(t, ntiles);
        if ((sb + 1) * PV_BLOCK <= nc) break;
        const uint32_t i0 = sb * PV_BLOCK + threadIdx.x;  // slot
        const bool active = i0 < n && i0 >= nc;
        const uint32_t i = active ? i0 : (uint32_t)n - 1;  // whole waves stay in step for the staging
        const DevDigits dig{wk.digits, (uint32_t)wk.stride, i};
        ge_p3 acc;
        pv_comb_b_acc_w<Bc2<W>::POS>(acc, DevB2Stage<Bc2<W>::ENT>{bcomb, &stg[wv][0][0], threadIdx.x & 63u},
                                     [&](int j) { return dig.fb(j); });
        if (active) {
#pragma unroll
            for (int q = 0; q < 10; q++) {
                qs.st(q, i, acc.X.v[q]);
                qs.st(10 + q, i, acc.Y.v[q]);
                qs.st(20 + q, i, acc.Z.v[q]);
                qs.st(30 + q, i, acc.T.v[q]);
            }
        }
    }
}

// Wide fixed-base comb build (pv_init): each thread makes PV_BC2_RUN consecutive entries d0.. of one
// row (base point P = [2^(W j)] B): start [d0] P by double-and-add, then P-steps, the projective
// points parked in the entries themselves and the running product of their Z in `scratch`; one
// inversion per run (Montgomery's trick) gives every entry's affine niels form (canonical limbs).
static constexpr uint32_t PV_BC2_RUN = 64;
struct PvPoint40 {
    uint32_t w[40];  // X, Y, Z, T limbs
};
struct DevBc2Row {  // one row of the wide comb, 32 words per entry
    uint32_t* r;
    __device__ __forceinline__ uint32_t* e(uint32_t d) const { return r + (uint64_t)d * PV_BCOMB_STRIDE; }
};
struct DevBc2Scratch {  // running Z products, 10 words per entry
    uint32_t* z;
    __device__ __forceinline__ void store(uint32_t d, const fe& f) const {
#pragma unroll
        for (int q = 0; q < 10; q++) z[(uint64_t)d * 10 + q] = f.v[q];
    }
    __device__ __forceinline__ void load(uint32_t d, fe& f) const {
#pragma unroll
        for (int q = 0; q < 10; q++) f.v[q] = z[(uint64_t)d * 10 + q];
    }
};
__global__ __launch_bounds__(PV_BLOCK) void pv_bc2_build_kernel(uint4* __restrict__ row, uint32_t ent, PvPoint40 base,
                                                                uint32_t* __restrict__ scratch) {
    const uint32_t d0 = (blockIdx.x * PV_BLOCK + threadIdx.x) * PV_BC2_RUN;
    if (d0 >= ent) return;
    ge_p3 P;
#pragma unroll
    for (int q = 0; q < 10; q++) {
        P.X.v[q] = base.w[q];
        P.Y.v[q] = base.w[10 + q];
        P.Z.v[q] = base.w[20 + q];
        P.T.v[q] = base.w[30 + q];
    }
    pv_bc2_build_run(DevBc2Row{reinterpret_cast<uint32_t*>(row)}, DevBc2Scratch{scratch}, P, d0,
                     min(PV_BC2_RUN, ent - d0));
}

// Key cache fill, third part: the radix-65536 rows of the slots below wcap (comb.h PV_KW_*), keys
// [j0, j0 + g) of the put batch: one thread per run of PV_BC2_RUN entries of one row, the row's base
// [65536^q](-A) = the chain's P_{2q}; pv_bc2_build_run (double-and-add start, P-steps, one inversion
// per run) writes affine niels entries, the Z products in scratch.
#ifndef PV_KC_WIDE_KEYS
#define PV_KC_WIDE_KEYS 1024  // keys that get wide rows (67 MB each)
#endif
static constexpr uint32_t PV_KW_GROUP = 64;  // keys per wide build launch (scratch: 1.35 GB)
static constexpr uint32_t PV_KW_RUNS = (PV_KW_ENT + PV_BC2_RUN - 1) / PV_BC2_RUN;  // runs per row
__global__ __launch_bounds__(PV_BLOCK) void pv_kc_wide_kernel(KeyWork kw, const uint32_t* __restrict__ slots,
                                                              uint32_t j0, uint32_t g, uint32_t wcap,
                                                              uint4* __restrict__ wtab, uint32_t* __restrict__ scr) {
    const uint32_t t = blockIdx.x * PV_BLOCK + threadIdx.x;
    const uint32_t per_key = PV_KW_POS * PV_KW_RUNS;
    if (t >= g * per_key) return;
    const uint32_t jj = t / per_key, q = (t % per_key) / PV_KW_RUNS, r = t % PV_KW_RUNS;
    const uint32_t j = j0 + jj, slot = slots[j];
    if (slot >= wcap) return;
    ge_p3 P;
    DevBases{kw.bases + (uint64_t)j * PV_COMB_POS * PV_COMB_PTS * 10}.load(2 * q, 0, P);
    const uint32_t d0 = r * PV_BC2_RUN;
    pv_bc2_build_run(DevBc2Row{reinterpret_cast<uint32_t*>(wtab + ((uint64_t)slot * PV_KW_POS + q) * PV_KW_ENT * 8)},
                     DevBc2Scratch{scr + ((uint64_t)jj * PV_KW_POS + q) * PV_KW_ENT * 10}, P, d0,
                     min(PV_BC2_RUN, PV_KW_ENT - d0));
}

// XCD-aware block order. Workgroups are dealt round-robin over the 8 XCDs (block b runs on the XCD
// of b % 8; MI355X_MICROARCH.md, workgroup dispatch), each XCD with its own 4 MB L2. Slot order is
// key-sorted, so mapping the blocks of XCD x to ONE contiguous range of slots keeps a key's table
// rows in one L2 instead of fetching them into all eight. A bijection on [0, gridDim.x).
#ifndef PV_XCD_REMAP
#define PV_XCD_REMAP 1
#endif
__device__ __forceinline__ uint32_t pv_xcd_block() {
#if PV_XCD_REMAP
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
#else
    return blockIdx.x;
#endif
}

// Second half: Q = acc + [k](-A) from the key's comb table (32 additions, no doublings), projective
// Q to q rows 0..29; the key's own libsodium checks are folded into flags[i] here.
__device__ __forceinline__ void pv_comb_a_from(const Work& wk, const KeyWork& kw, uint32_t i, const ge_p3& acc,
                                               uint4* stg_wave) {
    const uint32_t id = kw.skey[i];  // comb index
    const uint32_t cslot = kw.comb_cslot[id];
    const bool xt = cslot != PV_EMPTY && (cslot & PV_CSLOT_XT);
    const uint4* ktab = cslot == PV_EMPTY ? kw.ctab + (uint64_t)id * PV_COMB_POS * PV_COMB_ENT * 10
                        : xt ? kw.xt_tab + (uint64_t)(cslot & ~PV_CSLOT_XT) * PV_COMB_POS * PV_COMB_ENT * 10
                             : kw.kc_tab + (uint64_t)cslot * PV_COMB_POS * PV_COMB_ENT * 10;
    const Soa qs(wk.q, 40, wk.stride);
    const DevDigits dig{wk.digits, (uint32_t)wk.stride, i};
    fe X, Y, Z;
#if PV_COMB_PIPELINE
    // a cached key with affine rows: additions without the Z1 Z2 product (comb.h pv_comb_row_to_affine)
    const bool aff = cslot != PV_EMPTY && !xt && kw.kc_ntab;
    if (aff) ktab = kw.kc_ntab + (uint64_t)cslot * PV_COMB_POS * PV_COMB_ENT * 10;
    pv_comb_a_xyz_staged(X, Y, Z, acc, DevCombStage{ktab, stg_wave, threadIdx.x & 63u, aff}, dig);
#else
    const DevCombRows arows{const_cast<uint4*>(ktab)};
    pv_comb_a_xyz(X, Y, Z, acc, arows, dig);
#endif
    if (kw.key_flag[id] == 0) wk.flags[i] = 0;
#pragma unroll
    for (int q = 0; q < 10; q++) {
        qs.st(q, i, X.v[q]);
        qs.st(10 + q, i, Y.v[q]);
        qs.st(20 + q, i, Z.v[q]);
    }
}

// comb_a after a separate pv_comb_b_kernel: acc = [S]B from q rows 0..39 (or qb, PV_COMB_B_EARLY).
__device__ __forceinline__ void pv_comb_a_slot(const Work& wk, const KeyWork& kw, uint32_t i, uint4* stg_wave) {
    const uint32_t S = (uint32_t)wk.stride;
    const Soa qs(wk.q, 40, wk.stride);
    ge_p3 acc;
#if PV_COMB_B_EARLY
    {
        const uint4* a = wk.qb + (uint64_t)kw.slot_req[i] * 10u;  // [S]B of the slot's request
        uint32_t w[40];
#pragma unroll
        for (int q = 0; q < 10; q++) {
            const uint4 v = a[q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int q = 0; q < 10; q++) {
            acc.X.v[q] = w[q];
            acc.Y.v[q] = w[10 + q];
            acc.Z.v[q] = w[20 + q];
            acc.T.v[q] = w[30 + q];
        }
    }
#else
#pragma unroll
    for (int q = 0; q < 10; q++) {
        acc.X.v[q] = qs.ld(q, i);
        acc.Y.v[q] = qs.ld(10 + q, i);
        acc.Z.v[q] = qs.ld(20 + q, i);
        acc.T.v[q] = qs.ld(30 + q, i);
    }
#endif
    (void)S;
    pv_comb_a_from(wk, kw, i, acc, stg_wave);
}

__global__ __launch_bounds__(PV_BLOCK, PV_COMB_A_MINBLOCKS) void pv_comb_a_kernel(uint64_t n, Work wk, KeyWork kw,
                                                                               Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t i = pv_xcd_block() * PV_BLOCK + threadIdx.x;  // slot
    if (i >= gate.ncomb()) return;
    if (pv_kw_rows(kw, i)) {  // pv_comb_b_kernel added [k](-A) from the key's wide rows: Q is in q rows 0..29
        if (kw.key_flag[kw.skey[i]] == 0) wk.flags[i] = 0;
        return;
    }
    __shared__ uint4 stg[PV_BLOCK / 64][10][64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    pv_comb_a_slot(wk, kw, i, &stg[wv][0][0]);
}

// [S]B and [k](-A) of a comb slot in ONE kernel (PV_COMB_FUSED): the 10 niels additions from the wide
// fixed-base comb (random 128 B entries in HBM, LDS-staged one addition ahead in the first 8 rows of
// the wave's staging area) run inside the issue-bound comb kernel, where the other waves of the SIMD
// cover their fetch latency, instead of as a latency-bound kernel of their own between comb_prep and
// the per-key tables; and acc never round-trips through q. The kernel then starts as soon as the
// per-key tables are built.
#ifndef PV_COMB_FUSED
#define PV_COMB_FUSED 1
#endif
// ... for chunks above this many requests. Below it the two-kernel form stays: a small chunk's [S]B
// kernel is a latency-bound chain of 10 dependent HBM lookups that the split form hides beside the
// table fill, while the fused kernel would add it after the fill (4,096-32,768-request calls were
// 0.08-0.12 ms slower fused).
#ifndef PV_FUSED_MIN_REQ
#define PV_FUSED_MIN_REQ 262144
#endif
// Diagnostic build only (PV_CLOCK_PROBE=1, tools/clock_probe.py; MI355X_MICROARCH "DVFS give-back"
// item 6): wave 0 of every comb_ab workgroup stamps the shader clock (s_memtime) and the 100 MHz
// constant clock (s_memrealtime) at entry and exit into a buffer of its own, which no other code reads;
// the in-kernel clock is the median over workgroups of delta-memtime / delta-realtime x 100 MHz. The
// product build compiles no stamp.
#ifndef PV_CLOCK_PROBE
#define PV_CLOCK_PROBE 0
#endif
#if PV_CLOCK_PROBE
static constexpr uint32_t PV_CLOCK_SLOTS = 16384;  // workgroups stamped (block index mod this)
__device__ uint64_t pv_clock_stamps[PV_CLOCK_SLOTS * 4];
__device__ __forceinline__ void pv_clock_stamp(uint64_t& t, uint64_t& r) {
    __builtin_amdgcn_sched_barrier(0);
    t = __builtin_amdgcn_s_memtime();
    r = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) alone
    __builtin_amdgcn_sched_barrier(0);
}
#endif

#ifndef PV_COMB_AB_PRIO
#define PV_COMB_AB_PRIO 0
#endif
// 0: off; k: the last 1/k of the grid at priority 1. Measured slower (base 393.5-400.9 M/s, last 1/4
// 391.4-394.6, last 1/8 385.9-397.6: profiles/r06/ab/ab_comb_ab_tail_prio.txt): off
#ifndef PV_COMB_AB_TAIL_PRIO
#define PV_COMB_AB_TAIL_PRIO 0
#endif
// Workgroup size of the fused comb kernel (A/B knob): its waves share nothing (each stages its own
// rows in its own 10 KB of LDS), so one-wave workgroups release a slot per wave instead of per four.
// Measured: 64 within noise of 256, 128 3 % slower (profiles/r06/ab/ab_comb_ab_block.txt); 256 kept.
#ifndef PV_COMB_AB_BLOCK
#define PV_COMB_AB_BLOCK PV_BLOCK
#endif
template <int W>
__global__ __launch_bounds__(PV_COMB_AB_BLOCK, PV_COMB_A_MINBLOCKS) void pv_comb_ab_kernel(uint64_t n, Work wk,
                                                                                        KeyWork kw,
                                                                                        const uint4* __restrict__ bcomb,
                                                                                        Gate gate) {
    if (!gate.keyed() || gate.off()) return;
    const uint32_t i = pv_xcd_block() * PV_COMB_AB_BLOCK + threadIdx.x;  // slot
    if (i >= gate.ncomb()) return;
#if PV_CLOCK_PROBE
    uint64_t t0 = 0, r0 = 0;
    pv_clock_stamp(t0, r0);
#endif
    __shared__ uint4 stg[PV_COMB_AB_BLOCK / 64][10][64];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DevDigits dig{wk.digits, (uint32_t)wk.stride, i};
    ge_p3 acc;
    const uint4* wkey = pv_kw_rows(kw, i);
#if PV_COMB_AB_PRIO  // A/B knob: the [S]B phase at a higher issue priority than the [k](-A) phase
    __builtin_amdgcn_s_setprio(PV_COMB_AB_PRIO);
#endif
#if PV_COMB_AB_TAIL_PRIO  // A/B knob: the workgroups dispatched last (the final round) at a higher priority
    if (blockIdx.x >= gridDim.x - gridDim.x / PV_COMB_AB_TAIL_PRIO) __builtin_amdgcn_s_setprio(1);
#endif
    pv_comb_bw_acc<W>(acc, bcomb, wkey, dig, &stg[wv][0][0]);
#if PV_COMB_AB_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    if (wkey)  // [k](-A) came from the key's wide rows in the same loop
        pv_comb_store_q(wk, kw, i, acc);
    else
        pv_comb_a_from(wk, kw, i, acc, &stg[wv][0][0]);
#if PV_CLOCK_PROBE
    uint64_t t1 = 0, r1 = 0;
    pv_clock_stamp(t1, r1);
    if (threadIdx.x == 0) {
        uint64_t* o = pv_clock_stamps + 4ull * (blockIdx.x % PV_CLOCK_SLOTS);
        o[0] = t0;
        o[1] = t1;
        o[2] = r0;
        o[3] = r1;
    }
#endif
}

// Kernel 3: encode Q for B requests per lane with one shared inversion, compare with R, one __ballot
// per request group. Wave w covers requests [64 B w, 64 B (w + 1)): lane l handles 64 B w + l + 64 t,
// t = 0..B-1, so every load is coalesced and group t's ballot is verdict word B w + t. Points are
// re-read from q rather than held. B = 16 (two groups of 8 under one inversion, verify_core.h) for
// chunks of >= PV_ENC16_MIN requests, else PV_ENC_SMALL_B = 8. With each lane's own inversion chain 16
// won at 1M requests (0.185-0.190 ms against 0.191-0.198 for 2,048 waves of 8, profiles/r05/
// ab_encode_prefetch.txt); with the wave's limb-parallel inversion 8 wins everywhere (0.145-0.148 vs
// 0.159-0.161 ms at 1M, 4 per lane 0.185-0.191: profiles/r06/ab/ab_encode_batch.txt), so 16 is off.
#ifndef PV_ENC_SMALL_B
#define PV_ENC_SMALL_B 8
#endif
#ifndef PV_ENC16_MIN
#define PV_ENC16_MIN 0xffffffffu
#endif
template <int B>
struct DevEncSrc {
    Soa q;
    uint32_t w, l;
    uint64_t n;
    __device__ __forceinline__ uint32_t req(int t) const {
        const uint32_t r = w * (64u * B) + l + 64 * t;
        return r < n ? r : 0;
    }
    __device__ __forceinline__ void z(int t, fe& o) const {
        const uint32_t r = req(t);
#pragma unroll
        for (int k = 0; k < 10; k++) o.v[k] = q.ld(20 + k, r);
    }
    __device__ __forceinline__ void xy(int t, fe& x, fe& y) const {
        const uint32_t r = req(t);
#pragma unroll
        for (int k = 0; k < 10; k++) {
            x.v[k] = q.ld(k, r);
            y.v[k] = q.ld(10 + k, r);
        }
    }
};
template <int B>
struct DevEncSink {
    const uint8_t* sm;
    const uint64_t* off;
    uint64_t* verdict;
    const uint32_t* slot_req;  // comb path: slot -> request (verdict words are then slot-ordered)
    uint32_t w, l;
    uint64_t n;
    __device__ __forceinline__ void operator()(int t, const uint32_t enc[8], bool use) const {
        const uint32_t r = w * (64u * B) + l + 64 * t;
        const uint32_t rr0 = r < n ? r : 0;
        const uint32_t rr = slot_req ? slot_req[rr0] : rr0;
        const uint64_t raddr = reinterpret_cast<uint64_t>(sm + off[rr]);
        const DevMsg mw{reinterpret_cast<const uint32_t*>(raddr & ~3ull), (uint32_t)(raddr & 3)};
        uint32_t R[8];
#pragma unroll
        for (int q = 0; q < 8; q++) R[q] = mw.dw(q);
        const bool ok = use && pv_words_equal(enc, R);
        const uint64_t bits = __ballot(ok);
        const uint32_t r0 = w * (64u * B) + 64 * t;
        if (l == 0 && r0 < n) verdict[r0 >> 6] = bits;
    }
};
// The encode's one inversion per lane done by the whole wave (PV_ENC_WAVE_INV): the 64 lanes' products
// are multiplied pairwise across lanes (xor partners 32, 16, 8, 4, and 2 with PV_ENC_INV_DUAL) down to
// four products, one per lane residue mod 4 (two, mod 2), which are inverted at once in limb-parallel form
// (lp_invert: row r = the product of the lanes = r mod 4; DUAL: rows 0, 1 the two products, repeated in
// rows 2, 3, and five column terms per lane, a shorter dependent chain per product), and the inverses
// walked back down the same tree (one product per level). Where every lane ran its own ~27k-instruction
// exponentiation chain (the chain's latency was most of the kernel's time), the wave now runs ~265
// limb-parallel products. Every lane of the wave must be active (pv_encode_kernel: all lanes run the batch).
#ifndef PV_ENC_WAVE_INV
#define PV_ENC_WAVE_INV 1
#endif
#ifndef PV_ENC_INV_DUAL
#define PV_ENC_INV_DUAL 1
#endif
// A/B knob: one chain per workgroup (its 4 waves' products shared through LDS). Parity-green; encode stage
// 0.139-0.141 vs 0.143-0.145 ms, step within noise (profiles/r06/ab/ab_encode_wg_inv.txt): off, no barrier
#ifndef PV_ENC_WG_INV
#define PV_ENC_WG_INV 0
#endif
__device__ __forceinline__ void pv_shfl_xor_fe(fe& o, const fe& a, int m) {
#pragma unroll
    for (int k = 0; k < 10; k++) o.v[k] = __shfl_xor(a.v[k], m);
}
struct PvWaveInvert {
    __device__ void operator()(fe& x) const {
#if LP_DEVICE
        constexpr int LV = PV_ENC_INV_DUAL ? 5 : 4;  // tree levels
        constexpr uint32_t RES = PV_ENC_INV_DUAL ? 1u : 3u;  // lane residue a row's product covers
        const uint32_t lane = threadIdx.x & 63u;
        constexpr int M[5] = {32, 16, 8, 4, 2};
        fe p[LV + 1], q;
        p[0] = x;
#pragma unroll
        for (int i = 0; i < LV; i++) {
            pv_shfl_xor_fe(q, p[i], M[i]);
            fe_mul(p[i + 1], p[i], q);
        }
        const LpLane c = LpLane::make();
        const int src = (int)((lane >> 4) & RES);
        fe inv;
#if PV_ENC_WG_INV
        // the workgroup's waves share ONE chain: their (two) products meet in LDS, wave 0 inverts the
        // workgroup's products, and each wave takes its own inverse as that times the other waves' products
        static_assert(PV_ENC_INV_DUAL, "PV_ENC_WG_INV: the dual-row form (two products per wave)");
        constexpr int NW = PV_BLOCK / 64;
        __shared__ uint32_t wg_p[NW][2][10];
        __shared__ uint32_t wg_inv[2][10];
        const uint32_t wv = threadIdx.x >> 6, r = lane & 1u;
        if (lane < 2) {
#pragma unroll
            for (int k = 0; k < 10; k++) wg_p[wv][lane][k] = p[LV].v[k];
        }
        __syncthreads();
        fe others;  // the product of the other waves' products of residue r
        bool have = false;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            if ((uint32_t)w == wv) continue;
            fe o;
#pragma unroll
            for (int k = 0; k < 10; k++) o.v[k] = wg_p[w][r][k];
            if (have) fe_mul(others, others, o);
            else others = o;
            have = true;
        }
        if (wv == 0) {  // wave-uniform
            fe tot;
            fe_mul(tot, others, p[LV]);
            uint32_t z = 0;
#pragma unroll
            for (int k = 0; k < 10; k++) {
                const uint32_t t = __shfl(tot.v[k], src);
                z = (lane & 15u) == (uint32_t)k ? t : z;
            }
            const lu zi = lp_invert<true>(c, lu(z));
            if ((lane >> 4) < 2u && (lane & 15u) < 10u) wg_inv[lane >> 4][lane & 15u] = static_cast<uint32_t>(zi);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 10; k++) inv.v[k] = wg_inv[r][k];
        fe_mul(inv, inv, others);
#else
        // row r (lanes 16 r + k) gets limb k of lane (r & RES)'s product
        uint32_t z = 0;
#pragma unroll
        for (int k = 0; k < 10; k++) {
            const uint32_t t = __shfl(p[LV].v[k], src);
            z = (lane & 15u) == (uint32_t)k ? t : z;
        }
        const lu zi = lp_invert<PV_ENC_INV_DUAL != 0>(c, lu(z));
#pragma unroll
        for (int k = 0; k < 10; k++) inv.v[k] = __shfl(static_cast<uint32_t>(zi), (int)(16u * (lane & RES)) + k);
#endif
#pragma unroll
        for (int i = LV - 1; i >= 0; i--) {
            pv_shfl_xor_fe(q, p[i], M[i]);
            fe_mul(inv, inv, q);
        }
        x = inv;
#else
        fe_invert(x, x);
#endif
    }
};

template <int B>
__global__ __launch_bounds__(PV_BLOCK, 2) void pv_encode_kernel(const uint8_t* __restrict__ sm,
                                                                 const uint64_t* __restrict__ off, uint64_t n,
                                                                 Work wk, uint64_t* __restrict__ verdict,
                                                                 KeyWork kw, Gate gate) {
    if (gate.off()) return;
    const bool comb = gate.keyed();  // slot order
    const uint32_t g = blockIdx.x * PV_BLOCK + threadIdx.x;
    const uint32_t w = g >> 6, l = g & 63;
    const DevEncSrc<B> src{Soa(wk.q, 40, wk.stride), w, l, n};
    bool use[B];
#pragma unroll
    for (int t = 0; t < B; t++) {
        const uint32_t r = w * (64u * B) + l + 64 * t;
        use[t] = r < n && wk.flags[r < n ? r : 0] != 0;
    }
#if PV_ENC_WAVE_INV
    pv_encode_batch_stream_b<B>(src, use, DevEncSink<B>{sm, off, comb ? kw.sverdict : verdict,
                                                        comb ? kw.slot_req : nullptr, w, l, n}, PvWaveInvert{});
#else
    pv_encode_batch_stream_b<B>(src, use, DevEncSink<B>{sm, off, comb ? kw.sverdict : verdict,
                                                        comb ? kw.slot_req : nullptr, w, l, n});
#endif
}

// ------------------------------------------------------------------------------------------ host

namespace {

struct Ctx {
    int device = -1;
    int cus = 0;
    hipStream_t stream = nullptr;
    hipStream_t kstream = nullptr;           // per-key pipeline (chain + table fill), overlapped
    hipEvent_t ev_keys_ready = nullptr;      // dedup done (main -> Straus side stream)
    hipEvent_t ev_scan_done = nullptr;       // comb keys chosen (main -> kstream, before the scatter)
    hipEvent_t ev_tables_ready = nullptr;    // comb tables done (fstream -> main)
    hipStream_t fstream = nullptr;           // table fill, one launch per chain part
    hipEvent_t ev_chain[PV_CHAIN_PARTS] = {};  // chain part done (kstream -> fstream)
    hipEvent_t ev_prep_done = nullptr;        // comb_prep done: need masks ready (main -> fstream)
    hipStream_t bstream = nullptr;           // [S]B per request of a keyed chunk (PV_COMB_B_EARLY)
    hipEvent_t ev_b_start = nullptr, ev_b_done = nullptr;
    hipStream_t sstream = nullptr;           // Straus-path slots of a split chunk, overlapped
    hipEvent_t ev_straus_done = nullptr;     // their q / flags written (sstream -> main)
    // Workspace hand-over between callers' streams: every launch ends by recording ev_launch_done
    // on its stream; a launch on a DIFFERENT stream first makes its stream wait for it, so two
    // batches enqueued on two caller streams never share the workspace at the same time.
    hipEvent_t ev_launch_done = nullptr;
    hipStream_t last_stream = nullptr;
    uint32_t* d_btab = nullptr;
    Work work{nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr};
    KeyWork kw{};
    bool last_keyed = false;  // the most recent chunk ran the dedup / split kernels
    bool slots_dirty = true;  // the key hash table / need masks may hold entries (cleared before use)
    bool last_latency = false;  // the most recent launch took the latency path
    bool verdict_zeroed = false;  // the caller's verdict words are already 0 (pv_verify_batch)
    bool keyed_hint = false;      // pv_verify_batch saw few distinct keys: keyed path below PV_LATENCY_MAX
    bool hint_set = false;        // pv_verify_batch decided keyed_hint on the host (no device-side choice)
    bool last_dev_choice = false; // the last launch let its dedup pick latency vs keyed
    uint32_t last_split[3] = {0, 0, 0};  // PV_SPLIT_* of it, read back by pv_last_path
    uint4* d_bcomb = nullptr;  // fixed-base comb T_B (radix 65536; latency path)
    uint4* d_bc2 = nullptr;    // wide fixed-base comb T_B2 (radix 2^W; comb path's [S]B)
    int bc2_w = PV_BC2_W;      // its radix: PV_BC2_W, or 16 when d_bc2 aliases d_bcomb (fallback)
    uint32_t prep_lds_pad = PV_PREP_LDS_PAD;  // dynamic LDS per comb_prep workgroup (occupancy cap)
    int path = PV_PATH_AUTO;
    // host-entry staging
    uint8_t* h_stage = nullptr;  // pinned
    uint64_t h_stage_cap = 0;
    uint8_t* d_stage = nullptr;
    uint64_t d_stage_cap = 0;
    uint64_t* h_ver = nullptr;  // pinned verdict words of the pipelined host-buffer form
    uint64_t h_ver_cap = 0;
    // pipelined host-buffer form: H2D of sub-batch j on cstream, its kernels on `stream` after ev_copy[j]
    hipStream_t cstream = nullptr;
    hipEvent_t ev_cstart = nullptr;  // the engine stream's work so far (cstream waits: staging reuse)
    std::vector<hipEvent_t> ev_copy;
    int inject_stage = 0;  // pv_test_inject(PV_INJECT_STAGE): host-buffer stagings left to fail
    // the comb tables one pipelined host call's sub-batches share (pv_xtab_publish_kernel): room for
    // PV_XT_KEYS keys, allocated on first use; xt_fill: the next chunk builds its tables here and
    // publishes them; xt_use: the next chunks look keys up here (as in the node-side key cache)
    struct {
        uint32_t* htab = nullptr;
        uint32_t* keys = nullptr;
        uint32_t* flags = nullptr;
        uint4* tab = nullptr;
        bool failed = false;  // allocation failed once: the call's sub-batches build their own tables
    } xt;
    bool xt_fill = false, xt_use = false;
    bool timing = false;
    // PV_NSTAGES + 1 events per chunk launched since pv_set_timing(1) (stage boundaries, see
    // pv_stage_times); unused stages record back-to-back events
    std::vector<hipEvent_t> ev;
    int ev_used = 0;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // node-side key cache (keycache.h): device arrays + host index (LRU, most recent first)
    struct {
        uint32_t cap = 0;
        uint32_t* d_htab = nullptr;
        uint32_t* d_keys = nullptr;
        uint32_t* d_flags = nullptr;
        uint4* d_tab = nullptr;
        uint4* d_ntab = nullptr;      // the tables with every entry divided by its Z (comb path), or null
        uint4* d_wtab = nullptr;      // radix-65536 niels rows of slots < wcap (comb.h PV_KW_*), or null
        uint32_t wcap = 0;
        uint32_t* d_wscr = nullptr;   // Z products of one group of wide-row builds
        uint8_t* d_put_pk = nullptr;  // keys of one put batch
        uint32_t* d_put_slot = nullptr;
        uint32_t hmask = 0, seed = 0;
        bool enabled = true;  // consulted by the latency path
        std::unordered_map<std::string, std::list<uint32_t>::iterator> index;  // key bytes -> LRU node
        std::list<uint32_t> lru;                                                 // slots, most recent first
        std::vector<std::string> slot_key;
        std::vector<uint32_t> free_slots;
        bool broken = false;  // a failed hash-table upload left the device table stale: not consulted
        // automatic admission (pv_key_cache_auto): a key is put on its auto_min-th VERIFIED appearance
        // in pv_verify_batch calls (every request of calls of <= PV_KC_AUTO_MAX_BATCH requests, a
        // sample of larger ones). Appearances are counted in a SipHash-keyed table of full keys with
        // bounded probing (kc_admit.h); an evicted key is forgotten there, so it can be re-admitted
        uint32_t auto_min = 0;
        pvhost::AdmitTable seen;
        uint64_t auto_admitted = 0, auto_failed = 0;
        // LRU refresh on use: every launch that consults the cache stamps the slots it reads with its
        // epoch (d_stamp, pv_kc_lookup); before a put evicts, the slots stamped since the last fold
        // move to the front of the host LRU (kc_fold_hits)
        uint32_t* d_stamp = nullptr;
        uint32_t epoch = 1, fold_epoch = 1;
        // pinned staging of an asynchronous put (keys, slots, hash table), reused once ev_async is done
        uint8_t* h_async = nullptr;
        uint64_t h_async_cap = 0;
        hipEvent_t ev_async = nullptr;
        bool async_pending = false;
    } kc;
    // zero-copy verdict bytes (pinned, coherent: the host reads them while the kernel runs)
    uint8_t* h_zc_verdict = nullptr;
    bool last_zero_copy = false;  // the most recent pv_verify_batch took the zero-copy form
    // pv_verify_batch_multi_gpu: this device's gathered verdict words (device) and their host copy
    uint64_t* d_mg = nullptr;
    uint64_t d_mg_words = 0;
    uint64_t* h_mg = nullptr;
    uint64_t h_mg_words = 0;
    const uint32_t* last_nkeys = nullptr;  // split counters of the most recent keyed chunk
};

// One context per device. The single-device ABI (pv_init, pv_verify_batch, ...) works on the device
// pv_init bound (the primary); pv_init_devices adds contexts for more devices of the same process,
// which pv_verify_batch_multi_gpu drives from one worker thread per device. g_ctx / g_mu name the
// calling thread's context: a multi-GPU worker's device (t_dev), else the primary.
constexpr int PV_MAX_DEV = 16;
Ctx g_ctxs[PV_MAX_DEV];
std::mutex g_mus[PV_MAX_DEV];
std::atomic<int> g_primary{-1};
thread_local int t_dev = -1;
inline int pv_cur_dev() {
    if (t_dev >= 0) return t_dev;
    const int p = g_primary.load(std::memory_order_acquire);
    return p >= 0 ? p : 0;
}
#define g_ctx (g_ctxs[pv_cur_dev()])
#define g_mu (g_mus[pv_cur_dev()])
// Makes `dev` the calling thread's context for the scope (multi-GPU workers, per-device init).
struct DevScope {
    int prev;
    explicit DevScope(int dev) : prev(t_dev) { t_dev = dev; }
    ~DevScope() { t_dev = prev; }
};
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define PV_HIP(call, code)                                                                     \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) return fail(code, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

PvKeyCacheView kc_view() {
    auto& k = g_ctx.kc;
    PvKeyCacheView v{k.d_htab, k.d_keys, k.d_flags, k.d_tab, 0u, k.seed, k.d_wtab, k.wcap};
    if (k.enabled && !k.broken && k.cap > 0 && !k.index.empty()) {
        v.hmask = k.hmask;
        v.stamp = k.d_stamp;
        v.epoch = ++k.epoch;
    }
    return v;
}

void kc_free() {
    auto& k = g_ctx.kc;
    for (void* p : {(void*)k.d_htab, (void*)k.d_keys, (void*)k.d_flags, (void*)k.d_tab, (void*)k.d_ntab,
                    (void*)k.d_wtab, (void*)k.d_wscr, (void*)k.d_put_pk, (void*)k.d_put_slot, (void*)k.d_stamp})
        if (p) (void)hipFree(p);
    k.d_htab = k.d_keys = k.d_flags = k.d_put_slot = k.d_wscr = k.d_stamp = nullptr;
    k.d_tab = k.d_ntab = k.d_wtab = nullptr;
    k.wcap = 0;
    k.d_put_pk = nullptr;
    if (k.async_pending && k.ev_async) (void)hipEventSynchronize(k.ev_async);
    k.async_pending = false;
    if (k.h_async) (void)hipHostFree(k.h_async);
    k.h_async = nullptr;
    k.h_async_cap = 0;
    k.cap = k.hmask = 0;
    k.broken = false;
    k.seen.reset();
    k.epoch = k.fold_epoch = 1;
    k.index.clear();
    k.lru.clear();
    k.slot_key.clear();
    k.free_slots.clear();
}

// Rebuild the open-addressing table from the index and upload it (stream-ordered). hbuf: pinned
// room for hmask + 1 words whose copy the caller lets run asynchronously; nullptr = a local buffer
// and a synchronous upload.
int kc_upload_htab(hipStream_t s, uint32_t* hbuf = nullptr) {
    auto& k = g_ctx.kc;
    std::vector<uint32_t> local;
    uint32_t* h = hbuf;
    if (!h) {
        local.assign((size_t)k.hmask + 1, PV_KC_EMPTY);
        h = local.data();
    } else {
        std::fill(h, h + k.hmask + 1, PV_KC_EMPTY);
    }
    for (auto& e : k.index) {
        uint32_t A[8];
        memcpy(A, e.first.data(), 32);
        uint32_t p = pv_kc_hash(A, k.seed) & k.hmask;
        while (h[p] != PV_KC_EMPTY) p = (p + 1) & k.hmask;
        h[p] = *e.second;
    }
    PV_HIP(hipMemcpyAsync(k.d_htab, h, ((size_t)k.hmask + 1) * 4, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
    if (!hbuf) PV_HIP(hipStreamSynchronize(s), PV_ERR_LAUNCH);  // h is a local buffer
    return PV_OK;
}

int kc_auto_after_batch(const uint8_t* pk, uint64_t n, hipStream_t s, const uint8_t* vb, const uint64_t* hver);

int ensure_stage(uint64_t host_bytes, uint64_t dev_bytes) {
    if (host_bytes > g_ctx.h_stage_cap) {
        if (g_ctx.h_stage) (void)hipHostFree(g_ctx.h_stage);
        g_ctx.h_stage = nullptr;
        const uint64_t cap = std::max<uint64_t>(host_bytes, 1 << 20);
        PV_HIP(hipHostMalloc((void**)&g_ctx.h_stage, cap, hipHostMallocPortable), PV_ERR_ALLOC);
        g_ctx.h_stage_cap = cap;
    }
    if (dev_bytes > g_ctx.d_stage_cap) {
        if (g_ctx.d_stage) (void)hipFree(g_ctx.d_stage);
        g_ctx.d_stage = nullptr;
        const uint64_t cap = std::max<uint64_t>(dev_bytes, 1 << 20);
        PV_HIP(hipMalloc((void**)&g_ctx.d_stage, cap), PV_ERR_ALLOC);
        g_ctx.d_stage_cap = cap;
    }
    return PV_OK;
}

int ensure_events(int count) {
    while ((int)g_ctx.ev.size() < count) {
        hipEvent_t e;
        PV_HIP(hipEventCreate(&e), PV_ERR_NO_DEVICE);
        g_ctx.ev.push_back(e);
    }
    return PV_OK;
}

int launch_chunks(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk, uint64_t* d_verdict,
                  hipStream_t stream);

int lane_alloc_buffers(Work& w, KeyWork& kw);
void lane_free_buffers(Work& w, KeyWork& kw);

int launch_chunk(int c, uint64_t n, const uint8_t* d_sm, const uint64_t* d_off, const uint8_t* d_pk,
                 uint64_t* d_verdict, hipStream_t stream, bool latency, bool dev_choice, int evb);

// A kernel instantiated per wide-comb radix (Bc2<W>), launched for the radix pv_init chose.
#define PV_LAUNCH_BC2(k, ...)                                                                      \
    do {                                                                                           \
        if (g_ctx.bc2_w == 16) hipLaunchKernelGGL(k<16>, __VA_ARGS__);                             \
        else hipLaunchKernelGGL(k<PV_BC2_W>, __VA_ARGS__);                                          \
    } while (0)

// One batch on `stream` (caller holds g_mu). Chunks of at most work.stride requests (a multiple of
// 64, so verdict words never straddle).
int launch(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk, uint64_t* d_verdict,
           hipStream_t stream) {
    if (n == 0) return PV_OK;
    if (g_ctx.last_stream && g_ctx.last_stream != stream)
        PV_HIP(hipStreamWaitEvent(stream, g_ctx.ev_launch_done, 0), PV_ERR_LAUNCH);
    int rc = launch_chunks(d_sm, d_off, n, d_pk, d_verdict, stream);
    // recorded even after a failed enqueue: whatever did get enqueued is covered
    PV_HIP(hipEventRecord(g_ctx.ev_launch_done, stream), PV_ERR_LAUNCH);
    g_ctx.last_stream = stream;
    return rc;
}

int launch_chunks(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk, uint64_t* d_verdict,
                  hipStream_t stream) {
    const uint64_t cap = g_ctx.work.stride;
    const int nchunks = (int)((n + cap - 1) / cap);
    constexpr int NE = PV_NSTAGES + 1;
    // small batches: one wave pair per request (pv_latency.hip); forced LATENCY takes it at any size.
    // Between PV_KEYED_HINT_MIN and PV_LATENCY_MAX requests AUTO picks by key repeats: the host-buffer
    // call counted the keys (keyed_hint, hint_set); a device-buffer call lets the dedup kernels count
    // them and decide on the device (dev_choice: the keyed kernels exit at once and the latency kernel
    // runs when the scan picks latency; no host round trip). A non-empty key cache keeps the latency
    // path there (cached keys make it faster still).
    const bool kc_nonempty = kc_view().hmask != 0;
    const bool dev_choice = g_ctx.path == PV_PATH_AUTO && !g_ctx.hint_set && !kc_nonempty &&
                            n >= PV_KEYED_HINT_MIN && n <= PV_LATENCY_MAX;
    const bool latency = g_ctx.path == PV_PATH_LATENCY ||
                         (g_ctx.path == PV_PATH_AUTO && n <= PV_LATENCY_MAX && !g_ctx.keyed_hint && !dev_choice);
    g_ctx.last_latency = latency;
    g_ctx.last_dev_choice = dev_choice;
    int evb = 0;
    if (g_ctx.timing) {
        evb = g_ctx.ev_used;
        int rc = ensure_events(evb + NE * nchunks);
        if (rc) return rc;
        g_ctx.ev_used = evb + NE * nchunks;
    }
    int rc = PV_OK;
    for (int c = 0; c < nchunks && rc == PV_OK; c++)
        rc = launch_chunk(c, n, d_sm, d_off, d_pk, d_verdict, stream, latency, dev_choice, evb);
    return rc;
}

// kstream (key chain + fill) forks from the main stream right after the scan kernel instead of after
// the scatter (A/B switch; the chain is on the step's critical path, profiles/r06/).
#ifndef PV_FORK_AFTER_SCAN
#define PV_FORK_AFTER_SCAN 1
#endif

// Chunk c of the batch on `stream` (the workspace is the context's; key / fill / side streams join it).
int launch_chunk(int c, uint64_t n, const uint8_t* d_sm, const uint64_t* d_off, const uint8_t* d_pk,
                 uint64_t* d_verdict, hipStream_t stream, bool latency, bool dev_choice, int evb) {
    constexpr int NE = PV_NSTAGES + 1;
    const uint64_t cap = g_ctx.work.stride;
    {
        const uint64_t c0 = (uint64_t)c * cap;
        const uint64_t m = std::min<uint64_t>(cap, n - c0);
        const unsigned grid = (unsigned)((m + PV_BLOCK - 1) / PV_BLOCK);
        hipEvent_t* e = g_ctx.timing ? &g_ctx.ev[evb + NE * c] : nullptr;
        auto mark = [&](int k) -> int {
            if (e) PV_HIP(hipEventRecord(e[k], stream), PV_ERR_LAUNCH);
            return PV_OK;
        };
        int rc = mark(PV_STAGE_KEYS);
        if (rc) return rc;
        if (latency) {
            // one kernel: every stage of the verification inside it (timed as MSM)
            g_ctx.last_keyed = false;
            for (int k = PV_STAGE_PREP; k <= PV_STAGE_MSM; k++)
                if ((rc = mark(k))) return rc;
            rc = pv_latency_launch(d_sm, d_off + c0, m, d_pk + 32 * c0, g_ctx.d_bcomb, kc_view(),
                                   d_verdict + c0 / 64, g_ctx.verdict_zeroed, stream, nullptr);
            if (rc) return rc;
            if ((rc = mark(PV_STAGE_ENCODE)) || (rc = mark(PV_NSTAGES))) return rc;
            return PV_OK;
        }
        // Path split (measured round-1 costs on MI355X): a key's comb table costs ~0.47 us of device
        // time (chain + 4,128-entry fill) and then saves ~10 ns per request against the Straus
        // path (~3 vs ~13 ns), so AUTO gives a table to keys with >= PV_COMB_MIN_REQ requests in
        // the chunk and verifies every other request on the Straus path in the same launch. The
        // split is computed on the device by the dedup/sort kernels (Gate); nothing synchronises.
        // Chunks below PV_KEYED_MIN (the latency path's range; only the tail chunk of a large
        // batch can be that small) skip dedup and go Straus. A key in the node-side key cache has
        // its comb table already built: its requests take the comb path at any count.
        PvKeyCacheView kcv = kc_view();
        PvKeyCacheView xtv{nullptr, nullptr, nullptr, nullptr, 0u, 0u};
        const uint32_t* kc_flags = g_ctx.kc.d_flags;
        const uint4* kc_tab = g_ctx.kc.d_tab;
        const bool node_kc = kcv.hmask != 0;
        bool xt_only = false;
        if (g_ctx.xt_use) {  // a later sub-batch of a pipelined host call: the call's shared tables
            const PvKeyCacheView xv{g_ctx.xt.htab, g_ctx.xt.keys, g_ctx.xt.flags, g_ctx.xt.tab, PV_XT_HASH - 1,
                                    g_ctx.kw.seed};
            if (node_kc) {  // the node cache first, then the shared store for the keys it misses
                xtv = xv;
            } else {        // the shared store is the only view
                kcv = xv;
                kc_flags = g_ctx.xt.flags;
                kc_tab = g_ctx.xt.tab;
                xt_only = true;
            }
        }
        const bool kc_active = kcv.hmask != 0;
        const bool keyed = g_ctx.path == PV_PATH_COMB ||
                           (g_ctx.path == PV_PATH_AUTO &&
                            (m >= PV_KEYED_MIN || g_ctx.keyed_hint || dev_choice || kc_active));
        Gate gate{nullptr, nullptr};
        g_ctx.last_keyed = keyed;
        if (keyed) g_ctx.last_nkeys = g_ctx.kw.nkeys;
        KeyWork kw = g_ctx.kw;
        kw.min_req = g_ctx.path == PV_PATH_COMB ? 1u : (uint32_t)PV_COMB_MIN_REQ;
        kw.kc_on = kc_active ? 1u : 0u;
        kw.chunk_n = (uint32_t)m;
        // a key-id segment holds the owners among its waves (every PV_NSEG-th wave of the chunk)
        kw.seg_cap = (uint32_t)((((m + 63) / 64) + PV_NSEG - 1) / PV_NSEG * 64);
        kw.lat_choice = dev_choice ? 1u : 0u;
        kw.kc_tab = kc_tab;
        kw.kc_ntab = xt_only ? nullptr : g_ctx.kc.d_ntab;
        kw.kc_wtab = xt_only ? nullptr : g_ctx.kc.d_wtab;
        kw.kc_wcap = xt_only ? 0u : g_ctx.kc.wcap;
        kw.xt_flags = xtv.hmask ? g_ctx.xt.flags : nullptr;
        kw.xt_tab = xtv.hmask ? g_ctx.xt.tab : nullptr;
        kw.dense_only = 0;
        if (g_ctx.xt_fill) {  // sub-batch 0 of a pipelined host call: its tables go to the shared store, whole
            kw.ctab = g_ctx.xt.tab;
            kw.kcap = std::min<uint32_t>(kw.kcap, PV_XT_KEYS);
            kw.dense_only = 1;
        }
        const uint32_t limit = kw.kcap;  // comb keys a chunk can hold (launch grids of the key stream)
        const bool direct_fill = PV_CHAIN_MODE == 2 && PV_CHAIN_PARTS == 1 && PV_DIRECT_FILL && m > PV_SPARSE_CHUNK;
        if (keyed) {
            // the hash table and need masks are left empty by the previous keyed chunk (unpermute and
            // sparse fill kernels); after an enqueue failure they may not be, and are cleared here
            if (g_ctx.slots_dirty) {
                PV_HIP(hipMemsetAsync(kw.slot, 0xFF, (uint64_t)(kw.hmask + 1) * 4, stream), PV_ERR_LAUNCH);
                PV_HIP(hipMemsetAsync(kw.slot_cnt, 0, (uint64_t)(kw.hmask + 1) * 4 * PV_RANK_SUB, stream),
                       PV_ERR_LAUNCH);
                PV_HIP(hipMemsetAsync(kw.need, 0, (uint64_t)PV_ALLCOMB_KEYS * PV_COMB_POS * 5 * 4, stream),
                       PV_ERR_LAUNCH);
            }
            g_ctx.slots_dirty = true;  // until this chunk's unpermute kernel is enqueued
#if PV_COMB_B_EARLY
            // [S]B per request on bstream from the chunk's start (after everything already on the
            // main stream, e.g. the previous chunk's comb_a reading qb); joined before comb_a
            auto launch_b_early = [&]() -> int {
                PV_HIP(hipEventRecord(g_ctx.ev_b_start, stream), PV_ERR_LAUNCH);
                PV_HIP(hipStreamWaitEvent(g_ctx.bstream, g_ctx.ev_b_start, 0), PV_ERR_LAUNCH);
                PV_LAUNCH_BC2(pv_comb_b_req_kernel, dim3(grid), dim3(PV_BLOCK), 0, g_ctx.bstream, d_sm, d_off + c0, m,
                              g_ctx.work, g_ctx.d_bc2);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
                PV_HIP(hipEventRecord(g_ctx.ev_b_done, g_ctx.bstream), PV_ERR_LAUNCH);
                return PV_OK;
            };
#ifndef PV_COMB_B_AFTER
#define PV_COMB_B_AFTER 0  // 0: at the chunk's start, 1: after the insert kernel
#endif
            if (PV_COMB_B_AFTER == 0 && (rc = launch_b_early())) return rc;
#endif
            // kw.nkeys is cleared by pv_key_insert_kernel (m >= 1 here: the grid has a thread 0)
            if (PV_KEY_SEED > 0 && m > 16ull * PV_KEY_SEED) {  // small chunks: no contention worth a launch
                const uint64_t ms = std::min<uint64_t>(m, PV_KEY_SEED);
                hipLaunchKernelGGL(pv_key_seed_kernel, dim3((unsigned)((ms + PV_BLOCK - 1) / PV_BLOCK)), dim3(PV_BLOCK), 0,
                                   stream, d_pk + 32 * c0, ms, kw);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
#if PV_INSERT_LDS
            hipLaunchKernelGGL(pv_key_insert_lds_kernel, dim3((unsigned)((m + PV_INS_REQS - 1) / PV_INS_REQS)),
                               dim3(PV_INS_THREADS), 0, stream, d_pk + 32 * c0, m, kw);
#else
            hipLaunchKernelGGL(pv_key_insert_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, d_pk + 32 * c0, m, kw);
#endif
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#if PV_COMB_B_EARLY
            if (PV_COMB_B_AFTER == 1 && (rc = launch_b_early())) return rc;
#endif
            hipLaunchKernelGGL(pv_key_assign_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, kw);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            if (kc_active) {
                hipLaunchKernelGGL(pv_key_cache_probe_kernel, dim3((PV_NSEG * kw.seg_cap + PV_BLOCK - 1) / PV_BLOCK),
                                   dim3(PV_BLOCK), 0, stream, d_pk + 32 * c0,
                                   kw, kcv, xtv);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
            gate = Gate{kw.nkeys, kw.slot_req};
            // key-sorted slot order: comb keys' requests first, then the Straus requests
            hipLaunchKernelGGL(pv_key_scan_kernel, dim3(1), dim3(PV_SCAN_THREADS), 0, stream, kw, kc_flags);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            // the per-key chain (few, long-latency lanes) and the table fill run on kstream, overlapped
            // with the scatter and the per-request prep on the main stream: the chain needs only the
            // scan's comb-key list (comb_key, comb_cslot), so kstream forks before the scatter
#if PV_FORK_AFTER_SCAN
            PV_HIP(hipEventRecord(g_ctx.ev_scan_done, stream), PV_ERR_LAUNCH);
            PV_HIP(hipStreamWaitEvent(g_ctx.kstream, g_ctx.ev_scan_done, 0), PV_ERR_LAUNCH);
#endif
            hipLaunchKernelGGL(pv_key_scatter_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, kw);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            PV_HIP(hipEventRecord(g_ctx.ev_keys_ready, stream), PV_ERR_LAUNCH);
#if !PV_FORK_AFTER_SCAN
            PV_HIP(hipStreamWaitEvent(g_ctx.kstream, g_ctx.ev_keys_ready, 0), PV_ERR_LAUNCH);
#endif
            // a chunk above PV_SPARSE_CHUNK never fills sparsely: chain and fill back to back on kstream
            // and the tables-ready event right after the fill (no event hop to fstream, no gated
            // sparse-fill launch in the dependency chain of the comb kernel)
            // the chain runs in PV_CHAIN_PARTS launches of consecutive positions; the fill of a part
            // runs on fstream as soon as its chain part is done, beside the chain of the next part
#if PV_CHAIN_MODE == 2
            constexpr int parts = PV_CHAIN_PARTS;
#else
            constexpr int parts = 1;
#endif
            const uint64_t items = (uint64_t)limit * (PV_COMB_POS / parts) * PV_COMB_BLOCKS;
            const unsigned fgrid = (unsigned)std::min<uint64_t>((items + PV_BLOCK - 1) / PV_BLOCK, 4096);
            if (direct_fill) {  // one part, no sparse fill possible: the fill follows the chain on kstream
                hipLaunchKernelGGL(pv_key_chain_lp_kernel, dim3(std::min<uint32_t>(limit, PV_LP_CHAIN_BLOCKS)), dim3(64),
                                   0, g_ctx.kstream, d_pk + 32 * c0, kw, gate, 0, PV_COMB_POS);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
                hipLaunchKernelGGL(pv_key_fill_kernel, dim3(fgrid), dim3(PV_BLOCK), 0, g_ctx.kstream, kw, gate, 0,
                                   PV_COMB_POS);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
                PV_HIP(hipEventRecord(g_ctx.ev_tables_ready, g_ctx.kstream), PV_ERR_LAUNCH);
            }
            for (int part = 0; part < parts && !direct_fill; part++) {
                const int lo = part * PV_COMB_POS / parts, hi = (part + 1) * PV_COMB_POS / parts;
#if PV_CHAIN_MODE == 2
                hipLaunchKernelGGL(pv_key_chain_lp_kernel, dim3(std::min<uint32_t>(limit, PV_LP_CHAIN_BLOCKS)), dim3(64),
                                   0, g_ctx.kstream, d_pk + 32 * c0, kw, gate, lo, hi);
#elif PV_CHAIN_MODE == 1
                hipLaunchKernelGGL(pv_key_chain_quad_kernel, dim3((4 * limit + PV_BLOCK - 1) / PV_BLOCK),
                                   dim3(PV_BLOCK), 0, g_ctx.kstream, d_pk + 32 * c0, kw, gate);
#else
                hipLaunchKernelGGL(pv_key_chain_kernel, dim3((limit + PV_BLOCK - 1) / PV_BLOCK), dim3(PV_BLOCK), 0,
                                   g_ctx.kstream, d_pk + 32 * c0, kw, gate);
#endif
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
                PV_HIP(hipEventRecord(g_ctx.ev_chain[part], g_ctx.kstream), PV_ERR_LAUNCH);
                PV_HIP(hipStreamWaitEvent(g_ctx.fstream, g_ctx.ev_chain[part], 0), PV_ERR_LAUNCH);
                hipLaunchKernelGGL(pv_key_fill_kernel, dim3(fgrid), dim3(PV_BLOCK), 0, g_ctx.fstream, kw, gate, lo, hi);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
        }
        if ((rc = mark(PV_STAGE_PREP))) return rc;
        if (keyed) {
            // The Straus-path slots of a split chunk (keys without a table: usually a few
            // thousand one-off requests) run on their own stream beside the comb kernels: their
            // waves take ~1 ms from start to end however few they are, which on the main stream
            // would delay the whole comb path. Their blocks are dispatched from the END of the slot
            // range (where the Straus slots are), and blocks of comb slots exit at once.
            hipStream_t ss = g_ctx.sstream;
#ifndef PV_SIDE_GRID_PER_CU
#define PV_SIDE_GRID_PER_CU 2
#endif
            const unsigned sgrid = std::min<unsigned>(
                grid, std::max(1u, (unsigned)(PV_SIDE_GRID_PER_CU * std::max(1, g_ctx.cus))));
            PV_HIP(hipStreamWaitEvent(ss, g_ctx.ev_keys_ready, 0), PV_ERR_LAUNCH);
#ifndef PV_AB_NO_SIDE  // measurement-only switch: drops the Straus side (wrong verdicts if it has work)
            PV_LAUNCH_BC2(pv_prep_kernel, dim3(sgrid), dim3(PV_BLOCK), 0, ss, d_sm, d_off + c0, m,
                               d_pk + 32 * c0, g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#if PV_STRAUS_HALF
            PV_LAUNCH_BC2(pv_split_kernel, dim3(sgrid), dim3(PV_BLOCK), 0, ss, d_sm, d_off + c0, m, g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
            hipLaunchKernelGGL(pv_table_kernel, dim3(sgrid), dim3(PV_BLOCK), 0, ss, d_sm, d_off + c0, m, d_pk + 32 * c0,
                               g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#if PV_STRAUS_WIDE_B
#if !PV_MSM_FUSED_B
            PV_LAUNCH_BC2(pv_straus_b_kernel, dim3(sgrid), dim3(PV_BLOCK), 0, ss, m, g_ctx.work, g_ctx.d_bc2, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
#endif
            PV_LAUNCH_BC2(pv_msm_kernel, dim3(sgrid), dim3(PV_BLOCK), 0, ss, d_sm, d_off + c0, m, g_ctx.d_btab,
                          g_ctx.work, g_ctx.d_bc2, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
            PV_HIP(hipEventRecord(g_ctx.ev_straus_done, ss), PV_ERR_LAUNCH);
#if PV_PREP_REQ_ORDER
            PV_LAUNCH_BC2(pv_comb_prep_req_kernel, dim3(grid), dim3(PV_BLOCK), g_ctx.prep_lds_pad, stream, d_sm,
                          d_off + c0, m, d_pk + 32 * c0, g_ctx.work, kw, gate);
#else
            PV_LAUNCH_BC2(pv_comb_prep_kernel, dim3(grid), dim3(PV_BLOCK), g_ctx.prep_lds_pad, stream, d_sm,
                          d_off + c0, m, d_pk + 32 * c0, g_ctx.work, kw, gate);
#endif
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            if (!direct_fill) {
                // a small chunk's sparse table fill (needs the chain's bases and the need masks comb_prep
                // writes) runs on fstream after the full fill; for a large chunk it exits at once
                PV_HIP(hipEventRecord(g_ctx.ev_prep_done, stream), PV_ERR_LAUNCH);
                PV_HIP(hipStreamWaitEvent(g_ctx.fstream, g_ctx.ev_prep_done, 0), PV_ERR_LAUNCH);
                hipLaunchKernelGGL(pv_key_fill_sparse_kernel, dim3(PV_ALLCOMB_KEYS * PV_COMB_POS / PV_BLOCK),
                                   dim3(PV_BLOCK), 0, g_ctx.fstream, kw, gate);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
                PV_HIP(hipEventRecord(g_ctx.ev_tables_ready, g_ctx.fstream), PV_ERR_LAUNCH);
            }
#if PV_PREP_REQ_ORDER
            // the per-request results to slot-ordered rows, while the key stream finishes the tables
            PV_LAUNCH_BC2(pv_comb_digits_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, g_ctx.work, kw, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
            if ((rc = mark(PV_STAGE_TABLE))) return rc;
            const bool fused = PV_COMB_FUSED && !PV_COMB_B_EARLY && m > PV_FUSED_MIN_REQ;
#if PV_COMB_B_EARLY
            PV_HIP(hipStreamWaitEvent(stream, g_ctx.ev_b_done, 0), PV_ERR_LAUNCH);
#else
            if (!fused) {  // [S]B while the key stream finishes the tables, then join
                PV_LAUNCH_BC2(pv_comb_b_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, g_ctx.work, kw, g_ctx.d_bc2,
                              gate);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
#endif
            PV_HIP(hipStreamWaitEvent(stream, g_ctx.ev_tables_ready, 0), PV_ERR_LAUNCH);
            if ((rc = mark(PV_STAGE_MSM))) return rc;
            if (fused)  // [S]B + [k](-A) in one kernel as soon as the tables are built
                PV_LAUNCH_BC2(pv_comb_ab_kernel, dim3((unsigned)((m + PV_COMB_AB_BLOCK - 1) / PV_COMB_AB_BLOCK)),
                              dim3(PV_COMB_AB_BLOCK), 0, stream, m, g_ctx.work, kw, g_ctx.d_bc2, gate);
            else
                hipLaunchKernelGGL(pv_comb_a_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, g_ctx.work, kw, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            PV_HIP(hipStreamWaitEvent(stream, g_ctx.ev_straus_done, 0), PV_ERR_LAUNCH);
        } else {
            PV_LAUNCH_BC2(pv_prep_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m,
                               d_pk + 32 * c0, g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#if PV_STRAUS_HALF
            PV_LAUNCH_BC2(pv_split_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m, g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
            if ((rc = mark(PV_STAGE_TABLE))) return rc;
            hipLaunchKernelGGL(pv_table_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m, d_pk + 32 * c0,
                               g_ctx.work, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#if PV_STRAUS_WIDE_B && !PV_MSM_FUSED_B
            // (run beside the table kernel on the side stream it gains nothing: the table kernel's blocks hold
            // every slot, profiles/r05/ab_straus_fork_b.txt)
            PV_LAUNCH_BC2(pv_straus_b_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, g_ctx.work, g_ctx.d_bc2,
                               gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
#endif
            if ((rc = mark(PV_STAGE_MSM))) return rc;
            PV_LAUNCH_BC2(pv_msm_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m, g_ctx.d_btab,
                          g_ctx.work, g_ctx.d_bc2, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        }
        if ((rc = mark(PV_STAGE_ENCODE))) return rc;
        if (m >= PV_ENC16_MIN) {
            const unsigned egrid = (unsigned)((m + PV_BLOCK * 16 - 1) / (PV_BLOCK * 16));
            hipLaunchKernelGGL(pv_encode_kernel<16>, dim3(egrid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m,
                           g_ctx.work, d_verdict + c0 / 64, kw, gate);
        } else {
            const unsigned egrid = (unsigned)((m + PV_BLOCK * PV_ENC_SMALL_B - 1) / (PV_BLOCK * PV_ENC_SMALL_B));
            hipLaunchKernelGGL(pv_encode_kernel<PV_ENC_SMALL_B>, dim3(egrid), dim3(PV_BLOCK), 0, stream, d_sm, d_off + c0, m,
                           g_ctx.work, d_verdict + c0 / 64, kw, gate);
        }
        PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        if (keyed) {
            hipLaunchKernelGGL(pv_unpermute_kernel, dim3(grid), dim3(PV_BLOCK), 0, stream, m, kw,
                               d_verdict + c0 / 64, gate);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            g_ctx.slots_dirty = false;
            if (g_ctx.xt_fill) {  // publish this chunk's tables for the call's later sub-batches
                hipLaunchKernelGGL(pv_xtab_publish_kernel, dim3(PV_XT_KEYS / PV_BLOCK), dim3(PV_BLOCK), 0, stream,
                                   d_pk + 32 * c0, kw, g_ctx.xt.htab, PV_XT_HASH - 1, g_ctx.kw.seed, g_ctx.xt.keys,
                                   g_ctx.xt.flags);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
            if (dev_choice) {  // runs only when the scan picked latency (the words were zeroed above)
                rc = pv_latency_launch(d_sm, d_off + c0, m, d_pk + 32 * c0, g_ctx.d_bcomb, kc_view(),
                                       d_verdict + c0 / 64, true, stream, kw.nkeys + PV_SPLIT_LAT);
                if (rc) return rc;
            }
        }
        if ((rc = mark(PV_NSTAGES))) return rc;
    }
    return PV_OK;
}

}  // namespace

hipStream_t pv_engine_stream() { return g_ctx.stream; }
int pv_fail(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

int pv_abi_version(void) { return PV_ABI_VERSION; }
uint32_t pv_build_flags(void) { return (PV_COMB_FUSED && !PV_COMB_B_EARLY) ? PV_BUILD_COMB_FUSED : 0u; }

int pv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* pv_last_error(void) { return g_err.c_str(); }

}  // extern "C"

namespace {
int check_device_index(int device, const char* who) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(PV_ERR_NO_DEVICE, std::string(who) + ": no HIP device visible");
    if (device < 0 || device >= ndev || device >= PV_MAX_DEV)
        return fail(PV_ERR_ARG, std::string(who) + ": device index out of range");
    return PV_OK;
}

// The per-lane workspace: per-request rows (Work) and the keyed path's tables (KeyWork), ~15 GB.
int lane_alloc_buffers(Work& w, KeyWork& kw) {
    const uint64_t S = PV_CHUNK;
    w.stride = S;
    PV_HIP(hipMalloc((void**)&w.atab, S * PV_ATAB_ENT * 160), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&w.digits, S * PV_DIGIT_ROWS * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&w.flags, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&w.q, S * 40 * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&w.aos, S * PV_PREP_AOS_QMAX * 16), PV_ERR_ALLOC);
#if PV_COMB_B_EARLY
    PV_HIP(hipMalloc((void**)&w.qb, S * 160), PV_ERR_ALLOC);
#endif
    const uint64_t H = 2 * S;
    kw.hmask = (uint32_t)(H - 1);
    kw.kcap = PV_KEY_CAP;
    kw.seed = (uint32_t)std::random_device{}() | 1u;
    PV_HIP(hipMalloc((void**)&kw.slot, H * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.slot_id, H * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.slot_cnt, H * 4 * PV_RANK_SUB), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.req_key, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.req_rank, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.nkeys, PV_SPLIT_ALLOC_WORDS * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.key_owner, (S + 64 * PV_NSEG) * 4), PV_ERR_ALLOC);  // key ids: segment-major
    PV_HIP(hipMalloc((void**)&kw.key_cid, (S + 64 * PV_NSEG) * 4), PV_ERR_ALLOC);  // key ids: segment-major
    PV_HIP(hipMalloc((void**)&kw.comb_key, (uint64_t)kw.kcap * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.key_flag, (uint64_t)kw.kcap * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.bases, (uint64_t)kw.kcap * PV_COMB_POS * PV_COMB_PTS * 160), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.ctab, (uint64_t)kw.kcap * PV_COMB_POS * PV_COMB_ENT * 160), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.key_count, (S + 64 * PV_NSEG) * 4), PV_ERR_ALLOC);  // key ids: segment-major
    PV_HIP(hipMalloc((void**)&kw.key_cursor, (S + 64 * PV_NSEG) * 4), PV_ERR_ALLOC);  // key ids: segment-major
    PV_HIP(hipMalloc((void**)&kw.slot_req, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.req_pos, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.skey, S * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.sverdict, S / 64 * 8), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.key_cslot, (S + 64 * PV_NSEG) * 4), PV_ERR_ALLOC);  // key ids: segment-major
    PV_HIP(hipMalloc((void**)&kw.comb_cslot, (uint64_t)kw.kcap * 4), PV_ERR_ALLOC);
    PV_HIP(hipMalloc((void**)&kw.need, (uint64_t)PV_ALLCOMB_KEYS * PV_COMB_POS * 5 * 4), PV_ERR_ALLOC);
    PV_HIP(hipMemset(kw.comb_cslot, 0xFF, (uint64_t)kw.kcap * 4), PV_ERR_ALLOC);
    return PV_OK;
}

void lane_free_buffers(Work& w, KeyWork& kw) {
    for (void* p : {(void*)w.atab, (void*)w.digits, (void*)w.flags, (void*)w.q, (void*)w.qb, (void*)w.aos,
                    (void*)kw.slot, (void*)kw.slot_id, (void*)kw.slot_cnt, (void*)kw.req_key, (void*)kw.req_rank,
                    (void*)kw.nkeys, (void*)kw.key_owner, (void*)kw.key_cid, (void*)kw.comb_key, (void*)kw.key_flag,
                    (void*)kw.bases, (void*)kw.ctab, (void*)kw.key_count, (void*)kw.key_cursor, (void*)kw.slot_req,
                    (void*)kw.req_pos, (void*)kw.skey, (void*)kw.sverdict, (void*)kw.key_cslot, (void*)kw.comb_cslot,
                    (void*)kw.need})
        if (p) (void)hipFree(p);
    w = Work{nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr};
    kw = KeyWork{};
}

void ctx_free();
// Builds g_ctxs[device] (caller: g_mus[device] held, DevScope(device) active, context not built yet):
// streams and events, the fixed-base tables, the workspace. Sets the calling thread's HIP device.
bool env_flag_devscope() {
    const char* e = getenv("PV_EVENT_DEVSCOPE");
    return !(e && *e == '0');
}

int ctx_init_parts(int device) {
    PV_HIP(hipSetDevice(device), PV_ERR_NO_DEVICE);
    hipDeviceProp_t prop;
    PV_HIP(hipGetDeviceProperties(&prop, device), PV_ERR_NO_DEVICE);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(PV_ERR_NO_DEVICE, std::string("pv_init: built for gfx950, device is ") + prop.gcnArchName);
    g_ctx.cus = prop.multiProcessorCount;
    PV_HIP(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
#if PV_SIDE_PRIO >= 2
    {
        int least = 0, greatest = 0;
        PV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest), PV_ERR_NO_DEVICE);
        PV_HIP(hipStreamCreateWithPriority(&g_ctx.kstream, hipStreamNonBlocking, greatest), PV_ERR_NO_DEVICE);
    }
#else
    PV_HIP(hipStreamCreateWithFlags(&g_ctx.kstream, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
#endif
    // stream-to-stream hand-overs inside the engine (one device, never read by the host) are recorded with
    // a device-scope release instead of the default system-scope fence: headline step 2.612-2.618 against
    // 2.620-2.624 ms interleaved (profiles/r05/ab_event_devscope.txt); PV_EVENT_DEVSCOPE=0 restores it
    const unsigned evf = hipEventDisableTiming | (env_flag_devscope() ? hipEventReleaseToDevice : 0u);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_keys_ready, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_scan_done, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_tables_ready, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipStreamCreateWithFlags(&g_ctx.fstream, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
    for (auto& e : g_ctx.ev_chain) PV_HIP(hipEventCreateWithFlags(&e, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_prep_done, evf), PV_ERR_NO_DEVICE);
#if PV_SIDE_PRIO
    {
        // Straus-side requests (one-off keys) are a short dependent chain of small grids; a
        // high-priority queue lets their workgroups dispatch ahead of the comb grids so the
        // chain ends before comb_a instead of overlapping it.
        int least = 0, greatest = 0;
        PV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest), PV_ERR_NO_DEVICE);
        PV_HIP(hipStreamCreateWithPriority(&g_ctx.sstream, hipStreamNonBlocking, greatest), PV_ERR_NO_DEVICE);
    }
#else
    PV_HIP(hipStreamCreateWithFlags(&g_ctx.sstream, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
#endif
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_straus_done, evf), PV_ERR_NO_DEVICE);
#if PV_COMB_B_EARLY
    PV_HIP(hipStreamCreateWithFlags(&g_ctx.bstream, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
#endif
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_b_start, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_b_done, evf), PV_ERR_NO_DEVICE);
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_launch_done, evf), PV_ERR_NO_DEVICE);
    {
        // the host path's copy stream at the greatest priority: the runtime keeps such streams on hardware
        // queues of their own instead of round-robin over GPU_MAX_HW_QUEUES (4) with the engine's streams,
        // where a copy sat behind the key stream's table fill (profiles/r05/host_path)
        int least = 0, greatest = 0;
        PV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest), PV_ERR_NO_DEVICE);
        const char* pe = getenv("PV_CSTREAM_PRIO");  // A/B knob: 0 = normal priority
        const bool hi = !(pe && *pe == '0');
        PV_HIP(hipStreamCreateWithPriority(&g_ctx.cstream, hipStreamNonBlocking, hi ? greatest : least), PV_ERR_NO_DEVICE);
    }
    PV_HIP(hipEventCreateWithFlags(&g_ctx.ev_cstart, hipEventDisableTiming), PV_ERR_NO_DEVICE);
    std::vector<uint32_t> bt(PV_BTAB_ENTRIES * PV_BTAB_STRIDE);
    pv_build_b_table(bt.data());
    PV_HIP(hipMalloc((void**)&g_ctx.d_btab, bt.size() * 4), PV_ERR_ALLOC);
    PV_HIP(hipMemcpy(g_ctx.d_btab, bt.data(), bt.size() * 4, hipMemcpyHostToDevice), PV_ERR_ALLOC);
    {
        int rc = lane_alloc_buffers(g_ctx.work, g_ctx.kw);
        if (rc) return rc;
        std::vector<uint32_t> bc((size_t)PV_BCOMB_POS * PV_BCOMB_ENT * PV_BCOMB_STRIDE);
        {
            ge_p3 base[PV_BCOMB_POS];
            pv_bcomb_bases(base);
            std::vector<std::thread> th;
            for (int j = 0; j < PV_BCOMB_POS; j++)
                th.emplace_back(pv_bcomb_build_position, bc.data() + (size_t)j * PV_BCOMB_ENT * PV_BCOMB_STRIDE,
                                std::cref(base[j]));
            for (auto& t : th) t.join();
        }
        PV_HIP(hipMalloc((void**)&g_ctx.d_bcomb, bc.size() * 4), PV_ERR_ALLOC);
        PV_HIP(hipMemcpy(g_ctx.d_bcomb, bc.data(), bc.size() * 4, hipMemcpyHostToDevice), PV_ERR_ALLOC);
        // the wide fixed-base comb, built on the device row by row (one scratch row of Z products)
        {
            const uint64_t rows_ent = (uint64_t)(PV_BC2_POS - 1) * PV_BC2_ENT + PV_BC2_TOP_ENT;
            // not enough HBM for the wide table (a smaller part, several processes on one GPU) or
            // PV_FORCE_BCOMB16 set: [S]B from the radix-65536 comb T_B instead (16 lookups instead of
            // 11, same verdicts; profiles/r02/ab_bcomb_radix.txt: ~2 % slower per step)
            const char* force16 = getenv("PV_FORCE_BCOMB16");
            if (PV_BC2_W == 16 || (force16 && *force16 && *force16 != '0') ||
                hipMalloc((void**)&g_ctx.d_bc2, rows_ent * PV_BCOMB_STRIDE * 4) != hipSuccess) {
                (void)hipGetLastError();  // clear a failed allocation's sticky error
                g_ctx.d_bc2 = g_ctx.d_bcomb;
                g_ctx.bc2_w = 16;
            }
        }
        if (g_ctx.bc2_w != 16) {
            uint32_t* scratch = nullptr;
            PV_HIP(hipMalloc((void**)&scratch, (uint64_t)PV_BC2_ENT * 40), PV_ERR_ALLOC);
            ge_p3 negB, P;
            ge_frombytes_negate(negB, PV_B_ENC);
            P = negB;
            fe z;
            fe_0(z);
            fe_sub(P.X, z, negB.X);
            fe_carry(P.X, P.X);
            fe_sub(P.T, z, negB.T);
            fe_carry(P.T, P.T);
            int rc = PV_OK;
            for (int j = 0; j < PV_BC2_POS && rc == PV_OK; j++) {
                PvPoint40 arg;
                for (int q = 0; q < 10; q++) {
                    arg.w[q] = P.X.v[q];
                    arg.w[10 + q] = P.Y.v[q];
                    arg.w[20 + q] = P.Z.v[q];
                    arg.w[30 + q] = P.T.v[q];
                }
                const uint32_t ent = j + 1 < PV_BC2_POS ? PV_BC2_ENT : PV_BC2_TOP_ENT;
                const uint32_t threads = (ent + PV_BC2_RUN - 1) / PV_BC2_RUN;
                hipLaunchKernelGGL(pv_bc2_build_kernel, dim3((threads + PV_BLOCK - 1) / PV_BLOCK), dim3(PV_BLOCK), 0,
                                   g_ctx.stream, g_ctx.d_bc2 + (uint64_t)j * PV_BC2_ENT * (PV_BCOMB_STRIDE / 4), ent,
                                   arg, scratch);
                if (hipGetLastError() != hipSuccess || hipStreamSynchronize(g_ctx.stream) != hipSuccess)
                    rc = fail(PV_ERR_LAUNCH, "pv_init: wide fixed-base comb build failed");
                for (int r = 0; r < PV_BC2_W; r++) {  // next row's base: 2^W P
                    ge_p1p1 t;
                    ge_p2_dbl(t, P.X, P.Y, P.Z);
                    ge_p1p1_to_p3(P, t);
                }
            }
            (void)hipFree(scratch);
            if (rc != PV_OK) return rc;
        }
    }
    PV_HIP(hipHostMalloc((void**)&g_ctx.h_zc_verdict, PV_ZC_MAX_REQ, hipHostMallocCoherent | hipHostMallocPortable),
           PV_ERR_ALLOC);
    if (const char* pad = getenv("PV_PREP_LDS_PAD")) g_ctx.prep_lds_pad = (uint32_t)atoi(pad);  // A/B knob
    g_ctx.device = device;
    return PV_OK;
}

// ctx_init_parts, and on failure everything it had built is released (streams, events, the workspace,
// the tables): a retry of pv_init / pv_init_devices starts from an empty context instead of allocating
// ~25 GB on top of a half-built one.
int ctx_init(int device) {
    const int rc = ctx_init_parts(device);
    if (rc != PV_OK) {
        const std::string err = g_err;
        g_ctx.device = device;  // ctx_free releases a context of a known device
        ctx_free();
        g_err = err;
    }
    return rc;
}

// Frees g_ctxs[t_dev or primary] (caller holds its mutex).
void ctx_free() {
    if (g_ctx.device < 0) return;
    (void)hipSetDevice(g_ctx.device);
    if (g_ctx.comm) ncclCommDestroy(g_ctx.comm);
    if (g_ctx.h_zc_verdict) (void)hipHostFree(g_ctx.h_zc_verdict);
    if (g_ctx.d_mg) (void)hipFree(g_ctx.d_mg);
    if (g_ctx.h_mg) (void)hipHostFree(g_ctx.h_mg);
    kc_free();
    if (g_ctx.h_stage) (void)hipHostFree(g_ctx.h_stage);
    if (g_ctx.d_stage) (void)hipFree(g_ctx.d_stage);
    if (g_ctx.d_btab) (void)hipFree(g_ctx.d_btab);
    lane_free_buffers(g_ctx.work, g_ctx.kw);
    if (g_ctx.d_bcomb) (void)hipFree(g_ctx.d_bcomb);
    if (g_ctx.d_bc2 && g_ctx.d_bc2 != g_ctx.d_bcomb) (void)hipFree(g_ctx.d_bc2);
    for (hipEvent_t e : g_ctx.ev) (void)hipEventDestroy(e);
    if (g_ctx.stream) (void)hipStreamDestroy(g_ctx.stream);
    if (g_ctx.kstream) (void)hipStreamDestroy(g_ctx.kstream);
    if (g_ctx.ev_keys_ready) (void)hipEventDestroy(g_ctx.ev_keys_ready);
    if (g_ctx.ev_scan_done) (void)hipEventDestroy(g_ctx.ev_scan_done);
    if (g_ctx.ev_tables_ready) (void)hipEventDestroy(g_ctx.ev_tables_ready);
    if (g_ctx.fstream) (void)hipStreamDestroy(g_ctx.fstream);
    for (hipEvent_t e : g_ctx.ev_chain)
        if (e) (void)hipEventDestroy(e);
    if (g_ctx.ev_prep_done) (void)hipEventDestroy(g_ctx.ev_prep_done);
    if (g_ctx.sstream) (void)hipStreamDestroy(g_ctx.sstream);
    if (g_ctx.bstream) (void)hipStreamDestroy(g_ctx.bstream);
    if (g_ctx.ev_b_start) (void)hipEventDestroy(g_ctx.ev_b_start);
    if (g_ctx.ev_b_done) (void)hipEventDestroy(g_ctx.ev_b_done);
    if (g_ctx.ev_straus_done) (void)hipEventDestroy(g_ctx.ev_straus_done);
    if (g_ctx.ev_launch_done) (void)hipEventDestroy(g_ctx.ev_launch_done);
    if (g_ctx.cstream) (void)hipStreamDestroy(g_ctx.cstream);
    if (g_ctx.ev_cstart) (void)hipEventDestroy(g_ctx.ev_cstart);
    for (hipEvent_t e : g_ctx.ev_copy) (void)hipEventDestroy(e);
    if (g_ctx.h_ver) (void)hipHostFree(g_ctx.h_ver);
    for (void* p : {(void*)g_ctx.xt.htab, (void*)g_ctx.xt.keys, (void*)g_ctx.xt.flags, (void*)g_ctx.xt.tab})
        if (p) (void)hipFree(p);
    if (g_ctx.kc.ev_async) (void)hipEventDestroy(g_ctx.kc.ev_async);
    g_ctx = Ctx();
}

// In-process multi-GPU state (pv_init_devices): the devices in mask order and one RCCL communicator
// per device from ncclCommInitAll (a single-process clique).
struct MultiGpu {
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
};
MultiGpu g_mg;
std::mutex g_mg_mu;

void mg_destroy_comms() {
    for (ncclComm_t c : g_mg.comms)
        if (c) ncclCommDestroy(c);
    g_mg.comms.clear();
    g_mg.devs.clear();
}
}  // namespace

extern "C" {

int pv_init(int device) {
    const int p = g_primary.load();
    if (p == device) {
        PV_HIP(hipSetDevice(device), PV_ERR_NO_DEVICE);  // this thread's device as well
        return PV_OK;
    }
    if (p >= 0) return fail(PV_ERR_ARG, "pv_init: already bound to another device");
    int rc = check_device_index(device, "pv_init");
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(g_mus[device]);
        DevScope ds(device);
        if (g_ctx.device != device && (rc = ctx_init(device)) != PV_OK) return rc;
    }
    PV_HIP(hipSetDevice(device), PV_ERR_NO_DEVICE);
    g_primary.store(device);
    return PV_OK;
}

}  // extern "C"
namespace {
void pinned_cache_drain();
}
extern "C" {
void pv_shutdown(void) {
    pinned_cache_drain();  // freed pv_host_alloc blocks back to the system (live ones stay the caller's)
    {
        std::lock_guard<std::mutex> lk(g_mg_mu);
        mg_destroy_comms();
    }
    for (int d = 0; d < PV_MAX_DEV; d++) {
        std::lock_guard<std::mutex> lk(g_mus[d]);
        DevScope ds(d);
        ctx_free();
    }
    const int p = g_primary.exchange(-1);
    if (p >= 0) (void)hipSetDevice(p);
}

int pv_last_path(int* path, uint32_t* nkeys) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_last_path: call pv_init first");
    uint32_t u[PV_SPLIT_WORDS] = {};
    if (g_ctx.last_keyed) {
        PV_HIP(hipStreamSynchronize(g_ctx.stream), PV_ERR_LAUNCH);
        PV_HIP(hipDeviceSynchronize(), PV_ERR_LAUNCH);
        PV_HIP(hipMemcpy(u, g_ctx.last_nkeys ? g_ctx.last_nkeys : g_ctx.kw.nkeys, sizeof(u), hipMemcpyDeviceToHost),
               PV_ERR_LAUNCH);
    }
    if (nkeys) *nkeys = u[PV_SPLIT_KEYS];
    const bool lat = g_ctx.last_latency || (g_ctx.last_keyed && u[PV_SPLIT_LAT] != 0);
    if (path) *path = lat ? PV_PATH_LATENCY : u[PV_SPLIT_SLOTS] > 0 ? PV_PATH_COMB : PV_PATH_STRAUS;
    g_ctx.last_split[0] = u[PV_SPLIT_KEYS];
    g_ctx.last_split[1] = u[PV_SPLIT_COMB_KEYS];
    g_ctx.last_split[2] = u[PV_SPLIT_SLOTS];
    return PV_OK;
}

int pv_last_split(uint32_t* keys, uint32_t* comb_keys, uint32_t* comb_requests) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_last_split: call pv_init first");
    if (keys) *keys = g_ctx.last_split[0];
    if (comb_keys) *comb_keys = g_ctx.last_split[1];
    if (comb_requests) *comb_requests = g_ctx.last_split[2];
    return PV_OK;
}

int pv_set_path(int mode) {
    if (mode != PV_PATH_AUTO && mode != PV_PATH_STRAUS && mode != PV_PATH_COMB && mode != PV_PATH_LATENCY)
        return fail(PV_ERR_ARG, "pv_set_path: unknown mode");
    for (int d = 0; d < PV_MAX_DEV; d++) {  // every device context of the process
        std::lock_guard<std::mutex> lk(g_mus[d]);
        g_ctxs[d].path = mode;
    }
    return PV_OK;
}

int pv_set_timing(int enable) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ctx.timing = enable != 0;
    g_ctx.ev_used = 0;
    return PV_OK;
}

int pv_stage_times(double* ms, int max_stages, int* launches) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_stage_times: call pv_init first");
    constexpr int NE = PV_NSTAGES + 1;
    double acc[PV_NSTAGES] = {0};
    const int nq = g_ctx.ev_used / NE;
    for (int c = 0; c < nq; c++) {
        hipEvent_t* e = &g_ctx.ev[NE * c];
        PV_HIP(hipEventSynchronize(e[PV_NSTAGES]), PV_ERR_LAUNCH);
        for (int k = 0; k < PV_NSTAGES; k++) {
            float t = 0;
            PV_HIP(hipEventElapsedTime(&t, e[k], e[k + 1]), PV_ERR_LAUNCH);
            acc[k] += t;
        }
    }
    for (int k = 0; k < max_stages && k < PV_NSTAGES; k++) ms[k] = acc[k];
    if (launches) *launches = nq;
    return PV_OK;
}

int pv_kernel_times(double* prep_ms, double* table_ms, double* msm_ms, int* launches) {
    double t[PV_NSTAGES];
    const int rc = pv_stage_times(t, PV_NSTAGES, launches);
    if (rc) return rc;
    if (prep_ms) *prep_ms = t[PV_STAGE_KEYS] + t[PV_STAGE_PREP];
    if (table_ms) *table_ms = t[PV_STAGE_TABLE];
    if (msm_ms) *msm_ms = t[PV_STAGE_MSM] + t[PV_STAGE_ENCODE];
    return PV_OK;
}

int pv_verify_batch_device(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk,
                           uint64_t* d_verdict_words, void* stream) {
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_verify_batch_device: call pv_init first");
    if (n > 0 && (!d_sm || !d_off || !d_pk || !d_verdict_words)) return fail(PV_ERR_ARG, "null pointer");
    std::lock_guard<std::mutex> lk(g_mu);
    return launch(d_sm, d_off, n, d_pk, d_verdict_words, stream ? (hipStream_t)stream : g_ctx.stream);
}

// Host-side copy workers (copy_pool.h): one pool per device context, so the per-device workers of
// pv_verify_batch_multi_gpu stage their shards at the same time; pinned host ranges the library owns
// or registered (pv_host_alloc / pv_host_register), whose bytes the host-buffer entry DMAs directly.
}  // extern "C"
namespace {
pvhost::PinnedRegistry g_pinned_alloc, g_pinned_reg;
// freed pv_host_alloc blocks kept for reuse (copy_pool.h PinnedCache), up to PV_PINNED_CACHE_MB (4 GB)
pvhost::PinnedCache& pinned_cache() {
    static pvhost::PinnedCache* c = [] {
        const char* e = getenv("PV_PINNED_CACHE_MB");
        return new pvhost::PinnedCache((e && *e ? strtoull(e, nullptr, 10) : 4096ull) << 20);
    }();
    return *c;
}
void pinned_release(const std::vector<pvhost::PinnedCache::Block>& v) {
    for (const auto& b : v) (void)hipHostFree(b.p);
}
void pinned_cache_drain() { pinned_release(pinned_cache().drain()); }
bool pv_is_pinned(const void* p, uint64_t bytes) {
    return g_pinned_alloc.contains(p, bytes) || g_pinned_reg.contains(p, bytes);
}
pvhost::CopyPool& cur_pool() {
    static const unsigned ndev = (unsigned)std::max(1, pv_device_count());
    return pvhost::copy_pool_for<PV_MAX_DEV>(pv_cur_dev(), ndev);
}
}  // namespace
extern "C" {

// Move the request blob host -> pinned staging -> HBM. One host thread copies ~10 GB/s, so the blob is
// cut into pieces (256 KB - 4 MB) that the copy pool stages in parallel; with `dma`, each piece's DMA
// (hipMemcpyAsync from pinned memory) is enqueued as soon as it is staged, so the PCIe transfer of
// earlier pieces overlaps the staging of later ones (the pieces are disjoint: their order on the
// stream does not matter, and the kernels launched on the same stream afterwards see every piece).
static int pv_stage_to_device(uint8_t* d_dst, uint8_t* h_stage, const uint8_t* src, uint64_t bytes, hipStream_t s,
                              bool dma) {
    const uint64_t piece = std::min<uint64_t>(4ull << 20, std::max<uint64_t>(256ull << 10, bytes / 16));
    const unsigned k = (unsigned)((bytes + piece - 1) / piece);
    std::atomic<int> err{0};
    cur_pool().run(k, [&](unsigned i) {
        const uint64_t o = (uint64_t)i * piece, e = std::min(bytes, o + piece);
        memcpy(h_stage + o, src + o, e - o);
        if (dma && hipMemcpyAsync(d_dst + o, h_stage + o, e - o, hipMemcpyHostToDevice, s) != hipSuccess) err = 1;
    });
    return err.load() ? fail(PV_ERR_LAUNCH, "hipMemcpyAsync (request blob) failed") : PV_OK;
}

// AUTO between the latency path and the keyed path for a host batch of PV_KEYED_HINT_MIN..
// PV_LATENCY_MAX requests: the device cannot count keys before the path is chosen, the host can
// (~10 us for 4,096 keys). With >= 3 requests per key on average (and at most PV_ALLCOMB_KEYS keys:
// every key a comb key, sparse fill) the keyed path is faster -- MI355X, 1,024 signers, PCIe
// included (profiles/r02/latency_vs_keyed_crossover.txt): 3,072 requests 0.64 vs 0.71 ms, 4,096
// 0.65 vs 0.92; at 2 requests per key (2,048) the latency path still wins (0.58 vs 0.61). Keys in
// the node-side key cache make the latency path faster still: no hint while the cache holds keys.
#ifndef PV_KC_AUTO_MAX_BATCH
#define PV_KC_AUTO_MAX_BATCH 4096  // automatic admission counts every key of host batches up to this size (a sample above)
#endif
static int kc_put_locked(const uint8_t* pks, uint64_t n, bool async);
// Automatic admission: count the VERIFIED appearances of this batch's keys (idx: the sampled requests,
// or null for all n; pre: each one's entry located by kc_auto_locate while the kernels ran, or -1); the
// keys reaching auto_min appearances in the window are returned, at most kcap of them. The verdicts are
// vb[i] & 1 (zero-copy verdict bytes) or bit i of hver (verdict words).
static void kc_auto_count(const uint8_t* pk, const uint64_t* idx, uint64_t n, const int32_t* pre, uint64_t gen,
                          const uint8_t* vb, const uint64_t* hver, std::vector<uint8_t>& admit) {
    auto& k = g_ctx.kc;
    for (uint64_t j = 0; j < n; j++) {
        const uint64_t i = idx ? idx[j] : j;
        const bool ok = vb ? (vb[i] & 1u) != 0 : ((hver[i >> 6] >> (i & 63)) & 1u) != 0;
        if (!ok) continue;  // a key is never counted on the strength of a failing signature
        const auto o = pre && pre[j] >= 0 && k.seen.generation() == gen ? k.seen.bump_at(pre[j], k.auto_min)
                                                                         : k.seen.count(pk + 32 * i, k.auto_min);
        if (o == pvhost::AdmitTable::ADMIT) {
            admit.insert(admit.end(), pk + 32 * i, pk + 32 * i + 32);
            if (admit.size() >= 32ull * g_ctx.kw.kcap) break;
        }
    }
}
// The counting side's read-only lookups, run while the batch's kernels run (the verdicts decide later
// which of them count).
static void kc_auto_locate(const uint8_t* pk, const uint64_t* idx, uint64_t n, std::vector<int32_t>& pre) {
    pre.resize(n);
    for (uint64_t j = 0; j < n; j++) pre[j] = g_ctx.kc.seen.find(pk + 32 * (idx ? idx[j] : j));
}
static int stage_and_launch(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk, uint64_t* d_out,
                            uint64_t** dver_out, uint64_t** hver_out);

// sm_off[0..n] non-decreasing (the host-buffer entries refuse anything else before touching the
// device); large batches are checked in slices on the calling context's copy workers.
static bool offsets_nondecreasing(const uint64_t* off, uint64_t n) {
    auto ok = [off](uint64_t a, uint64_t b) {
        uint64_t bad = 0;
        for (uint64_t i = a; i < b; i++) bad |= off[i + 1] < off[i];
        return bad == 0;
    };
    if (n < (1u << 17)) return ok(0, n);
    pvhost::CopyPool& pool = cur_pool();
    const unsigned k = std::max(1u, pool.threads());
    std::atomic<bool> good{true};
    pool.run(k, [&](unsigned t) {
        if (!ok(n * t / k, n * (t + 1) / k)) good = false;
    });
    return good.load();
}

static bool pv_keyed_hint(const uint8_t* pk, uint64_t n) {
    if (g_ctx.path != PV_PATH_AUTO || n < PV_KEYED_HINT_MIN || n > PV_LATENCY_MAX) return false;
    if (g_ctx.kc.enabled && !g_ctx.kc.index.empty()) return false;
    // distinct keys by open addressing on the keys' first 16 bytes (a heuristic: a rare collision
    // only miscounts, the verdicts do not depend on the path)
    constexpr uint32_t H = 16384;  // > 2 x PV_LATENCY_MAX
    static_assert(H >= 2 * PV_LATENCY_MAX, "hint table too small");
    static thread_local std::vector<uint64_t> tab;
    tab.assign(2 * H, 0);
    uint64_t distinct = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t a, b;
        memcpy(&a, pk + 32 * i, 8);
        memcpy(&b, pk + 32 * i + 8, 8);
        a |= 1;  // (0, 0) marks an empty entry
        uint32_t h = (uint32_t)((a * 0x9E3779B97F4A7C15ull) >> 50) & (H - 1);
        while (tab[2 * h] && !(tab[2 * h] == a && tab[2 * h + 1] == b)) h = (h + 1) & (H - 1);
        if (!tab[2 * h]) {
            tab[2 * h] = a;
            tab[2 * h + 1] = b;
            distinct++;
        }
    }
    return distinct <= PV_ALLCOMB_KEYS && 3 * distinct <= n;
}

int pv_verify_batch(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk,
                    uint8_t* verdict_bits) {
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_verify_batch: call pv_init first");
    if (n == 0) return PV_OK;
    if (!sm || !sm_off || !pk || !verdict_bits) return fail(PV_ERR_ARG, "null pointer");
    if (!offsets_nondecreasing(sm_off, n)) return fail(PV_ERR_ARG, "sm_off must be non-decreasing");
    std::lock_guard<std::mutex> lk(g_mu);
#if PV_ZERO_COPY
    {
        // a small call that takes the latency path (the same choice launch_chunks makes for a host-buffer
        // call) and whose records fit a 2 KB slot: the kernel reads the pinned staging slots over PCIe
        // and stores one verdict byte per request back -- no copy kernels around it
        uint64_t maxlen = 0;
        for (uint64_t i = 0; i < n && n <= PV_ZC_MAX_REQ; i++) maxlen = std::max(maxlen, sm_off[i + 1] - sm_off[i]);
        const uint64_t stride = (4ull * PV_ZC_REC_WORD + maxlen + PV_ZC_SLACK + 63) & ~63ull;
        if (!g_ctx.timing && n <= PV_ZC_MAX_REQ && stride <= PV_ZC_MAX_STRIDE &&
            (g_ctx.path == PV_PATH_LATENCY ||
             (g_ctx.path == PV_PATH_AUTO && n <= PV_LATENCY_MAX && !pv_keyed_hint(pk, n)))) {
            int rc = ensure_stage(n * stride, 0);
            if (rc) return rc;
            uint8_t* vb = g_ctx.h_zc_verdict;  // coherent pinned memory, read while the kernel runs
            uint8_t* slots = g_ctx.h_stage;
            memset(vb, 0xFF, n);  // pending (PV_ZC_SPIN)
            auto fill_at = [&](uint8_t* base, uint64_t a, uint64_t b) {
                for (uint64_t i = a; i < b; i++) {
                    uint8_t* sl = base + i * stride;
                    const uint64_t len = sm_off[i + 1] - sm_off[i];
                    const uint32_t hdr[PV_ZC_PK_WORD] = {(uint32_t)len, 0u, 0u, 0u};
                    memcpy(sl, hdr, sizeof(hdr));
                    memcpy(sl + 4 * PV_ZC_PK_WORD, pk + 32 * i, 32);
                    memcpy(sl + 4 * PV_ZC_REC_WORD, sm + sm_off[i], len);
                    memset(sl + 4 * PV_ZC_REC_WORD + len, 0, stride - 4 * PV_ZC_REC_WORD - len);
                }
            };
            const bool one = n == 1 && stride <= sizeof(PvZcOne);  // the slot goes in the kernel arguments
            PvZcOne one_slot;
            if (one) {
                fill_at(reinterpret_cast<uint8_t*>(one_slot.w), 0, 1);
            } else if (n * stride < (128u << 10)) {
                fill_at(slots, 0, n);
            } else {  // node-quota sizes: the slots are written by the copy pool's threads
                const unsigned k = 8;
                cur_pool().run(k, [&](unsigned t) { fill_at(slots, n * t / k, n * (t + 1) / k); });
            }
            hipStream_t s = g_ctx.stream;
            if (g_ctx.last_stream && g_ctx.last_stream != s)
                PV_HIP(hipStreamWaitEvent(s, g_ctx.ev_launch_done, 0), PV_ERR_LAUNCH);
            g_ctx.last_latency = true;
            g_ctx.last_keyed = false;
            g_ctx.last_dev_choice = false;
            g_ctx.last_zero_copy = true;
            rc = one ? pv_latency_launch_zc_one(one_slot, (uint32_t)stride, g_ctx.d_bcomb, kc_view(), vb, s)
                     : pv_latency_launch_zc(slots, (uint32_t)stride, n, g_ctx.d_bcomb, kc_view(), vb, s);
            PV_HIP(hipEventRecord(g_ctx.ev_launch_done, s), PV_ERR_LAUNCH);
            g_ctx.last_stream = s;
            if (rc) {
                (void)hipStreamSynchronize(s);
                return rc;
            }
            rc = kc_auto_after_batch(pk, n, s, vb, nullptr);  // returns once the verdict bytes are written
            if (rc) return rc;
            memset(verdict_bits, 0, (n + 7) / 8);
            for (uint64_t i = 0; i < n; i++) verdict_bits[i >> 3] |= (uint8_t)((vb[i] & 1u) << (i & 7));
            return PV_OK;
        }
    }
#endif
    uint64_t *dver = nullptr, *hver = nullptr;
    int rc = stage_and_launch(sm, sm_off, n, pk, nullptr, &dver, &hver);
    if (rc) return rc;
    PV_HIP(hipMemcpyAsync(hver, dver, (n + 63) / 64 * 8, hipMemcpyDeviceToHost, g_ctx.stream), PV_ERR_LAUNCH);
    rc = kc_auto_after_batch(pk, n, g_ctx.stream, nullptr, hver);
    if (rc) return rc;
    memcpy(verdict_bits, hver, (n + 7) / 8);  // little-endian words, LSB-first bits
    return PV_OK;
}

// Requests per sub-batch of the pipelined host-buffer form (a multiple of 64; env PV_PIPE_SUB overrides
// it for A/Bs). Sub-batch j's H2D runs on the copy stream while sub-batch j-1's kernels run, so a large
// host batch costs about its PCIe time plus the last sub-batch's kernels instead of their sum.
#ifndef PV_PIPE_SUB
#define PV_PIPE_SUB 262144
#endif
#ifndef PV_PIPE_END_DEFAULT
#define PV_PIPE_END_DEFAULT (PV_PIPE_SUB / 2)
#endif
static constexpr uint64_t PV_PIPE_MAX = 64;                // sub-batches per call (copy events)
static constexpr uint64_t PV_PIPE_MIN_BLOB = 8ull << 20;   // smaller blobs: one piece
static uint64_t pipe_sub() {
    static const uint64_t v = [] {
        const char* e = getenv("PV_PIPE_SUB");
        const uint64_t x = e && *e ? strtoull(e, nullptr, 10) : (uint64_t)PV_PIPE_SUB;
        return std::max<uint64_t>(8192, x / 64 * 64);
    }();
    return v;
}

// The shared-table store of the pipelined host path (on first use; a failed allocation is not retried:
// the sub-batches then build their own tables, same verdicts).
static int ensure_xtab() {
    auto& x = g_ctx.xt;
    if (x.tab) return PV_OK;
    if (x.failed) return PV_ERR_ALLOC;
    if (hipMalloc((void**)&x.htab, PV_XT_HASH * 4) != hipSuccess ||
        hipMalloc((void**)&x.keys, PV_XT_KEYS * 32) != hipSuccess ||
        hipMalloc((void**)&x.flags, PV_XT_KEYS * 4) != hipSuccess ||
        hipMalloc((void**)&x.tab, (uint64_t)PV_XT_KEYS * PV_COMB_POS * PV_COMB_ENT * 160) != hipSuccess) {
        (void)hipGetLastError();
        for (void* p : {(void*)x.htab, (void*)x.keys, (void*)x.flags, (void*)x.tab})
            if (p) (void)hipFree(p);
        x.htab = x.keys = x.flags = nullptr;
        x.tab = nullptr;
        x.failed = true;
        return PV_ERR_ALLOC;
    }
    return PV_OK;
}

static int ensure_hver(uint64_t bytes) {
    if (bytes <= g_ctx.h_ver_cap) return PV_OK;
    if (g_ctx.h_ver) (void)hipHostFree(g_ctx.h_ver);
    g_ctx.h_ver = nullptr;
    g_ctx.h_ver_cap = 0;
    const uint64_t cap = std::max<uint64_t>(bytes, 64 << 10);
    PV_HIP(hipHostMalloc((void**)&g_ctx.h_ver, cap, hipHostMallocPortable), PV_ERR_ALLOC);
    g_ctx.h_ver_cap = cap;
    return PV_OK;
}

// The copy form of a host-buffer batch on the calling thread's context: moves the keys, offsets and
// records to the device staging area and enqueues the verification on the context's stream. d_out:
// where the verdict words go (nullptr = the staging area's own verdict section); *dver / *hver receive
// the device verdict section and a pinned buffer for the caller's copy back.
//   * small batches (blob < 8 MB, no input in pinned memory): one host copy into pinned staging in the
//     device layout, one DMA, the kernels (the quota sizes: fewest packets on the path);
//   * otherwise, in sub-batches of pipe_sub() requests: the copy workers stage sub-batch j's pageable
//     inputs (inputs inside pv_host_alloc / pv_host_register memory are not copied: the DMA reads them
//     where they are), its H2D goes on the copy stream, and its kernels on the engine stream after an
//     event -- so PCIe, host staging and kernels of consecutive sub-batches overlap.
// Staging layout (host and device, 256-B aligned sections): [pk n*32][off (n+1) u64][verdict][blob +
// PV_BLOB_SLACK]. A failure after DMAs were enqueued returns only after both streams drained, so no copy
// still reads the caller's or the staging buffers.
static int stage_and_launch(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk, uint64_t* d_out,
                            uint64_t** dver_out, uint64_t** hver_out) {
    Ctx& c = g_ctx;
    c.last_zero_copy = false;
    auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t pk_bytes = up(n * 32), off_bytes = up((n + 1) * 8), vwords = (n + 63) / 64;
    const uint64_t v_bytes = up(vwords * 8);
    const uint64_t base = sm_off[0], blob = sm_off[n] - base;
    const uint64_t total = pk_bytes + off_bytes + v_bytes + blob + PV_BLOB_SLACK;
    const bool pin_sm = pv_is_pinned(sm + base, blob), pin_pk = pv_is_pinned(pk, 32 * n);
    const bool pin_off = base == 0 && pv_is_pinned(sm_off, 8 * (n + 1));
    const bool any_pin = pin_sm || pin_pk || pin_off, all_pin = pin_sm && pin_pk && pin_off;
    const uint64_t sub = pipe_sub();
    // sub-batch bounds (64-aligned). The call ends one sub-batch's kernels after the last H2D, and
    // the first sub-batch's kernels (which also build the shared tables) start only after the first
    // H2D, so with >= 2 full sub-batches the first and the last are half-size
    // (profiles/r05/host_path: 1M requests, 0.5 + 3 x 1 + 0.5 of 262,144)
    std::vector<uint64_t> bnd{0};
    static const bool halves = env_int("PV_PIPE_HALF_ENDS", 1) != 0;
    // first / last piece size (env PV_PIPE_END, A/B): half a sub-batch by default. Smaller ends are slower
    // (1M arena: 116.8-119.1 M/s at 131,072, 113.6-114.1 at 65,536, 110.4-112.7 at 32,768; profiles/r06/
    // host_path/ab_pipe_end.txt): the copies are the critical path and a sub-batch's kernels beside a DMA
    // take longer than a small last piece's copy, so the last FULL piece's kernels become the tail
    static const uint64_t end_req = (uint64_t)std::max(8192, env_int("PV_PIPE_END", (int)(PV_PIPE_END_DEFAULT)));
    if (blob >= PV_PIPE_MIN_BLOB && halves && n >= 3 * sub) {
        const uint64_t h = std::min<uint64_t>(end_req, sub) / 64 * 64;
        const uint64_t mid = n - 2 * h;
        const uint64_t k = std::min<uint64_t>(PV_PIPE_MAX - 2, std::max<uint64_t>(1, (mid + sub / 2) / sub));
        bnd.push_back(h);
        for (uint64_t j = 1; j < k; j++) bnd.push_back(h + (mid * j / k) / 64 * 64);
        bnd.push_back((n - h) & ~63ull);  // every bound a whole verdict word (n itself need not be)
    } else if (blob >= PV_PIPE_MIN_BLOB) {
        const uint64_t k = std::min<uint64_t>(PV_PIPE_MAX, std::max<uint64_t>(1, n / sub));
        for (uint64_t j = 1; j < k; j++) bnd.push_back((n * j / k) & ~63ull);
    }
    bnd.push_back(n);
    const uint64_t np = bnd.size() - 1;
    hipStream_t s = c.stream;
    int rc = ensure_stage(all_pin ? 0 : total, total);
    if (rc) return rc;
    uint8_t* h = c.h_stage;
    uint8_t* d = c.d_stage;
    uint64_t* dver = reinterpret_cast<uint64_t*>(d + pk_bytes + off_bytes);
    uint8_t* dblob = d + pk_bytes + off_bytes + v_bytes;
    auto finish_piece = [&](uint64_t lo, uint64_t hi) -> int {
        c.verdict_zeroed = d_out == nullptr;
        c.keyed_hint = pv_keyed_hint(pk + 32 * lo, hi - lo);
        c.hint_set = true;
        const int r = launch(dblob, reinterpret_cast<const uint64_t*>(d + pk_bytes) + lo, hi - lo, d + 32 * lo,
                             (d_out ? d_out : dver) + lo / 64, s);
        c.verdict_zeroed = false;
        c.keyed_hint = false;
        c.hint_set = false;
        return r;
    };
    if (np == 1 && !any_pin) {
        // the quota sizes: everything in the device layout in pinned staging, one DMA
        uint64_t* hoff = reinterpret_cast<uint64_t*>(h + pk_bytes);
        const unsigned k = n >= (1u << 16) ? 8u : 1u;
        cur_pool().run(k, [&](unsigned t) {
            const uint64_t a = n * t / k, b = n * (t + 1) / k;
            memcpy(h + 32 * a, pk + 32 * a, 32 * (b - a));
            for (uint64_t i = a; i < b; i++) hoff[i] = sm_off[i] - base;
        });
        hoff[n] = sm_off[n] - base;
        uint8_t* hblob = h + pk_bytes + off_bytes + v_bytes;
        memset(h + pk_bytes + off_bytes, 0, v_bytes);  // the verdict words travel zeroed
        memset(hblob + blob, 0, PV_BLOB_SLACK);
        if (c.inject_stage > 0) {
            c.inject_stage--;
            return fail(PV_ERR_ALLOC, "stage_and_launch: injected staging failure (pv_test_inject)");
        }
        if (blob < (256ull << 10)) {
            memcpy(hblob, sm + base, blob);
        } else {
            rc = pv_stage_to_device(dblob, hblob, sm + base, blob, s, false);
            if (rc) return rc;
        }
        PV_HIP(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
        if ((rc = finish_piece(0, n))) return rc;
        *dver_out = dver;
        *hver_out = reinterpret_cast<uint64_t*>(h + pk_bytes + off_bytes);
        return PV_OK;
    }
    if ((rc = ensure_hver(v_bytes))) return rc;
    while (c.ev_copy.size() < np) {
        hipEvent_t e;
        PV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), PV_ERR_LAUNCH);
        c.ev_copy.push_back(e);
    }
    hipStream_t cs = c.cstream;
    const uint8_t* spk = pin_pk ? pk : h;
    const uint64_t* soff = pin_off ? sm_off : reinterpret_cast<const uint64_t*>(h + pk_bytes);
    const uint8_t* sblob = pin_sm ? sm + base : h + pk_bytes + off_bytes + v_bytes;
    uint64_t* hoff = reinterpret_cast<uint64_t*>(h + pk_bytes);
    uint8_t* hblob = h + pk_bytes + off_bytes + v_bytes;
    uint64_t* doff = reinterpret_cast<uint64_t*>(d + pk_bytes);
    // the copy stream starts after everything enqueued so far (the previous users of the staging area)
    PV_HIP(hipEventRecord(c.ev_cstart, s), PV_ERR_LAUNCH);
    PV_HIP(hipStreamWaitEvent(cs, c.ev_cstart, 0), PV_ERR_LAUNCH);
    if (c.last_stream && c.last_stream != s) PV_HIP(hipStreamWaitEvent(cs, c.ev_launch_done, 0), PV_ERR_LAUNCH);
    // sub-batch j = requests [lo(j), lo(j + 1))
    auto lo_of = [&](uint64_t j) -> uint64_t { return bnd[std::min<uint64_t>(j, np)]; };
    pvhost::CopyPool& pool = cur_pool();
    // sub-batch j's pageable inputs into pinned staging (copy workers), its H2D on the copy stream, then
    // ev_copy[j]
    auto stage_copy = [&](uint64_t j) -> int {
        const uint64_t lo = lo_of(j), hi = lo_of(j + 1);
        const uint64_t b0 = sm_off[lo] - base, b1 = sm_off[hi] - base;
        if (!all_pin) {  // this sub-batch's pageable inputs into pinned staging, on the copy workers
            const unsigned k = std::max(1u, std::min(pool.threads(), (unsigned)((b1 - b0) >> 22)));
            pool.run(k, [&](unsigned t) {
                const uint64_t a = lo + (hi - lo) * t / k, b = lo + (hi - lo) * (t + 1) / k;
                if (!pin_pk) memcpy(h + 32 * a, pk + 32 * a, 32 * (b - a));
                if (!pin_off)
                    for (uint64_t i = a; i < b; i++) hoff[i] = sm_off[i] - base;
                if (!pin_sm) memcpy(hblob + (sm_off[a] - base), sm + sm_off[a], sm_off[b] - sm_off[a]);
            });
            if (!pin_off) hoff[hi] = sm_off[hi] - base;
        }
        PV_HIP(hipMemcpyAsync(d + 32 * lo, spk + 32 * lo, 32 * (hi - lo), hipMemcpyHostToDevice, cs), PV_ERR_LAUNCH);
        PV_HIP(hipMemcpyAsync(doff + lo, soff + lo, 8 * (hi - lo + 1), hipMemcpyHostToDevice, cs), PV_ERR_LAUNCH);
        if (b1 > b0)
            PV_HIP(hipMemcpyAsync(dblob + b0, sblob + b0, b1 - b0, hipMemcpyHostToDevice, cs), PV_ERR_LAUNCH);
        PV_HIP(hipEventRecord(c.ev_copy[j], cs), PV_ERR_LAUNCH);
        return PV_OK;
    };
    // PV_PIPE_TRACE=1 (development): timing events after each sub-batch's copies and kernels, printed to
    // stderr relative to the call's first event -- the untraced pipeline timeline
    static const bool ptrace = env_int("PV_PIPE_TRACE", 0) != 0;
    static const int lookahead = env_int("PV_PIPE_LOOKAHEAD", 1);
    std::vector<hipEvent_t> tev;
    auto tmark = [&](hipStream_t st) {
        if (!ptrace) return;
        hipEvent_t e;
        if (hipEventCreate(&e) == hipSuccess) {
            (void)hipEventRecord(e, st);
            tev.push_back(e);
        }
    };
    // the sub-batches share one set of comb tables: sub-batch 0 builds the tables of its comb keys that
    // the node-side key cache does not hold, the later ones read the cache's for cached keys and the
    // shared store's for the rest (pv_key_cache_probe_kernel's two views)
    static const bool share_env = env_int("PV_PIPE_SHARE", 1) != 0;
    const bool share = share_env && np > 1 && (c.path == PV_PATH_AUTO || c.path == PV_PATH_COMB) &&
                       ensure_xtab() == PV_OK;
    auto run = [&]() -> int {
        tmark(cs);
        if (share) PV_HIP(hipMemsetAsync(c.xt.htab, 0xFF, PV_XT_HASH * 4, s), PV_ERR_LAUNCH);
        if (!d_out) PV_HIP(hipMemsetAsync(dver, 0, vwords * 8, s), PV_ERR_LAUNCH);  // the latency path ORs bits
        PV_HIP(hipMemsetAsync(dblob + blob, 0, PV_BLOB_SLACK, cs), PV_ERR_LAUNCH);
        int r = stage_copy(0);
        tmark(cs);
        // sub-batch j + 1's copies are enqueued BEFORE sub-batch j's kernels: should the copy stream share a
        // hardware queue with one of the engine's streams, no copy waits behind kernels enqueued before it
        for (uint64_t j = 0; j < np && r == PV_OK; j++) {
            if (lookahead && j + 1 < np) {
                if ((r = stage_copy(j + 1)) != PV_OK) break;
                tmark(cs);
            }
            if (c.inject_stage > 0 && j == std::min<uint64_t>(1, np - 1)) {  // sub-batch 0's kernels in flight
                c.inject_stage--;
                return fail(PV_ERR_ALLOC, "stage_and_launch: injected staging failure (pv_test_inject)");
            }
            PV_HIP(hipStreamWaitEvent(s, c.ev_copy[j], 0), PV_ERR_LAUNCH);
            c.xt_fill = share && j == 0;
            c.xt_use = share && j > 0;
            r = finish_piece(lo_of(j), lo_of(j + 1));
            c.xt_fill = c.xt_use = false;
            tmark(s);
            if (!lookahead && r == PV_OK && j + 1 < np) {
                if ((r = stage_copy(j + 1)) != PV_OK) break;
                tmark(cs);
            }
        }
        return r;
    };
    if ((rc = run()) != PV_OK) {
        (void)hipStreamSynchronize(cs);  // no DMA may still read the caller's or the staging buffers
        (void)hipStreamSynchronize(s);
        return rc;
    }
    if (ptrace && !tev.empty()) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(cs);
        std::string line = "pv_pipe: n " + std::to_string(n) + " pieces " + std::to_string(np) + " us:";
        for (size_t i = 1; i < tev.size(); i++) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, tev[0], tev[i]);
            line += " " + std::to_string((int)(ms * 1000));
        }
        fprintf(stderr, "%s\n", line.c_str());
        for (hipEvent_t e : tev) (void)hipEventDestroy(e);
    }
    *dver_out = dver;
    *hver_out = c.h_ver;
    return PV_OK;
}

namespace {
// Zero-copy verdict bytes start at 0xFF and each workgroup's last store sets its byte: the host spins
// on them instead of the runtime's completion wait (a kernel fault surfaces at the next call's
// synchronisation); bounded at 50 ms, then false and the caller waits on the stream.
bool pv_spin_verdict_bytes(const uint8_t* vb, uint64_t n) {
#if PV_ZC_SPIN
    const auto t0 = std::chrono::steady_clock::now();
    volatile const uint8_t* vv = vb;
    uint64_t i = 0;
    while (i < n) {
        if (vv[i] != 0xFFu) {
            i++;
            continue;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) return false;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return true;
#else
    (void)vb;
    (void)n;
    return false;
#endif
}

// Automatic key-cache admission after a host-buffer batch whose verdicts are the last thing enqueued on
// `s`. Waits for the verdicts first (vb: zero-copy verdict bytes, spun on; else the verdict words hver
// copied back on `s`), then counts the keys of the requests that VERIFIED -- a request with a failing
// signature never counts towards its key's admission, so senders without a valid signature cannot make
// the node build tables or evict its signers (plenum/server/client_authn.py:84-118: every signature is
// untrusted input). The admitted keys' tables are built right behind the batch on the engine stream;
// the call does not wait for the build (the next launch is stream-ordered after it).
int kc_auto_after_batch(const uint8_t* pk, uint64_t n, hipStream_t s, const uint8_t* vb, const uint64_t* hver) {
    auto& k = g_ctx.kc;
    const bool on = k.auto_min > 0 && k.cap > 0 && k.enabled && !k.broken;
    // the requests counted: all of a batch of <= 4,096, else a sample of one request from each block of
    // ceil(n / 4,096), at a hashed position in the block (a fixed stride would alias with periodic
    // signer orders); their table entries are located while the kernels still run
    std::vector<uint64_t> sample;
    std::vector<int32_t> pre;
    uint64_t gen = 0;
    if (on) {
        if (n > PV_KC_AUTO_MAX_BATCH) {
            const uint64_t stride = (n + PV_KC_AUTO_MAX_BATCH - 1) / PV_KC_AUTO_MAX_BATCH;
            sample.reserve(n / stride + 1);
            for (uint64_t b = 0, t = 0; b < n; b += stride, t++)
                sample.push_back(b + ((t * 0x9E3779B97F4A7C15ull) >> 40) % std::min(stride, n - b));
        }
        gen = k.seen.generation();
        kc_auto_locate(pk, sample.empty() ? nullptr : sample.data(), sample.empty() ? n : sample.size(), pre);
    }
    if (!(vb && pv_spin_verdict_bytes(vb, n))) PV_HIP(hipStreamSynchronize(s), PV_ERR_LAUNCH);
    if (!on) return PV_OK;
    std::vector<uint8_t> admit;
    kc_auto_count(pk, sample.empty() ? nullptr : sample.data(), sample.empty() ? n : sample.size(), pre.data(), gen,
                  vb, hver, admit);
    if (admit.empty()) return PV_OK;
    const std::string err = g_err;
    if (kc_put_locked(admit.data(), admit.size() / 32, true) == PV_OK) {
        k.auto_admitted += admit.size() / 32;
    } else {
        k.auto_failed += admit.size() / 32;  // the verdicts stand; the keys stay uncached and re-admissible
        for (size_t j = 0; j < admit.size(); j += 32) k.seen.forget(admit.data() + j);
        g_err = err;
    }
    return PV_OK;
}
}  // namespace

int pv_comm_unique_id(uint8_t out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return fail(PV_ERR_COMM, "ncclGetUniqueId failed");
    static_assert(sizeof(id.internal) == 128, "ncclUniqueId size");
    memcpy(out, id.internal, 128);
    return PV_OK;
}

int pv_comm_init(int nranks, int rank, const uint8_t id_bytes[128]) {
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_comm_init: call pv_init first");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PV_ERR_ARG, "pv_comm_init: bad rank");
    ncclUniqueId id;
    memcpy(id.internal, id_bytes, 128);
    ncclResult_t r = ncclCommInitRank(&g_ctx.comm, nranks, id, rank);
    if (r != ncclSuccess) return fail(PV_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    g_ctx.nranks = nranks;
    g_ctx.rank = rank;
    return PV_OK;
}

int pv_allgather_verdicts(const uint64_t* d_local, uint64_t words_per_rank, uint64_t* d_all, void* stream) {
    if (!g_ctx.comm) return fail(PV_ERR_NOT_INIT, "pv_allgather_verdicts: call pv_comm_init first");
    ncclResult_t r = ncclAllGather(d_local, d_all, words_per_rank, ncclUint64, g_ctx.comm,
                                   stream ? (hipStream_t)stream : g_ctx.stream);
    if (r != ncclSuccess) return fail(PV_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    return PV_OK;
}

int pv_comm_count(int* nranks, int* rank) {
    if (!g_ctx.comm) return fail(PV_ERR_NOT_INIT, "pv_comm_count: call pv_comm_init first");
    int c = 0, r = -1;
    ncclResult_t e = ncclCommCount(g_ctx.comm, &c);
    if (e == ncclSuccess) e = ncclCommUserRank(g_ctx.comm, &r);
    if (e != ncclSuccess) return fail(PV_ERR_COMM, std::string("ncclCommCount / ncclCommUserRank: ") + ncclGetErrorString(e));
    if (nranks) *nranks = c;
    if (rank) *rank = r;
    return PV_OK;
}

void pv_comm_destroy(void) {
    if (g_ctx.comm) ncclCommDestroy(g_ctx.comm);
    g_ctx.comm = nullptr;
}

int pv_shard_plan(uint64_t n, int ndev, uint64_t* bounds, uint64_t* words_per_shard) {
    if (ndev < 1 || ndev > PV_MAX_DEV || !bounds || !words_per_shard) return fail(PV_ERR_ARG, "pv_shard_plan: bad arguments");
    // whole 64-request verdict words per shard (sharding.py shard_bounds): word ranges
    // [words r / G, words (r + 1) / G), so every shard but the last is a multiple of 64 requests
    const uint64_t words = (n + 63) / 64;
    uint64_t wmax = 0;
    for (int r = 0; r <= ndev; r++) bounds[r] = std::min<uint64_t>(n, 64 * (words * (uint64_t)r / (uint64_t)ndev));
    for (int r = 0; r < ndev; r++)
        wmax = std::max<uint64_t>(wmax, words * (uint64_t)(r + 1) / ndev - words * (uint64_t)r / ndev);
    *words_per_shard = wmax;
    return PV_OK;
}

int pv_init_devices(uint32_t device_mask) {
    std::vector<int> devs;
    for (int d = 0; d < PV_MAX_DEV; d++)
        if ((device_mask >> d) & 1u) devs.push_back(d);
    if (devs.empty() || (device_mask >> PV_MAX_DEV) != 0) return fail(PV_ERR_ARG, "pv_init_devices: bad device mask");
    for (int d : devs) {
        const int rc = check_device_index(d, "pv_init_devices");
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> mg(g_mg_mu);
    // the missing contexts are built in parallel, one host thread per device (tables built on each GPU)
    std::vector<int> rcs(devs.size(), PV_OK);
    std::vector<std::string> errs(devs.size());
    {
        std::vector<std::thread> th;
        for (size_t i = 0; i < devs.size(); i++)
            th.emplace_back([&, i] {
                const int d = devs[i];
                std::lock_guard<std::mutex> lk(g_mus[d]);
                DevScope ds(d);
                if (g_ctx.device != d && (rcs[i] = ctx_init(d)) != PV_OK) errs[i] = g_err;
            });
        for (auto& t : th) t.join();
    }
    for (size_t i = 0; i < devs.size(); i++)
        if (rcs[i]) return fail(rcs[i], "pv_init_devices: device " + std::to_string(devs[i]) + ": " + errs[i]);
    if (g_mg.devs != devs) {
        mg_destroy_comms();
        int cur = 0;
        (void)hipGetDevice(&cur);
        std::vector<ncclComm_t> comms(devs.size(), nullptr);
        const ncclResult_t r = ncclCommInitAll(comms.data(), (int)devs.size(), devs.data());
        (void)hipSetDevice(cur);  // the caller's current device is unchanged
        if (r != ncclSuccess) return fail(PV_ERR_COMM, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        g_mg.comms = comms;
        g_mg.devs = devs;
    }
    return PV_OK;
}

int pv_multi_gpu_devices(int* devices, int max_devices) {
    std::lock_guard<std::mutex> mg(g_mg_mu);
    for (int i = 0; i < (int)g_mg.devs.size() && i < max_devices && devices; i++) devices[i] = g_mg.devs[i];
    return (int)g_mg.devs.size();
}

int pv_multi_gpu_comm_ranks(int* nranks, int* ranks, int max_devices) {
    std::lock_guard<std::mutex> mg(g_mg_mu);
    if (g_mg.comms.empty()) return fail(PV_ERR_NOT_INIT, "pv_multi_gpu_comm_ranks: call pv_init_devices first");
    int c = 0;
    ncclResult_t e = ncclCommCount(g_mg.comms[0], &c);
    for (int i = 0; e == ncclSuccess && i < (int)g_mg.comms.size() && i < max_devices && ranks; i++)
        e = ncclCommUserRank(g_mg.comms[i], &ranks[i]);
    if (e != ncclSuccess) return fail(PV_ERR_COMM, std::string("ncclCommCount / ncclCommUserRank: ") + ncclGetErrorString(e));
    if (nranks) *nranks = c;
    return PV_OK;
}

int pv_verify_batch_multi_gpu(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk,
                              uint8_t* verdict_bits) {
    if (n == 0) return PV_OK;
    if (!sm || !sm_off || !pk || !verdict_bits) return fail(PV_ERR_ARG, "null pointer");
    if (!offsets_nondecreasing(sm_off, n)) return fail(PV_ERR_ARG, "sm_off must be non-decreasing");
    std::lock_guard<std::mutex> mg(g_mg_mu);
    const int G = (int)g_mg.devs.size();
    if (G == 0) return fail(PV_ERR_NOT_INIT, "pv_verify_batch_multi_gpu: call pv_init_devices first");
    std::vector<uint64_t> b(G + 1);
    uint64_t wpr = 0;
    int rc = pv_shard_plan(n, G, b.data(), &wpr);
    if (rc) return rc;
    // every device's context for the whole call (ascending device order: no lock-order inversion)
    std::vector<std::unique_lock<std::mutex>> locks;
    for (int d : g_mg.devs) locks.emplace_back(g_mus[d]);
    // one worker per device: stage its shard (host -> pinned -> HBM, its own stream) and enqueue the
    // shard's verification with the verdict words landing in its slot of the gather buffer
    std::vector<int> rcs(G, PV_OK);
    std::vector<std::string> errs(G);
    {
        std::vector<std::thread> th;
        for (int r = 0; r < G; r++)
            th.emplace_back([&, r] {
                const int d = g_mg.devs[r];
                DevScope ds(d);
                auto run = [&]() -> int {
                    PV_HIP(hipSetDevice(d), PV_ERR_NO_DEVICE);
                    Ctx& c = g_ctx;
                    const uint64_t need = (uint64_t)G * wpr;
                    if (c.d_mg_words < need) {
                        if (c.d_mg) (void)hipFree(c.d_mg);
                        c.d_mg = nullptr;
                        c.d_mg_words = 0;
                        PV_HIP(hipMalloc((void**)&c.d_mg, need * 8), PV_ERR_ALLOC);
                        c.d_mg_words = need;
                    }
                    if (c.last_stream && c.last_stream != c.stream)
                        PV_HIP(hipStreamWaitEvent(c.stream, c.ev_launch_done, 0), PV_ERR_LAUNCH);
                    PV_HIP(hipMemsetAsync(c.d_mg + (uint64_t)r * wpr, 0, wpr * 8, c.stream), PV_ERR_LAUNCH);
                    const uint64_t lo = b[r], hi = b[r + 1];
                    if (hi == lo) return PV_OK;
                    uint64_t *dv = nullptr, *hv = nullptr;
                    return stage_and_launch(sm, sm_off + lo, hi - lo, pk + 32 * lo, c.d_mg + (uint64_t)r * wpr, &dv, &hv);
                };
                if ((rcs[r] = run()) != PV_OK) errs[r] = g_err;
            });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < G; r++)
        if (rcs[r]) {
            for (int d : g_mg.devs) (void)hipStreamSynchronize(g_ctxs[d].stream);  // no DMA still reads staging
            return fail(rcs[r], "pv_verify_batch_multi_gpu: device " + std::to_string(g_mg.devs[r]) + ": " + errs[r]);
        }
    // ONE all-gather of the per-shard verdict words over the devices' RCCL clique (in place: shard r
    // sits at r * wpr on every device), then the gathered words come back from the first device
    ncclResult_t nr = ncclGroupStart();
    for (int r = 0; r < G && nr == ncclSuccess; r++) {
        Ctx& c = g_ctxs[g_mg.devs[r]];
        nr = ncclAllGather(c.d_mg + (uint64_t)r * wpr, c.d_mg, wpr, ncclUint64, g_mg.comms[r], c.stream);
    }
    const ncclResult_t ne = ncclGroupEnd();
    if (nr == ncclSuccess) nr = ne;
    Ctx& c0 = g_ctxs[g_mg.devs[0]];
    int cur = 0;
    (void)hipGetDevice(&cur);
    rc = PV_OK;
    if (nr != ncclSuccess) rc = fail(PV_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
    if (rc == PV_OK && c0.h_mg_words < (uint64_t)G * wpr) {
        if (c0.h_mg) (void)hipHostFree(c0.h_mg);
        c0.h_mg = nullptr;
        c0.h_mg_words = 0;
        if (hipSetDevice(c0.device) != hipSuccess ||
            hipHostMalloc((void**)&c0.h_mg, (uint64_t)G * wpr * 8, hipHostMallocPortable) != hipSuccess)
            rc = fail(PV_ERR_ALLOC, "pv_verify_batch_multi_gpu: pinned verdict buffer");
        else
            c0.h_mg_words = (uint64_t)G * wpr;
    }
    if (rc == PV_OK && hipMemcpyAsync(c0.h_mg, c0.d_mg, (uint64_t)G * wpr * 8, hipMemcpyDeviceToHost, c0.stream) != hipSuccess)
        rc = fail(PV_ERR_LAUNCH, "pv_verify_batch_multi_gpu: verdict copy");
    for (int r = 0; r < G; r++) {
        Ctx& c = g_ctxs[g_mg.devs[r]];
        const hipError_t e = hipStreamSynchronize(c.stream);
        if (e != hipSuccess && rc == PV_OK)
            rc = fail(PV_ERR_LAUNCH, std::string("pv_verify_batch_multi_gpu: ") + hipGetErrorString(e));
    }
    (void)hipSetDevice(cur);
    if (rc) return rc;
    for (int r = 0; r < G; r++) {  // shard r's words start at bit b[r] (a multiple of 64)
        const uint64_t lo = b[r], hi = b[r + 1];
        if (hi > lo) memcpy(verdict_bits + lo / 8, c0.h_mg + (uint64_t)r * wpr, (hi - lo + 7) / 8);
    }
    return PV_OK;
}

int pv_host_alloc(void** p, uint64_t bytes) {
    if (!p) return fail(PV_ERR_ARG, "pv_host_alloc: null pointer");
    *p = nullptr;
    bytes = std::max<uint64_t>(bytes, 64);
    pvhost::PinnedCache::Block b = pinned_cache().take(bytes);  // a block an earlier pv_host_free released
    if (!b.p) {
        b.bytes = bytes;
        if (hipHostMalloc(&b.p, bytes, hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            pinned_release(pinned_cache().drain());  // the cached blocks back to the system, then once more
            PV_HIP(hipHostMalloc(&b.p, bytes, hipHostMallocPortable), PV_ERR_ALLOC);
        }
    }
    g_pinned_alloc.add(b.p, b.bytes);
    *p = b.p;
    return PV_OK;
}
int pv_host_free(void* p) {
    if (!p) return PV_OK;
    const uint64_t bytes = g_pinned_alloc.size_of(p);
    if (!bytes || !g_pinned_alloc.remove(p)) return fail(PV_ERR_ARG, "pv_host_free: not a pv_host_alloc block");
    pinned_release(pinned_cache().put(p, bytes));  // kept pinned for the next allocation of a similar size
    return PV_OK;
}
int pv_host_register(void* p, uint64_t bytes) {
    if (!p || bytes == 0) return fail(PV_ERR_ARG, "pv_host_register: empty range");
    PV_HIP(hipHostRegister(p, bytes, hipHostRegisterPortable), PV_ERR_ALLOC);
    g_pinned_reg.add(p, bytes);
    return PV_OK;
}
int pv_host_unregister(void* p) {
    if (!p || g_pinned_reg.size_of(p) == 0) return fail(PV_ERR_ARG, "pv_host_unregister: not a registered range");
    // the runtime first: if it refuses, the registry still describes what is pinned
    PV_HIP(hipHostUnregister(p), PV_ERR_ALLOC);
    (void)g_pinned_reg.remove(p);
    return PV_OK;
}
int pv_host_is_pinned(const void* p, uint64_t bytes) { return pv_is_pinned(p, bytes) ? 1 : 0; }

int pv_test_clock_stamps(uint64_t* out, uint32_t max_blocks) {
#if PV_CLOCK_PROBE
    const uint32_t k = std::min<uint32_t>(max_blocks, PV_CLOCK_SLOTS);
    if (!out || k == 0) return (int)PV_CLOCK_SLOTS;
    PV_HIP(hipDeviceSynchronize(), PV_ERR_LAUNCH);
    PV_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(pv_clock_stamps), (size_t)k * 32, 0, hipMemcpyDeviceToHost), PV_ERR_LAUNCH);
    return (int)k;
#else
    (void)out;
    (void)max_blocks;
    return 0;
#endif
}

int pv_test_inject(int what, int device, int count) {
    const char* on = getenv("PV_ENABLE_TEST_HOOKS");
    if (!on || strcmp(on, "1") != 0) return fail(PV_ERR_ARG, "pv_test_inject: test hooks are disabled (PV_ENABLE_TEST_HOOKS=1)");
    if (what != PV_INJECT_STAGE) return fail(PV_ERR_ARG, "pv_test_inject: unknown fault");
    if (device < 0 || device >= PV_MAX_DEV || count < 0) return fail(PV_ERR_ARG, "pv_test_inject: bad device / count");
    std::lock_guard<std::mutex> lk(g_mus[device]);
    g_ctxs[device].inject_stage = count;
    return PV_OK;
}

int pv_dev_alloc(void** p, uint64_t bytes) {
    PV_HIP(hipMalloc(p, std::max<uint64_t>(bytes, 16)), PV_ERR_ALLOC);
    return PV_OK;
}
int pv_dev_free(void* p) {
    PV_HIP(hipFree(p), PV_ERR_ALLOC);
    return PV_OK;
}
}  // extern "C"

namespace {
// A copy ordered after every launch enqueued so far on the primary context, whatever stream the caller
// gave it: the library stream first waits for the last launch's completion event, then copies; the
// call returns once the copy is done. (A plain null-stream hipMemcpy is not ordered after the
// library's non-blocking streams: a D2H could read verdict words before the launch wrote them, an H2D
// could overwrite inputs a running launch still reads.)
int ordered_copy(void* dst, const void* src, uint64_t bytes, hipMemcpyKind kind) {
    if (bytes == 0) return PV_OK;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) {
        PV_HIP(hipMemcpy(dst, src, bytes, kind), PV_ERR_LAUNCH);
        return PV_OK;
    }
    hipStream_t s = g_ctx.stream;
    if (g_ctx.last_stream && g_ctx.last_stream != s) PV_HIP(hipStreamWaitEvent(s, g_ctx.ev_launch_done, 0), PV_ERR_LAUNCH);
    PV_HIP(hipMemcpyAsync(dst, src, bytes, kind, s), PV_ERR_LAUNCH);
    PV_HIP(hipStreamSynchronize(s), PV_ERR_LAUNCH);
    return PV_OK;
}
}  // namespace

extern "C" {
int pv_memcpy_h2d(void* dst, const void* src, uint64_t bytes) { return ordered_copy(dst, src, bytes, hipMemcpyHostToDevice); }
int pv_memcpy_d2h(void* dst, const void* src, uint64_t bytes) { return ordered_copy(dst, src, bytes, hipMemcpyDeviceToHost); }
int pv_last_zero_copy(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_ctx.last_zero_copy ? 1 : 0;
}
int pv_sync(void) {
    PV_HIP(hipDeviceSynchronize(), PV_ERR_LAUNCH);
    return PV_OK;
}
int pv_key_cache_configure(uint32_t capacity) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_key_cache_configure: call pv_init first");
    PV_HIP(hipDeviceSynchronize(), PV_ERR_LAUNCH);  // no launch may still read the old tables
    kc_free();
    if (capacity == 0) return PV_OK;
    if (capacity > (1u << 20)) return fail(PV_ERR_ARG, "pv_key_cache_configure: capacity above 2^20 keys");
    auto& k = g_ctx.kc;
    uint32_t H = 2;
    while (H < 2 * capacity) H <<= 1;
    const uint64_t per = (uint64_t)PV_COMB_POS * PV_COMB_ENT * 160;  // bytes per key table
    hipError_t e;
    if ((e = hipMalloc((void**)&k.d_tab, per * capacity)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_keys, (uint64_t)capacity * 32)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_flags, (uint64_t)capacity * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_htab, (uint64_t)H * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_stamp, (uint64_t)capacity * 4)) != hipSuccess ||
        (e = hipMemset(k.d_stamp, 0, (uint64_t)capacity * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_put_pk, (uint64_t)g_ctx.kw.kcap * 32)) != hipSuccess ||
        (e = hipMalloc((void**)&k.d_put_slot, (uint64_t)g_ctx.kw.kcap * 4)) != hipSuccess ||
        (e = hipHostMalloc((void**)&k.h_async, (uint64_t)g_ctx.kw.kcap * 36 + (uint64_t)H * 4,
                           hipHostMallocDefault)) != hipSuccess ||
        (!k.ev_async && (e = hipEventCreateWithFlags(&k.ev_async, hipEventDisableTiming)) != hipSuccess)) {
        kc_free();
        return fail(PV_ERR_ALLOC, std::string("pv_key_cache_configure: hipMalloc: ") + hipGetErrorString(e));
    }
    k.h_async_cap = (uint64_t)g_ctx.kw.kcap * 36 + (uint64_t)H * 4;
    // the affine rows (660 KB per key): optional -- without them cached keys use the cached-form rows
    static const bool affine = env_int("PV_KC_AFFINE", 1) != 0;
    if (affine && hipMalloc((void**)&k.d_ntab, per * capacity) != hipSuccess) {
        (void)hipGetLastError();
        k.d_ntab = nullptr;
    }
    // the wide rows (67 MB per key) for the first min(capacity, PV_KC_WIDE_KEYS) slots: optional
    {
        const uint32_t want = std::min<uint32_t>(capacity, (uint32_t)std::max(0, env_int("PV_KC_WIDE_KEYS", PV_KC_WIDE_KEYS)));
        const uint64_t per_w = (uint64_t)PV_KW_POS * PV_KW_ENT * 128;
        if (want > 0 && hipMalloc((void**)&k.d_wtab, per_w * want) == hipSuccess &&
            hipMalloc((void**)&k.d_wscr, (uint64_t)PV_KW_GROUP * PV_KW_POS * PV_KW_ENT * 40) == hipSuccess) {
            k.wcap = want;
        } else {
            (void)hipGetLastError();
            if (k.d_wtab) (void)hipFree(k.d_wtab);
            k.d_wtab = nullptr;
            k.wcap = 0;
        }
    }
    k.cap = capacity;
    k.hmask = H - 1;
    k.seed = (uint32_t)std::random_device{}() | 1u;
    k.slot_key.assign(capacity, std::string());
    for (uint32_t i = capacity; i-- > 0;) k.free_slots.push_back(i);
    return kc_upload_htab(g_ctx.stream);
}

// Builds the fresh keys' tables (slot PV_KC_EMPTY = evicted again within the same put) into their
// cache slots, in batches of the workspace's comb capacity. async: one batch only (the caller caps
// the keys), staged through the pinned h_async area and left running on the engine stream (the
// next launch is stream-ordered after it). PV_TEST_FAIL_KC_PUT_BATCH=b (tests only) reports a
// failure after batch b has been enqueued, to exercise the rollback.
static int kc_build_tables(const std::vector<std::string>& fresh, const std::vector<uint32_t>& fresh_slot,
                           bool async) {
    auto& k = g_ctx.kc;
    hipStream_t s = g_ctx.stream;
    if (g_ctx.last_stream && g_ctx.last_stream != s) PV_HIP(hipStreamWaitEvent(s, g_ctx.ev_launch_done, 0), PV_ERR_LAUNCH);
    const char* fail_env = getenv("PV_TEST_FAIL_KC_PUT_BATCH");
    const long fail_batch = fail_env ? atol(fail_env) : -1;
    KeyWork kw = g_ctx.kw;
    std::vector<uint8_t> lpk;
    std::vector<uint32_t> lslot;
    long batch = 0;
    for (size_t f0 = 0; f0 < fresh.size();) {
        uint8_t* bpk;
        uint32_t* bslot;
        if (async) {  // pinned: keys [kcap][32], then slots [kcap]
            bpk = k.h_async;
            bslot = reinterpret_cast<uint32_t*>(k.h_async + (uint64_t)kw.kcap * 32);
        } else {
            lpk.resize((uint64_t)kw.kcap * 32);
            lslot.resize(kw.kcap);
            bpk = lpk.data();
            bslot = lslot.data();
        }
        uint32_t m = 0;
        size_t f = f0;
        for (; f < fresh.size() && m < kw.kcap; f++) {
            if (fresh_slot[f] == PV_KC_EMPTY) continue;
            memcpy(bpk + 32ull * m, fresh[f].data(), 32);
            bslot[m++] = fresh_slot[f];
        }
        f0 = f;
        if (m == 0) continue;
        if (async && f0 < fresh.size()) return fail(PV_ERR_ARG, "kc_build_tables: asynchronous put above one batch");
        PV_HIP(hipMemcpyAsync(k.d_put_pk, bpk, 32ull * m, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
        PV_HIP(hipMemcpyAsync(k.d_put_slot, bslot, (uint64_t)m * 4, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
        hipLaunchKernelGGL(pv_kc_put_prep_kernel, dim3((m + PV_BLOCK - 1) / PV_BLOCK), dim3(PV_BLOCK), 0, s, kw, m);
        PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        const Gate gate{kw.nkeys, kw.slot_req};
        hipLaunchKernelGGL(pv_key_chain_lp_kernel, dim3(std::min<uint32_t>(m, PV_LP_CHAIN_BLOCKS)), dim3(64), 0, s,
                           k.d_put_pk, kw, gate, 0, PV_COMB_POS);
        PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        const uint64_t items = (uint64_t)m * PV_COMB_POS * PV_COMB_BLOCKS;
        hipLaunchKernelGGL(pv_key_fill_kernel, dim3((unsigned)std::min<uint64_t>((items + PV_BLOCK - 1) / PV_BLOCK, 4096)),
                           dim3(PV_BLOCK), 0, s, kw, gate, 0, PV_COMB_POS);
        PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        hipLaunchKernelGGL(pv_kc_scatter_kernel, dim3(64, m), dim3(PV_BLOCK), 0, s, kw.ctab, kw.key_flag, k.d_put_pk,
                           k.d_put_slot, m, k.d_tab, k.d_flags, k.d_keys);
        PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        if (k.d_ntab) {
            hipLaunchKernelGGL(pv_kc_affine_kernel, dim3((m * PV_COMB_POS + 63) / 64), dim3(64), 0, s, k.d_tab,
                               k.d_put_slot, m, k.d_ntab);
            PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
        }
        if (k.d_wtab) {
            bool any = false;
            for (uint32_t j = 0; j < m && !any; j++) any = bslot[j] < k.wcap;
            for (uint32_t j0 = 0; any && j0 < m; j0 += PV_KW_GROUP) {
                const uint32_t g = std::min<uint32_t>(PV_KW_GROUP, m - j0);
                const uint64_t threads = (uint64_t)g * PV_KW_POS * PV_KW_RUNS;
                hipLaunchKernelGGL(pv_kc_wide_kernel, dim3((unsigned)((threads + PV_BLOCK - 1) / PV_BLOCK)), dim3(PV_BLOCK),
                                   0, s, kw, k.d_put_slot, j0, g, k.wcap, k.d_wtab, k.d_wscr);
                PV_HIP(hipGetLastError(), PV_ERR_LAUNCH);
            }
        }
        if (!async) PV_HIP(hipStreamSynchronize(s), PV_ERR_LAUNCH);  // bpk / bslot are host locals
        if (batch++ == fail_batch) return fail(PV_ERR_LAUNCH, "pv_key_cache_put: injected failure (PV_TEST_FAIL_KC_PUT_BATCH)");
    }
    return PV_OK;
}

// LRU refresh on use: the slots that launches read since the last fold (d_stamp newer than
// fold_epoch) move to the front of the LRU, least recently read first, so eviction takes the least
// recently USED keys rather than the least recently put. Launches still running on other streams are
// folded at the next eviction.
static int kc_fold_hits() {
    auto& k = g_ctx.kc;
    if (!k.d_stamp || k.cap == 0) return PV_OK;
    std::vector<uint32_t> st(k.cap);
    PV_HIP(hipMemcpyAsync(st.data(), k.d_stamp, (uint64_t)k.cap * 4, hipMemcpyDeviceToHost, g_ctx.stream), PV_ERR_LAUNCH);
    PV_HIP(hipStreamSynchronize(g_ctx.stream), PV_ERR_LAUNCH);
    std::vector<std::pair<uint32_t, uint32_t>> used;  // (age of the stamp past the fold, slot), LRU order
    for (auto it = k.lru.rbegin(); it != k.lru.rend(); ++it) {
        const uint32_t age = st[*it] - k.fold_epoch;
        if ((int32_t)age > 0) used.emplace_back(age, *it);
    }
    std::stable_sort(used.begin(), used.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& u : used) {
        auto it = k.index.find(k.slot_key[u.second]);
        if (it != k.index.end() && *it->second == u.second) k.lru.splice(k.lru.begin(), k.lru, it->second);
    }
    k.fold_epoch = k.epoch;
    return PV_OK;
}

// pv_key_cache_put under g_mu. async (automatic admission): at most kcap new keys, nothing waited
// for (pinned staging; the hash-table upload and ev_launch_done are stream-ordered after the build).
static int kc_put_locked(const uint8_t* pks, uint64_t n, bool async) {
    auto& k = g_ctx.kc;
    if (async) {
        if (k.async_pending) PV_HIP(hipEventSynchronize(k.ev_async), PV_ERR_LAUNCH);  // h_async is free again
        k.async_pending = false;
    }
    // slots for the new keys (at most cap of them: the last cap distinct keys of the call win).
    // The device hash table still holds the state before this call until kc_upload_htab below.
    std::vector<std::string> fresh;
    std::vector<uint32_t> fresh_slot, touched;
    if (k.free_slots.size() < n && !k.lru.empty()) {
        const int rc = kc_fold_hits();  // evictions ahead: take the launches' reads into account
        if (rc != PV_OK) return rc;
    }
    for (uint64_t i = 0; i < n; i++) {
        std::string key(reinterpret_cast<const char*>(pks + 32 * i), 32);
        auto it = k.index.find(key);
        if (it != k.index.end()) {  // refresh
            k.lru.splice(k.lru.begin(), k.lru, it->second);
            continue;
        }
        uint32_t slot;
        if (!k.free_slots.empty()) {
            slot = k.free_slots.back();
            k.free_slots.pop_back();
        } else {  // evict the least recently put key
            slot = k.lru.back();
            k.lru.pop_back();
            k.index.erase(k.slot_key[slot]);
            k.seen.forget(reinterpret_cast<const uint8_t*>(k.slot_key[slot].data()));  // re-admissible
            for (size_t f = 0; f < fresh.size(); f++)
                if (fresh_slot[f] == slot) fresh_slot[f] = PV_KC_EMPTY;  // evicted before it was built
        }
        k.lru.push_front(slot);
        k.index[key] = k.lru.begin();
        k.slot_key[slot] = key;
        fresh.push_back(key);
        fresh_slot.push_back(slot);
        touched.push_back(slot);
    }
    int rc = kc_build_tables(fresh, fresh_slot, async);
    if (rc != PV_OK) {
        // roll back to a state in which every indexed key's table is built: every slot this call
        // assigned (its new key's table may be unbuilt, and its evicted key's table may already be
        // overwritten) leaves the index and returns to the free list; the keys this call did not
        // touch keep their slots. Then the device hash table is re-uploaded; if even that fails,
        // the cache is switched off (kc_view() reports it empty) until configure / clear.
        const std::string err = g_err;
        std::vector<char> seen(k.cap, 0);
        for (uint32_t slot : touched) {
            if (seen[slot]) continue;
            seen[slot] = 1;
            auto it = k.index.find(k.slot_key[slot]);
            if (it != k.index.end() && *it->second == slot) {
                k.lru.erase(it->second);
                k.index.erase(it);
            }
            k.slot_key[slot].clear();
            k.free_slots.push_back(slot);
        }
        (void)hipStreamSynchronize(g_ctx.stream);
        if (kc_upload_htab(g_ctx.stream) != PV_OK) k.broken = true;
        g_err = err;
        return rc;
    }
    g_ctx.last_keyed = false;
    if (async) {
        rc = kc_upload_htab(g_ctx.stream, reinterpret_cast<uint32_t*>(k.h_async + (uint64_t)g_ctx.kw.kcap * 36));
        if (rc == PV_OK) {
            PV_HIP(hipEventRecord(k.ev_async, g_ctx.stream), PV_ERR_LAUNCH);
            k.async_pending = true;
        }
    } else {
        rc = kc_upload_htab(g_ctx.stream);
    }
    PV_HIP(hipEventRecord(g_ctx.ev_launch_done, g_ctx.stream), PV_ERR_LAUNCH);
    g_ctx.last_stream = g_ctx.stream;
    k.broken = rc != PV_OK;  // a complete upload also repairs an earlier failed one
    return rc;
}

int pv_key_cache_put(const uint8_t* pks, uint64_t n) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& k = g_ctx.kc;
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_key_cache_put: call pv_init first");
    if (k.cap == 0) return fail(PV_ERR_NOT_INIT, "pv_key_cache_put: cache not configured");
    if (n > 0 && !pks) return fail(PV_ERR_ARG, "pv_key_cache_put: null pointer");
    return kc_put_locked(pks, n, false);
}

int pv_key_cache_auto(uint32_t min_seen) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx.device < 0) return fail(PV_ERR_NOT_INIT, "pv_key_cache_auto: call pv_init first");
    if (min_seen > 254) return fail(PV_ERR_ARG, "pv_key_cache_auto: min_seen above 254");
    g_ctx.kc.auto_min = min_seen;
    g_ctx.kc.seen.reset();
    return PV_OK;
}

int pv_key_cache_auto_stats(uint64_t* admitted, uint64_t* failed) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (admitted) *admitted = g_ctx.kc.auto_admitted;
    if (failed) *failed = g_ctx.kc.auto_failed;
    return PV_OK;
}

int pv_key_cache_clear(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& k = g_ctx.kc;
    if (k.cap == 0) return PV_OK;
    PV_HIP(hipDeviceSynchronize(), PV_ERR_LAUNCH);
    k.index.clear();
    k.lru.clear();
    k.free_slots.clear();
    for (uint32_t i = k.cap; i-- > 0;) k.free_slots.push_back(i);
    for (auto& sk : k.slot_key) sk.clear();
    k.seen.reset();  // every key may be admitted again
    const int rc = kc_upload_htab(g_ctx.stream);
    k.broken = rc != PV_OK;
    return rc;
}

int pv_key_cache_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ctx.kc.enabled = enable != 0;
    return PV_OK;
}

int pv_key_cache_stats(uint32_t* size, uint32_t* capacity) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (size) *size = (uint32_t)g_ctx.kc.index.size();
    if (capacity) *capacity = g_ctx.kc.cap;
    return PV_OK;
}

int pv_key_cache_contains(const uint8_t* pk) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!pk) return 0;
    return g_ctx.kc.index.count(std::string(reinterpret_cast<const char*>(pk), 32)) ? 1 : 0;
}

int pv_stream_create(void** stream) {
    if (!stream) return fail(PV_ERR_ARG, "pv_stream_create: null pointer");
    hipStream_t s = nullptr;
    PV_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), PV_ERR_NO_DEVICE);
    *stream = (void*)s;
    return PV_OK;
}
int pv_stream_destroy(void* stream) {
    if (!stream) return PV_OK;
    PV_HIP(hipStreamSynchronize((hipStream_t)stream), PV_ERR_LAUNCH);
    {
        // a later launch must not wait on an event of a destroyed stream
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_ctx.last_stream == (hipStream_t)stream) g_ctx.last_stream = nullptr;
    }
    pv_ingress_forget_stream(stream);
    PV_HIP(hipStreamDestroy((hipStream_t)stream), PV_ERR_LAUNCH);
    return PV_OK;
}
int pv_stream_sync(void* stream) {
    PV_HIP(hipStreamSynchronize(stream ? (hipStream_t)stream : g_ctx.stream), PV_ERR_LAUNCH);
    return PV_OK;
}

}  // extern "C"
