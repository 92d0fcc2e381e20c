// pv_ingress: the request-authentication front end on the device.
//
// Replaces, for a whole batch, the per-signature host work the reference does before libsodium:
//   plenum/server/client_authn.py:97      raw = b58decode(sig)            -> per verification, GPU
//   plenum/common/verifier.py:24-51       DidVerifier key resolution      -> per distinct signer, GPU
//   stp_core/crypto/nacl_wrappers.py:108  sm = signature + msg            -> device-side assembly
// and then runs pv_verify_batch_device on the assembled records. Base58 follows the PyPI base58 2.x
// b58decode semantics the reference calls (setup.py:98-99, restated in oracle/base58_ref.py): trailing
// ASCII whitespace stripped (bytes.rstrip), each leading '1' -> 0x00, Bitcoin alphabet.
//
// Kernels (one stream, no host round trip):
//   pv_ing_signer_kernel   one lane per distinct signer: decode identifier / verkey / '~' tail and
//                          apply the DidVerifier rules -> 32-byte key + status (pv_resolve_verkeys codes)
//   pv_ing_sig_kernel      one lane per verification: decode the signature (5 characters per
//                          multiply-accumulate pass over 24 x 32-bit limbs, 58^5 < 2^32), gather the
//                          signer's key, record length = |b58decode(sig)| + |M|
//   pv_ing_scan_*          exclusive prefix sum of the record lengths (tile of 1,024, then tile sums)
//   pv_ing_assemble_kernel 16 lanes per record: sm = b58decode(sig) || M at its final offset
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "pv_internal.h"
#include "../../include/plenum_verify.h"

namespace {

constexpr int PV_B58_LIMBS = 24;  // decode capacity: 96 bytes
constexpr int ING_BLOCK = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = ING_BLOCK * SCAN_ITEMS;  // 1,024 records per scan tile
constexpr int SCAN_TOP = 1024;                     // threads of the tile-sum scan
constexpr uint64_t ING_MAX_N = 1ull << 26;          // 65,536 tiles: 64 tile sums per top-scan thread
constexpr int ASM_LANES = 16;                       // lanes per record in the assembly kernel

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ------------------------------------------------------------------------------------- device

__device__ __forceinline__ int pv_b58_digit(uint32_t c) {
    int d = -1;
    d = (c >= '1' && c <= '9') ? (int)(c - '1') : d;
    d = (c >= 'A' && c <= 'H') ? (int)(c - 'A' + 9) : d;
    d = (c >= 'J' && c <= 'N') ? (int)(c - 'J' + 17) : d;
    d = (c >= 'P' && c <= 'Z') ? (int)(c - 'P' + 22) : d;
    d = (c >= 'a' && c <= 'k') ? (int)(c - 'a' + 33) : d;
    d = (c >= 'm' && c <= 'z') ? (int)(c - 'm' + 44) : d;
    return d;
}

__device__ __forceinline__ bool pv_ascii_ws(uint32_t c) { return c == 32u || (c - 9u) <= 4u; }

// b58decode of s[0..len): value little-endian in limb[], `zeros` leading 0x00 bytes, `nbytes` the
// minimal big-endian length of the value. status 0 ok, 1 invalid character, 2 longer than 96 bytes
// (every character is still checked, so an invalid character wins, as in the reference).
struct B58Dec {
    uint32_t limb[PV_B58_LIMBS];
    uint32_t zeros;
    uint32_t nbytes;
    uint32_t status;
    __device__ __forceinline__ uint32_t len() const { return zeros + nbytes; }
};

// Character sources for the decoder: global memory, or a workgroup's span staged in LDS.
struct GlobalChars {
    const uint8_t* p;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return p[i]; }
};

template <class Src>
__device__ void pv_b58_decode(const Src& s, uint64_t len, B58Dec& o) {
    while (len > 0 && pv_ascii_ws(s(len - 1))) len--;
    uint64_t z = 0;
    while (z < len && s(z) == '1') z++;
#pragma unroll
    for (int l = 0; l < PV_B58_LIMBS; l++) o.limb[l] = 0;
    bool bad = false, ovf = false;
    for (uint64_t i = z; i < len; i += 5) {
        const uint32_t g = (uint32_t)umin64(5, len - i);
        uint32_t mul = 1, add = 0;
        for (uint32_t k = 0; k < g; k++) {
            const int d = pv_b58_digit(s(i + k));
            bad |= d < 0;
            add = add * 58u + (uint32_t)(d & 63);
            mul *= 58u;
        }
        uint64_t carry = add;
#pragma unroll
        for (int l = 0; l < PV_B58_LIMBS; l++) {
            const uint64_t t = (uint64_t)o.limb[l] * mul + carry;
            o.limb[l] = (uint32_t)t;
            carry = t >> 32;
        }
        ovf |= carry != 0;
    }
    uint32_t nb = 0;
#pragma unroll
    for (int l = 0; l < PV_B58_LIMBS; l++)
        if (o.limb[l]) nb = 4u * l + (32u - __clz(o.limb[l]) + 7u) / 8u;
    o.zeros = (uint32_t)umin64(z, 0xFFFFu);
    o.nbytes = nb;
    o.status = bad ? 1u : ((ovf || z + nb > 4u * PV_B58_LIMBS) ? 2u : 0u);
}

__device__ __forceinline__ void pv_b58_decode(const uint8_t* s, uint64_t len, B58Dec& o) {
    pv_b58_decode(GlobalChars{s}, len, o);
}

__device__ __forceinline__ int pv_hexval(uint32_t c) {
    int v = -1;
    v = (c >= '0' && c <= '9') ? (int)(c - '0') : v;
    v = (c >= 'a' && c <= 'f') ? (int)(c - 'a' + 10) : v;
    v = (c >= 'A' && c <= 'F') ? (int)(c - 'A' + 10) : v;
    return v;
}

// Byte k (big-endian, 0 = most significant) of the L-byte fixed-width encoding of a little-endian
// limb value.
__device__ __forceinline__ uint32_t pv_be_byte(const uint32_t* num, uint32_t L, uint32_t k) {
    const uint32_t b = L - 1 - k;  // little-endian byte index
    return (num[b >> 2] >> (8 * (b & 3))) & 0xFFu;
}

// stp_core Verifier(raw) (nacl_wrappers.py:62-84, 212-229) on the L raw bytes whose value is num[]:
// 0 ok, 2 InvalidKey (neither 32 raw bytes nor 64 hex characters), 3 empty key (verify -> False).
__device__ uint32_t pv_key_from_raw(const uint32_t num[16], uint32_t L, uint32_t pk[8]) {
    if (L == 0) return 3;
    if (L == 32) {
#pragma unroll
        for (int w = 0; w < 8; w++) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) v |= pv_be_byte(num, 32, 4 * w + j) << (8 * j);
            pk[w] = v;
        }
        return 0;
    }
    if (L != 64) return 2;
    bool bad = false;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int hi = pv_hexval(pv_be_byte(num, 64, 2 * (4 * w + j)));
            const int lo = pv_hexval(pv_be_byte(num, 64, 2 * (4 * w + j) + 1));
            bad |= (hi | lo) < 0;
            v |= (uint32_t)((hi << 4) | (lo & 15)) << (8 * j);
        }
        pk[w] = v;
    }
    return bad ? 2u : 0u;
}

// One lane per distinct signer: DidVerifier(verkey, identifier) (verifier.py:24-51). Status codes
// as pv_resolve_verkeys: 0 ok, 1 ValueError (empty verkey), 2 InvalidKey, 3 empty key, 4 identifier
// or abbreviated tail not base58.
__global__ __launch_bounds__(ING_BLOCK) void pv_ing_signer_kernel(
    const uint8_t* __restrict__ idr_chars, const uint64_t* __restrict__ idr_off,
    const uint8_t* __restrict__ vk_chars, const uint64_t* __restrict__ vk_off,
    const uint8_t* __restrict__ vk_present, uint64_t nsig, uint4* __restrict__ kpk, uint8_t* __restrict__ kstatus) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nsig) return;
    const uint8_t* idr = idr_chars + idr_off[u];
    const uint64_t idr_len = idr_off[u + 1] - idr_off[u];
    const uint8_t* vk = vk_chars + vk_off[u];
    const uint64_t vk_len = vk_off[u + 1] - vk_off[u];
    const bool vk_truthy = vk_present[u] && vk_len > 0;
    uint32_t pk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t num[16];
    uint32_t st;
    B58Dec a;
    bool done = false;
    st = 0;
    if (idr_len > 0) {  // `if identifier:`
        pv_b58_decode(idr, idr_len, a);
        if (a.status == 1) {
            st = 4;
            done = true;
        } else if (a.status == 0 && a.len() == 32 && !vk_truthy) {  // cryptonym: verkey = identifier
#pragma unroll
            for (int l = 0; l < 16; l++) num[l] = l < 8 ? a.limb[l] : 0;
            st = pv_key_from_raw(num, 32, pk);
            done = true;
        } else if (!vk_truthy) {
            st = 1;
            done = true;
        } else if (vk[0] == '~') {  // abbreviated: b58decode(identifier) || b58decode(verkey[1:])
            B58Dec t;
            pv_b58_decode(vk + 1, vk_len - 1, t);
            if (t.status == 1) {
                st = 4;
            } else {
                const uint32_t L1 = a.len(), L2 = t.len();
                if (a.status != 0 || t.status != 0 || (L1 + L2 != 0 && L1 + L2 != 32 && L1 + L2 != 64)) {
                    st = 2;
                } else {
                    // value = N_idr * 256^L2 + N_tail, then the fixed-width (L1 + L2)-byte encoding
                    const uint32_t q = L2 >> 2, r = 8 * (L2 & 3);
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        uint32_t hi = 0, lo = 0;
#pragma unroll
                        for (int qq = 0; qq <= 16; qq++) {
                            if ((uint32_t)qq == q) {
                                hi = (j - qq >= 0) ? a.limb[j - qq] : 0u;
                                lo = (j - qq - 1 >= 0) ? a.limb[j - qq - 1] : 0u;
                            }
                        }
                        const uint32_t sh = r ? ((hi << r) | (lo >> (32 - r))) : hi;
                        num[j] = sh | (j < PV_B58_LIMBS ? t.limb[j] : 0u);
                    }
                    st = pv_key_from_raw(num, L1 + L2, pk);
                }
            }
            done = true;
        }
    }
    if (!done) {  // the setter: NaclVerifier(b58decode(verkey))
        if (!vk_present[u]) {
            st = 2;  // b58decode(None) raises inside the setter -> InvalidKey
        } else {
            pv_b58_decode(vk, vk_len, a);
            if (a.status != 0) {
                st = 2;
            } else {
#pragma unroll
                for (int l = 0; l < 16; l++) num[l] = a.limb[l];
                st = pv_key_from_raw(num, a.len(), pk);
            }
        }
    }
    kpk[2 * u] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    kpk[2 * u + 1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    kstatus[u] = (uint8_t)st;
}

// One lane per verification: decode the signature, gather the key, record length.
//   status: 0 verified, 1 signature not base58, 2 signature decodes to > 96 bytes (not assembled),
//           3 index out of range, 16 + k signer status k != 0 (k = 3: no key, verify() is False)
//   siginfo: zeros | nbytes << 16 of the decoded signature; rec_len: 0 unless status == 0
constexpr uint32_t SIG_SPAN_WORDS = 8192;  // 32 KB of LDS: the signature strings of one workgroup

struct LdsChars {
    const uint8_t* lds;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return lds[i]; }
};

__global__ __launch_bounds__(ING_BLOCK) void pv_ing_sig_kernel(
    const uint8_t* __restrict__ sig_chars, const uint64_t* __restrict__ sig_off,
    const uint32_t* __restrict__ msg_idx, const uint32_t* __restrict__ signer_idx, uint64_t n,
    const uint64_t* __restrict__ msg_off, uint64_t nmsg, const uint4* __restrict__ kpk,
    const uint8_t* __restrict__ kstatus, uint64_t nsig, uint4* __restrict__ sigfix, uint4* __restrict__ pk_out,
    uint32_t* __restrict__ siginfo, uint64_t* __restrict__ rec_len, uint8_t* __restrict__ status) {
    // The workgroup's strings are contiguous: stage them in LDS with coalesced dword loads (each
    // lane then parses its string from LDS instead of 88 scattered byte loads from HBM).
    __shared__ uint32_t span[SIG_SPAN_WORDS];
    const uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t b1 = umin64(n, b0 + blockDim.x);
    const uintptr_t first = (uintptr_t)(sig_chars + sig_off[b0]);
    const uintptr_t lo = first & ~(uintptr_t)3;  // inside the allocation (allocations are 256-B aligned)
    const uintptr_t hi = (uintptr_t)(sig_chars + sig_off[b1]);
    const bool staged = hi - lo <= 4ull * SIG_SPAN_WORDS;
    if (staged) {
        const uint64_t full = (hi - lo) / 4;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(lo);
        for (uint64_t w = threadIdx.x; w < full; w += blockDim.x) span[w] = src[w];
        uint8_t* sb = reinterpret_cast<uint8_t*>(span);
        for (uint64_t b = 4 * full + threadIdx.x; b < hi - lo; b += blockDim.x)
            sb[b] = reinterpret_cast<const uint8_t*>(lo)[b];
    }
    __syncthreads();
    const uint64_t i = b0 + threadIdx.x;
    if (i >= n) return;
    const uint32_t mi = msg_idx[i], si = signer_idx[i];
    uint32_t st = 0;
    uint64_t len = 0;
    uint4 k0 = make_uint4(0, 0, 0, 0), k1 = k0;
    if (mi >= nmsg || si >= nsig) {
        st = 3;
    } else {
        B58Dec d;
        const uint64_t sl = sig_off[i + 1] - sig_off[i];
        if (staged)
            pv_b58_decode(LdsChars{reinterpret_cast<const uint8_t*>(span) +
                                   ((uintptr_t)(sig_chars + sig_off[i]) - lo)}, sl, d);
        else
            pv_b58_decode(sig_chars + sig_off[i], sl, d);
        if (d.status) {
            st = d.status;
        } else {
            const uint32_t ks = kstatus[si];
            if (ks) {
                st = 16 + ks;
            } else {
                k0 = kpk[2 * si];
                k1 = kpk[2 * si + 1];
                len = d.len() + (msg_off[mi + 1] - msg_off[mi]);
                // big-endian 96-byte fixed-width value: decoded bytes are its last nbytes
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    const int l = PV_B58_LIMBS - 1 - 4 * q;
                    sigfix[6 * i + q] = make_uint4(__builtin_bswap32(d.limb[l]), __builtin_bswap32(d.limb[l - 1]),
                                                   __builtin_bswap32(d.limb[l - 2]), __builtin_bswap32(d.limb[l - 3]));
                }
                siginfo[i] = d.zeros | (d.nbytes << 16);
            }
        }
    }
    pk_out[2 * i] = k0;
    pk_out[2 * i + 1] = k1;
    rec_len[i] = len;
    status[i] = (uint8_t)st;
}

// Wave-level inclusive scan (wave64).
__device__ __forceinline__ uint64_t pv_wave_incl_scan(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((unsigned long long)v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total the sum.
template <int NT>
__device__ __forceinline__ uint64_t pv_block_excl_scan(uint64_t v, uint64_t* lds, uint64_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t inc = pv_wave_incl_scan(v);
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int w = 0; w < NT / 64; w++) {
            const uint64_t t = lds[w];
            lds[w] = s;
            s += t;
        }
        lds[NT / 64] = s;
    }
    __syncthreads();
    const uint64_t r = lds[wave] + inc - v;
    *total = lds[NT / 64];
    __syncthreads();
    return r;
}

// Tile-local exclusive offsets (rec_len -> local) and one sum per tile.
__global__ __launch_bounds__(ING_BLOCK) void pv_ing_scan_tiles_kernel(const uint64_t* __restrict__ rec_len,
                                                                      uint64_t n, uint64_t* __restrict__ local,
                                                                      uint64_t* __restrict__ tile_sum) {
    __shared__ uint64_t lds[ING_BLOCK / 64 + 1];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        v[k] = base + k < n ? rec_len[base + k] : 0;
        s += v[k];
    }
    uint64_t total;
    uint64_t p = pv_block_excl_scan<ING_BLOCK>(s, lds, &total);
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        if (base + k < n) local[base + k] = p;
        p += v[k];
    }
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// Exclusive scan of the tile sums (one workgroup, <= 65,536 tiles); writes off[n] = total and flags
// an overrun of the assembly buffer (cap bytes).
__global__ __launch_bounds__(SCAN_TOP) void pv_ing_scan_top_kernel(uint64_t* __restrict__ tile_sum, uint64_t ntiles,
                                                                   uint64_t n, uint64_t* __restrict__ off,
                                                                   uint64_t cap, uint32_t* __restrict__ overrun) {
    __shared__ uint64_t lds[SCAN_TOP / 64 + 1];
    const uint64_t per = (ntiles + SCAN_TOP - 1) / SCAN_TOP;
    const uint64_t lo = umin64(ntiles, threadIdx.x * per), hi = umin64(ntiles, lo + per);
    uint64_t s = 0;
    for (uint64_t t = lo; t < hi; t++) s += tile_sum[t];
    uint64_t total;
    uint64_t p = pv_block_excl_scan<SCAN_TOP>(s, lds, &total);
    for (uint64_t t = lo; t < hi; t++) {
        const uint64_t x = tile_sum[t];
        tile_sum[t] = p;
        p += x;
    }
    if (threadIdx.x == 0) {
        const bool bad = total > cap;
        *overrun = bad ? 1u : 0u;
        off[n] = bad ? 0 : total;
    }
}

// 16 lanes per record: final offset, then sm = b58decode(sig) || M. Destination dwords that lie
// wholly inside the record are written as dwords (the message part read as an unaligned 4-byte
// window: two aligned loads + v_alignbyte_b32); the first and last dword of a record are shared
// with its neighbours and written byte by byte. On an overrun every record is emptied (verdict 0,
// status 3).
__global__ __launch_bounds__(ING_BLOCK) void pv_ing_assemble_kernel(
    uint64_t n, const uint64_t* __restrict__ local, const uint64_t* __restrict__ tile_excl,
    const uint64_t* __restrict__ rec_len, const uint32_t* __restrict__ siginfo, const uint8_t* __restrict__ sigfix,
    const uint32_t* __restrict__ msg_idx, const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ overrun, uint8_t* __restrict__ blob, uint64_t* __restrict__ off,
    uint8_t* __restrict__ status) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = gid / ASM_LANES;
    const uint32_t sub = (uint32_t)(gid % ASM_LANES);
    if (i >= n) return;
    if (*overrun) {
        if (sub == 0) {
            off[i] = 0;
            status[i] = 3;
        }
        return;
    }
    const uint64_t o = tile_excl[i / SCAN_TILE] + local[i];
    if (sub == 0) off[i] = o;
    const uint64_t L = rec_len[i];
    if (L == 0) return;
    const uint32_t info = siginfo[i];
    const uint32_t z = info & 0xFFFFu, nb = info >> 16, sl = z + nb;
    const uint8_t* F = sigfix + 96 * i + (96 - nb) - z;  // F[p] for z <= p < sl
    const uint8_t* M = msg + msg_off[msg_idx[i]] - sl;  // M[p] for p >= sl
    auto byte_at = [&](int64_t p) -> uint32_t { return p < (int64_t)z ? 0u : (p < (int64_t)sl ? F[p] : M[p]); };
    uint32_t* dst32 = reinterpret_cast<uint32_t*>(blob);
    const uint64_t d0 = o >> 2, d1 = (o + L + 3) >> 2;
    for (uint64_t D = d0 + sub; D < d1; D += ASM_LANES) {
        const int64_t p0 = (int64_t)(4 * D) - (int64_t)o;  // record position of the dword's first byte
        if (p0 >= 0 && p0 + 4 <= (int64_t)L) {
            uint32_t w;
            if (p0 >= (int64_t)sl) {
                const uintptr_t a = (uintptr_t)(M + p0);
                const uint32_t* ap = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
                w = __builtin_amdgcn_alignbyte(ap[1], ap[0], (uint32_t)(a & 3));
            } else {
                w = byte_at(p0) | byte_at(p0 + 1) << 8 | byte_at(p0 + 2) << 16 | byte_at(p0 + 3) << 24;
            }
            dst32[D] = w;
        } else {
            for (int b = 0; b < 4; b++) {
                const int64_t p = p0 + b;
                if (p >= 0 && p < (int64_t)L) blob[4 * D + b] = (uint8_t)byte_at(p);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------ host

struct IngWork {
    uint64_t n_cap = 0, sig_cap = 0, blob_cap = 0;
    uint4* sigfix = nullptr;
    uint4* pk = nullptr;
    uint32_t* siginfo = nullptr;
    uint64_t* rec_len = nullptr;
    uint64_t* local = nullptr;
    uint64_t* off = nullptr;
    uint64_t* tile_sum = nullptr;
    uint32_t* overrun = nullptr;
    uint4* kpk = nullptr;
    uint8_t* kstatus = nullptr;
    uint8_t* blob = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    // workspace hand-over between callers' streams (as the engine's ev_launch_done)
    hipEvent_t ev_done = nullptr;
    hipStream_t last_stream = nullptr;
    // host-entry staging (pv_ingress_verify)
    uint8_t* h_stage = nullptr;
    uint64_t h_cap = 0;
    uint8_t* d_stage = nullptr;
    uint64_t d_cap = 0;
};

IngWork g_ing;
std::mutex g_ing_mu;

#define ING_HIP(call, code)                                                                         \
    do {                                                                                            \
        hipError_t e_ = (call);                                                                     \
        if (e_ != hipSuccess) return pv_fail(code, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
int regrow(T*& p, uint64_t bytes) {
    if (p) (void)hipFree(p);
    p = nullptr;
    ING_HIP(hipMalloc((void**)&p, std::max<uint64_t>(bytes, 256)), PV_ERR_ALLOC);
    return PV_OK;
}

int ensure_work(uint64_t n, uint64_t nsig, uint64_t blob_bytes) {
    int rc;
    if (n > g_ing.n_cap) {
        const uint64_t c = std::max<uint64_t>(n, 1 << 16);
        const uint64_t tiles = (c + SCAN_TILE - 1) / SCAN_TILE;
        if ((rc = regrow(g_ing.sigfix, c * 96)) || (rc = regrow(g_ing.pk, c * 32)) ||
            (rc = regrow(g_ing.siginfo, c * 4)) || (rc = regrow(g_ing.rec_len, c * 8)) ||
            (rc = regrow(g_ing.local, c * 8)) || (rc = regrow(g_ing.off, (c + 1) * 8)) ||
            (rc = regrow(g_ing.tile_sum, tiles * 8)))
            return rc;
        g_ing.n_cap = c;
    }
    if (!g_ing.overrun && (rc = regrow(g_ing.overrun, 256))) return rc;
    if (nsig > g_ing.sig_cap) {
        const uint64_t c = std::max<uint64_t>(nsig, 1 << 12);
        if ((rc = regrow(g_ing.kpk, c * 32)) || (rc = regrow(g_ing.kstatus, c))) return rc;
        g_ing.sig_cap = c;
    }
    if (blob_bytes > g_ing.blob_cap) {
        const uint64_t c = std::max<uint64_t>(blob_bytes, 1 << 20);
        if ((rc = regrow(g_ing.blob, c + PV_BLOB_SLACK))) return rc;
        g_ing.blob_cap = c;
    }
    if (!g_ing.ev0) {
        ING_HIP(hipEventCreate(&g_ing.ev0), PV_ERR_NO_DEVICE);
        ING_HIP(hipEventCreate(&g_ing.ev1), PV_ERR_NO_DEVICE);
        ING_HIP(hipEventCreateWithFlags(&g_ing.ev_done, hipEventDisableTiming), PV_ERR_NO_DEVICE);
    }
    return PV_OK;
}

int ingress_enqueue(const uint8_t* sig_chars, const uint64_t* sig_off, const uint32_t* msg_idx,
                    const uint32_t* signer_idx, uint64_t n, const uint8_t* msg, const uint64_t* msg_off, uint64_t nmsg,
                    uint64_t cap, const uint8_t* idr_chars, const uint64_t* idr_off, const uint8_t* vk_chars,
                    const uint64_t* vk_off, const uint8_t* vk_present, uint64_t nsig, uint8_t* status,
                    uint64_t* verdict, hipStream_t s);

// Caller holds g_ing_mu.
int ingress_device(const uint8_t* sig_chars, const uint64_t* sig_off, const uint32_t* msg_idx,
                   const uint32_t* signer_idx, uint64_t n, const uint8_t* msg, const uint64_t* msg_off, uint64_t nmsg,
                   uint64_t msg_bytes_total, const uint8_t* idr_chars, const uint64_t* idr_off,
                   const uint8_t* vk_chars, const uint64_t* vk_off, const uint8_t* vk_present, uint64_t nsig,
                   uint8_t* status, uint64_t* verdict, hipStream_t s) {
    if (n == 0) return PV_OK;
    if (n > ING_MAX_N) return pv_fail(PV_ERR_ARG, "pv_ingress: more than 2^26 verifications in one call");
    const uint64_t cap = 96 * n + msg_bytes_total;
    int rc = ensure_work(n, nsig, cap);
    if (rc) return rc;
    if (g_ing.last_stream && g_ing.last_stream != s) ING_HIP(hipStreamWaitEvent(s, g_ing.ev_done, 0), PV_ERR_LAUNCH);
    rc = ingress_enqueue(sig_chars, sig_off, msg_idx, signer_idx, n, msg, msg_off, nmsg, cap, idr_chars, idr_off,
                         vk_chars, vk_off, vk_present, nsig, status, verdict, s);
    ING_HIP(hipEventRecord(g_ing.ev_done, s), PV_ERR_LAUNCH);
    g_ing.last_stream = s;
    return rc;
}

int ingress_enqueue(const uint8_t* sig_chars, const uint64_t* sig_off, const uint32_t* msg_idx,
                    const uint32_t* signer_idx, uint64_t n, const uint8_t* msg, const uint64_t* msg_off, uint64_t nmsg,
                    uint64_t cap, const uint8_t* idr_chars, const uint64_t* idr_off, const uint8_t* vk_chars,
                    const uint64_t* vk_off, const uint8_t* vk_present, uint64_t nsig, uint8_t* status,
                    uint64_t* verdict, hipStream_t s) {
    ING_HIP(hipEventRecord(g_ing.ev0, s), PV_ERR_LAUNCH);
    if (nsig > 0) {
        hipLaunchKernelGGL(pv_ing_signer_kernel, dim3((unsigned)((nsig + ING_BLOCK - 1) / ING_BLOCK)), dim3(ING_BLOCK),
                           0, s, idr_chars, idr_off, vk_chars, vk_off, vk_present, nsig, g_ing.kpk, g_ing.kstatus);
        ING_HIP(hipGetLastError(), PV_ERR_LAUNCH);
    }
    const unsigned grid = (unsigned)((n + ING_BLOCK - 1) / ING_BLOCK);
    hipLaunchKernelGGL(pv_ing_sig_kernel, dim3(grid), dim3(ING_BLOCK), 0, s, sig_chars, sig_off, msg_idx, signer_idx,
                       n, msg_off, nmsg, g_ing.kpk, g_ing.kstatus, nsig, g_ing.sigfix, g_ing.pk, g_ing.siginfo,
                       g_ing.rec_len, status);
    ING_HIP(hipGetLastError(), PV_ERR_LAUNCH);
    const uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(pv_ing_scan_tiles_kernel, dim3((unsigned)tiles), dim3(ING_BLOCK), 0, s, g_ing.rec_len, n,
                       g_ing.local, g_ing.tile_sum);
    ING_HIP(hipGetLastError(), PV_ERR_LAUNCH);
    hipLaunchKernelGGL(pv_ing_scan_top_kernel, dim3(1), dim3(SCAN_TOP), 0, s, g_ing.tile_sum, tiles, n, g_ing.off, cap,
                       g_ing.overrun);
    ING_HIP(hipGetLastError(), PV_ERR_LAUNCH);
    const uint64_t athreads = n * ASM_LANES;
    hipLaunchKernelGGL(pv_ing_assemble_kernel, dim3((unsigned)((athreads + ING_BLOCK - 1) / ING_BLOCK)),
                       dim3(ING_BLOCK), 0, s, n, g_ing.local, g_ing.tile_sum, g_ing.rec_len, g_ing.siginfo,
                       reinterpret_cast<const uint8_t*>(g_ing.sigfix), msg_idx, msg, msg_off, g_ing.overrun, g_ing.blob,
                       g_ing.off, status);
    ING_HIP(hipGetLastError(), PV_ERR_LAUNCH);
    ING_HIP(hipEventRecord(g_ing.ev1, s), PV_ERR_LAUNCH);
    g_ing.timed = true;
    return pv_verify_batch_device(g_ing.blob, g_ing.off, n, reinterpret_cast<const uint8_t*>(g_ing.pk), verdict, s);
}

}  // namespace

void pv_ingress_forget_stream(void* stream) {
    std::lock_guard<std::mutex> lk(g_ing_mu);
    if (g_ing.last_stream == (hipStream_t)stream) g_ing.last_stream = nullptr;
}

extern "C" {

int pv_ingress_verify_device(const char* d_sig_chars, const uint64_t* d_sig_off, const uint32_t* d_msg_idx,
                             const uint32_t* d_signer_idx, uint64_t n, const uint8_t* d_msg, const uint64_t* d_msg_off,
                             uint64_t n_msgs, uint64_t msg_bytes_total, const char* d_idr_chars,
                             const uint64_t* d_idr_off, const char* d_vk_chars, const uint64_t* d_vk_off,
                             const uint8_t* d_vk_present, uint64_t n_signers, uint8_t* d_status,
                             uint64_t* d_verdict_words, void* stream) {
    if (!pv_engine_stream()) return pv_fail(PV_ERR_NOT_INIT, "pv_ingress_verify_device: call pv_init first");
    if (n > 0 && (!d_sig_chars || !d_sig_off || !d_msg_idx || !d_signer_idx || !d_msg || !d_msg_off || !d_status ||
                  !d_verdict_words))
        return pv_fail(PV_ERR_ARG, "pv_ingress_verify_device: null pointer");
    if (n_signers > 0 && (!d_idr_chars || !d_idr_off || !d_vk_chars || !d_vk_off || !d_vk_present))
        return pv_fail(PV_ERR_ARG, "pv_ingress_verify_device: null signer pointer");
    std::lock_guard<std::mutex> lk(g_ing_mu);
    return ingress_device(reinterpret_cast<const uint8_t*>(d_sig_chars), d_sig_off, d_msg_idx, d_signer_idx, n, d_msg,
                          d_msg_off, n_msgs, msg_bytes_total, reinterpret_cast<const uint8_t*>(d_idr_chars), d_idr_off,
                          reinterpret_cast<const uint8_t*>(d_vk_chars), d_vk_off, d_vk_present, n_signers, d_status,
                          d_verdict_words, stream ? (hipStream_t)stream : pv_engine_stream());
}

int pv_ingress_front_ms(double* ms) {
    if (!g_ing.timed) return pv_fail(PV_ERR_NOT_INIT, "pv_ingress_front_ms: no ingress call yet");
    ING_HIP(hipEventSynchronize(g_ing.ev1), PV_ERR_LAUNCH);
    float t = 0;
    ING_HIP(hipEventElapsedTime(&t, g_ing.ev0, g_ing.ev1), PV_ERR_LAUNCH);
    if (ms) *ms = t;
    return PV_OK;
}

int pv_ingress_verify(const char* sig_chars, const uint64_t* sig_off, const uint32_t* msg_idx,
                      const uint32_t* signer_idx, uint64_t n, const uint8_t* msg, const uint64_t* msg_off,
                      uint64_t n_msgs, const char* idr_chars, const uint64_t* idr_off, const char* vk_chars,
                      const uint64_t* vk_off, const uint8_t* vk_present, uint64_t n_signers, uint8_t* status,
                      uint8_t* verdict_bits) {
    if (!pv_engine_stream()) return pv_fail(PV_ERR_NOT_INIT, "pv_ingress_verify: call pv_init first");
    if (n == 0) return PV_OK;
    if (!sig_chars || !sig_off || !msg_idx || !signer_idx || !msg_off || !status || !verdict_bits)
        return pv_fail(PV_ERR_ARG, "pv_ingress_verify: null pointer");
    if (n_signers > 0 && (!idr_chars || !idr_off || !vk_chars || !vk_off || !vk_present))
        return pv_fail(PV_ERR_ARG, "pv_ingress_verify: null signer pointer");
    // validate everything the kernels index with, so a bad argument is an error and never a fault
    auto monotone = [](const uint64_t* o, uint64_t k) {
        for (uint64_t i = 0; i < k; i++)
            if (o[i + 1] < o[i]) return false;
        return true;
    };
    if (!monotone(sig_off, n) || !monotone(msg_off, n_msgs) || (n_signers && (!monotone(idr_off, n_signers) ||
                                                                              !monotone(vk_off, n_signers))))
        return pv_fail(PV_ERR_ARG, "pv_ingress_verify: offsets must be non-decreasing");
    uint64_t mtotal = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (msg_idx[i] >= n_msgs || signer_idx[i] >= n_signers)
            return pv_fail(PV_ERR_ARG, "pv_ingress_verify: message or signer index out of range");
        mtotal += msg_off[msg_idx[i] + 1] - msg_off[msg_idx[i]];
    }
    std::lock_guard<std::mutex> lk(g_ing_mu);
    // staging: [sig_off][msg_off][idr_off][vk_off] u64, [msg_idx][signer_idx] u32, [vk_present][status],
    // [verdict words], then the byte blobs; every section 256-B aligned
    auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t b_sigoff = up((n + 1) * 8), b_msgoff = up((n_msgs + 1) * 8);
    const uint64_t b_idroff = up((n_signers + 1) * 8), b_vkoff = b_idroff;
    const uint64_t b_idx = up(n * 4), b_vkp = up(n_signers + 1), b_status = up(n), b_ver = up((n + 63) / 64 * 8);
    const uint64_t sig_base = sig_off[0], msg_base = n_msgs ? msg_off[0] : 0;
    const uint64_t b_sig = up(sig_off[n] - sig_base + 8), b_msg = up((n_msgs ? msg_off[n_msgs] - msg_base : 0) + 8);
    const uint64_t idr_base = n_signers ? idr_off[0] : 0, vk_base = n_signers ? vk_off[0] : 0;
    const uint64_t b_idr = up((n_signers ? idr_off[n_signers] - idr_base : 0) + 8);
    const uint64_t b_vk = up((n_signers ? vk_off[n_signers] - vk_base : 0) + 8);
    const uint64_t total = b_sigoff + b_msgoff + b_idroff + b_vkoff + 2 * b_idx + b_vkp + b_status + b_ver + b_sig +
                           b_msg + b_idr + b_vk;
    if (total > g_ing.h_cap) {
        if (g_ing.h_stage) (void)hipHostFree(g_ing.h_stage);
        g_ing.h_stage = nullptr;
        ING_HIP(hipHostMalloc((void**)&g_ing.h_stage, total, hipHostMallocDefault), PV_ERR_ALLOC);
        g_ing.h_cap = total;
    }
    if (total > g_ing.d_cap) {
        int rc = regrow(g_ing.d_stage, total);
        if (rc) return rc;
        g_ing.d_cap = total;
    }
    uint8_t* h = g_ing.h_stage;
    uint64_t at = 0;
    auto sec = [&](uint64_t bytes) {
        const uint64_t p = at;
        at += bytes;
        return p;
    };
    const uint64_t o_sigoff = sec(b_sigoff), o_msgoff = sec(b_msgoff), o_idroff = sec(b_idroff),
                   o_vkoff = sec(b_vkoff), o_midx = sec(b_idx), o_sidx = sec(b_idx), o_vkp = sec(b_vkp),
                   o_status = sec(b_status), o_ver = sec(b_ver), o_sig = sec(b_sig), o_msg = sec(b_msg),
                   o_idr = sec(b_idr), o_vk = sec(b_vk);
    auto rebase = [&](uint64_t o, const uint64_t* src, uint64_t k, uint64_t base) {
        uint64_t* d = reinterpret_cast<uint64_t*>(h + o);
        for (uint64_t i = 0; i <= k; i++) d[i] = src[i] - base;
    };
    rebase(o_sigoff, sig_off, n, sig_base);
    if (n_msgs) rebase(o_msgoff, msg_off, n_msgs, msg_base);
    if (n_signers) {
        rebase(o_idroff, idr_off, n_signers, idr_base);
        rebase(o_vkoff, vk_off, n_signers, vk_base);
        memcpy(h + o_vkp, vk_present, n_signers);
        memcpy(h + o_idr, idr_chars + idr_base, idr_off[n_signers] - idr_base);
        memcpy(h + o_vk, vk_chars + vk_base, vk_off[n_signers] - vk_base);
    }
    memcpy(h + o_midx, msg_idx, n * 4);
    memcpy(h + o_sidx, signer_idx, n * 4);
    memcpy(h + o_sig, sig_chars + sig_base, sig_off[n] - sig_base);
    if (n_msgs) memcpy(h + o_msg, msg + msg_base, msg_off[n_msgs] - msg_base);
    uint8_t* d = g_ing.d_stage;
    const hipStream_t s = pv_engine_stream();
    ING_HIP(hipMemcpyAsync(d, h, o_status, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
    ING_HIP(hipMemcpyAsync(d + o_sig, h + o_sig, total - o_sig, hipMemcpyHostToDevice, s), PV_ERR_LAUNCH);
    int rc = ingress_device(d + o_sig, reinterpret_cast<const uint64_t*>(d + o_sigoff),
                            reinterpret_cast<const uint32_t*>(d + o_midx), reinterpret_cast<const uint32_t*>(d + o_sidx),
                            n, d + o_msg, reinterpret_cast<const uint64_t*>(d + o_msgoff), n_msgs, mtotal, d + o_idr,
                            reinterpret_cast<const uint64_t*>(d + o_idroff), d + o_vk,
                            reinterpret_cast<const uint64_t*>(d + o_vkoff), d + o_vkp, n_signers, d + o_status,
                            reinterpret_cast<uint64_t*>(d + o_ver), s);
    if (rc) return rc;
    ING_HIP(hipMemcpyAsync(h + o_status, d + o_status, b_status + b_ver, hipMemcpyDeviceToHost, s), PV_ERR_LAUNCH);
    ING_HIP(hipStreamSynchronize(s), PV_ERR_LAUNCH);
    memcpy(status, h + o_status, n);
    memcpy(verdict_bits, h + o_ver, (n + 7) / 8);
    return PV_OK;
}

}  // extern "C"
