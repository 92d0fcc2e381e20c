// Internal (non-ABI) hooks shared between the engine translation units of libplenum_verify.so.
#ifndef PV_INTERNAL_H
#define PV_INTERNAL_H

#include <hip/hip_runtime.h>

#include <string>

// The library's main stream (valid after pv_init).
hipStream_t pv_engine_stream();
// Records `msg` as the calling thread's pv_last_error() and returns `code`.
int pv_fail(int code, const std::string& msg);
// A caller stream is being destroyed: the ingress workspace stops handing over through it.
void pv_ingress_forget_stream(void* stream);
// The latency path (pv_latency.hip): n requests on device buffers, verdict words written on `stream`.
// run_if (device word, may be null): the kernel exits at once unless *run_if != 0 (AUTO's device-side
// latency-vs-keyed choice).
struct PvKeyCacheView;
int pv_latency_launch(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk,
                      const void* d_bcomb, const PvKeyCacheView& kc, uint64_t* d_verdict, bool verdict_zeroed,
                      hipStream_t stream, const uint32_t* run_if);
// Zero-copy latency path for a host-buffer call of n <= PV_ZC_MAX_REQ requests in pinned host memory,
// request r in the slot h_slots + r * stride: word 0 = smlen, words PV_ZC_PK_WORD.. the 32-byte key, the
// record's bytes from word PV_ZC_REC_WORD, then >= PV_ZC_SLACK zero bytes (the hash reads ahead); stride a
// multiple of 64, <= PV_ZC_MAX_STRIDE. The kernel reads the slots directly and stores one verdict byte
// per request to h_vbytes (pinned host memory).
int pv_latency_launch_zc(const uint8_t* h_slots, uint32_t stride, uint64_t n, const void* d_bcomb,
                         const PvKeyCacheView& kc, uint8_t* h_vbytes, hipStream_t stream);
// the largest zero-copy call: the latency range AUTO uses for host buffers without a key-repeat hint
// (PV_KEYED_HINT_MIN - 1 = 2,048; PV_LATENCY_MAX, 4,096, bounds the device-side choice). The four-wave
// form runs up to PV_LAT4_MAX, the two-wave form above it
static constexpr uint64_t PV_ZC_MAX_REQ = 2048;
static constexpr uint32_t PV_ZC_MAX_STRIDE = 2048;  // bytes per slot (the LDS copy)
static constexpr uint32_t PV_ZC_PK_WORD = 4, PV_ZC_REC_WORD = 12, PV_ZC_SLACK = 160;
// A one-request zero-copy call whose slot (same layout) fits PvZcOne travels in the kernel arguments
// (pv_latency_launch_zc_one): records up to 1,024 - 48 - 160 = 816 bytes.
struct PvZcOne {
    uint32_t w[256];
};
int pv_latency_launch_zc_one(const PvZcOne& one, uint32_t stride, const void* d_bcomb, const PvKeyCacheView& kc,
                             uint8_t* h_vbytes, hipStream_t stream);

#endif  // PV_INTERNAL_H
