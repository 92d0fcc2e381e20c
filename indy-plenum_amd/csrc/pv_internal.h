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

#endif  // PV_INTERNAL_H
