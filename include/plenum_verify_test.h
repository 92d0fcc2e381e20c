/* Test-only entry points of libplenum_verify.so (not part of the product interface in
 * plenum_verify.h). They are exported so the failure-path tests can drive them through the same
 * ctypes binding, and refuse to act unless the process environment has PV_ENABLE_TEST_HOOKS=1 at the
 * call (PV_ERR_ARG otherwise), so no production caller can arm them by accident. */
#ifndef PLENUM_VERIFY_TEST_H
#define PLENUM_VERIFY_TEST_H
#include "plenum_verify.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection: PV_INJECT_STAGE makes the next `count` host-buffer stagings on `device`
 * (pv_verify_batch's copy form, a shard of pv_verify_batch_multi_gpu) fail as an allocation failure
 * would -- in the pipelined form after the first sub-batch's DMA and kernels were enqueued -- so the
 * tests can check that the call returns an error only after no copy still reads the buffers, and
 * that the next call is exact. count 0 clears it. */
#define PV_INJECT_STAGE 1
int pv_test_inject(int what, int device, int count);

/* In-kernel clock of the dominant comb kernel, in a diagnostic build only (make EXTRA=-DPV_CLOCK_PROBE=1,
 * tools/clock_probe.py): wave 0 of each pv_comb_ab_kernel workgroup stamps (s_memtime, s_memrealtime)
 * at entry and exit; this copies (t0, t1, r0, r1) of up to max_blocks workgroups (block index mod
 * 16,384, the last launch's) into out and returns how many; 0 in the product build (no stamps). Read-only:
 * no environment switch needed. */
int pv_test_clock_stamps(uint64_t* out, uint32_t max_blocks);

#ifdef __cplusplus
}
#endif
#endif
