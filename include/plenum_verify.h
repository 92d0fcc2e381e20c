/*
 * plenum_verify.h — C ABI of the MI355X batch Ed25519 request-verification engine
 * (libplenum_verify.so). Plain pointers and sizes only; no torch/HIP types cross this boundary
 * (streams are passed as void*). All functions return 0 on success and a negative PV_ERR_* code on
 * infrastructure failure; a bad signature is NEVER an error, it is a 0 verdict bit. No exceptions
 * cross the ABI; pv_last_error() describes the last failure of the calling thread.
 *
 * What each entry point replaces in the reference (swcurran/indy-plenum):
 *   pv_verify_batch        the per-signature ctypes call chain
 *                          stp_core/crypto/nacl_wrappers.py:232-242 Verifier.verify
 *                          -> :86-108 VerifyKey.verify(signature + msg)
 *                          -> libnacl.crypto_sign_open(sm, pk) (libnacl 1.6.1, setup.py:107-108)
 *                          -> libsodium 1.0.18 crypto_sign_open, batched: request i is the byte
 *                          string sm[sm_off[i] : sm_off[i+1]] (exactly the `signature + msg`
 *                          concatenation the reference builds, so the sig/msg split point is
 *                          libsodium's: the first 64 bytes) verified against pk[32 i : 32 i + 32].
 *                          verdict bit i (LSB-first within each byte) = 1 iff crypto_sign_open
 *                          would return 0 (libnacl would not raise ValueError).
 *   pv_verify_batch_device the same on device-resident inputs (the hot path the benchmark times).
 *   pv_b58decode_batch     base58.b58decode (PyPI base58, unpinned; setup.py:98-99) as called from
 *                          plenum/server/client_authn.py:97 (signature) and
 *                          plenum/common/verifier.py:27,37,50 (identifier / verkey).
 *   pv_resolve_verkeys     plenum/common/verifier.py:24-50 DidVerifier key resolution (cryptonym,
 *                          abbreviated '~' verkey expansion, full verkey) for a batch.
 *   pv_comm_* / pv_allgather_verdicts
 *                          new: the cross-GPU gather of per-shard verdict bitmaps (one RCCL
 *                          all-gather over xGMI). The reference has no equivalent.
 *   pv_init_devices / pv_verify_batch_multi_gpu
 *                          the same batched crypto_sign_open as pv_verify_batch, sharded over several
 *                          GPUs driven from ONE process (the reference's node is one process with one
 *                          asyncio Looper, stp_core/loop/looper.py:142-213, fed from
 *                          plenum/server/node.py:1518-1527 and stp_zmq/zstack.py:606-646), the
 *                          per-shard verdict bitmaps gathered with one in-process RCCL all-gather.
 * Threading: the reference caller is the single-threaded asyncio Looper (stp_core/loop/looper.py);
 * the library is synchronous per call. It keeps one context per device: pv_init binds the primary
 * device that every single-device call uses; pv_init_devices adds contexts for the multi-GPU call.
 */
#ifndef PLENUM_VERIFY_H
#define PLENUM_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PV_OK 0
#define PV_ERR_NO_DEVICE (-1)
#define PV_ERR_ALLOC (-2)
#define PV_ERR_LAUNCH (-3)
#define PV_ERR_ARG (-4)
#define PV_ERR_NOT_INIT (-5)
#define PV_ERR_COMM (-6)
#define PV_ERR_DECODE (-7)

/* Bytes that must be readable past sm_off[n] in a device blob (SHA-512 reads whole 8-byte words). */
#define PV_BLOB_SLACK 256

/* ABI version of this header. */
#define PV_ABI_VERSION 1
int pv_abi_version(void);
/* Build configuration of the library's kernels (bit set = compiled in):
 *   PV_BUILD_COMB_FUSED  the keyed comb path computes [S]B and [k](-A) in ONE kernel
 *                        (pv_comb_ab_kernel, the MSM stage) for chunks above 262,144 requests instead
 *                        of pv_comb_b_kernel (TABLE stage) + pv_comb_a_kernel (MSM stage); smaller
 *                        chunks keep the two kernels */
#define PV_BUILD_COMB_FUSED 1u
uint32_t pv_build_flags(void);

/* Number of visible GPUs (0 when none; never an error). */
int pv_device_count(void);

/* Bind this process to `device`, build the fixed-base table, allocate the workspace. Idempotent
 * for the same device. */
int pv_init(int device);
void pv_shutdown(void);
const char* pv_last_error(void);

/* Host buffers in, host bitmap out (ceil(n/8) bytes). sm_off has n+1 entries, non-decreasing;
 * offsets need no alignment. Synchronous. Inputs in ordinary (pageable) memory are copied into the
 * library's pinned staging buffer by per-device copy threads; inputs that lie in pinned memory the
 * library allocated or registered (pv_host_alloc / pv_host_register below) are DMA'd from where they
 * are, without that copy (the offsets too when sm_off[0] == 0). Batches whose blob is >= 8 MB are
 * verified in sub-batches of 262,144 requests (the first and the last half-size) whose H2D transfers
 * (on a copy stream) overlap the previous sub-batch's kernels, so a large host batch costs about its
 * PCIe time plus one sub-batch's kernels.
 * A call of <= 2,048 requests that takes the latency path (AUTO's range for host buffers without a
 * key-repeat hint, or PV_PATH_LATENCY) and whose records are all <= 1,840 bytes is zero-copy: the
 * requests go into fixed-stride slots of the pinned staging buffer that the kernel reads over PCIe,
 * and each request's verdict byte is stored back into coherent pinned memory (no copy kernels around
 * the verification); the host returns as soon as every byte is written (a fault of such a call is
 * reported by the next call's synchronisation). With stage timing on or key-cache auto-admission
 * active the host waits on the stream as for any other call. pv_last_zero_copy() returns 1 if the
 * most recent pv_verify_batch took the zero-copy form. */
int pv_verify_batch(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk,
                    uint8_t* verdict_bits);
int pv_last_zero_copy(void);

/* Several GPUs from one process (SURVEY.md §8b pv_init(device_mask) / pv_verify_batch_multi_gpu).
 *   pv_init_devices(mask)       bit d set = use device d (d < 16); builds each missing device context
 *                               (tables, workspace, streams; in parallel) and one RCCL communicator per
 *                               device with ncclCommInitAll. A primary bound by pv_init may be in the
 *                               mask: its context is shared. Calling it again with another mask
 *                               rebuilds the communicators only.
 *   pv_verify_batch_multi_gpu   pv_verify_batch's contract (host buffers, synchronous, same verdict
 *                               bits), sharded over those devices: shard r = requests
 *                               [bounds[r], bounds[r+1]) of pv_shard_plan (contiguous, whole 64-request
 *                               verdict words), staged and verified on device r's own stream by one host
 *                               worker per device; the per-shard verdict words are gathered with ONE
 *                               ncclAllGather over the clique (group call) and copied back from the first
 *                               device. No other cross-GPU traffic.
 *   pv_multi_gpu_devices        the devices in use (up to max), returns their count (0 = none).
 *   pv_multi_gpu_comm_ranks     what RCCL itself reports for the clique: ncclCommCount of the first
 *                               device's communicator, and ncclCommUserRank of each device's (up to max).
 *   pv_shard_plan               host-only: the shard bounds (ndev + 1 entries) and the verdict words
 *                               per shard (the all-gather's count) for n requests over ndev devices. */
int pv_init_devices(uint32_t device_mask);
int pv_verify_batch_multi_gpu(const uint8_t* sm, const uint64_t* sm_off, uint64_t n, const uint8_t* pk,
                              uint8_t* verdict_bits);
int pv_multi_gpu_devices(int* devices, int max_devices);
int pv_multi_gpu_comm_ranks(int* nranks, int* ranks, int max_devices);
int pv_shard_plan(uint64_t n, int ndev, uint64_t* bounds, uint64_t* words_per_shard);

/* Library-owned pinned host memory: the host-fed path's input arena. A node that receives its
 * requests straight into such buffers (the signature + message blob, the offsets, the keys) lets
 * pv_verify_batch / pv_verify_batch_multi_gpu DMA them to HBM without a pageable -> pinned copy. The
 * blocks are portable (every device of the process can DMA from them). Any range inside a block is
 * recognised per call.
 *   pv_host_alloc(p, bytes)      allocate a pinned block (*p = its address)
 *   pv_host_free(p)              release a pv_host_alloc block (PV_ERR_ARG for any other pointer);
 *                                it stays pinned in a cache (4 GB, PV_PINNED_CACHE_MB) for the next
 *                                pv_host_alloc of a similar size, returned to the system at pv_shutdown
 *   pv_host_register(p, bytes)   pin an existing host range in place (hipHostRegister; ~50 ms per GB,
 *                                for long-lived receive buffers)
 *   pv_host_unregister(p)        undo pv_host_register (p = the registered start); a registered
 *                                range must be unregistered before its memory is freed, or the
 *                                library keeps treating that address range as pinned
 *   pv_host_is_pinned(p, bytes)  1 if [p, p + bytes) lies inside one such block or range */
int pv_host_alloc(void** p, uint64_t bytes);
int pv_host_free(void* p);
int pv_host_register(void* p, uint64_t bytes);
int pv_host_unregister(void* p);
int pv_host_is_pinned(const void* p, uint64_t bytes);

/* Device buffers in, device bitmap out. Requirements: d_sm 4-byte aligned and readable up to
 * sm_off[n] + PV_BLOB_SLACK (records themselves need no alignment), d_pk 16-byte aligned,
 * verdict_words holds ceil(n/64) 64-bit words. Enqueued on `stream` (a hipStream_t, NULL = the
 * library stream); returns without synchronising. Thread-safe: calls are serialised on a library
 * mutex, and a call on a different stream than the previous call first makes its stream wait for
 * the previous launch (the workspace is shared), so concurrent callers get correct verdicts. */
int pv_verify_batch_device(const uint8_t* d_sm, const uint64_t* d_off, uint64_t n, const uint8_t* d_pk,
                           uint64_t* d_verdict_words, void* stream);

/* pv_set_timing(1) (re)starts timing: from then on every launch records HIP events on its own
 * stream at each stage boundary. pv_stage_times returns the device time (ms) of each stage summed
 * over all launches since then, in this order (PV_STAGE_*):
 *   KEYS    per-batch key deduplication and per-key expansion (keyed comb path only)
 *   PREP    per-request checks, SHA-512, reduction mod L, recoding (Straus path: also A's
 *           decompression and the half-size split of k, pv_split_kernel)
 *   TABLE   per-request [j](+-A) and [j](-R') multiples with R's decompression, and [k2 S]B from the
 *           wide fixed-base comb (Straus path) / comb path: [S]B from the fixed-base comb while the
 *           per-key comb tables are built on a second stream, then the join
 *   MSM     the double-scalar multiplication to projective coordinates (Straus path: ~33 windows of
 *           both half-size scalars; comb path: the [k](-A) half, 32 table additions)
 *   ENCODE  batched inversion, canonical encoding, compare with R, verdict bits
 * and the number of launches (chunks). pv_kernel_times is the coarse three-way view
 * (KEYS+PREP, TABLE, MSM+ENCODE). pv_set_timing(0) stops recording. */
#define PV_STAGE_KEYS 0
#define PV_STAGE_PREP 1
#define PV_STAGE_TABLE 2
#define PV_STAGE_MSM 3
#define PV_STAGE_ENCODE 4
#define PV_NSTAGES 5
/* Arithmetic path for subsequent launches. Every path gives bit-identical verdicts:
 *   PV_PATH_STRAUS  per request: decompress A and R (R must decode to R' with encode(R') == R, else
 *                   reject), split k = k1 / k2 (mod 8L) with |k1|, k2 < ~2^128 and k2 odd (extended
 *                   Euclid in Lehmer blocks), 9-entry tables of [j](+-A) and [j](-R'), [k2 S mod L]B
 *                   from the wide fixed-base comb (11 radix-2^24 lookups: the top entry converted +
 *                   10 niels additions), then a regular-window loop over both scalars: ~33 x (4
 *                   doublings + 2 cached additions), + [k2 S]B + R', and encode(.) == R: equal iff
 *                   [k2](SB - kA - R') = 0 iff libsodium's encode(SB - kA) == R (any A, R of the
 *                   curve: 8L kills every point, k2 is odd and below L). A lane whose split is not
 *                   settled takes (k, 1) and the full-length loop, same verdict
 *   PV_PATH_COMB    per batch: deduplicate keys; per DISTINCT key: libsodium's key checks,
 *                   decompression and a radix-256 comb table T_A[i][d] = [d 256^i](-A) (32 x 129
 *                   entries); per request: [S]B as above (10 niels additions) and [k](-A) as 32
 *                   cached table additions, no doublings (keys beyond the PV_KEY_CAP = 16,384 tables
 *                   a chunk holds take the Straus path in the same launch)
 *   PV_PATH_LATENCY per request: one workgroup with limb-parallel arithmetic, every field element
 *                   spread over 10 lanes of a 16-lane row; decompression of A and R in one chain,
 *                   the same half-size split as the Straus path, [k1](+-A) and [k2](-R') (~33 x 4
 *                   doublings + ~33 additions each) on two waves at once -- batches of <= 512
 *                   requests (PV_LAT4_MAX): four waves, each scalar cut again at 2^68 (~17 windows per wave) --
 *                   [k2 S]B from the radix-65536 fixed-base comb, and the comparison with R' without
 *                   an inversion. A key in the node-side key cache keeps the full k: [k](-A) as 32
 *                   table additions, no doublings. One kernel launch; the fastest path for small
 *                   batches (Plenum's 100 / 1,000-message quotas). In the comb kernels a cached key's
 *                   additions read the cache's affine rows (entries divided by Z: no Z1 Z2 product)
 *   PV_PATH_AUTO    (default) batches of <= 2,048 requests take the latency path. From 2,049 to
 *                   4,096 requests AUTO picks by key repeats: the keyed path with >= 3 requests per
 *                   key (and <= 2,048 keys), else the latency path; pv_verify_batch counts the keys
 *                   on the host, pv_verify_batch_device lets its dedup kernels count them and choose
 *                   on the device (the other path's kernels exit at once; no host round trip). A
 *                   non-empty key cache keeps such batches on the latency path. Larger batches, per
 *                   chunk: deduplicate keys, give a comb table to every key with >= 48 requests in
 *                   the chunk (a table costs about what ~50 requests save) -- to every key when the
 *                   chunk has <= 2,048 keys and <= 256k requests -- and verify the other requests on
 *                   the Straus path in the same launch; a tail chunk of <= 4,096 requests goes
 *                   Straus unless the key cache holds keys (then keyed). Split on the device, so
 *                   pv_verify_batch_device stays asynchronous.
 * Every path returns bit-identical verdicts. */
#define PV_PATH_AUTO 0
#define PV_PATH_STRAUS 1
#define PV_PATH_COMB 2
#define PV_PATH_LATENCY 3
int pv_set_path(int mode);
/* The path the most recent chunk took (PV_PATH_COMB if any of its requests used a comb table, else
 * PV_PATH_STRAUS) and its distinct-key count (0 when no key kernels ran). Synchronises the device. */
int pv_last_path(int* path, uint32_t* nkeys);
/* The split of the most recent chunk, as read by the last pv_last_path call: distinct keys, keys
 * given a comb table, requests verified with those tables (the rest took the Straus path). */
int pv_last_split(uint32_t* keys, uint32_t* comb_keys, uint32_t* comb_requests);
int pv_set_timing(int enable);
int pv_stage_times(double* ms, int max_stages, int* launches);
int pv_kernel_times(double* prep_ms, double* table_ms, double* msm_ms, int* launches);

/* Node-side key cache (persistent across calls). A node verifies requests from a fairly stable set
 * of signers whose verkeys it already holds (the domain ledger's NYM records,
 * plenum/server/request_handlers/utils.py:30-39). For a cached key the latency path computes [k](-A)
 * with 32 additions from the key's radix-256 comb table (660 KB of HBM per key, built once by the
 * engine's key-chain and fill kernels) instead of ~132 doublings + ~66 additions; verdicts are
 * unchanged (the table holds exact multiples of -A, and libsodium's key checks ran when it was built).
 * Above the latency path's range (AUTO: batches > 4,096 requests) a non-empty cache also makes every
 * chunk keyed, the tail chunk of a multi-chunk batch included: a cached key's requests take the comb
 * path at any request count and its table is read from the cache instead of being built (no key
 * chain / table fill for it); uncached keys are handled as without the cache. A put that fails part
 * way (an error from a build step) leaves only keys whose tables were built: every slot the call
 * assigned is dropped. The benchmark's headline never configures it.
 *   pv_key_cache_configure(capacity)  allocate room for `capacity` keys (0 = free, disabled)
 *   pv_key_cache_put(pks, n)          host keys (n x 32 B): build and insert the missing ones, refresh
 *                                     the present ones; when full, the least recently USED keys are
 *                                     evicted (every launch stamps the cache slots it reads; the stamps
 *                                     are folded into the LRU order before a put evicts). Synchronous: a
 *                                     batch of keys is built in parallel, ~0.1 ms of GPU time per key with
 *                                     the affine and radix-65536 rows (1,024 keys in 0.10-0.12 s)
 *   pv_key_cache_clear()              drop every key (capacity kept)
 *   pv_key_cache_enable(on)           whether launches consult the cache (default on)
 *   pv_key_cache_stats(size, cap)     keys held / capacity
 *   pv_key_cache_contains(pk)         1 if the 32-byte key is cached
 *   pv_key_cache_auto(min_seen)       automatic admission (0 = off, the default): once a
 *                                     pv_verify_batch call's verdicts are back, the keys of its requests
 *                                     that VERIFIED are counted (every request of calls of <= 4,096
 *                                     requests, a sample of 4,096 of larger ones: one request per block of
 *                                     ceil(n / 4,096)); a request with a failing signature never counts,
 *                                     so senders without valid signatures cannot make the node build
 *                                     tables or evict its signers (plenum/server/client_authn.py:84-118:
 *                                     every signature is untrusted input). A key verified min_seen times
 *                                     within the counting window (the last ~32k distinct keys) is put
 *                                     into the cache behind that batch on the engine stream: the call
 *                                     returns with its verdicts, the build (~0.1 ms of GPU time per key)
 *                                     overlaps the caller's next steps and the next launch is ordered
 *                                     after it. The count table is keyed by a per-process random secret
 *                                     with bounded probing (csrc/kc_admit.h); an evicted key, or one whose
 *                                     admission failed, counts from zero again and is re-admitted on its
 *                                     next min_seen verified appearances. A failed admission leaves the
 *                                     verdicts unchanged and the keys uncached. Verkeys come from NYM
 *                                     records (plenum/server/request_handlers/utils.py:30-39): signers repeat
 *   pv_key_cache_auto_stats(a, f)     keys admitted automatically / admissions that failed */
int pv_key_cache_configure(uint32_t capacity);
int pv_key_cache_put(const uint8_t* pks, uint64_t n);
int pv_key_cache_clear(void);
int pv_key_cache_enable(int enable);
int pv_key_cache_stats(uint32_t* size, uint32_t* capacity);
int pv_key_cache_contains(const uint8_t* pk);
int pv_key_cache_auto(uint32_t min_seen);
int pv_key_cache_auto_stats(uint64_t* admitted, uint64_t* failed);

/* Batched base58 decode (Bitcoin alphabet, PyPI base58 2.x b58decode semantics: trailing ASCII
 * whitespace stripped, each leading '1' -> 0x00). Input: strings concatenated in `chars` with
 * n+1 offsets. Output: out[i * out_stride ...], out_len[i] bytes, status[i] = 0 ok, 1 invalid
 * character, 2 longer than out_stride. */
int pv_b58decode_batch(const char* chars, const uint64_t* off, uint64_t n, uint8_t* out,
                       uint64_t out_stride, uint32_t* out_len, uint8_t* status);

/* base58.b58encode of data[0..len): writes min(cap, result) chars, returns the full encoded length. */
int64_t pv_b58encode(const uint8_t* data, uint64_t len, char* out, uint64_t cap);

/* Batched DidVerifier key resolution (plenum/common/verifier.py:24-50) for n (identifier, verkey)
 * string pairs (concatenated + offsets; an empty identifier means None, has_verkey[i] = 0 means
 * verkey None). pk_out receives 32-byte raw keys. status[i]:
 *   0 ok, raw 32-byte key in pk_out
 *   1 ValueError("'verkey' should be a non-empty string")
 *   2 InvalidKey (key resolution failed: bad base58, wrong length, bad hex)
 *   3 empty key: the stp_core Verifier has no key and verify() returns False
 *   4 identifier is not valid base58 (b58decode raises ValueError in DidVerifier.__init__)
 * has_verkey/pk_out/status are per request. */
int pv_resolve_verkeys(const char* idr_chars, const uint64_t* idr_off, const char* vk_chars,
                       const uint64_t* vk_off, const uint8_t* has_verkey, uint64_t n, uint8_t* pk_out,
                       uint8_t* status);

/* Device ingress front end: everything between the received strings and
 * crypto_sign_open, for a whole batch, on the GPU, then the verification itself. Replaces per
 * signature: plenum/server/client_authn.py:97 b58decode(sig), plenum/common/verifier.py:24-51
 * DidVerifier(verkey, identifier) key resolution, stp_core/crypto/nacl_wrappers.py:108
 * `signature + msg`. Inputs (device pointers, offsets relative to their blob):
 *   n verifications: sig_chars/sig_off  base58 signature strings (after str.rstrip(); non-ASCII
 *                                       bytes are invalid characters)
 *                    msg_idx[n]         message M of verification i (signing-serialized request)
 *                    signer_idx[n]      signer of verification i
 *   n_msgs messages: msg/msg_off        (readable for 8 bytes past msg_off[n_msgs];
 *                                       msg_bytes_total = sum over i of len(M[msg_idx[i]]), it
 *                                       sizes the assembly buffer; an understatement empties
 *                                       every record and reports status 3, never a fault)
 *   n_signers:       idr_chars/idr_off  identifier strings ("" = None), vk_chars/vk_off verkey
 *                                       strings as getVerkey returned them, vk_present[u] = 0 when
 *                                       the verkey is None
 * Outputs: verdict bit i (as pv_verify_batch: crypto_sign_open(b58decode(sig) || M, key) == 0) and
 * status[i]:
 *   0       verified (the verdict bit is the result)
 *   1       the signature is not base58 (InvalidSignatureFormat)
 *   2       the signature decodes to more than 96 bytes (not assembled; verdict 0)
 *   3       msg_idx / signer_idx out of range, or msg_bytes_total too small (verdict 0)
 *   16 + k  signer key resolution status k (pv_resolve_verkeys codes; k = 3: no key, verify() is
 *           False) — the verdict bit is 0
 * Enqueued on `stream` (NULL = the library stream); the workspace is the library's and is handed
 * over between streams as for pv_verify_batch_device, so calls on different streams and threads are
 * safe. pv_ingress_verify is the same on host buffers (synchronous; validates
 * offsets and indices and returns PV_ERR_ARG instead of launching on bad input).
 * pv_ingress_front_ms: device time of the most recent call's front end (decode, resolve, scan,
 * assembly), excluding the verification kernels. */
int pv_ingress_verify_device(const char* d_sig_chars, const uint64_t* d_sig_off, const uint32_t* d_msg_idx,
                             const uint32_t* d_signer_idx, uint64_t n, const uint8_t* d_msg, const uint64_t* d_msg_off,
                             uint64_t n_msgs, uint64_t msg_bytes_total, const char* d_idr_chars,
                             const uint64_t* d_idr_off, const char* d_vk_chars, const uint64_t* d_vk_off,
                             const uint8_t* d_vk_present, uint64_t n_signers, uint8_t* d_status,
                             uint64_t* d_verdict_words, void* stream);
int pv_ingress_verify(const char* sig_chars, const uint64_t* sig_off, const uint32_t* msg_idx,
                      const uint32_t* signer_idx, uint64_t n, const uint8_t* msg, const uint64_t* msg_off,
                      uint64_t n_msgs, const char* idr_chars, const uint64_t* idr_off, const char* vk_chars,
                      const uint64_t* vk_off, const uint8_t* vk_present, uint64_t n_signers, uint8_t* status,
                      uint8_t* verdict_bits);
int pv_ingress_front_ms(double* ms);

/* Signing serialization of received JSON requests on the host, many threads:
 * request i is the JSON text json[off[i] : off[i+1]] that ZStack.deserializeMsg decodes
 * (stp_zmq/zstack.py:881-885); the output is the signing-serialized message
 * (common/serializers/signing_serializer.py:35-92, serialization.py:27-36) of
 *   PV_SER_DICT     json.loads(text)
 *   PV_SER_AUTHN    json.loads(text) minus top-level {signature, signatures, fees}
 *                   (CoreAuthMixin.authenticate, plenum/server/client_authn.py:198,232)
 *   PV_SER_REQUEST  Request(**json.loads(text)).as_dict minus those keys (Node.verifySignature,
 *                   plenum/server/node.py:2636-2650), and digest[32 i .. 32 i + 32) =
 *                   sha256(serialize(signingState())) (plenum/common/request.py:86-121)
 * written to msg_out[msg_off[i] : msg_off[i+1]]. plugin_fields: NUL-separated names ending with an
 * empty name (PLUGIN_CLIENT_REQUEST_FIELDS, request.py:37-39), or NULL. status[i]:
 *   PV_SER_OK          serialized
 *   PV_SER_INVALID     json.loads would raise (bad UTF-8, bad JSON, control characters...)
 *   PV_SER_NOT_OBJECT  the document is not a JSON object
 *   PV_SER_DEFER       valid, but outside what is reproduced bit-for-bit here (floats, NaN/Infinity,
 *                      lone surrogates, nesting > 512, ints > 4,300 digits, a request-mode digest
 *                      whose Python evaluation raises): the caller serializes it in Python
 * Returns PV_ERR_ARG with msg_off[n] = the bytes needed when msg_cap is too small. */
#define PV_SER_DICT 0
#define PV_SER_AUTHN 1
#define PV_SER_REQUEST 2
#define PV_SER_OK 0
#define PV_SER_INVALID 1
#define PV_SER_NOT_OBJECT 2
#define PV_SER_DEFER 3
int pv_signing_serialize_json(const char* json, const uint64_t* off, uint64_t n, int mode, const char* plugin_fields,
                              int threads, uint8_t* msg_out, uint64_t msg_cap, uint64_t* msg_off, uint8_t* digest,
                              uint8_t* status);

/* Fused ingress planning (replaces the per-request Python planning of the wire
 * path: json.loads -> Request(**msg).as_dict -> CoreAuthMixin._select_signatures,
 * plenum/server/client_authn.py:240-264, node.py:1643,2636-2650). ONE parse of every received
 * request gives what pv_signing_serialize_json(PV_SER_REQUEST) gives (msg, msg_off, digest, status)
 * and its signature plan:
 *   kind[i]  PV_PLAN_SINGLE  {identifier: signature}: both non-empty strings (the first branch of
 *                            _select_signatures)
 *            PV_PLAN_MULTI   the `signatures` object (non-empty, string values, no duplicate
 *                            names) of a request without a usable identifier/signature pair and
 *                            without a `signature` value (so the verified-request cache stores None)
 *            PV_PLAN_PY      anything else: the caller runs the reference's Python path for it
 *                            (serialization status not OK, not an object, a `self` key, plugin
 *                            fields registered, operation not an object or its type not a string,
 *                            non-ASCII or escaped identifier/signature text, trailing whitespace, ...)
 *   type_id[i]      operation["type"] of a SINGLE/MULTI request, as an index into the distinct type
 *                   strings types[type_off[t] : type_off[t+1]] (first-appearance order)
 *   pair_off[i]     request i's (identifier, signature) pairs are [pair_off[i], pair_off[i+1])
 *                   (dict order); pair_name[p] indexes the distinct identifier strings
 *                   names[name_off[k] : name_off[k+1]]; sigs[sig_off[p] : sig_off[p+1]] is the
 *                   signature text (ASCII)
 * Capacities: msg_cap as pv_signing_serialize_json; sigs_cap, names_cap and types_cap are byte
 * capacities and off[n] always suffices (every string is a substring of its request); pair_cap =
 * off[n] / 6 + 1 always suffices (a pair takes at least 6 bytes of JSON). name_off holds
 * pair_cap + 1 entries (distinct names <= pairs), type_off n + 1 (distinct types <= requests).
 * Returns PV_ERR_ARG with msg_off[n] = bytes needed when msg_cap is too small. */
#define PV_PLAN_PY 0
#define PV_PLAN_SINGLE 1
#define PV_PLAN_MULTI 2
typedef struct {
    uint8_t* msg_out; /* in: buffers */
    uint64_t msg_cap;
    uint64_t* msg_off;  /* [n + 1] */
    uint8_t* digest;    /* [32 n] */
    uint8_t* status;    /* [n] PV_SER_* */
    uint8_t* kind;      /* [n] PV_PLAN_* */
    uint32_t* type_id;  /* [n] */
    uint64_t* pair_off; /* [n + 1] */
    uint32_t* pair_name; /* [pair_cap] */
    uint64_t* sig_off;   /* [pair_cap + 1] */
    uint64_t pair_cap;
    char* sigs;
    uint64_t sigs_cap;
    char* names;
    uint64_t* name_off; /* [pair_cap + 1] */
    uint64_t names_cap;
    char* types;
    uint64_t* type_off; /* [n + 1] */
    uint64_t types_cap;
    char* keys_hex;   /* [65 n] or NULL: Request.digest of request i as 64 lowercase hex digits + '\n' */
    char* sig_lines;  /* [sigs_cap + pair_cap] or NULL: every signature text followed by '\n' */
    uint64_t n_pairs; /* out */
    uint64_t n_names; /* out */
    uint64_t n_types; /* out */
} PvWirePlan;
int pv_wire_plan(const char* json, const uint64_t* off, uint64_t n, const char* plugin_fields, int threads,
                 PvWirePlan* plan);

/* Multi-GPU: one process per GPU. pv_comm_unique_id on rank 0, broadcast the 128 bytes by any
 * channel, pv_comm_init on every rank (after pv_init). pv_allgather_verdicts gathers
 * words_per_rank 64-bit verdict words from every rank into d_all (nranks * words_per_rank) with
 * one RCCL all-gather on `stream`. pv_comm_count reports what RCCL itself sees for this rank's
 * communicator (ncclCommCount / ncclCommUserRank), so a multi-GPU run can show the ranks RCCL joined
 * (plenum/server/node.py:1518-1527 is the batch feed these shards come from). */
int pv_comm_unique_id(uint8_t out[128]);
int pv_comm_init(int nranks, int rank, const uint8_t id[128]);
int pv_allgather_verdicts(const uint64_t* d_local, uint64_t words_per_rank, uint64_t* d_all, void* stream);
int pv_comm_count(int* nranks, int* rank);
void pv_comm_destroy(void);

/* Device memory helpers so hosts without a GPU framework can stage data (bench, smoke).
 * pv_memcpy_h2d / pv_memcpy_d2h are ordered after every launch enqueued before them (on any stream:
 * the copy runs on the library stream after the last launch's completion event) and return once the
 * copy is done. So pv_verify_batch_device(..., NULL) followed by pv_memcpy_d2h of its verdict words
 * needs no pv_sync, and pv_memcpy_h2d right after a launch never overwrites inputs that launch still
 * reads. pv_sync waits for all work on the calling thread's current device. */
int pv_dev_alloc(void** p, uint64_t bytes);
int pv_dev_free(void* p);
int pv_memcpy_h2d(void* dst, const void* src, uint64_t bytes);
int pv_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
int pv_sync(void);
/* Caller streams for the *_device entry points, for hosts without a GPU framework. A stream handed
 * to pv_verify_batch_device / pv_ingress_verify_device may be any stream of this device: batches
 * enqueued on DIFFERENT streams are ordered by the library (each launch waits for the previous one
 * to release the shared workspace), so they never race; pv_stream_destroy synchronises first. */
int pv_stream_create(void** stream);
int pv_stream_destroy(void* stream);
int pv_stream_sync(void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PLENUM_VERIFY_H */
