"""ctypes binding of libplenum_verify.so (include/plenum_verify.h).

This is the only way the package reaches the verification arithmetic: there is no CPU fallback.
If the library is missing, or no gfx950 GPU is visible, verification calls raise
``NativeUnavailable`` instead of silently computing elsewhere.
"""
import ctypes
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PLENUM_AMD_LIB", os.path.join(_HERE, "libplenum_verify.so"))

PV_OK = 0
PV_ERR_ARG = -4
PV_BLOB_SLACK = 256
PV_ABI_VERSION = 1
PV_BUILD_COMB_FUSED = 1  # pv_build_flags(): [S]B and [k](-A) of the comb path in one kernel

PV_STAGES = ("keys", "prep", "table", "msm", "encode")  # PV_STAGE_* order
PV_PATH_AUTO, PV_PATH_STRAUS, PV_PATH_COMB, PV_PATH_LATENCY = 0, 1, 2, 3
PATH_NAMES = ("straus", "comb", "latency")  # forced arithmetic paths (tests run every one)

# exported symbol -> (restype, argtypes); kept in sync with include/plenum_verify.h
_c_u8p = ctypes.POINTER(ctypes.c_uint8)
_c_u64p = ctypes.POINTER(ctypes.c_uint64)
_c_u32p = ctypes.POINTER(ctypes.c_uint32)
SIGNATURES = {
    "pv_abi_version": (ctypes.c_int, []),
    "pv_build_flags": (ctypes.c_uint32, []),
    "pv_device_count": (ctypes.c_int, []),
    "pv_init": (ctypes.c_int, [ctypes.c_int]),
    "pv_shutdown": (None, []),
    "pv_last_error": (ctypes.c_char_p, []),
    "pv_verify_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_void_p]),
    "pv_verify_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "pv_set_timing": (ctypes.c_int, [ctypes.c_int]),
    "pv_set_path": (ctypes.c_int, [ctypes.c_int]),
    "pv_last_path": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32)]),
    "pv_last_split": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32)] * 3),
    "pv_stage_times": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "pv_kernel_times": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "pv_b58decode_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "pv_b58encode": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]),
    "pv_resolve_verkeys": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "pv_ingress_verify_device": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
                                 + [ctypes.c_void_p] * 5 + [ctypes.c_uint64] + [ctypes.c_void_p] * 3),
    "pv_ingress_verify": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64] + [ctypes.c_void_p] * 5 + [ctypes.c_uint64]
                          + [ctypes.c_void_p] * 2),
    "pv_signing_serialize_json": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                                 ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "pv_wire_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.c_void_p]),
    "pv_ingress_front_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double)]),
    "pv_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_comm_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "pv_allgather_verdicts": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "pv_comm_destroy": (None, []),
    "pv_dev_alloc": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64]),
    "pv_dev_free": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_memcpy_h2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "pv_memcpy_d2h": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "pv_sync": (ctypes.c_int, []),
    "pv_key_cache_configure": (ctypes.c_int, [ctypes.c_uint32]),
    "pv_key_cache_put": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "pv_key_cache_clear": (ctypes.c_int, []),
    "pv_key_cache_enable": (ctypes.c_int, [ctypes.c_int]),
    "pv_key_cache_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "pv_key_cache_contains": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_key_cache_auto": (ctypes.c_int, [ctypes.c_uint32]),
    "pv_key_cache_auto_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "pv_last_zero_copy": (ctypes.c_int, []),
    "pv_init_devices": (ctypes.c_int, [ctypes.c_uint32]),
    "pv_verify_batch_multi_gpu": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "pv_multi_gpu_devices": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "pv_multi_gpu_comm_ranks": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "pv_comm_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "pv_shard_plan": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, _c_u64p, _c_u64p]),
    "pv_host_alloc": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64]),
    "pv_host_free": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "pv_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_host_is_pinned": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "pv_test_inject": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "pv_test_clock_stamps": (ctypes.c_int, [_c_u64p, ctypes.c_uint32]),
    "pv_stream_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "pv_stream_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pv_stream_sync": (ctypes.c_int, [ctypes.c_void_p]),
}


class NativeUnavailable(RuntimeError):
    """The HIP engine cannot run here (library missing or no gfx950 device)."""


class NativeError(RuntimeError):
    """An infrastructure failure inside libplenum_verify (allocation, launch, comm)."""


_lib = None
_lock = threading.Lock()
_device = None


def lib():
    """The loaded library (loading does not touch the GPU)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise NativeUnavailable(
                        "libplenum_verify.so not built at %s (run __graft_entry__.build() or make -C indy-plenum_amd)"
                        % LIB_PATH)
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                if L.pv_abi_version() != PV_ABI_VERSION:
                    raise NativeUnavailable("ABI version mismatch")
                _lib = L
    return _lib


def check(rc, what):
    if rc != PV_OK:
        msg = lib().pv_last_error()
        raise NativeError("%s failed (%d): %s" % (what, rc, msg.decode(errors="replace") if msg else ""))


def ensure_device(device=None):
    """Bind this process to a GPU (once). Raises NativeUnavailable when none is visible."""
    global _device
    if _device is not None:
        return _device
    L = lib()
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = L.pv_device_count()
    if ndev <= 0:
        raise NativeUnavailable("no HIP device visible: the verification engine is GPU-only")
    rc = L.pv_init(device % ndev)
    if rc != PV_OK:
        raise NativeUnavailable("pv_init failed: %s" % L.pv_last_error().decode(errors="replace"))
    _device = device % ndev
    return _device


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


_U8, _U64 = np.dtype(np.uint8), np.dtype(np.uint64)
_fast = None  # the CPython binding (_fastcall) once bound to the loaded library, False if not built


def _fastcall():
    global _fast
    if _fast is None:
        if os.environ.get("PLENUM_AMD_NO_FASTCALL"):  # the ctypes path (A/B, debugging)
            _fast = False
            return _fast
        try:
            from . import _fastcall as fc
            fc.bind(ctypes.cast(lib().pv_verify_batch, ctypes.c_void_p).value)
            _fast = fc
        except ImportError:
            _fast = False
    return _fast


def verify_sm_batch(blob, offsets, pks):
    """crypto_sign_open verdicts for n concatenated (sig || msg) records.

    blob: uint8 array; offsets: uint64 array of n+1 prefix offsets into blob; pks: uint8 (n, 32).
    Returns a bool array of n verdicts (True = libnacl.crypto_sign_open would not raise)."""
    if _device is None:
        ensure_device()
    # numpy inputs of the right type and layout pass through untouched (Plenum's small calls: every
    # microsecond here is on the request's latency)
    if type(offsets) is not np.ndarray or offsets.dtype != _U64 or not offsets.flags.c_contiguous:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.shape[0] - 1
    if n <= 0:
        return np.zeros(0, dtype=bool)
    if type(blob) is not np.ndarray or blob.dtype != _U8 or not blob.flags.c_contiguous:
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, dtype=np.uint8)
    if type(pks) is not np.ndarray or pks.dtype != _U8 or not pks.flags.c_contiguous:
        pks = np.ascontiguousarray(pks, dtype=np.uint8)
    if pks.size != 32 * n:
        raise ValueError("pks must hold n x 32 key bytes")
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    fc = _fast if _fast is not None else _fastcall()
    if fc:  # the same C ABI call without ctypes' per-array marshalling
        rc = fc.verify(blob, offsets, pks, bits)
    else:
        if int(offsets[n]) > blob.size:
            raise ValueError("verify: inconsistent blob / offsets / keys / verdict sizes")
        rc = lib().pv_verify_batch(_ptr(blob), _ptr(offsets), n, _ptr(pks), _ptr(bits))
    if rc:
        check(rc, "pv_verify_batch")
    return np.unpackbits(bits, count=n, bitorder="little").view(bool)


def verify_one(pk, sm):
    """crypto_sign_open verdict of ONE (32-byte key, sig || msg) pair: the unbatched drop-in's call
    (Verifier.verify outside an authenticate_batch), without the arrays verify_sm_batch builds."""
    if _device is None:
        ensure_device()
    fc = _fast if _fast is not None else _fastcall()
    if fc and hasattr(fc, "verify_one"):
        rc = fc.verify_one(pk, sm)
        if rc < 0:
            check(rc, "pv_verify_batch")
        return bool(rc)
    off = np.array([0, len(sm)], dtype=np.uint64)
    return bool(verify_sm_batch(np.frombuffer(bytes(sm) or b"\0", dtype=np.uint8), off,
                                np.frombuffer(bytes(pk), dtype=np.uint8))[0])


PV_INJECT_STAGE = 1  # pv_test_inject: fail the next host-buffer stagings of a device


class HostArena:
    """numpy arrays in the library's pinned host memory (pv_host_alloc). pv_verify_batch /
    pv_verify_batch_multi_gpu DMA inputs that live there straight to HBM (no pageable -> pinned
    staging copy): a node that receives its requests into such buffers, or builds its batch there,
    feeds the GPUs at PCIe rate. The block is freed when the last array viewing it is collected."""

    @staticmethod
    def empty(shape, dtype=np.uint8):
        dtype = np.dtype(dtype)
        count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
        nbytes = max(1, count * dtype.itemsize)
        p = ctypes.c_void_p()
        check(lib().pv_host_alloc(ctypes.byref(p), nbytes), "pv_host_alloc")
        buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
        weakref.finalize(buf, lib().pv_host_free, p.value)
        return np.frombuffer(buf, dtype=np.uint8, count=count * dtype.itemsize).view(dtype).reshape(shape)

    @staticmethod
    def is_pinned(arr):
        arr = np.asarray(arr)
        return bool(lib().pv_host_is_pinned(arr.ctypes.data, arr.nbytes))

    @classmethod
    def batch(cls, blob, offsets, pks):
        """(blob, offsets, pks) copied into arena arrays, offsets rebased to 0 (the form whose offsets
        are DMA'd as they are)."""
        offsets = np.asarray(offsets, dtype=np.uint64)
        base, end = int(offsets[0]), int(offsets[-1])
        b = cls.empty(max(1, end - base))
        b[:end - base] = np.asarray(blob, np.uint8)[base:end]
        o = cls.empty(offsets.shape, np.uint64)
        np.subtract(offsets, np.uint64(base), out=o)
        k = cls.empty((len(offsets) - 1, 32))
        k[:] = np.asarray(pks, np.uint8).reshape(-1, 32)
        return b, o, k


def inject_stage_failures(device, count):
    """Test hook: the next `count` host-buffer stagings on `device` fail (pv_test_inject, declared in
    include/plenum_verify_test.h; the library refuses it unless PV_ENABLE_TEST_HOOKS=1 is set)."""
    check(lib().pv_test_inject(PV_INJECT_STAGE, int(device), int(count)), "pv_test_inject")


def comb_fused():
    """True if the library computes the comb path's [S]B and [k](-A) in one kernel (pv_comb_ab_kernel)."""
    return bool(lib().pv_build_flags() & PV_BUILD_COMB_FUSED)


def last_zero_copy():
    """True if the most recent host-buffer call (pv_verify_batch) took the zero-copy form."""
    return bool(lib().pv_last_zero_copy())


def shard_plan(n, ndev):
    """(bounds uint64[ndev + 1], verdict words per shard) of pv_verify_batch_multi_gpu's split of n
    requests over ndev devices (host-only, no GPU needed)."""
    b = np.zeros(ndev + 1, np.uint64)
    w = ctypes.c_uint64()
    check(lib().pv_shard_plan(int(n), int(ndev), b.ctypes.data_as(_c_u64p), ctypes.byref(w)), "pv_shard_plan")
    return b, w.value


_multi_devices = None


def ensure_devices(devices):
    """Bind this process to several GPUs for pv_verify_batch_multi_gpu (one context and one RCCL
    communicator per device, ncclCommInitAll). Raises NativeUnavailable when they are not visible."""
    global _multi_devices
    devices = tuple(sorted(set(int(d) for d in devices)))
    if _multi_devices == devices:
        return devices
    L = lib()
    ndev = L.pv_device_count()
    if ndev <= 0:
        raise NativeUnavailable("no HIP device visible: the verification engine is GPU-only")
    if not devices or devices[-1] >= ndev or devices[0] < 0:
        raise NativeUnavailable("devices %s not visible (%d GPUs)" % (list(devices), ndev))
    mask = 0
    for d in devices:
        mask |= 1 << d
    rc = L.pv_init_devices(mask)
    if rc != PV_OK:
        raise NativeUnavailable("pv_init_devices failed: %s" % L.pv_last_error().decode(errors="replace"))
    _multi_devices = devices
    return devices


def multi_gpu_clique():
    """The in-process clique as RCCL reports it: {"devices": [...], "nranks": ncclCommCount,
    "user_ranks": [ncclCommUserRank per device]} (pv_multi_gpu_devices / pv_multi_gpu_comm_ranks)."""
    L = lib()
    devs = (ctypes.c_int * 16)()
    nd = L.pv_multi_gpu_devices(devs, 16)
    nr, ranks = ctypes.c_int(), (ctypes.c_int * 16)()
    check(L.pv_multi_gpu_comm_ranks(ctypes.byref(nr), ranks, 16), "pv_multi_gpu_comm_ranks")
    return {"devices": list(devs[:nd]), "nranks": nr.value, "user_ranks": list(ranks[:nd])}


def comm_count():
    """(nranks, rank) of this process's rank communicator as RCCL reports them (pv_comm_count)."""
    nr, rk = ctypes.c_int(), ctypes.c_int()
    check(lib().pv_comm_count(ctypes.byref(nr), ctypes.byref(rk)), "pv_comm_count")
    return nr.value, rk.value


def verify_sm_batch_multi(blob, offsets, pks, devices=None):
    """verify_sm_batch sharded over several GPUs of this process (pv_verify_batch_multi_gpu: one shard
    per device, verdict bitmaps gathered with one RCCL all-gather). devices: the GPUs to use (default:
    every visible one, or the set already bound)."""
    if devices is None:
        devices = _multi_devices or range(max(1, lib().pv_device_count()))
    ensure_devices(devices)
    L = lib()
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    if n <= 0:
        return np.zeros(0, dtype=bool)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(n, 32)
    bits = np.zeros((n + 7) // 8, dtype=np.uint8)
    check(L.pv_verify_batch_multi_gpu(_ptr(blob), _ptr(offsets), n, _ptr(pks), _ptr(bits)),
          "pv_verify_batch_multi_gpu")
    return np.unpackbits(bits, bitorder="little")[:n].astype(bool)


def multi_gpu_engine(devices):
    """An engine callable (blob, off, pks) -> verdicts for authenticate_batch(engine=...) that shards
    every batch over `devices` (SURVEY.md §8b pv_verify_batch_multi_gpu)."""
    devices = tuple(devices)

    def engine(blob, off, pks):
        return verify_sm_batch_multi(blob, off, pks, devices)

    engine.devices = devices
    return engine


def set_path(mode):
    """Select the arithmetic path (PV_PATH_AUTO / PV_PATH_STRAUS / PV_PATH_COMB / PV_PATH_LATENCY);
    verdicts are identical on every path."""
    check(lib().pv_set_path(int(mode)), "pv_set_path")


def last_path():
    """(path, distinct keys) of the most recent chunk: path is PV_PATH_STRAUS or PV_PATH_COMB."""
    p, u = ctypes.c_int(), ctypes.c_uint32()
    check(lib().pv_last_path(ctypes.byref(p), ctypes.byref(u)), "pv_last_path")
    return p.value, u.value


def last_split():
    """(distinct keys, keys with a comb table, requests verified with them) of the most recent
    chunk; the remaining requests took the Straus path. Synchronises (via pv_last_path)."""
    last_path()
    v = [ctypes.c_uint32() for _ in range(3)]
    check(lib().pv_last_split(*[ctypes.byref(x) for x in v]), "pv_last_split")
    return tuple(x.value for x in v)


def _blob(items):
    """Concatenate byte strings -> (uint8 blob (never empty), uint64 offsets)."""
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        np.cumsum(np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items)), out=off[1:])
    joined = b"".join(items)
    return (np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, np.uint8)), off


def ingress_verify_arrays(sig_blob, sig_off, msg_blob, msg_off, msg_idx, signer_idx, idr_blob, idr_off, vk_blob,
                          vk_off, vk_present):
    """pv_ingress_verify on packed arrays (uint8 blobs, uint64 offsets, uint32 indices, uint8 flags):
    GPU base58 decode of every signature, GPU key resolution per signer, device-side sm assembly
    and verification. Returns (status uint8[n], verdict bool[n]); status codes in
    include/plenum_verify.h."""
    ensure_device()
    n = len(sig_off) - 1
    if n <= 0:
        return np.zeros(0, np.uint8), np.zeros(0, bool)
    status = np.zeros(n, np.uint8)
    bits = np.zeros((n + 7) // 8, np.uint8)
    c = np.ascontiguousarray
    args = [c(sig_blob, np.uint8), c(sig_off, np.uint64), c(msg_idx, np.uint32), c(signer_idx, np.uint32),
            c(msg_blob, np.uint8), c(msg_off, np.uint64), c(idr_blob, np.uint8), c(idr_off, np.uint64),
            c(vk_blob, np.uint8), c(vk_off, np.uint64), c(vk_present, np.uint8)]
    sb, so, mi, si, mb, mo, ib, io, vb, vo, vp = [a if a.size else np.zeros(1, a.dtype) for a in args]
    check(lib().pv_ingress_verify(_ptr(sb), _ptr(so), _ptr(mi), _ptr(si), n, _ptr(mb), _ptr(mo), len(msg_off) - 1,
                                  _ptr(ib), _ptr(io), _ptr(vb), _ptr(vo), _ptr(vp), len(idr_off) - 1,
                                  _ptr(status), _ptr(bits)), "pv_ingress_verify")
    return status, np.unpackbits(bits, bitorder="little")[:n].astype(bool)


def ingress_verify(sigs, msgs, msg_idx, signer_idx, idrs, vks):
    """ingress_verify_arrays on Python lists: sigs (n byte strings), msgs (byte strings),
    msg_idx / signer_idx (n ints), idrs (identifier bytes per signer, b"" = None), vks (verkey
    bytes or None per signer)."""
    sig_b, sig_o = _blob(list(sigs))
    msg_b, msg_o = _blob(list(msgs))
    idr_b, idr_o = _blob(list(idrs))
    vk_b, vk_o = _blob([v if v is not None else b"" for v in vks])
    vkp = np.array([v is not None for v in vks], dtype=np.uint8)
    return ingress_verify_arrays(sig_b, sig_o, msg_b, msg_o, np.asarray(msg_idx, np.uint32),
                                 np.asarray(signer_idx, np.uint32), idr_b, idr_o, vk_b, vk_o, vkp)


class KeyCache:
    """The engine's node-side key cache (include/plenum_verify.h pv_key_cache_*): known signers'
    keys verified with 32 comb-table additions on the latency path instead of 252 doublings."""

    @staticmethod
    def configure(capacity):
        ensure_device()
        check(lib().pv_key_cache_configure(int(capacity)), "pv_key_cache_configure")

    @staticmethod
    def put(pks):
        """pks: iterable of 32-byte keys, or a uint8 array (n, 32)."""
        ensure_device()
        a = np.frombuffer(b"".join(pks), np.uint8) if not isinstance(pks, np.ndarray) else pks
        a = np.ascontiguousarray(a, np.uint8).reshape(-1)
        if a.size % 32:
            raise ValueError("keys must be 32 bytes each")
        n = a.size // 32
        check(lib().pv_key_cache_put(_ptr(a if a.size else np.zeros(32, np.uint8)), n), "pv_key_cache_put")

    @staticmethod
    def clear():
        check(lib().pv_key_cache_clear(), "pv_key_cache_clear")

    @staticmethod
    def enable(on=True):
        check(lib().pv_key_cache_enable(1 if on else 0), "pv_key_cache_enable")

    @staticmethod
    def stats():
        size, cap = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().pv_key_cache_stats(ctypes.byref(size), ctypes.byref(cap)), "pv_key_cache_stats")
        return size.value, cap.value

    @staticmethod
    def auto(min_seen):
        """Automatic admission: a key seen min_seen times in host batches of <= 4,096 requests is put
        into the cache behind that batch (0 = off)."""
        check(lib().pv_key_cache_auto(int(min_seen)), "pv_key_cache_auto")

    @staticmethod
    def auto_stats():
        a, f = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().pv_key_cache_auto_stats(ctypes.byref(a), ctypes.byref(f)), "pv_key_cache_auto_stats")
        return a.value, f.value

    @staticmethod
    def contains(pk):
        b = np.frombuffer(bytes(pk), np.uint8)
        if b.size != 32:
            raise ValueError("keys must be 32 bytes each")
        return bool(lib().pv_key_cache_contains(_ptr(b)))

