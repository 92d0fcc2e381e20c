"""Multi-GPU sharding of a verification batch: one process per GPU, contiguous
shards by request index, each rank verifies its shard, then ONE all-gather of the per-shard verdict
bitmaps (RCCL over xGMI through libplenum_verify's pv_allgather_verdicts). No other cross-GPU
traffic. Shard boundaries fall on 64-request verdict words, so every rank's bitmap is a whole
number of 64-bit words and the gathered words concatenate into the global bitmap.

The gather is pluggable so the same logic runs under torch.distributed/gloo on CPU in tests.
"""
import ctypes

import numpy as np


def shard_bounds(n, world, rank):
    """Requests [lo, hi) of ``rank``'s shard of an n-request batch."""
    words = (n + 63) // 64
    w_lo = words * rank // world
    w_hi = words * (rank + 1) // world
    return min(n, 64 * w_lo), min(n, 64 * w_hi)


def words_per_rank(n, world):
    words = (n + 63) // 64
    return max(words * (r + 1) // world - words * r // world for r in range(world))


def assemble(gathered, n, world):
    """gathered: (world, words_per_rank) uint64 words, rank r's shard in row r (padded) -> n bools."""
    gathered = np.asarray(gathered, dtype=np.uint64).reshape(world, -1)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(n, world, r)
        w = (hi - lo + 63) // 64
        parts.append(gathered[r, :w])
    words = np.concatenate(parts) if parts else np.zeros(0, np.uint64)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    out = np.zeros(n, dtype=bool)
    pos = 0
    for r in range(world):
        lo, hi = shard_bounds(n, world, r)
        w = (hi - lo + 63) // 64
        out[lo:hi] = bits[64 * pos: 64 * pos + (hi - lo)]
        pos += w
    return out


def slice_batch(blob, off, pks, lo, hi):
    """The sub-batch [lo, hi) with offsets rebased to its own blob slice."""
    base = int(off[lo])
    sub_off = (np.asarray(off[lo:hi + 1], dtype=np.uint64) - np.uint64(base))
    return blob[base:int(off[hi])], sub_off, pks[lo:hi]


def pack_words(verdicts, nwords):
    bits = np.zeros(nwords * 64, dtype=np.uint8)
    bits[:len(verdicts)] = verdicts
    return np.packbits(bits, bitorder="little").view(np.uint64)


def verify_sharded(blob, off, pks, rank, world, verify_fn, allgather_fn):
    """Verify this rank's shard with ``verify_fn(blob, off, pks) -> bools`` and gather everyone's
    verdict words with ``allgather_fn(local_words uint64[wpr]) -> uint64[world, wpr]``.
    Returns the full n-request verdict array on every rank."""
    n = len(off) - 1
    lo, hi = shard_bounds(n, world, rank)
    wpr = words_per_rank(n, world)
    local = verify_fn(*slice_batch(blob, off, pks, lo, hi)) if hi > lo else np.zeros(0, dtype=bool)
    gathered = allgather_fn(pack_words(np.asarray(local, dtype=np.uint8), wpr))
    return assemble(gathered, n, world)


class RcclGather:
    """allgather_fn over libplenum_verify's RCCL communicator (device buffers, one ncclAllGather)."""

    def __init__(self, world, rank, unique_id: bytes):
        from . import _native
        self._n = _native
        self.L = _native.lib()
        self.world = world
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        _native.check(self.L.pv_comm_init(world, rank, uid), "pv_comm_init")

    def comm_count(self):
        """(nranks, rank) as RCCL itself reports them for this communicator."""
        return self._n.comm_count()

    @staticmethod
    def unique_id() -> bytes:
        from . import _native
        uid = (ctypes.c_uint8 * 128)()
        _native.check(_native.lib().pv_comm_unique_id(uid), "pv_comm_unique_id")
        return bytes(uid)

    def __call__(self, local_words):
        L, nat = self.L, self._n
        local_words = np.ascontiguousarray(local_words, dtype=np.uint64)
        wpr = len(local_words)
        d_loc, d_all = ctypes.c_void_p(), ctypes.c_void_p()
        nat.check(L.pv_dev_alloc(ctypes.byref(d_loc), wpr * 8), "pv_dev_alloc")
        nat.check(L.pv_dev_alloc(ctypes.byref(d_all), wpr * 8 * self.world), "pv_dev_alloc")
        try:
            nat.check(L.pv_memcpy_h2d(d_loc, local_words.ctypes.data, wpr * 8), "pv_memcpy_h2d")
            nat.check(L.pv_allgather_verdicts(d_loc, wpr, d_all, None), "pv_allgather_verdicts")
            nat.check(L.pv_sync(), "pv_sync")
            out = np.zeros((self.world, wpr), dtype=np.uint64)
            nat.check(L.pv_memcpy_d2h(out.ctypes.data, d_all, out.nbytes), "pv_memcpy_d2h")
            return out
        finally:
            L.pv_dev_free(d_loc)
            L.pv_dev_free(d_all)
