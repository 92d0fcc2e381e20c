"""The N > 1 path on CPU: world_size-2 (and 3) torch.distributed/gloo processes shard a batch by
request index (plenum_amd.sharding), verify their shards (C oracle as the engine here; the HIP
engine on GPUs) and all-gather the verdict words; every rank must end with the single-process
verdicts. On GPUs the gather is pv_allgather_verdicts (RCCL); here torch's gloo all_gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from plenum_amd.sharding import assemble, pack_words, shard_bounds, verify_sharded, words_per_rank


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def make_batch(n, seed):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from oracle.oracle import Oracle
    from vectors import pack
    o = Oracle()
    rng = np.random.default_rng(seed)
    L = 2 ** 252 + 27742317777372353535851937790883648493
    keys = []
    for _ in range(8):
        a = int.from_bytes(rng.bytes(32), "little") % L or 1
        keys.append((a, o.scalarmult_base(a.to_bytes(32, "little"))))
    cases = []
    for i in range(n):
        a, A = keys[i % len(keys)]
        r = int.from_bytes(rng.bytes(32), "little") % L or 1
        m = rng.bytes(int(rng.integers(0, 120)))
        sig = bytearray(o.sign_raw(r.to_bytes(32, "little"), a.to_bytes(32, "little"), A, m))
        if i % 5 == 2:
            sig[40] ^= 4
        cases.append((bytes(sig) + m, A))
    return pack(cases), o


def worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        (blob, off, pks), o = make_batch(n, seed=5)

        def engine(b, of, pk):
            return o.verify_batch(b, of, pk).astype(bool)

        def gather(local_words):
            t = torch.from_numpy(local_words.view(np.int64).copy())
            out = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return np.stack([x.numpy().view(np.uint64) for x in out])

        got = verify_sharded(blob, off, pks, rank, world, engine, gather)
        q.put((rank, got.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 200), (3, 130)])
def test_sharded_verdicts_equal_single_process(world, n):
    (blob, off, pks), o = make_batch(n, seed=5)
    want = o.verify_batch(blob, off, pks).astype(bool)
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert np.array_equal(np.array(results[r], dtype=bool), want), r


def test_shard_bounds_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 4097):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a % 64 == 0
            wpr = words_per_rank(n, world)
            verd = np.arange(n) % 3 == 0
            rows = [pack_words(verd[a:b].astype(np.uint8), wpr) for a, b in spans]
            assert np.array_equal(assemble(np.stack(rows) if rows else np.zeros((world, 0)), n, world), verd)


def test_sharded_world8_gloo():
    """The 8-rank split of configs[4] in miniature: 8 gloo ranks, one all-gather, every rank ends with
    the single-process verdicts."""
    test_sharded_verdicts_equal_single_process(8, 600)


def test_config5_shard_arithmetic():
    """bench.py's N > 1 default is configs[4]: 64M requests over N GPUs, i.e. ceil(64M / N) per GPU
    in 64-aligned contiguous shards (8M per rank at N = 8, 8 launch chunks of 2^20), and the
    shards tile the 64M batch exactly as plenum_amd.sharding splits it."""
    import bench
    total = bench.CONFIG5_TOTAL
    assert total == 64 * 2 ** 20
    for world in (2, 4, 8):
        per = (total + world * 64 - 1) // (world * 64) * 64
        spans = [shard_bounds(total, world, r) for r in range(world)]
        assert all(hi - lo == per for lo, hi in spans), (world, spans[:2])
        assert spans[-1][1] == total and words_per_rank(total, world) * 64 == per
    assert (total // 8) == 8 * 2 ** 20 and (total // 8) // 2 ** 20 == 8


def test_bench_expected_bits_match_tamper():
    """The headline's must-reject records: every rank (re)computes each shard's expected bitmap from
    the seed alone, and it equals the set adversarial_batch.tamper() corrupted."""
    import bench
    import adversarial_batch
    n = 5000
    blob = np.zeros(n * 100, np.uint8)
    off = np.arange(0, n * 100 + 1, 100, dtype=np.uint64)
    for rank in (0, 3, 7):
        b2, idx = adversarial_batch.tamper(blob, off, bench.tamper_count(n), seed=1000 + rank)
        want = bench.expected_bits(n, rank)
        assert np.array_equal(np.nonzero(~want)[0], idx)
        changed = np.nonzero((b2 != blob).reshape(n, 100).any(axis=1))[0]
        assert np.array_equal(changed, idx)
