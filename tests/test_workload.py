"""The bench workloads' known answers on CPU (libsodium 1.0.18 as the checker): the configs[3]
multi-signature generator's corrupted records are exactly the ones libsodium rejects, and the
bench's authenticate_multi reduction follows client_authn.py:84-118 (threshold None)."""
import numpy as np


def test_multisig_corruption_is_exactly_what_libsodium_rejects(sodium):
    import nym_workload
    from oracle.oracle import cpu_verdicts
    n, k = 3000, 3
    blob, off, pks, bad = nym_workload.generate_multisig(0, n, k, workers=1, bad_frac=0.01, seed=4)
    assert bad.shape == (n, k) and bad.sum() == 90
    assert len(off) == n * k + 1 and pks.shape == (n * k, 32)
    want = cpu_verdicts(blob, off, pks).reshape(n, k)
    assert np.array_equal(want, ~bad)
    # records of one request share the payload; signers are the author and two endorsers
    for i in (0, 17, n - 1):
        msgs = {blob[int(off[i * k + j]) + 64:int(off[i * k + j + 1])].tobytes() for j in range(k)}
        assert len(msgs) == 1
        assert [pks[i * k + j].tobytes() for j in range(k)] == \
            [nym_workload._pool()[s]["vk"] for s in nym_workload.endorsers(i, k)]
    clean = nym_workload.generate_multisig(0, 200, k, workers=1)
    assert not clean[3].any() and cpu_verdicts(*clean[:3]).all()


def test_multisig_reduction_rule():
    import bench
    got = np.array([[1, 1, 1], [1, 0, 1], [0, 0, 0], [1, 1, 0]], bool)
    acc, correct = bench.multisig_reduce(got)
    assert acc.tolist() == [True, False, False, False]
    assert correct.tolist() == [3, 2, 0, 2]

