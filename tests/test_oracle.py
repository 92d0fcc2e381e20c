"""The oracle is pinned before it is trusted: golden libsodium verdicts, libsodium differential runs,
hashlib SHA-512, Python big-int scalar reduction, and the reference's own base58 KAT
(plenum/test/common/test_verifier.py:6-29)."""
import hashlib
import json
import os
import random

import pytest

from oracle.base58_ref import b58decode, b58encode

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
L = 2 ** 252 + 27742317777372353535851937790883648493


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_oracle_matches_golden_verdicts(oracle):
    cases = load("verdicts.json")
    assert len(cases) >= 200
    classes = set()
    for c in cases:
        got = oracle.sign_open_ok(bytes.fromhex(c["sm"]), bytes.fromhex(c["pk"]))
        assert got == c["ok"], c["cls"]
        classes.add((c["cls"], c["ok"]))
    # mixed-order keys with honest signatures verify sometimes (8 | k) and fail otherwise
    assert ("mixed_order_A", True) in classes and ("mixed_order_A", False) in classes


def test_oracle_vs_libsodium_random(oracle, sodium):
    from vectors import VectorGen
    g = VectorGen(sodium, oracle, seed=99)
    for cls in VectorGen.CLASSES:
        for _ in range(6):
            sm, pk = g.make(cls)
            assert oracle.sign_open_ok(sm, pk) == sodium.sign_open_ok(sm, pk), cls


def test_oracle_sha512_and_reduce(oracle):
    rng = random.Random(3)
    for n in (0, 1, 111, 112, 127, 128, 129, 239, 240, 255, 256, 363, 1000):
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.sha512(d) == hashlib.sha512(d).digest()
    for x in [0, L - 1, L, L + 1, 2 ** 512 - 1, 2 ** 252, L * 7 + 3] + [rng.getrandbits(512) for _ in range(200)]:
        assert int.from_bytes(oracle.sc_reduce64(x.to_bytes(64, "little")), "little") == x % L


def test_base58_reference_kat():
    # plenum/test/common/test_verifier.py: '~8zH9ZSyZTFPGJ4ZPL5Rvxx' + '99BgFBg35BehzfSADV5nM4'
    full = b58encode(b58decode("99BgFBg35BehzfSADV5nM4") + b58decode("8zH9ZSyZTFPGJ4ZPL5Rvxx")).decode()
    assert full == "5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdock"
    assert b58decode("1112") == b"\0\0\0\x01"
    assert b58decode("") == b"" and b58decode("111") == b"\0\0\0"
    assert b58decode("2 \n") == b"\x01"
    with pytest.raises(ValueError, match="Invalid character '0'"):
        b58decode("10")
    for data in (b"", b"\0", b"\0\0ab", bytes(range(40))):
        assert b58decode(b58encode(data).decode()) == data


def test_sodium_forger_matches_oracle(oracle, sodium):
    """bench.py builds configs[2] with tools/adversarial_batch.SodiumForger (libsodium's group API);
    the tests use the C oracle's raw signer: same keys and signatures for the same scalars."""
    import numpy as np
    from adversarial_batch import ORDER8, SodiumForger
    f = SodiumForger()
    rng = np.random.default_rng(9)
    L = 2 ** 252 + 27742317777372353535851937790883648493
    for _ in range(20):
        a = (int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % L).to_bytes(32, "little")
        r = (int(rng.integers(1, 2 ** 62)) * 7919 % L).to_bytes(32, "little")
        A = f.scalarmult_base(a)
        assert A == oracle.scalarmult_base(a)
        A2 = f.point_add(A, ORDER8)
        assert A2 == oracle.point_add(A, ORDER8)
        m = rng.bytes(int(rng.integers(0, 300)))
        s = f.sign_raw(r, a, A2, m)
        assert s == oracle.sign_raw(r, a, A2, m)
        assert sodium.sign_open_ok(s + m, A2) == oracle.sign_open_ok(s + m, A2)


def test_config3_batch_with_sodium_forger(oracle):
    """configs[2] as bench.py builds it (libsodium forger), small: untouched records valid, mutated
    ones rejected except mixed-order keys whose k happens to be a multiple of 8 and mixed-order
    (A, R) pairs whose torsion parts cancel."""
    import numpy as np
    import nym_workload
    from adversarial_batch import inject
    from oracle.oracle import cpu_verdicts
    blob, off, pks = nym_workload.generate(0, 3000, workers=1)
    blob2, pks2, idx, labels = inject(blob, off, pks, 0.05, seed=3)
    got = cpu_verdicts(blob2, off, pks2)
    mask = np.ones(len(got), bool)
    mask[idx] = False
    assert got[mask].all()
    lab = np.array(labels)
    assert not got[idx[(lab != "mixed_order_A") & (lab != "mixed_order_AR")]].any()
    o = np.array([oracle.sign_open_ok(blob2[off[i]:off[i + 1]].tobytes(), pks2[i].tobytes()) for i in idx])
    assert np.array_equal(o, got[idx])
