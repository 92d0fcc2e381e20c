"""Synthetic NYM-style signed requests for bench.py and the large GPU tests.

Template (signing-serialized with the reference's rules: sorted keys, "k:v" joined by "|"):
  {identifier: DID_s, reqId: 1700000000000000 + i, protocolVersion: 2,
   operation: {type: '1', dest: DID_i, verkey: '~' + b58(16 B), alias: 'u%08d' % i},
   taaAcceptance: {taaDigest: 64 hex, mechanism: 'service_agreement', time: 1700000000}}
The signer pool has 1024 DidSigner-style identities: seed_s = SHA-512("plenum-bench" || u64 s)[:32],
vk = Ed25519 public key, DID = b58(vk[:16]), abbreviated verkey = '~' + b58(vk[16:]).
Messages are rendered directly in signing-serialized form (checked against
plenum_amd.serialization.serialize_msg_for_signing on a sample), then signed with the image's
libsodium (crypto_sign_detached) in worker processes. Everything is seeded and deterministic.
"""
import ctypes
import hashlib
import multiprocessing as mp
import os
import struct

import numpy as np

B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
POOL = 1024
TAA_DIGEST = hashlib.sha256(b"plenum-bench-taa").hexdigest()
_SODIUM = None


def b58(data: bytes) -> str:
    n0 = len(data) - len(data.lstrip(b"\0"))
    v = int.from_bytes(data, "big")
    out = ""
    while v:
        v, r = divmod(v, 58)
        out = B58[r] + out
    return "1" * n0 + out


def sodium():
    global _SODIUM
    if _SODIUM is None:
        for p in ("/opt/conda/lib/libsodium.so.23", "/usr/lib/x86_64-linux-gnu/libsodium.so.23"):
            if os.path.exists(p):
                lib = ctypes.CDLL(p)
                lib.sodium_init()
                _SODIUM = lib
                break
        else:
            raise OSError("libsodium.so.23 is needed to sign the synthetic workload")
    return _SODIUM


def signer(s):
    seed = hashlib.sha512(b"plenum-bench" + struct.pack("<Q", s)).digest()[:32]
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    sodium().crypto_sign_seed_keypair(pk, sk, seed)
    vk = pk.raw
    return {"sk": sk.raw, "vk": vk, "did": b58(vk[:16]), "abbr": "~" + b58(vk[16:])}


def request_dict(i, s):
    h = hashlib.sha256(struct.pack("<Q", i)).digest()
    return {
        "identifier": s["did"], "reqId": 1700000000000000 + i, "protocolVersion": 2,
        "operation": {"type": "1", "dest": b58(h[:16]), "verkey": "~" + b58(h[16:]), "alias": "u%08d" % i},
        "taaAcceptance": {"taaDigest": TAA_DIGEST, "mechanism": "service_agreement", "time": 1700000000},
    }


def message(i, s):
    """serialize_msg_for_signing(request_dict(i, s)) rendered directly."""
    h = hashlib.sha256(struct.pack("<Q", i)).digest()
    return ("identifier:%s|operation:alias:u%08d|dest:%s|type:1|verkey:~%s|protocolVersion:2|reqId:%d|"
            "taaAcceptance:mechanism:service_agreement|taaDigest:%s|time:1700000000"
            % (s["did"], i, b58(h[:16]), b58(h[16:]), 1700000000000000 + i, TAA_DIGEST)).encode()


_POOL_CACHE = None


def _pool():
    global _POOL_CACHE
    if _POOL_CACHE is None:
        _POOL_CACHE = [signer(s) for s in range(POOL)]
    return _POOL_CACHE


def wire_text(i, s, sig_b58):
    """The request as a client sends it: json.dumps(request_dict(i, s) + signature), rendered
    directly (checked against json.dumps on a sample)."""
    h = hashlib.sha256(struct.pack("<Q", i)).digest()
    return ('{"identifier": "%s", "reqId": %d, "protocolVersion": 2, "operation": {"type": "1", "dest": "%s", '
            '"verkey": "~%s", "alias": "u%08d"}, "taaAcceptance": {"taaDigest": "%s", "mechanism": '
            '"service_agreement", "time": 1700000000}, "signature": "%s"}'
            % (s["did"], 1700000000000000 + i, b58(h[:16]), b58(h[16:]), i, TAA_DIGEST, sig_b58)).encode()


def _sign_range(args):
    lo, hi, wire = args
    pool = _pool()
    lib = sodium()
    sig = ctypes.create_string_buffer(64)
    out_sm, out_pk, out_wire, out_sig = [], [], [], []
    for i in range(lo, hi):
        s = pool[i % POOL]
        m = message(i, s)
        lib.crypto_sign_detached(sig, None, m, ctypes.c_ulonglong(len(m)), s["sk"])
        out_sm.append(sig.raw + m)
        out_pk.append(s["vk"])
        if wire:
            sb = b58(sig.raw)
            out_sig.append(sb.encode())
            out_wire.append(wire_text(i, s, sb))
    extra = ((b"".join(out_wire), [len(x) for x in out_wire], b"".join(out_sig), [len(x) for x in out_sig])
             if wire else None)
    return b"".join(out_sm), [len(x) for x in out_sm], b"".join(out_pk), extra


def endorsers(i, k=3):
    """Signers of multi-signature request i (configs[3]): its author and k - 1 endorsers."""
    return [(i + 341 * j) % POOL for j in range(k)]


def _sign_multi_range(args):
    lo, hi, k = args
    pool = _pool()
    lib = sodium()
    sig = ctypes.create_string_buffer(64)
    out_sm, out_pk = [], []
    for i in range(lo, hi):
        m = message(i, pool[i % POOL])  # the payload every signer signs (serializeForSig ignores the signer)
        for s in endorsers(i, k):
            lib.crypto_sign_detached(sig, None, m, ctypes.c_ulonglong(len(m)), pool[s]["sk"])
            out_sm.append(sig.raw + m)
            out_pk.append(pool[s]["vk"])
    return b"".join(out_sm), [len(x) for x in out_sm], b"".join(out_pk)


def generate_multisig(lo, n, k=3, workers=None, bad_frac=0.0, seed=4):
    """configs[3]: requests [lo, lo + n) with k signatures each over the same payload, expanded to
    one (sig || msg, pk) record per (request, signer), request-major.

    With bad_frac > 0, that fraction of the n * k records (seeded positions, any of a request's k
    signatures) gets one flipped bit in its signature's R or S half, so libsodium rejects exactly
    those records. Returns (blob, off, pks, bad) with bad a bool (n, k) array of the corrupted
    records (all False when bad_frac == 0)."""
    workers = workers or min(16, max(1, (os.cpu_count() or 1)))
    chunk = max(1, (n + workers * 4 - 1) // (workers * 4))
    ranges = [(a, min(a + chunk, lo + n), k) for a in range(lo, lo + n, chunk)]
    if workers > 1 and n > 20000:
        with mp.get_context("fork").Pool(workers) as p:
            parts = p.map(_sign_multi_range, ranges)
    else:
        parts = [_sign_multi_range(r) for r in ranges]
    blob = np.frombuffer(b"".join(p[0] for p in parts), dtype=np.uint8)
    off = _offsets([x for p in parts for x in p[1]])
    pks = np.frombuffer(b"".join(p[2] for p in parts), dtype=np.uint8).reshape(n * k, 32)
    bad = np.zeros(n * k, bool)
    if bad_frac > 0:
        rng = np.random.default_rng(seed)
        idx = rng.choice(n * k, size=max(1, int(n * k * bad_frac)), replace=False)
        byte = rng.integers(0, 64, size=len(idx))
        bit = rng.integers(0, 8, size=len(idx))
        blob = blob.copy()
        pos = off[idx].astype(np.int64) + byte
        blob[pos] ^= (np.uint8(1) << bit.astype(np.uint8))
        bad[idx] = True
    return blob, off, pks, bad.reshape(n, k)


def _offsets(lens):
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(np.asarray(lens, dtype=np.uint64), out=off[1:])
    return off


def generate_wire(lo, n, workers=None):
    """As generate(), plus what arrives on the wire: (blob, off, pks, wire blob, wire offsets,
    b58 signature blob, signature offsets)."""
    return generate(lo, n, workers, wire=True)


def generate(lo, n, workers=None, wire=False):
    """Requests [lo, lo + n): (blob uint8, offsets uint64[n+1], pks uint8[n, 32])."""
    workers = workers or min(16, max(1, (os.cpu_count() or 1)))
    chunk = max(1, (n + workers * 4 - 1) // (workers * 4))
    ranges = [(a, min(a + chunk, lo + n), wire) for a in range(lo, lo + n, chunk)]
    if workers > 1 and n > 20000:
        ctx = mp.get_context("fork")
        with ctx.Pool(workers) as p:
            parts = p.map(_sign_range, ranges)
    else:
        parts = [_sign_range(r) for r in ranges]
    blob = np.frombuffer(b"".join(p[0] for p in parts), dtype=np.uint8)
    lens = np.array([x for p in parts for x in p[1]], dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    pks = np.frombuffer(b"".join(p[2] for p in parts), dtype=np.uint8).reshape(n, 32)
    if not wire:
        return blob, off, pks
    wblob = np.frombuffer(b"".join(p[3][0] for p in parts), dtype=np.uint8)
    woff = _offsets([x for p in parts for x in p[3][1]])
    sblob = np.frombuffer(b"".join(p[3][2] for p in parts), dtype=np.uint8)
    soff = _offsets([x for p in parts for x in p[3][3]])
    return blob, off, pks, wblob, woff, sblob, soff


def save(path, lo, n, workers=None):
    blob, off, pks = generate(lo, n, workers)
    np.savez(path, blob=blob, off=off, pks=pks, lo=np.array([lo]))


def load(path):
    d = np.load(path, allow_pickle=False)
    return d["blob"], d["off"], d["pks"], int(d["lo"][0])


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--lo", type=int, default=0)
    a = ap.parse_args()
    save(a.out, a.lo, a.n)
