"""Test-vector generation: normal and adversarial Ed25519 (sm, pk) cases.

TEST INFRASTRUCTURE. Uses libsodium 1.0.18 (the reference's pinned native dependency, reached via
ctypes exactly as libnacl does) for keys/signatures and the C oracle's raw signer to forge
vectors libsodium's signer cannot produce (mixed-order keys with honest signatures).
Every generator is seeded and deterministic.
"""
import hashlib
import random
import struct

import numpy as np

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493

# the 7 libsodium small-order encodings (ge25519_has_small_order)
BLACKLIST = [
    bytes(32),
    bytes([1]) + bytes(31),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    (P - 1).to_bytes(32, "little"),
    P.to_bytes(32, "little"),
    (P + 1).to_bytes(32, "little"),
]
ORDER8 = BLACKLIST[2]


def seed_for(tag, i):
    return hashlib.sha512(tag + struct.pack("<Q", i)).digest()[:32]


class VectorGen:
    CLASSES = ("valid", "flip_R", "flip_S", "flip_A", "flip_M", "S_plus_L", "S_big", "R_blacklist",
               "A_blacklist", "A_noncanonical", "A_offcurve", "R_noncanonical", "mixed_order_A", "short_sm",
               "empty_msg", "long_msg", "mixed_order_AR", "mixed_order_R")

    def __init__(self, sodium, oracle, seed=1):
        self.ls = sodium
        self.o = oracle
        self.rng = random.Random(seed)
        self._keys = []

    def key(self, i=None):
        if i is None:
            i = self.rng.randrange(1 << 30)
        return self.ls.seed_keypair(seed_for(b"vectors", i))

    def msg(self, lo=0, hi=400):
        return bytes(self.rng.getrandbits(8) for _ in range(self.rng.randrange(lo, hi)))

    def valid(self, msg=None):
        pk, sk = self.key()
        m = self.msg() if msg is None else msg
        return self.ls.sign_detached(m, sk) + m, pk

    def make(self, cls):
        r = self.rng
        if cls == "valid":
            return self.valid()
        if cls == "empty_msg":
            return self.valid(b"")
        if cls == "long_msg":
            return self.valid(self.msg(900, 2200))
        sm, pk = self.valid()
        sig, m = bytearray(sm[:64]), sm[64:]
        if cls == "flip_R":
            sig[r.randrange(32)] ^= 1 << r.randrange(8)
        elif cls == "flip_S":
            sig[32 + r.randrange(32)] ^= 1 << r.randrange(8)
        elif cls == "flip_A":
            pk = bytearray(pk)
            pk[r.randrange(32)] ^= 1 << r.randrange(8)
            pk = bytes(pk)
        elif cls == "flip_M":
            if not m:
                m = b"x"
            m = bytearray(m)
            m[r.randrange(len(m))] ^= 1 << r.randrange(8)
            m = bytes(m)
        elif cls == "S_plus_L":
            s = int.from_bytes(sig[32:], "little") + L
            sig[32:] = s.to_bytes(32, "little")
        elif cls == "S_big":
            s = r.choice([L, L + 1, 2 ** 253 - 1, 2 ** 256 - 1, L - 1 + (r.getrandbits(200) << 54) % 2 ** 256])
            sig[32:] = (s % 2 ** 256).to_bytes(32, "little")
        elif cls == "R_blacklist":
            b = bytearray(r.choice(BLACKLIST))
            if r.random() < 0.5:
                b[31] |= 0x80
            sig[:32] = b
        elif cls == "A_blacklist":
            b = bytearray(r.choice(BLACKLIST))
            if r.random() < 0.5:
                b[31] |= 0x80
            pk = bytes(b)
        elif cls == "A_noncanonical":
            y = r.randrange(P, 2 ** 255)
            b = bytearray(y.to_bytes(32, "little"))
            if r.random() < 0.5:
                b[31] |= 0x80
            pk = bytes(b)
        elif cls == "A_offcurve":
            # y with (y^2-1)/(dy^2+1) a non-square
            d = (-121665 * pow(121666, P - 2, P)) % P
            while True:
                y = r.randrange(P)
                u = (y * y - 1) % P
                v = (d * y * y + 1) % P
                t = u * pow(v, P - 2, P) % P
                if t != 0 and pow(t, (P - 1) // 2, P) != 1:
                    break
            pk = y.to_bytes(32, "little")
        elif cls == "R_noncanonical":
            y = int.from_bytes(bytes(sig[:32]), "little") & (2 ** 255 - 1)
            if y < 19:
                y += P
            else:
                y = P + r.randrange(19)
            b = bytearray(y.to_bytes(32, "little"))
            b[31] |= sig[31] & 0x80
            sig[:32] = b
        elif cls == "mixed_order_A":
            # A' = A + T8 with an honest signature under A' (passes iff 8 | k)
            a = r.randrange(1, L)
            A = self.o.scalarmult_base(a.to_bytes(32, "little"))
            A2 = self.o.point_add(A, ORDER8)
            rr = r.randrange(1, L).to_bytes(32, "little")
            m = self.msg()
            sig = bytearray(self.o.sign_raw(rr, a.to_bytes(32, "little"), A2, m))
            pk = A2
        elif cls in ("mixed_order_AR", "mixed_order_R"):
            # R' = rB + [j]T8 (j = 1..7) with S = r + k a: libsodium compares encode(SB - kA) with R,
            # so for A = aB + T8 the signature passes iff [j]T8 = -[k]T8 (about 1 in 8 -- half of
            # these cases retry until it passes), and for a prime-order A (mixed_order_R) never.
            a = r.randrange(1, L)
            A = self.o.scalarmult_base(a.to_bytes(32, "little"))
            pk = self.o.point_add(A, ORDER8) if cls == "mixed_order_AR" else A
            m = self.msg()
            want_pass = cls == "mixed_order_AR" and r.random() < 0.5
            for _ in range(200):
                rr = r.randrange(1, L)
                T = ORDER8
                for _ in range(r.randrange(7)):
                    T = self.o.point_add(T, ORDER8)
                R = self.o.point_add(self.o.scalarmult_base(rr.to_bytes(32, "little")), T)
                k = int.from_bytes(hashlib.sha512(R + pk + m).digest(), "little") % L
                sig = bytearray(R + ((rr + k * a) % L).to_bytes(32, "little"))
                if not want_pass or self.ls.sign_open_ok(bytes(sig) + m, pk):
                    break
        elif cls == "short_sm":
            smb = bytes(sig) + m
            return smb[: r.randrange(0, 64)], pk
        else:
            raise ValueError(cls)
        return bytes(sig) + m, pk

    def batch(self, n, adversarial_frac=0.0):
        cases = []
        for _ in range(n):
            if self.rng.random() < adversarial_frac:
                cls = self.rng.choice(self.CLASSES[1:])
            else:
                cls = "valid"
            cases.append(self.make(cls))
        return cases


def pack(cases):
    """[(sm, pk)] -> (blob uint8, offsets uint64[n+1], pks uint8[n,32])"""
    lens = np.array([len(sm) for sm, _ in cases], dtype=np.uint64)
    off = np.zeros(len(cases) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(sm for sm, _ in cases), dtype=np.uint8) if cases else np.zeros(0, np.uint8)
    pks = np.frombuffer(b"".join(pk for _, pk in cases), dtype=np.uint8).reshape(len(cases), 32)
    return blob, off, pks
