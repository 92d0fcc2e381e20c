"""In-place adversarial mutation of a large packed batch (SURVEY.md §8c iv, config 3: ~2 %).

TEST INFRASTRUCTURE. Every class keeps the record length, so the packed blob/offsets stay valid:
bit flips in R/S/A/M, S + L, S in {L, L+1, 2^253-1, 2^256-1}, small-order R / A (with and without
bit 255), non-canonical A, off-curve A, non-canonical R, and mixed-order keys A + T8 with an
honest signature over the record's own message (forged with the C oracle).
"""
import numpy as np

from vectors import BLACKLIST, ORDER8, P, L

CLASSES = ("flip_R", "flip_S", "flip_A", "flip_M", "S_plus_L", "S_big", "R_blacklist", "A_blacklist",
           "A_noncanonical", "A_offcurve", "R_noncanonical", "mixed_order_A")


def _offcurve_ys(rng, k):
    d = (-121665 * pow(121666, P - 2, P)) % P
    ys = []
    while len(ys) < k:
        y = int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % P
        u = (y * y - 1) % P
        v = (d * y * y + 1) % P
        t = u * pow(v, P - 2, P) % P
        if t and pow(t, (P - 1) // 2, P) != 1:
            ys.append(y)
    return ys


def inject(blob, off, pks, frac, seed, oracle):
    """Mutates copies of blob/pks; returns (blob, pks, idx, classes)."""
    rng = np.random.default_rng(seed)
    blob = blob.copy()
    pks = pks.copy()
    n = len(off) - 1
    k = max(len(CLASSES), int(n * frac))
    idx = np.sort(rng.choice(n, size=k, replace=False))
    labels = []
    offc = _offcurve_ys(rng, 64)
    for j, i in enumerate(idx):
        cls = CLASSES[j % len(CLASSES)]
        labels.append(cls)
        o0, o1 = int(off[i]), int(off[i + 1])
        sig = blob[o0:o0 + 64]
        if cls == "flip_R":
            sig[int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_S":
            sig[32 + int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_A":
            pks[i, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "flip_M":
            if o1 > o0 + 64:
                blob[int(rng.integers(o0 + 64, o1))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif cls == "S_plus_L":
            s = int.from_bytes(sig[32:].tobytes(), "little") + L
            sig[32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif cls == "S_big":
            s = [L, L + 1, 2 ** 253 - 1, 2 ** 256 - 1][j % 4]
            sig[32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif cls == "R_blacklist":
            b = bytearray(BLACKLIST[j % 7])
            b[31] |= 0x80 * (j % 2)
            sig[:32] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_blacklist":
            b = bytearray(BLACKLIST[j % 7])
            b[31] |= 0x80 * (j % 2)
            pks[i] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_noncanonical":
            b = bytearray((P + j % 19).to_bytes(32, "little"))
            b[31] |= 0x80 * (j % 2)
            pks[i] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "A_offcurve":
            pks[i] = np.frombuffer(offc[j % len(offc)].to_bytes(32, "little"), np.uint8)
        elif cls == "R_noncanonical":
            y = P + j % 19
            b = bytearray(y.to_bytes(32, "little"))
            b[31] |= int(sig[31]) & 0x80
            sig[:32] = np.frombuffer(bytes(b), np.uint8)
        elif cls == "mixed_order_A":
            a = int(rng.integers(1, 2 ** 62)) * int(rng.integers(1, 2 ** 62)) % L or 1
            A = oracle.scalarmult_base(a.to_bytes(32, "little"))
            A2 = oracle.point_add(A, ORDER8)
            r = (int(rng.integers(1, 2 ** 62)) * 7919 % L or 1).to_bytes(32, "little")
            msg = blob[o0 + 64:o1].tobytes()
            s2 = oracle.sign_raw(r, a.to_bytes(32, "little"), A2, msg)
            sig[:] = np.frombuffer(s2, np.uint8)
            pks[i] = np.frombuffer(A2, np.uint8)
    return blob, pks, idx, labels
