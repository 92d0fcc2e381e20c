"""ORACLE / TEST INFRASTRUCTURE ONLY: restatement of PyPI ``base58`` 2.1.x (Bitcoin alphabet),
the package the reference imports (plenum/server/client_authn.py:7, plenum/common/verifier.py:4;
unpinned in setup.py:98-99, 2.1.0 is the commented-out pin). The package is absent from this
image, so this restatement of its published algorithm serves (a) as the ``base58`` module when
importing the reference to generate golden vectors (tests/golden/make_golden.py) and (b) as the
checker for the product's C++ base58 (indy-plenum_amd/csrc/host_prep.cpp).

b58decode: v.rstrip() (str: Unicode whitespace), str -> ASCII bytes (UnicodeEncodeError
otherwise), strip leading '1's (each is one 0x00 byte), big-endian integer of the rest,
ValueError("Invalid character 'c'") for a character outside the alphabet.
b58encode: leading 0x00 bytes -> '1', then base-58 digits of the integer; returns bytes.
"""
BITCOIN_ALPHABET = b'123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
alphabet = BITCOIN_ALPHABET


def scrub_input(v):
    if isinstance(v, str):
        v = v.encode('ascii')
    return v


def b58encode_int(i, default_one=True, alphabet=BITCOIN_ALPHABET):
    if not i and default_one:
        return alphabet[0:1]
    out = b""
    while i:
        i, r = divmod(i, 58)
        out = alphabet[r:r + 1] + out
    return out


def b58encode(v, alphabet=BITCOIN_ALPHABET):
    v = scrub_input(v)
    n0 = len(v)
    v = v.lstrip(b'\0')
    zeros = n0 - len(v)
    acc = int.from_bytes(v, 'big')
    body = b58encode_int(acc, default_one=False, alphabet=alphabet)
    return alphabet[0:1] * zeros + body


def b58decode_int(v, alphabet=BITCOIN_ALPHABET):
    if b' ' not in alphabet:
        v = v.rstrip()
    v = scrub_input(v)
    table = {c: i for i, c in enumerate(alphabet)}
    acc = 0
    for ch in v:
        if ch not in table:
            raise ValueError("Invalid character {!r}".format(chr(ch)))
        acc = acc * 58 + table[ch]
    return acc


def b58decode(v, alphabet=BITCOIN_ALPHABET):
    v = v.rstrip()
    v = scrub_input(v)
    n0 = len(v)
    v = v.lstrip(alphabet[0:1])
    zeros = n0 - len(v)
    acc = b58decode_int(v, alphabet=alphabet)
    return b'\0' * zeros + acc.to_bytes((acc.bit_length() + 7) // 8, 'big')
