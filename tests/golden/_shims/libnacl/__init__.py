"""TEST-ONLY shim: libnacl 1.6.1's ctypes API over the image's libsodium 1.0.18, used only to import
the reference (/root/reference) when generating golden vectors. Restates libnacl's behaviour for
the functions the reference's hot path and signers call."""
import ctypes
import os

for _p in ("/opt/conda/lib/libsodium.so.23", "/usr/lib/x86_64-linux-gnu/libsodium.so.23"):
    if os.path.exists(_p):
        nacl = ctypes.CDLL(_p)
        break
else:
    raise OSError("libsodium not found")
nacl.sodium_init()

crypto_sign_BYTES = 64
crypto_sign_SEEDBYTES = 32
crypto_sign_PUBLICKEYBYTES = 32
crypto_sign_SECRETKEYBYTES = 64
crypto_box_PUBLICKEYBYTES = 32
crypto_box_SECRETKEYBYTES = 32
crypto_box_NONCEBYTES = 24
crypto_box_BEFORENMBYTES = 32
crypto_box_ZEROBYTES = 32
crypto_box_BOXZEROBYTES = 16
crypto_secretbox_KEYBYTES = 32
crypto_secretbox_NONCEBYTES = 24


def randombytes(size):
    buf = ctypes.create_string_buffer(size)
    nacl.randombytes_buf(buf, ctypes.c_size_t(size))
    return buf.raw


def crypto_sign_seed_keypair(seed):
    if len(seed) != crypto_sign_SEEDBYTES:
        raise ValueError('Invalid Seed')
    pk = ctypes.create_string_buffer(crypto_sign_PUBLICKEYBYTES)
    sk = ctypes.create_string_buffer(crypto_sign_SECRETKEYBYTES)
    if nacl.crypto_sign_seed_keypair(pk, sk, seed):
        raise ValueError('Failed to generate keypair from seed')
    return pk.raw, sk.raw


def crypto_sign_keypair():
    return crypto_sign_seed_keypair(randombytes(32))


def crypto_sign(msg, sk):
    if len(sk) != crypto_sign_SECRETKEYBYTES:
        raise ValueError('Invalid secret key')
    sig = ctypes.create_string_buffer(len(msg) + crypto_sign_BYTES)
    slen = ctypes.pointer(ctypes.c_ulonglong())
    if nacl.crypto_sign(sig, slen, msg, ctypes.c_ulonglong(len(msg)), sk):
        raise ValueError('Failed to sign message')
    return sig.raw


def crypto_sign_open(sig, vk):
    if len(vk) != crypto_sign_PUBLICKEYBYTES:
        raise ValueError('Invalid public key')
    msg = ctypes.create_string_buffer(len(sig))
    msglen = ctypes.c_ulonglong()
    msglenp = ctypes.pointer(msglen)
    if nacl.crypto_sign_open(msg, msglenp, sig, ctypes.c_ulonglong(len(sig)), vk):
        raise ValueError('Failed to validate message')
    return msg.raw[:msglen.value]


def crypto_sign_ed25519_pk_to_curve25519(ed25519_pk):
    out = ctypes.create_string_buffer(32)
    nacl.crypto_sign_ed25519_pk_to_curve25519(out, ed25519_pk)
    return out.raw


def crypto_sign_ed25519_sk_to_curve25519(ed25519_sk):
    out = ctypes.create_string_buffer(32)
    nacl.crypto_sign_ed25519_sk_to_curve25519(out, ed25519_sk)
    return out.raw


def randombytes_uniform(upper_bound):
    nacl.randombytes_uniform.restype = ctypes.c_uint32
    return nacl.randombytes_uniform(ctypes.c_uint32(upper_bound))
