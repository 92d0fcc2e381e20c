"""Drop-in for the verification half of ``stp_core/crypto/nacl_wrappers.py``.

  VerifyKey (nacl_wrappers.py:62-108)   32-byte Ed25519 public key; ``verify(smessage, signature=None)``
                                        returns the message or raises ValueError, like libnacl.
  Verifier  (nacl_wrappers.py:212-242)  ``verify(signature, msg) -> bool``; never raises on a bad
                                        signature; a falsy key makes every verify False.
  crypto_sign_open                      libnacl 1.6.1 ``crypto_sign_open(sm, vk)`` semantics
                                        (ValueError('Invalid public key') / ('Failed to validate
                                        message')), computed by the HIP engine.

Every verification goes to the GPU engine. Inside an ``authenticate_batch`` call the verdicts were
already computed in one batched launch and are looked up (plenum_amd.batch); outside one, a
single-request launch is made. There is no CPU fallback: without the library/GPU this raises
``plenum_amd._native.NativeUnavailable``.
"""
import binascii

from . import batch

crypto_sign_PUBLICKEYBYTES = 32
crypto_sign_BYTES = 64


class RawEncoder:
    @staticmethod
    def encode(data):
        return data

    @staticmethod
    def decode(data):
        return data


class HexEncoder:
    @staticmethod
    def encode(data):
        return binascii.hexlify(data)

    @staticmethod
    def decode(data):
        return binascii.unhexlify(data)


class Encodable:
    def encode(self, encoder=RawEncoder):
        return encoder.encode(bytes(self))


def crypto_sign_open(sm, vk):
    """libnacl.crypto_sign_open: returns the message part of ``sm`` or raises ValueError."""
    if len(vk) != crypto_sign_PUBLICKEYBYTES:
        raise ValueError('Invalid public key')
    sm = bytes(sm)
    if not batch.verdict(bytes(vk), sm):
        raise ValueError('Failed to validate message')
    return sm[crypto_sign_BYTES:]


class VerifyKey(Encodable):
    def __init__(self, key, encoder=RawEncoder):
        key = encoder.decode(key)
        if len(key) != crypto_sign_PUBLICKEYBYTES:
            raise ValueError("The key must be exactly %s bytes long" % crypto_sign_PUBLICKEYBYTES)
        self._key = key

    def __bytes__(self):
        return self._key

    def verify(self, smessage, signature=None, encoder=RawEncoder):
        if signature is not None:
            smessage = signature + smessage
        smessage = encoder.decode(smessage)
        return crypto_sign_open(smessage, self._key)


class Verifier:
    def __init__(self, key=None):
        if key and not isinstance(key, VerifyKey):
            key = VerifyKey(key, RawEncoder) if len(key) == 32 else VerifyKey(key, HexEncoder)
        self.key = key
        if isinstance(key, VerifyKey):
            self.keyhex = key.encode(HexEncoder)
            self.keyraw = key.encode(RawEncoder)
        else:
            self.keyhex = ''
            self.keyraw = ''

    def verify(self, signature, msg):
        if not self.key:
            return False
        try:
            self.key.verify(signature + msg)
        except ValueError:
            return False
        return True
