"""Drop-in for ``plenum/common/verifier.py`` (Verifier ABC, DidVerifier).

DidVerifier resolution rules (verifier.py:24-50), kept exactly, including which errors surface as
``ValueError`` (identifier / abbreviated tail not base58, empty verkey with an identifier) and which
as ``InvalidKey`` (anything failing inside the verkey setter):
  * identifier given: its base58 decoding is 32 bytes and no verkey -> cryptonym, verkey = identifier
  * still no verkey -> ValueError("'verkey' should be a non-empty string")
  * verkey starting with '~' -> full key = b58decode(identifier) || b58decode(verkey[1:])
  * setter: stp_core Verifier(b58decode(verkey)); 32 bytes raw, else hex; any error -> InvalidKey
"""
from abc import abstractmethod

from .base58 import b58decode, b58encode
from .exceptions import InvalidKey
from .nacl_wrappers import Verifier as NaclVerifier
from .serialization import serialize_msg_for_signing


class Verifier:
    @abstractmethod
    def __init__(self, *args, **kwargs):
        pass

    @abstractmethod
    def verify(self, sig, msg) -> bool:
        pass

    def verifyMsg(self, sig, msg):
        return self.verify(sig, serialize_msg_for_signing(msg))


class DidVerifier(Verifier):
    def __init__(self, verkey, identifier=None):
        given = verkey
        self._verkey = None
        self._vr = None
        if identifier:
            idr_raw = b58decode(identifier)
            if not verkey and len(idr_raw) == 32:
                verkey = identifier  # cryptonym: the DID is the full key
            if not verkey:
                raise ValueError("'verkey' should be a non-empty string")
            if verkey[0] == '~':
                verkey = b58encode(b58decode(identifier) + b58decode(verkey[1:])).decode("utf-8")
        try:
            self.verkey = verkey
        except Exception as ex:
            raise InvalidKey("verkey {}".format(given)) from ex

    @property
    def verkey(self):
        return self._verkey

    @verkey.setter
    def verkey(self, value):
        self._verkey = value
        self._vr = NaclVerifier(b58decode(value))

    @property
    def raw_key(self):
        """32-byte public key or None (no key: every verify is False)."""
        key = self._vr.key
        return bytes(key) if key else None

    def verify(self, sig, msg) -> bool:
        return self._vr.verify(sig, msg)
