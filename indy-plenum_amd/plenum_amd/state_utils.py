"""Verkey lookup helpers used by SimpleAuthNr.getVerkey (plenum/server/request_handlers/utils.py:
30-39, 58-67). The state backend itself (Patricia trie over leveldb/rocksdb) is out of scope; any
object with ``get(key: bytes, isCommitted: bool) -> bytes|None`` holding the reference's JSON
encoding of NYM records works (domain_state_serializer = JsonSerializer,
common/serializers/serialization.py:13)."""
import json
from hashlib import sha256

from .constants import IDENTIFIER, OPERATION, TARGET_NYM, TXN_TYPE, VERKEY


def nym_to_state_key(nym: str) -> bytes:
    return sha256(nym.encode()).digest()


def get_nym_details(state, nym, is_committed: bool = False):
    if state is None:
        raise AttributeError("'NoneType' object has no attribute 'get'")
    data = state.get(nym_to_state_key(nym), is_committed)
    if not data:
        return {}
    if isinstance(data, (bytes, bytearray)):
        data = data.decode()
    return json.loads(data)


def get_request_type(req: dict):
    return req[OPERATION][TXN_TYPE]


def nym_ident_is_dest(req: dict):
    return req[IDENTIFIER] == req[OPERATION].get(TARGET_NYM)


def get_target_verkey(req: dict):
    return req[OPERATION].get(VERKEY)


class DictState:
    """Minimal in-memory state: {nym: {"verkey": ..., "role": ...}} (tests, bench)."""

    def __init__(self, nyms=None):
        self._kv = {}
        for nym, rec in (nyms or {}).items():
            self.put_nym(nym, rec)

    def put_nym(self, nym, record):
        self._kv[nym_to_state_key(nym)] = json.dumps(record, sort_keys=True, separators=(',', ':')).encode()

    def get(self, key, isCommitted=True):
        return self._kv.get(key)
