"""Drop-in for ``plenum/server/req_authenticator.py`` with ``authenticate_batch``.

ReqAuthenticator (req_authenticator.py:11-72): ordered authenticator list (the first is the core
one), a verified-request cache keyed by request digest that short-circuits re-verification when
the same signature comes again (PROPAGATEs), query types -> empty set, NoAuthenticatorFound when
no authenticator produced an identifier.

``authenticate_batch(items)`` takes [(req_data, key)] — e.g. the client messages of one
ZStack.processReceived quota or the PROPAGATEs of one node ``Batch`` (SURVEY.md §8b feed points) —
plans every signature check of every authenticator that can run them, verifies them in one GPU
launch, then calls ``authenticate`` for each item in order: identical results, exceptions and
``_verified_reqs`` side effects, and one authenticator call per request, as in the sequential path.
"""
from copy import deepcopy
from typing import Optional

from . import batch
from .client_authn import ClientAuthNr
from .constants import OPERATION, SIGNATURE, TXN_TYPE
from .exceptions import NoAuthenticatorFound


class ReqAuthenticator:
    def __init__(self):
        self._authenticators = []
        self._verified_reqs = {}  # key -> {'signature': ..., 'identifiers': set}

    def register_authenticator(self, authenticator: ClientAuthNr):
        self._authenticators.append(authenticator)

    def authenticate(self, req_data, key=None):
        typ = req_data.get(OPERATION, {}).get(TXN_TYPE)
        if key and self._check_and_verify_existing_req(req_data, key):
            return self._verified_reqs[key]['identifiers']

        identifiers = set()
        for authnr in self._authenticators:
            if authnr.is_query(typ):
                return set()
            if authnr.is_write(typ) or authnr.is_action(typ):
                # the reference hands each authenticator a deep copy; a request whose outcome the
                # batch already holds is answered without reading the dict, so the copy is skipped
                arg = req_data if batch.answer(authnr, req_data) is not None else deepcopy(req_data)
                identifiers.update(authnr.authenticate(arg) or set())

        if not identifiers:
            raise NoAuthenticatorFound
        if key:
            self._verified_reqs[key] = {'signature': req_data.get(SIGNATURE), 'identifiers': identifiers}
        return identifiers

    def _check_and_verify_existing_req(self, req_data: dict, key: str):
        seen = self._verified_reqs.get(key)
        return seen is not None and req_data.get(SIGNATURE) == seen['signature']

    @property
    def core_authenticator(self):
        if not self._authenticators:
            raise RuntimeError('No authenticator registered yet')
        return self._authenticators[0]

    def get_authnr_by_type(self, authnr_type) -> Optional[ClientAuthNr]:
        for authnr in self._authenticators:
            if isinstance(authnr, authnr_type):
                return authnr
        return None

    def clean_from_verified(self, key):
        self._verified_reqs.pop(key, None)

    def authenticate_batch(self, items, engine=None, devices=None):
        """[(req_data, key)] -> per item: the identifier set authenticate() returns, or the
        exception instance it raises. ``devices`` (a list of GPU indices): shard the batch's
        signature checks over those GPUs of this process (pv_verify_batch_multi_gpu), unless an
        ``engine`` is given."""
        if engine is None and devices is not None:
            from . import _native
            engine = _native.multi_gpu_engine(devices)
        per_authnr = {}
        for req_data, key in items:
            if key and self._check_and_verify_existing_req(req_data, key):
                continue
            try:
                typ = req_data.get(OPERATION, {}).get(TXN_TYPE)
            except Exception:
                continue
            for idx, authnr in enumerate(self._authenticators):
                if authnr.is_query(typ):
                    break
                if (authnr.is_write(typ) or authnr.is_action(typ)) and hasattr(authnr, "plan_verifications"):
                    per_authnr.setdefault(idx, []).append(req_data)
        pairs = []
        for idx, reqs in per_authnr.items():
            pairs.extend(self._authenticators[idx].plan_verifications(reqs))
        cache = batch.VerdictCache()
        cache.fill(pairs, engine)
        results = []
        with batch.active(cache, engine):
            for req_data, key in items:
                try:
                    results.append(self.authenticate(req_data, key))
                except Exception as ex:
                    results.append(ex)
        return results
