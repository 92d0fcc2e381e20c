"""Drop-in for ``plenum/server/client_authn.py`` with a batched entry point.

Classes and semantics of the reference (client_authn.py:21-276):
  ClientAuthNr       interface: authenticate / authenticate_multi / addIdr / getVerkey
  NaclAuthNr         authenticate_multi: per-signature loop in dict order; threshold None = all;
                     InsufficientSignatures if fewer provided than required; InvalidSignatureFormat
                     for undecodable base58; CouldNotAuthenticate if no verkey; DidVerifier errors
                     propagate; stops at the threshold; InsufficientCorrectSignatures when the loop
                     runs out (also for an empty dict)
  SimpleAuthNr       clients registry + uncommitted-state lookup + NYM self-verkey rule
  CoreAuthMixin      picks `signature` (with `identifier`) or `signatures`, strips
                     {signature, signatures, fees} from the signed payload
  CoreAuthNr         CoreAuthMixin + SimpleAuthNr
New: ``CoreAuthMixin.plan_verifications`` and ``CoreAuthMixin.authenticate_batch`` — every
Ed25519 check of a batch of requests runs in one GPU launch, then each request goes through the
unchanged ``authenticate`` (once per request) answering from the precomputed verdicts.
"""
from abc import abstractmethod
from typing import Dict, Optional

from . import batch
from .base58 import b58decode, b58decode_many
from .constants import NYM, ROLE, VERKEY, IDENTIFIER, SIGNATURE, SIGNATURES, FEES
from .exceptions import (CouldNotAuthenticate, EmptyIdentifier, EmptySignature, InsufficientCorrectSignatures,
                         InsufficientSignatures, InvalidSignatureFormat, MissingIdentifier, MissingSignature)
from .serialization import serialize_msg_for_signing
from .state_utils import get_nym_details, get_request_type, get_target_verkey, nym_ident_is_dest
from .verifier import DidVerifier, Verifier


class ClientAuthNr:
    """Interface for client authenticators (client_authn.py:21-79)."""

    @abstractmethod
    def authenticate(self, msg: Dict, identifier: Optional[str] = None, signature: Optional[str] = None,
                     threshold: Optional[int] = None, key: Optional[str] = None) -> str:
        """Verify the signature(s) of ``msg``; return the identifier(s) or raise SigningException."""

    @abstractmethod
    def authenticate_multi(self, msg: Dict, signatures: Dict[str, str], threshold: Optional[int] = None):
        """Return the identifiers whose signatures verified; raise if the threshold is not met."""

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        """Register a client's verification key."""

    @abstractmethod
    def getVerkey(self, identifier):
        """Verification key of a client."""


class NaclAuthNr(ClientAuthNr):

    def authenticate_multi(self, msg: Dict, signatures: Dict[str, str], threshold: Optional[int] = None,
                           verifier: Verifier = DidVerifier):
        provided = len(signatures)
        if threshold is None:
            threshold = provided
        elif provided < threshold:
            raise InsufficientSignatures(provided, threshold)

        accepted, rejected = [], {}
        for idr, sig in signatures.items():
            try:
                raw_sig = b58decode(sig)
            except Exception as ex:
                raise InvalidSignatureFormat from ex
            payload = self.serializeForSig(msg, identifier=idr)
            verkey = self.getVerkey(idr, msg)
            if verkey is None:
                raise CouldNotAuthenticate(idr)
            if verifier(verkey, identifier=idr).verify(raw_sig, payload):
                accepted.append(idr)
                if len(accepted) == threshold:
                    return accepted
            else:
                rejected[idr] = sig
        raise InsufficientCorrectSignatures(threshold, len(accepted), rejected)

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        pass

    @abstractmethod
    def getVerkey(self, ident, request):
        pass

    def serializeForSig(self, msg, identifier=None, topLevelKeysToIgnore=None):
        return serialize_msg_for_signing(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)


class SimpleAuthNr(NaclAuthNr):
    """Client registry backed by uncommitted state (client_authn.py:121-192)."""

    def __init__(self, state=None):
        self.clients = {}  # identifier -> {verkey, role}
        self.state = state
        self.specific_verkey_validation = {NYM: self.nym_specific_auth}

    def addIdr(self, identifier, verkey, role=None):
        self.clients[identifier] = {VERKEY: verkey, ROLE: role}

    def getVerkey(self, ident, request):
        record = self.clients.get(ident)
        if not record:
            # uncommitted batches may create the DID a later request in the batch signs with
            record = get_nym_details(self.state, ident, is_committed=False)
            if not record:
                # not on the ledger: a non-ledger NYM may carry its own verkey
                return self.get_verkey_specific(request)
        return record.get(VERKEY)

    def authenticate(self, msg: Dict, identifier: Optional[str] = None, signature: Optional[str] = None,
                     threshold: Optional[int] = None):
        return self.authenticate_multi(msg, signatures={identifier: signature}, threshold=threshold)

    def get_verkey_specific(self, request):
        rule = self.specific_verkey_validation.get(get_request_type(request))
        return None if rule is None else rule(request)

    def nym_specific_auth(self, request):
        return get_target_verkey(request) if nym_ident_is_dest(request) else None

    def verkey_resolver(self):
        """A batch-scoped getVerkey: see VerkeyResolver."""
        return VerkeyResolver(self)


_MISS = object()
_PER_REQUEST = object()


class VerkeyResolver:
    """Batched ``SimpleAuthNr.getVerkey`` (client_authn.py:154-168, request_handlers/utils.py:30-39)
    for the requests of ONE batch: a DID's registry entry or uncommitted-state NYM record is read
    and JSON-decoded once per batch instead of once per signature. Only the request-dependent tail
    (a DID with no record -> the NYM self-verkey rule) runs per request. ``get(idr, request)``
    returns what ``getVerkey(idr, request)`` returns, or raises ``LookupError`` where getVerkey
    would raise, so the caller sends that request down the sequential path (which raises the
    exact exception). Valid while the registry and state do not change (one ingress batch); an
    authenticator that overrides getVerkey is called per signature, unchanged."""

    def __init__(self, authnr):
        self.authnr = authnr
        self.memo = {}  # idr -> verkey | _PER_REQUEST | LookupError
        self.batched = type(authnr).getVerkey is SimpleAuthNr.getVerkey
        self.reads = 0

    def _record(self, idr):
        a = self.authnr
        try:
            record = a.clients.get(idr)
            if not record:
                self.reads += 1
                record = get_nym_details(a.state, idr, is_committed=False)
                if not record:
                    return _PER_REQUEST
            return record.get(VERKEY)
        except Exception as ex:
            return LookupError(ex)

    def static(self, idr):
        """The verkey of ``idr`` when it does not depend on the request (a registry or state
        record: what getVerkey returns for every request of the batch), else None (request-
        dependent, or getVerkey would raise: the caller takes the per-request path)."""
        if not self.batched:
            return None
        r = self.memo.get(idr, _MISS)
        if r is _MISS:
            r = self.memo[idr] = self._record(idr)
        return None if r is _PER_REQUEST or isinstance(r, LookupError) else r

    def get(self, idr, request):
        if not self.batched:
            try:
                return self.authnr.getVerkey(idr, request)
            except Exception as ex:
                raise LookupError(ex)
        r = self.memo.get(idr, _MISS)
        if r is _MISS:
            r = self.memo[idr] = self._record(idr)
        if r is _PER_REQUEST:
            try:
                return self.authnr.get_verkey_specific(request)
            except Exception as ex:
                raise LookupError(ex)
        if isinstance(r, LookupError):
            raise r
        return r


class CoreAuthMixin:
    excluded_from_signing = {SIGNATURE, SIGNATURES, FEES}

    def __init__(self, write_types, query_types, action_types) -> None:
        self._write_types = set(write_types)
        self._query_types = set(query_types)
        self._action_types = set(action_types)

    def is_query(self, typ):
        return typ in self._query_types

    def is_write(self, typ):
        return typ in self._write_types

    def is_action(self, typ):
        return typ in self._action_types

    @staticmethod
    def _extract_signature(msg):
        if SIGNATURE not in msg:
            raise MissingSignature
        if not msg[SIGNATURE]:
            raise EmptySignature
        return msg[SIGNATURE]

    @staticmethod
    def _extract_identifier(msg):
        if IDENTIFIER not in msg:
            raise MissingIdentifier
        if not msg[IDENTIFIER]:
            raise EmptyIdentifier
        return msg[IDENTIFIER]

    def _signing_view(self, req_data):
        return {k: v for k, v in req_data.items() if k not in self.excluded_from_signing}

    def _select_signatures(self, req_data, identifier, signature):
        """The {identifier: signature} mapping authenticate() verifies (client_authn.py:240-264)."""
        if req_data.get(SIGNATURE) is None and req_data.get(SIGNATURES) is None and signature is None:
            raise MissingSignature
        if req_data.get(IDENTIFIER) and (req_data.get(SIGNATURE) or signature):
            identifier = identifier or self._extract_identifier(req_data)
            signature = signature or self._extract_signature(req_data)
            return {identifier: signature}
        return req_data.get(SIGNATURES, None)

    def authenticate(self, req_data, identifier: Optional[str] = None, signature: Optional[str] = None,
                     threshold: Optional[int] = None, verifier: Verifier = DidVerifier):
        if identifier is None and signature is None and threshold is None and verifier is DidVerifier:
            known = batch.answer(self, req_data)  # a wire batch already finished this request
            if known is not None:
                return known
        payload = self._signing_view(req_data)
        signatures = self._select_signatures(req_data, identifier, signature)
        return self.authenticate_multi(payload, signatures=signatures, threshold=threshold, verifier=verifier)

    def serializeForSig(self, msg, identifier=None, topLevelKeysToIgnore=None):
        return serialize_msg_for_signing(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)

    # ----------------------------------------------------------------- batched entry point

    def plan_verifications(self, reqs, verifier=DidVerifier):
        """(public key, signature || message) pairs that authenticate() will check for each request
        in ``reqs``; requests or signatures that would fail before reaching the verifier are
        skipped (authenticate() raises for them in the second pass)."""
        todo = []  # (payload bytes, idr, sig, request view)
        for req_data in reqs:
            try:
                signatures = self._select_signatures(req_data, None, None)
                if not signatures:
                    continue
                view = self._signing_view(req_data)
                items = list(signatures.items())
            except Exception:
                continue
            payload = None
            for idr, sig in items:
                if payload is None:
                    try:
                        payload = self.serializeForSig(view, identifier=idr)
                    except Exception:
                        break
                todo.append((payload, idr, sig, view))
        decoded = b58decode_many([sig for _, _, sig, _ in todo])
        make_resolver = getattr(self, "verkey_resolver", None)
        get_verkey = make_resolver().get if make_resolver else self.getVerkey
        raw_keys = {}  # (verkey, idr) -> DidVerifier's raw key: resolved once per signer per batch
        pairs = []
        for (payload, idr, _, view), raw_sig in zip(todo, decoded):
            if isinstance(raw_sig, Exception):
                continue
            try:
                verkey = get_verkey(idr, view)
                if verkey is None:
                    continue
                if verifier is DidVerifier:
                    key = raw_keys.get((verkey, idr), _MISS)
                    if key is _MISS:
                        key = raw_keys[(verkey, idr)] = getattr(verifier(verkey, identifier=idr), "raw_key", None)
                else:
                    key = getattr(verifier(verkey, identifier=idr), "raw_key", None)
            except Exception:
                continue
            if key:
                pairs.append((key, raw_sig + payload))
        return pairs

    def authenticate_batch(self, reqs, threshold: Optional[int] = None, verifier: Verifier = DidVerifier,
                           engine=None, devices=None):
        """authenticate() for every request in ``reqs`` with all signature checks in one GPU launch.
        Returns, per request, what authenticate() returns or the exception instance it raises.
        ``devices``: shard the checks over those GPUs of this process (pv_verify_batch_multi_gpu)."""
        if engine is None and devices is not None:
            from . import _native
            engine = _native.multi_gpu_engine(devices)
        cache = batch.VerdictCache()
        cache.fill(self.plan_verifications(reqs, verifier), engine)
        results = []
        with batch.active(cache, engine):
            for req_data in reqs:
                try:
                    results.append(self.authenticate(req_data, threshold=threshold, verifier=verifier))
                except Exception as ex:
                    results.append(ex)
        return results


class CoreAuthNr(CoreAuthMixin, SimpleAuthNr):
    def __init__(self, write_types, query_types, action_types, state=None):
        SimpleAuthNr.__init__(self, state)
        CoreAuthMixin.__init__(self, write_types, query_types, action_types)
