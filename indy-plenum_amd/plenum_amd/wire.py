"""The ingress batch path: received JSON bytes -> authentication results.

Per received client request the reference does, at the authentication step,
    msg = json.loads(raw)                                   stp_zmq/zstack.py:881-885
    req = Request(**msg)                                    plenum/server/node.py:1643
    req_authnr.authenticate(req.as_dict, key=req.key)       node.py:2636-2650 verifySignature
one request at a time. ``authenticate_wire_packed`` / ``authenticate_wire_batch`` do it for a whole
ZStack quota (or the requests of a PROPAGATE batch) with the per-request work split by where it
runs best:
  1. C++, many threads (pv_wire_plan): one parse of each JSON text gives the signing-serialized M,
     Request.digest and the signature plan (CoreAuthMixin._select_signatures).
  2. Python, once per distinct txn type and per distinct signer: which authenticators run, the
     verkey (getVerkey via the batch's VerkeyResolver) — state lookups stay on the host.
  3. GPU, one launch: base58 decode of every signature, DidVerifier key resolution per signer, sm
     assembly and verification (pv_ingress_verify).
  4. Python, in request order: the verified-request cache and the result.
A request whose signatures all decode, resolve and verify completes in step 4 with exactly the
value the sequential path returns, without being decoded in Python. Every other request (a bad or
undecodable signature, a missing or request-dependent key, an unusual field, several
authenticators for its type, ...) is decoded and goes through the unchanged sequential
``ReqAuthenticator.authenticate`` — with its remaining signature checks batched into one more
launch — so results, exception classes and messages, and cache side effects are the sequential
ones.
"""
import ctypes
import gc
import json
import time
from hashlib import sha256

import numpy as np

from . import _native, batch
from .constants import (ENDORSER, IDENTIFIER, OPERATION, PROTOCOL_VERSION, REQ_ID, SIGNATURE, SIGNATURES,
                        TAA_ACCEPTANCE, TXN_TYPE)
from .serialization import serialize_msg_for_signing

PV_SER_DICT, PV_SER_AUTHN, PV_SER_REQUEST = 0, 1, 2
PV_SER_OK, PV_SER_INVALID, PV_SER_NOT_OBJECT, PV_SER_DEFER = 0, 1, 2, 3
PV_ERR_ARG = -4

# plenum/__init__.py:20 — names plugins register as extra client request fields
PLUGIN_CLIENT_REQUEST_FIELDS = {}

_OPTIONAL_FIELDS = (PROTOCOL_VERSION, TAA_ACCEPTANCE, ENDORSER)
_EXCLUDED = frozenset((SIGNATURE, SIGNATURES, "fees"))  # CoreAuthMixin.excluded_from_signing


class Request:
    """The fields, dict views and digests of plenum/common/request.py:13-168 that authentication
    uses (as_dict :53-74, digest/key :41-45,83-87, signingState/signingPayloadState :95-121,
    identifier :144-160)."""
    idr_delimiter = ','

    def __init__(self, identifier=None, reqId=None, operation=None, signature=None, signatures=None,
                 protocolVersion=None, taaAcceptance=None, endorser=None, **kwargs):
        self._identifier, self.reqId, self.operation = identifier, reqId, operation
        self.signature, self.signatures = signature, signatures
        self.protocolVersion, self.taaAcceptance, self.endorser = protocolVersion, taaAcceptance, endorser
        self._digest = self._payload_digest = None
        for name in PLUGIN_CLIENT_REQUEST_FIELDS:
            if name in kwargs:
                setattr(self, name, kwargs[name])

    @staticmethod
    def gen_idr_from_sigs(signatures):
        return Request.idr_delimiter.join(sorted(signatures.keys())) if signatures else None

    @property
    def identifier(self):
        return self._identifier or self.gen_idr_from_sigs(self.signatures)

    @property
    def all_identifiers(self):
        return [] if self.signatures is None else sorted(self.signatures.keys())

    def _given_optionals(self):
        return {k: getattr(self, k) for k in _OPTIONAL_FIELDS if getattr(self, k) is not None}

    @property
    def as_dict(self):
        view = {REQ_ID: self.reqId, OPERATION: self.operation}
        for name, value in ((IDENTIFIER, self._identifier), (SIGNATURES, self.signatures),
                            (SIGNATURE, self.signature)):
            if value is not None:
                view[name] = value
        for name in PLUGIN_CLIENT_REQUEST_FIELDS:
            if hasattr(self, name):
                view[name] = getattr(self, name)
        view.update(self._given_optionals())
        return view

    def signingPayloadState(self, identifier=None):
        state = {IDENTIFIER: identifier or self.identifier, REQ_ID: self.reqId, OPERATION: self.operation}
        state.update(self._given_optionals())
        return state

    def signingState(self, identifier=None):
        state = self.signingPayloadState(identifier)
        if self.signatures is not None:
            state[SIGNATURES] = self.signatures
        if self.signature is not None:
            state[SIGNATURE] = self.signature
        for name in PLUGIN_CLIENT_REQUEST_FIELDS:
            if getattr(self, name, None):
                state[name] = getattr(self, name)
        return state

    @property
    def digest(self):
        if self._digest is None:
            self._digest = sha256(serialize_msg_for_signing(self.signingState())).hexdigest()
        return self._digest

    @property
    def payload_digest(self):
        if self._payload_digest is None:
            self._payload_digest = sha256(serialize_msg_for_signing(self.signingPayloadState())).hexdigest()
        return self._payload_digest

    @property
    def key(self):
        return self.digest

    @property
    def txn_type(self):
        return self.operation.get(TXN_TYPE)


def signing_bytes(req: Request) -> bytes:
    """What verifySignature verifies for ``req``: serialize(as_dict minus the excluded keys)."""
    return serialize_msg_for_signing({k: v for k, v in req.as_dict.items() if k not in _EXCLUDED})


def signing_serialize_json(raws, mode=PV_SER_REQUEST, threads=16, plugin_fields=None):
    """pv_signing_serialize_json over JSON texts (bytes). Returns (status uint8[n], message blob
    uint8, offsets uint64[n+1], digests uint8[n, 32]) — message i is blob[off[i]:off[i+1]]."""
    blob, off = _native._blob([r if isinstance(r, (bytes, bytearray)) else r.encode() for r in raws])
    return signing_serialize_packed(blob, off, mode, threads, plugin_fields)


def signing_serialize_packed(blob, off, mode=PV_SER_REQUEST, threads=16, plugin_fields=None):
    """signing_serialize_json on texts already packed as (uint8 blob, uint64 offsets[n+1])."""
    L = _native.lib()
    n = len(off) - 1
    blob = np.ascontiguousarray(blob, np.uint8) if len(blob) else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    names = PLUGIN_CLIENT_REQUEST_FIELDS if plugin_fields is None else plugin_fields
    pf = b"".join(x.encode() + b"\0" for x in names) + b"\0"
    status = np.zeros(max(n, 1), np.uint8)
    digests = np.zeros((max(n, 1), 32), np.uint8)
    moff = np.zeros(n + 1, np.uint64)
    cap = 2 * int(off[-1]) + 64 * n + 64
    for _ in range(2):
        msg = np.zeros(cap, np.uint8)
        rc = L.pv_signing_serialize_json(blob.ctypes.data, off.ctypes.data, n, mode, pf, threads, msg.ctypes.data, cap,
                                         moff.ctypes.data, digests.ctypes.data, status.ctypes.data)
        if rc == PV_ERR_ARG and int(moff[n]) > cap:
            cap = int(moff[n])
            continue
        _native.check(rc, "pv_signing_serialize_json")
        return status[:n], msg, moff, digests[:n]
    raise _native.NativeError("pv_signing_serialize_json: output size changed between calls")


PV_PLAN_PY, PV_PLAN_SINGLE, PV_PLAN_MULTI = 0, 1, 2


class _PvWirePlan(ctypes.Structure):
    """include/plenum_verify.h PvWirePlan."""
    _fields_ = [("msg_out", ctypes.c_void_p), ("msg_cap", ctypes.c_uint64), ("msg_off", ctypes.c_void_p),
                ("digest", ctypes.c_void_p), ("status", ctypes.c_void_p), ("kind", ctypes.c_void_p),
                ("type_id", ctypes.c_void_p), ("pair_off", ctypes.c_void_p), ("pair_name", ctypes.c_void_p),
                ("sig_off", ctypes.c_void_p), ("pair_cap", ctypes.c_uint64), ("sigs", ctypes.c_void_p),
                ("sigs_cap", ctypes.c_uint64), ("names", ctypes.c_void_p), ("name_off", ctypes.c_void_p),
                ("names_cap", ctypes.c_uint64), ("types", ctypes.c_void_p), ("type_off", ctypes.c_void_p),
                ("types_cap", ctypes.c_uint64), ("keys_hex", ctypes.c_void_p), ("sig_lines", ctypes.c_void_p),
                ("n_pairs", ctypes.c_uint64), ("n_names", ctypes.c_uint64), ("n_types", ctypes.c_uint64)]


class WirePlan:
    """pv_wire_plan over packed JSON texts: per request the signing message (msg[moff[i]:moff[i+1]]),
    Request.digest (digests[i]), the serializer status, and the signature plan — kind[i]
    (PV_PLAN_*), type_id[i] into `types`, pairs [pair_off[i], pair_off[i+1]) with pair_name[p] into
    `names` and signature text signatures()[p] (bytes sig_blob[sig_off[p]:sig_off[p+1]])."""

    def __init__(self, blob, off, threads=16, plugin_fields=None):
        L = _native.lib()
        n = self.n = len(off) - 1
        blob = np.ascontiguousarray(blob, np.uint8) if len(blob) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        names = PLUGIN_CLIENT_REQUEST_FIELDS if plugin_fields is None else plugin_fields
        pf = b"".join(x.encode() + b"\0" for x in names) + b"\0"
        total = int(off[-1]) if n else 0
        self.status = np.zeros(max(n, 1), np.uint8)
        self.digests = np.zeros((max(n, 1), 32), np.uint8)
        self.moff = np.zeros(n + 1, np.uint64)
        self.kind = np.zeros(max(n, 1), np.uint8)
        self.type_id = np.zeros(max(n, 1), np.uint32)
        self.pair_off = np.zeros(n + 1, np.uint64)
        pair_cap = total // 6 + 1
        self.pair_name = np.zeros(pair_cap, np.uint32)
        self.sig_off = np.zeros(pair_cap + 1, np.uint64)
        sigs = np.empty(total + 1, np.uint8)
        nbuf = np.empty(total + 1, np.uint8)
        name_off = np.zeros(pair_cap + 1, np.uint64)
        tbuf = np.empty(total + 1, np.uint8)
        type_off = np.zeros(n + 1, np.uint64)
        p = lambda a: a.ctypes.data  # noqa: E731
        keys_hex = np.empty(65 * n + 1, np.uint8)
        sig_lines = np.empty(total + 1 + pair_cap, np.uint8)
        cap = total + 64 * n + 64
        for _ in range(2):
            self.msg = np.empty(cap, np.uint8)
            P = _PvWirePlan(p(self.msg), cap, p(self.moff), p(self.digests), p(self.status), p(self.kind),
                            p(self.type_id), p(self.pair_off), p(self.pair_name), p(self.sig_off), pair_cap, p(sigs),
                            total + 1, p(nbuf), p(name_off), total + 1, p(tbuf), p(type_off), total + 1, p(keys_hex), p(sig_lines), 0, 0, 0)
            rc = L.pv_wire_plan(p(blob), p(off), n, pf, threads, ctypes.byref(P))
            if rc == PV_ERR_ARG and int(self.moff[n]) > cap:
                cap = int(self.moff[n])
                continue
            _native.check(rc, "pv_wire_plan")
            break
        else:
            raise _native.NativeError("pv_wire_plan: output size changed between calls")
        self.status, self.digests = self.status[:n], self.digests[:n]
        self.kind, self.type_id = self.kind[:n], self.type_id[:n]
        np_ = self.n_pairs = int(P.n_pairs)
        self.pair_name, self.sig_off = self.pair_name[:np_], self.sig_off[:np_ + 1]
        self.sig_blob = sigs[:max(int(self.sig_off[-1]), 1)]
        self._keys_hex = keys_hex[:65 * n]
        self._sig_lines = sig_lines[:int(self.sig_off[-1]) + np_]
        no, to = name_off[:int(P.n_names) + 1].tolist(), type_off[:int(P.n_types) + 1].tolist()
        nb, tb = bytes(nbuf[:no[-1]]), bytes(tbuf[:to[-1]])
        self.names = [nb[no[k]:no[k + 1]].decode("ascii") for k in range(len(no) - 1)]
        self.names_blob = nbuf[:max(no[-1], 1)]
        self.name_off = name_off[:len(no)]
        self.types = [tb[to[k]:to[k + 1]].decode() for k in range(len(to) - 1)]

    def keys(self):
        """Request.digest of every request as a hex str (the verified-request cache key)."""
        return self._keys_hex.tobytes().decode("ascii").split("\n")[:self.n]

    def signatures(self):
        """The signature text of every pair, as str."""
        return self._sig_lines.tobytes().decode("ascii").split("\n")[:self.n_pairs]


def _plain(s):
    """A str the device decoder sees exactly as base58.b58decode does (ASCII, nothing stripped)."""
    return isinstance(s, str) and s.isascii() and s == s.rstrip()


_FAST, _QUERY, _SLOW, _FAILED = 0, 1, 2, 3
_scan_once = json.JSONDecoder().scan_once  # the C scanner json.loads drives


def _loads(raw):
    """json.loads(raw.decode()) — the same object or the same exception — calling the C scanner
    directly when the text is exactly one JSON value (no surrounding whitespace); anything else
    goes through json.loads itself."""
    s = raw.decode() if isinstance(raw, (bytes, bytearray)) else raw
    try:
        obj, end = _scan_once(s, 0)
        if end == len(s):
            return obj
    except (StopIteration, ValueError):
        pass
    return json.loads(s)
_REQUEST_PARAMS = frozenset(("self",))  # JSON keys Request(**msg) cannot take as keywords


def _request_view(msg):
    """``Request(**msg).as_dict`` for a JSON object, without building the Request (same keys, same
    insertion order); None when only the Request constructor gives the exact result or exception
    (not an object, a key colliding with a constructor parameter, plugin fields registered)."""
    if type(msg) is not dict or PLUGIN_CLIENT_REQUEST_FIELDS or "self" in msg:
        return None
    get = msg.get
    view = {REQ_ID: get(REQ_ID), OPERATION: get(OPERATION)}
    for name in (IDENTIFIER, SIGNATURES, SIGNATURE, PROTOCOL_VERSION, TAA_ACCEPTANCE, ENDORSER):
        v = get(name)
        if v is not None:
            view[name] = v
    return view


def authenticate_wire_batch(req_authnr, raws, threads=16, timings=None, one_call_per_request=False):
    """For each received request (JSON bytes), what the reference's ingress produces at the
    authentication step. Returns [(request dict or None, result)]: result is the identifier set
    ``req_authnr.authenticate(Request(**msg).as_dict, key=Request(**msg).key)`` returns, or the
    exception instance raised by json.loads, Request(**msg), .key or authenticate.

    By default a request whose signatures all verify on the device completes without calling
    ``req_authnr.authenticate`` (zero calls; the verified-request cache is filled as authenticate
    fills it). ``one_call_per_request=True`` keeps the reference's call pattern — authenticate
    exactly once per request that is not a cache hit (the spy of
    plenum/test/node_request/test_propagate/test_no_reauth.py:11-23) — with every signature check
    of the batch still in one launch.

    The cyclic garbage collector is paused for the call: the batch allocates a few dicts per
    request and creates no garbage cycles of its own, and generation scans triggered by those
    allocations cost as much as the per-request work itself (collection resumes afterwards)."""
    blob, off = _native._blob([r if isinstance(r, (bytes, bytearray)) else r.encode() for r in raws])
    res = authenticate_wire_packed(req_authnr, blob, off, threads, timings, one_call_per_request)
    return [(res.msg(i), r) for i, r in enumerate(res.results)]


class WireResults:
    """authenticate_wire_packed's outcome for n received requests: ``results[i]`` is the identifier
    set (or the exception instance) authenticate_wire_batch returns for request i, ``msg(i)`` the
    json.loads dict of its text (None when json.loads raises). A request the device completed was
    never decoded in Python: its dict is built on first access — the decode the reference does in
    ZStack.deserializeMsg (stp_zmq/zstack.py:881-885), not part of authentication. Indexing gives
    authenticate_wire_batch's (msg, result) pairs."""

    def __init__(self, blob, off, results, msgs):
        self._blob, self._off, self.results, self._msgs = blob, off, results, msgs

    def __len__(self):
        return len(self.results)

    def msg(self, i):
        m = self._msgs.get(i, _MISSING)
        if m is _MISSING:
            try:
                m = _loads(self._blob[int(self._off[i]):int(self._off[i + 1])].tobytes())
            except Exception:
                m = None
            self._msgs[i] = m
        return m

    def __getitem__(self, i):
        return self.msg(i), self.results[i]

    def __iter__(self):
        return (self[i] for i in range(len(self.results)))


_MISSING = object()


def _fast_capable(core, one_call_per_request):
    """The device may finish a request for `core` only where pv_wire_plan reproduces its Python
    planning: CoreAuthMixin's signature selection and signing view, batched verkey lookup."""
    if core is None or not hasattr(core, "plan_verifications"):
        return None
    from .client_authn import CoreAuthMixin
    cls = type(core)
    if one_call_per_request and getattr(cls, "authenticate", None) is not CoreAuthMixin.authenticate:
        return None  # only CoreAuthMixin.authenticate takes the batch's precomputed answer
    if (getattr(cls, "_select_signatures", None) is not CoreAuthMixin._select_signatures
            or getattr(cls, "_signing_view", None) is not CoreAuthMixin._signing_view
            or set(getattr(core, "excluded_from_signing", ())) != _EXCLUDED):
        return None
    make_resolver = getattr(core, "verkey_resolver", None)
    resolver = make_resolver() if make_resolver else None
    if resolver is None or not getattr(resolver, "batched", False):
        return None
    return resolver


def authenticate_wire_packed(req_authnr, blob, off, threads=16, timings=None, one_call_per_request=False):
    """authenticate_wire_batch on texts already packed as (uint8 blob, uint64 offsets[n+1]),
    returning a WireResults. The per-request work is split by where it runs best:
      1. C++, many threads (pv_wire_plan): one parse of each text gives the signing message,
         Request.digest and the signature plan (SINGLE / MULTI / Python).
      2. Python, per distinct txn type and per distinct identifier (not per request): which
         authenticators run, the batch's verkey of each signer (VerkeyResolver).
      3. GPU, one launch: base58 decode of every planned signature, DidVerifier key resolution
         per signer, sm assembly and verification (pv_ingress_verify).
      4. Python, in request order: the verified-request cache and the identifier set of each
         device-finished request; every other request (undecodable, unusual fields, a failing or
         request-dependent check, ...) is decoded here and goes through the unchanged sequential
         ``authenticate`` — its remaining checks batched into one more launch — so results,
         exceptions and cache side effects are the sequential ones."""
    was_enabled = gc.isenabled()
    gc.disable()
    try:
        return _authenticate_packed(req_authnr, blob, off, threads, timings, one_call_per_request)
    finally:
        if was_enabled:
            gc.enable()


def _authenticate_packed(req_authnr, blob, off, threads, timings, one_call_per_request):
    t0 = time.perf_counter()
    off = np.ascontiguousarray(off, np.uint64)
    P = WirePlan(blob, off, threads)
    n = P.n
    t1 = time.perf_counter()
    authnrs = req_authnr._authenticators
    core = authnrs[0] if authnrs else None
    resolver = _fast_capable(core, one_call_per_request)
    fast = np.zeros(n, bool)
    nver = 0
    t2 = t1
    if resolver is not None and P.n_pairs:
        kinds = [_type_kind(authnrs, core, t) for t in P.types]
        tk = np.array(kinds, np.uint8)
        name_vk = []
        for idr in P.names:
            vk = resolver.static(idr)
            name_vk.append(vk if type(vk) is str and _plain(vk) else None)
        name_ok = np.array([v is not None for v in name_vk], bool)
        lo = P.pair_off[:-1].astype(np.int64)
        hi = P.pair_off[1:].astype(np.int64)
        bad = np.zeros(P.n_pairs + 1, np.int64)
        np.cumsum(~name_ok[P.pair_name], out=bad[1:])
        cand = (P.kind != PV_PLAN_PY) & (tk[P.type_id] == _FAST) & (bad[hi] == bad[lo])
        sel = np.nonzero(np.repeat(cand, hi - lo))[0]
        t2 = time.perf_counter()
        if sel.size:
            if sel.size == P.n_pairs:
                sb, so = P.sig_blob, P.sig_off
            else:
                starts = P.sig_off[sel].astype(np.int64)
                lens = P.sig_off[sel + 1].astype(np.int64) - starts
                so = np.zeros(sel.size + 1, np.uint64)
                np.cumsum(lens, out=so[1:])
                sb = P.sig_blob[np.repeat(starts - so[:-1].astype(np.int64), lens) + np.arange(int(so[-1]))]
            msg_idx = np.repeat(np.arange(n, dtype=np.uint32), hi - lo)[sel]
            vb, vo = _native._blob([v.encode() if v is not None else b"" for v in name_vk])
            vp = name_ok.astype(np.uint8)
            vstat, verdict = _native.ingress_verify_arrays(sb, so, P.msg, P.moff, msg_idx, P.pair_name[sel],
                                                           P.names_blob, P.name_off, vb, vo, vp)
            nver = int(sel.size)
            good = np.zeros(P.n_pairs, bool)
            good[sel] = (vstat == 0) & verdict
            np.cumsum(~good, out=bad[1:])
            fast = cand & (bad[hi] == bad[lo])
    t3 = time.perf_counter()
    verified = req_authnr._verified_reqs
    fc = _native._fastcall()
    # the device-verified single-signature requests are finished in C (_fastcall.finish_single: the
    # same per-request dict operations, without the interpreter) when the cache is a plain dict
    c_finish = bool(fc) and hasattr(fc, "finish_single") and type(verified) is dict and not one_call_per_request
    # request i's key (Request.digest, hex) when its serialization succeeded; only the requests that
    # are not finished in C need it as a str
    keys_all = P.keys() if not (c_finish and (fast & (P.kind == PV_PLAN_SINGLE)).all()) else None
    ser_ok = (P.status == PV_SER_OK).tolist()
    msgs, other, slow_views = {}, {}, []
    names = P.names
    pn, po = P.pair_name, P.pair_off
    answers = {}
    if one_call_per_request and fast.any():
        # the reference's call pattern: every request still goes through req_authnr.authenticate
        # once, with the request dict it would get; for a device-finished request the core
        # authenticator answers from the plan (identifiers in signature-dict order) instead of
        # re-serializing and re-resolving every signer
        for i in np.nonzero(fast)[0].tolist():
            msg = None
            try:
                msg = _loads(blob[int(off[i]):int(off[i + 1])].tobytes())
                view = _request_view(msg)
                if view is None:
                    view = Request(**msg).as_dict
            except Exception as ex:
                msgs[i] = msg
                other[i] = (_FAILED, None, ex)
                continue
            msgs[i] = msg
            answers[id(view)] = (view, core, [names[q] for q in pn[int(po[i]):int(po[i + 1])].tolist()])
            other[i] = (_SLOW, view, keys_all[i])
    for i in np.nonzero(~fast)[0].tolist():  # decoded and classified as the sequential path does
        msg = None
        try:
            msg = _loads(blob[int(off[i]):int(off[i + 1])].tobytes())
            view = _request_view(msg)
            req = None
            if view is None:
                req = Request(**msg)
                view = req.as_dict
        except Exception as ex:
            msgs[i] = msg
            other[i] = (_FAILED, None, ex)
            continue
        msgs[i] = msg
        if ser_ok[i]:
            key = keys_all[i]
        else:
            try:
                key = (req or Request(**msg)).key
            except Exception as ex:
                other[i] = (_FAILED, view, ex)
                continue
        other[i] = (_SLOW, view, key)
        slow_views.append(view)
    cache = batch.VerdictCache()
    if slow_views and core is not None and hasattr(core, "plan_verifications"):
        cache.fill(core.plan_verifications(slow_views))
    if one_call_per_request:
        fast[:] = False  # every request takes one authenticate call
    results = [None] * n
    vget = verified.get
    kind = P.kind
    sigs_all = P.signatures() if fast.any() and not c_finish else []

    def one(i):  # request i in order, as the sequential path would finish it
        if fast[i]:
            key = keys_all[i]
            p = int(po[i])
            if kind[i] == PV_PLAN_SINGLE:
                sig, ids = sigs_all[p], None
            else:
                sig, ids = None, {names[q] for q in pn[p:int(po[i + 1])].tolist()}
            seen = vget(key)
            if seen is not None and seen['signature'] == sig:
                results[i] = seen['identifiers']
                return
            if ids is None:
                ids = {names[int(pn[p])]}
            verified[key] = {'signature': sig, 'identifiers': ids}
            results[i] = ids
            return
        k, view, key = other[i]
        if k == _FAILED:
            results[i] = key
            return
        try:
            results[i] = req_authnr.authenticate(view, key)
        except Exception as ex:
            results[i] = ex

    simple = fast & (kind == PV_PLAN_SINGLE)
    if simple.any() and not c_finish:
        # distinct keys among the device-finished requests (a 64-bit prefix suffices to prove it)
        pre = P.digests[simple, :8].copy().view(np.uint64).ravel()
        keys_distinct = np.unique(pre).size == pre.size

    def run(a, b):
        """Requests a..b-1, all device-finished single-signature ones: when their keys are new
        and distinct (the usual batch), the cache entries go in with one dict.update in request
        order — the state the per-request sequence leaves — else one by one."""
        if c_finish:
            fc.finish_single(verified, results, a, b, P._keys_hex, P._sig_lines, P.sig_off, po, pn, names)
            return
        keys = keys_all[a:b]
        if not keys_distinct or not verified.keys().isdisjoint(keys):
            for i in range(a, b):
                one(i)
            return
        p0, p1 = int(po[a]), int(po[b])  # single-signature requests: consecutive pairs
        ids = [{names[j]} for j in pn[p0:p1].tolist()]
        verified.update(zip(keys, [{'signature': s, 'identifiers': d} for s, d in zip(sigs_all[p0:p1], ids)]))
        results[a:b] = ids

    with batch.active(cache, answers=answers):
        start = 0
        for j in np.nonzero(~simple)[0].tolist() + [n]:
            if j > start:
                run(start, j)
            if j < n:
                one(j)
            start = j + 1
    t4 = time.perf_counter()
    if timings is not None:
        timings.update({"serialize_s": t1 - t0, "plan_s": t2 - t1, "gpu_s": t3 - t2, "finish_s": t4 - t3,
                        "requests": n, "verifications": nver, "slow": len(slow_views)})
    return WireResults(blob, off, results, msgs)


def _type_kind(authnrs, core, typ):
    """How ReqAuthenticator.authenticate (req_authenticator.py:23-51) treats a txn type: _QUERY if
    an authenticator reports it as a query before any runs, _FAST if the core authenticator is the
    only one that runs, _SLOW otherwise."""
    runners = []
    for a in authnrs:
        if a.is_query(typ):
            return _QUERY if not runners else _SLOW
        if a.is_write(typ) or a.is_action(typ):
            runners.append(a)
    return _FAST if len(runners) == 1 and runners[0] is core else _SLOW
