"""The ingress batch path: received JSON bytes -> authentication results.

Per received client request the reference does, at the authentication step,
    msg = json.loads(raw)                                   stp_zmq/zstack.py:881-885
    req = Request(**msg)                                    plenum/server/node.py:1643
    req_authnr.authenticate(req.as_dict, key=req.key)       node.py:2636-2650 verifySignature
one request at a time. ``authenticate_wire_batch`` does it for a whole ZStack quota (or the
requests of a PROPAGATE batch) with the per-request work split by where it runs best:
  1. C++, many threads: JSON text -> signing-serialized M and Request.digest
     (pv_signing_serialize_json, PV_SER_REQUEST). Requests it defers (floats, ...) use the Python
     mirror below.
  2. Python: json.loads (the node keeps the dicts), signature selection
     (CoreAuthMixin._select_signatures) and getVerkey per signer — state lookups stay on the host.
  3. GPU, one launch: base58 decode of every signature, DidVerifier key resolution per distinct
     (identifier, verkey), sm assembly and verification (pv_ingress_verify).
  4. Python, in request order: the verified-request cache, query/write dispatch, the result.
A request whose signatures all decode, resolve and verify completes in step 4 with exactly the
value the sequential path returns. Every other request (a bad or undecodable signature, a missing
key, an unusual field, several authenticators for its type, ...) goes through the unchanged
sequential ``ReqAuthenticator.authenticate`` — with its remaining signature checks batched into
one more launch — so results, exception classes and messages, and cache side effects are the
sequential ones.
"""
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
    was_enabled = gc.isenabled()
    gc.disable()
    try:
        return _authenticate_wire_batch(req_authnr, raws, threads, timings, one_call_per_request)
    finally:
        if was_enabled:
            gc.enable()


def _authenticate_wire_batch(req_authnr, raws, threads, timings, one_call_per_request=False):
    t0 = time.perf_counter()
    n = len(raws)
    ser_status, mblob, moff, digs = signing_serialize_json(raws, PV_SER_REQUEST, threads)
    ser_ok = (ser_status == PV_SER_OK).tolist()
    hexd = digs.tobytes().hex()  # request i's key (Request.digest) = hexd[64 i : 64 i + 64]
    t1 = time.perf_counter()
    authnrs = req_authnr._authenticators
    core = authnrs[0] if authnrs else None
    fast_capable = (not one_call_per_request and core is not None and hasattr(core, "_select_signatures")
                    and hasattr(core, "plan_verifications"))
    if fast_capable:
        make_resolver = getattr(core, "verkey_resolver", None)
        get_verkey = make_resolver().get if make_resolver else _unbatched_get(core)
        select = core._select_signatures
    type_kind = {}  # txn type -> _FAST (core alone runs it) / _QUERY / _SLOW, per batch
    entries = []  # (kind, msg dict, as_dict, key or exception, identifiers)
    sig_strs, v_msg, v_signer = [], [], []
    lo_hi = []  # verification range of each _FAST entry, in entry order
    signers, idr_list, vk_list, fixed = {}, [], [], {}
    for i, raw in enumerate(raws):
        msg = None
        try:
            msg = _loads(raw)
            view = _request_view(msg)
            if view is None:
                req = Request(**msg)
                view = req.as_dict
            else:
                req = None
        except Exception as ex:
            entries.append((_FAILED, msg, None, ex, None))
            continue
        ok_ser = ser_ok[i]
        if ok_ser:
            key = hexd[64 * i:64 * i + 64]
        else:
            try:
                key = (req or Request(**msg)).key
            except Exception as ex:
                entries.append((_FAILED, msg, view, ex, None))
                continue
        kind = _SLOW
        ids = None
        op = view[OPERATION]
        if fast_capable and ok_ser and type(op) is dict:
            typ = op.get(TXN_TYPE)
            try:
                k = type_kind.get(typ)
                if k is None:
                    k = type_kind[typ] = _type_kind(authnrs, core, typ)
            except TypeError:  # an unhashable type: the sequential path raises for it
                k = _SLOW
            if k == _QUERY:
                kind = _QUERY
            elif k == _FAST:
                ids = _plan_signatures(select, get_verkey, fixed, view, i, sig_strs, v_msg, v_signer, signers, idr_list,
                                       vk_list, lo_hi)
                if ids is not None:
                    kind = _FAST
        entries.append((kind, msg, view, key, ids))
    t2 = time.perf_counter()
    if sig_strs:
        sb, so = _native._blob(sig_strs)
        ib, io = _native._blob(idr_list)
        vb, vo = _native._blob([v if v is not None else b"" for v in vk_list])
        vp = np.array([v is not None for v in vk_list], np.uint8)
        vstat, verdict = _native.ingress_verify_arrays(sb, so, mblob, moff, np.array(v_msg, np.uint32),
                                                       np.array(v_signer, np.uint32), ib, io, vb, vo, vp)
        bad = np.zeros(len(sig_strs) + 1, np.int64)
        np.cumsum(~((vstat == 0) & verdict), out=bad[1:])
        rng = np.array(lo_hi, np.int64).reshape(-1, 2)
        fast_ok = iter((bad[rng[:, 1]] == bad[rng[:, 0]]).tolist())
    else:
        fast_ok = iter(())
    t3 = time.perf_counter()
    # requests the fast path cannot finish: their remaining checks in one more launch
    slow_views = []
    for idx, e in enumerate(entries):
        kind = e[0]
        if kind == _FAST and not next(fast_ok):
            entries[idx] = e = (_SLOW, e[1], e[2], e[3], None)
            kind = _SLOW
        if kind == _SLOW:
            slow_views.append(e[2])
    cache = batch.VerdictCache()
    if slow_views and core is not None and hasattr(core, "plan_verifications"):
        cache.fill(core.plan_verifications(slow_views))
    results = []
    verified = req_authnr._verified_reqs
    existing = req_authnr._check_and_verify_existing_req
    with batch.active(cache):
        for kind, msg, view, key, ids in entries:
            if kind == _FAILED:
                results.append((msg, key))
            elif kind == _SLOW:
                try:
                    results.append((msg, req_authnr.authenticate(view, key)))
                except Exception as ex:
                    results.append((msg, ex))
            elif key and existing(view, key):
                results.append((msg, verified[key]['identifiers']))
            elif kind == _QUERY:
                results.append((msg, set()))
            else:
                ids = set(ids)
                verified[key] = {'signature': view.get(SIGNATURE), 'identifiers': ids}
                results.append((msg, ids))
    t4 = time.perf_counter()
    if timings is not None:
        timings.update({"serialize_s": t1 - t0, "plan_s": t2 - t1, "gpu_s": t3 - t2, "finish_s": t4 - t3,
                        "requests": n, "verifications": len(sig_strs), "slow": len(slow_views)})
    return results


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


def _unbatched_get(core):
    def get(idr, request):
        try:
            return core.getVerkey(idr, request)
        except Exception as ex:
            raise LookupError(ex)
    return get


def _plan_signatures(select, get_verkey, fixed, view, i, sig_strs, v_msg, v_signer, signers, idr_list, vk_list,
                     lo_hi):
    """Queue request i's signatures for the device; returns the identifiers it authenticates, or
    None when the request needs the sequential path (selection or key lookup raising, non-str
    fields, a missing key). ``fixed`` maps an identifier whose verkey does not depend on the
    request (registry or state record, as the batch's VerkeyResolver found) to its signer index."""
    try:
        sigmap = select(view, None, None)
    except Exception:
        return None
    if type(sigmap) is not dict or not sigmap:
        return None
    staged = []
    for idr, sig in sigmap.items():
        if type(sig) is not str or type(idr) is not str:
            return None
        s = fixed.get(idr)
        if s is None:
            if not _plain(idr):
                return None
            try:
                vk = get_verkey(idr, view)
            except Exception:
                return None
            if vk is None or not _plain(vk):
                return None
            s = signers.get((idr, vk))
            if s is None:
                s = signers[(idr, vk)] = len(idr_list)
                idr_list.append(idr.encode())
                vk_list.append(vk.encode())
            memo = getattr(get_verkey, "__self__", None)
            if memo is not None and getattr(memo, "memo", {}).get(idr) is vk:
                fixed[idr] = s
        staged.append((s, sig))
    lo = len(sig_strs)
    for s, sig in staged:
        sig_strs.append(sig.rstrip().encode("utf-8", "surrogatepass"))
        v_msg.append(i)
        v_signer.append(s)
    lo_hi.append(lo)
    lo_hi.append(len(sig_strs))
    return list(sigmap)
