"""Generate the committed golden fixtures by running the REFERENCE itself (/root/reference).

TEST INFRASTRUCTURE, run in the build container only (the reference never ships to the GPU box):
    python tests/golden/make_golden.py
The reference's missing third-party modules are provided by tests/golden/_shims: libnacl (ctypes
over the image's libsodium 1.0.18, the version the reference pins), base58 (oracle/base58_ref.py),
and stubs for zmq/jsonpickle that the hot path never calls. Outputs (all JSON, data only):
  serializer.json    serialize_msg_for_signing KATs (incl. the INDY-1469 nested-dict ambiguity)
  didverifier.json   DidVerifier resolution results / exception class + message
  authn.json         CoreAuthNr.authenticate / authenticate_multi outcomes on signed requests
  reqauth.json       ReqAuthenticator.authenticate sequences (cache, query, NoAuthenticatorFound)
  verdicts.json      libsodium crypto_sign_open verdicts on normal + adversarial (sm, pk) vectors
  request.json       Request(**json.loads(text)): signing bytes of as_dict minus the excluded keys,
                     digest, payload_digest (the wire path's C++ serializer and Request mirror)
  feed.json          the node's feed points (plenum_amd/feed.py): a client quota through
                     Node.handleOneClientMsg and PROPAGATEs through Node.handleOneNodeMsg — the
                     reference's own methods, compiled from plenum/server/node.py's source and run
                     on a stub node (node.py itself cannot be imported here: ursa, rocksdb absent)
Run all generators, or name some: python tests/golden/make_golden.py request.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "_shims"), REF, ROOT, os.path.join(ROOT, "tests")]

import base58  # noqa: E402  (the shim)
from common.serializers.serialization import serialize_msg_for_signing  # noqa: E402
from plenum.common.exceptions import InvalidKey  # noqa: E402,F401
from plenum.common.request import Request  # noqa: E402
from plenum.common.signer_did import DidSigner  # noqa: E402
from plenum.common.signer_simple import SimpleSigner  # noqa: E402
from plenum.common.verifier import DidVerifier  # noqa: E402
from plenum.server.client_authn import CoreAuthNr  # noqa: E402
from plenum.server.req_authenticator import ReqAuthenticator  # noqa: E402

from oracle.libsodium_ref import LibSodium  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from vectors import VectorGen  # noqa: E402


def outcome(fn):
    try:
        r = fn()
        if isinstance(r, set):
            return {"set": sorted(r)}
        if isinstance(r, list):
            return {"list": r}
        return {"value": r}
    except Exception as ex:
        return {"exc": type(ex).__name__, "msg": str(ex)}


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)  # insertion order matters (signature dicts)
    print("wrote", name, len(obj) if hasattr(obj, "__len__") else "")


# ----------------------------------------------------------------------------- serializer
def gen_serializer():
    from collections import OrderedDict  # noqa: F401  (literal inputs may use it)
    inputs = [
        "1", "'aaa'", "None", "{1: 'a', 2: 'b'}", "{'2': 'b', '1': 'a'}", "[1, 5, 3, 4, 2]",
        "OrderedDict([('1', 'a'), ('2', 'b')])", "OrderedDict([('2', 'b'), ('1', 'a')])",
        "{1: 'a', 2: 'b', 3: [1, {2: 'k'}]}", "{'1': 'a', '2': 'b', '3': ['1', {'2': 'k'}]}",
        "{1: 'a', 2: {3: 'b', 4: {5: {6: 'c'}}}}", "{1: 'a', 2: {3: 'b'}, 4: {5: {6: 'c'}}}",
        "{'1': 'a', '2': 'b', '3': {'4': 'c', '5': 'd', '6': {'7': {'8': 'e', '9': 'f'}, "
        "'10': {'11': 'g', '12': 'h'}}, '13': {'13': {'13': 'i'}}}}",
        "OrderedDict([('2', OrderedDict([('4', 'c'), ('3', 'b')])), ('1', 'a')])",
        "{'a': True, 'b': False, 'c': 1.5, 'd': None, 'e': [], 'f': {}, 'g': [None, 2.25, 'x']}",
        "{'identifier': 'V4SGRU86Z58d6TV7PBUe6f', 'reqId': 1700000000000001, 'protocolVersion': 2, "
        "'operation': {'type': '1', 'dest': 'V4SGRU86Z58d6TV7PBUe6f', 'verkey': '~CoRER63DVYnWZtK8uAzNbx', "
        "'alias': 'u00000001'}, 'taaAcceptance': {'taaDigest': '" + "ab" * 32 + "', "
        "'mechanism': 'service_agreement', 'time': 1700000000}}",
        "{'x': 'ünïcödé', 'y': ['€', 1e100, -0.0, 10**30]}",
        "{'signature': 'S', 'signatures': {'a': 'b'}, 'fees': [1], 'k': 'v'}",
        "(1, 2)", "b'bytes'", "{'k': (1, 2)}", "{1: 'a', '2': 'b'}",
    ]
    ignore_sets = [None, ["signature"], ["signature", "signatures", "fees"]]
    out = []
    for src in inputs:
        for ign in ignore_sets:
            obj = eval(src)  # literal fixtures defined above
            res = outcome(lambda: serialize_msg_for_signing(obj, topLevelKeysToIgnore=ign).hex())
            out.append({"input": src, "ignore": ign, "out": res})
    return out


# ----------------------------------------------------------------------------- DidVerifier
def gen_didverifier():
    cases = [("~8zH9ZSyZTFPGJ4ZPL5Rvxx", "99BgFBg35BehzfSADV5nM4"),  # test_verifier.py KAT
             (None, "99BgFBg35BehzfSADV5nM4"), ("", "99BgFBg35BehzfSADV5nM4"),
             ("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF", None),  # odd-length verkey KAT
             ("5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdock", None),
             ("5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdock", "99BgFBg35BehzfSADV5nM4"),
             (None, None), ("", None), ("~", "99BgFBg35BehzfSADV5nM4"), ("~0OIl", "99BgFBg35BehzfSADV5nM4"),
             ("~8zH9ZSyZTFPGJ4ZPL5Rvxx", "0OIl"), ("~8zH9ZSyZTFPGJ4ZPL5Rvxx", None),
             ("~8zH9ZSyZTFPGJ4ZPL5Rvxx", "   "), ("5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdock  ", None),
             ("5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdoc", None), ("11111111111111111111111111111111", None),
             ("1111111111111111111111111111111111", None)]
    # cryptonyms (identifier = full b58 verkey) and DidSigner pairs
    for i in range(6):
        s = DidSigner(seed=bytes([65 + i]) * 32)
        cases.append((s.verkey, s.identifier))
        ss = SimpleSigner(seed=bytes([97 + i]) * 32)
        cases.append((None, ss.identifier))
        cases.append(("", ss.identifier))
        cases.append((ss.verkey, None))
    # hex-encoded verkey: b58(hex string of a 32-byte key) goes through VerifyKey(key, HexEncoder)
    hexkey = base58.b58encode(b"ab" * 32).decode()
    cases += [(hexkey, None), (base58.b58encode(b"ab" * 31 + b"zz").decode(), None),
              (base58.b58encode(b"abc").decode(), None)]
    out = []
    for vk, idr in cases:
        def run():
            v = DidVerifier(vk, identifier=idr)
            key = v._vr.key
            return {"verkey": v.verkey, "raw": bytes(key).hex() if key else None}
        out.append({"verkey": vk, "identifier": idr, "out": outcome(run)})
    return out


# ----------------------------------------------------------------------------- authn
class RefState:
    """state.get(key, isCommitted) over {sha256(nym): json} (request_handlers/utils.py:30-39)."""

    def __init__(self, nyms):
        from hashlib import sha256
        self.kv = {sha256(n.encode()).digest(): json.dumps(r).encode() for n, r in nyms.items()}

    def get(self, key, isCommitted=True):
        return self.kv.get(key)


def nym_op(signer, i):
    return {"type": "1", "dest": signer.identifier, "verkey": signer.verkey, "alias": "u%08d" % i}


def signed_request(signer, i, extra=None, op=None):
    req = Request(identifier=signer.identifier, reqId=1700000000000000 + i, operation=op or nym_op(signer, i),
                  protocolVersion=2)
    if extra:
        for k, v in extra.items():
            setattr(req, k, v)
    req.signature = signer.sign(req.signingPayloadState())
    return req.as_dict


def multi_signed(signers, i, bad=()):
    req = Request(identifier=signers[0].identifier, reqId=1700000000100000 + i,
                  operation={"type": "101", "x": i}, protocolVersion=2)
    sigs = {}
    for j, s in enumerate(signers):
        sig = s.sign(req.signingPayloadState())
        if j in bad:
            raw = bytearray(base58.b58decode(sig))
            raw[5] ^= 1
            sig = base58.b58encode(bytes(raw)).decode()
        sigs[s.identifier] = sig
    d = req.as_dict
    d["signatures"] = sigs
    return d


def gen_authn():
    signers = [DidSigner(seed=("signer%026d" % i).encode()) for i in range(5)]
    crypt = SimpleSigner(seed=b"c" * 32)
    unregistered = DidSigner(seed=b"u" * 32)
    clients = {s.identifier: s.verkey for s in signers[:4]}
    clients[crypt.identifier] = ""  # cryptonym: DidVerifier uses the identifier itself
    clients[signers[4].identifier] = base58.b58encode(base58.b58decode(signers[4].identifier) + base58.b58decode(
        signers[4].verkey[1:])).decode()  # full (non-abbreviated) verkey
    state_nyms = {unregistered.identifier: {"verkey": unregistered.verkey, "role": None}}
    cases = []

    def add(kind, req, **kw):
        cases.append({"kind": kind, "req": req, "kw": kw})

    for i, s in enumerate(signers + [crypt]):
        add("authenticate", signed_request(s, i))
    add("authenticate", signed_request(unregistered, 10))  # verkey from uncommitted state
    fresh = DidSigner(seed=b"f" * 32)
    add("authenticate", signed_request(fresh, 11))  # NYM dest == identifier: self verkey
    fresh2 = DidSigner(seed=b"g" * 32)
    r = signed_request(fresh2, 12, op={"type": "101", "dest": fresh2.identifier})
    add("authenticate", r)  # not NYM, unknown DID -> CouldNotAuthenticate
    r = signed_request(signers[0], 13)
    r["reqId"] += 1
    add("authenticate", r)  # tampered -> InsufficientCorrectSignatures
    r = signed_request(signers[0], 14)
    r["identifier"] = signers[1].identifier
    add("authenticate", r)  # wrong key
    r = signed_request(signers[0], 15)
    r["signature"] = "0OIl" + r["signature"][4:]
    add("authenticate", r)  # invalid base58 -> InvalidSignatureFormat
    r = signed_request(signers[0], 16)
    raw = base58.b58decode(r["signature"])
    r2 = dict(r, signature=base58.b58encode(raw[:63]).decode())
    add("authenticate", r2)  # 63-byte signature: sm split point shifts
    r3 = dict(r, signature=base58.b58encode(raw + b"\x00").decode())
    add("authenticate", r3)  # 65 bytes
    r4 = dict(r, signature=base58.b58encode(raw[:10]).decode())
    add("authenticate", r4)
    r = signed_request(signers[0], 17)
    del r["signature"]
    add("authenticate", r)  # MissingSignature
    r = signed_request(signers[0], 18)
    r["signature"] = ""
    add("authenticate", r)  # empty signature with identifier -> signatures None -> TypeError
    r = signed_request(signers[0], 19)
    r["fees"] = [["utxo", 1]]
    add("authenticate", r)  # fees excluded from signing
    r = signed_request(signers[0], 20)
    r["signature"] = r["signature"] + "  "
    add("authenticate", r)  # trailing whitespace stripped by b58decode
    r = signed_request(signers[0], 21)
    del r["identifier"]
    add("authenticate", r)  # signature without identifier -> signatures None
    r = signed_request(signers[0], 22)
    add("authenticate", r, identifier=signers[0].identifier, signature=r["signature"])
    ms = signers[:3]
    for bad in [(), (0,), (1,), (2,), (0, 2), (0, 1, 2)]:
        d = multi_signed(ms, 30 + len(cases), bad)
        add("authenticate", d)
        for th in (None, 1, 2, 3, 4):
            payload = {k: v for k, v in d.items() if k not in ("signature", "signatures", "fees")}
            add("authenticate_multi", payload, signatures=d["signatures"], threshold=th)
    d = multi_signed(ms, 50)
    d["signatures"] = {}
    add("authenticate", d)
    d = multi_signed(ms + [unregistered], 51)
    add("authenticate", d)  # 4th signer resolved from state
    d = multi_signed(ms + [DidSigner(seed=b"h" * 32)], 52)
    add("authenticate", d)  # unknown co-signer -> CouldNotAuthenticate (after 3 good ones)
    d = multi_signed(ms, 53)
    d["signatures"][signers[1].identifier] = "invalid!!"
    add("authenticate", d)  # invalid base58 in position 2
    out = []
    for c in cases:
        authnr = CoreAuthNr(["1", "101"], ["105"], ["action"], state=RefState(state_nyms))
        for idr, vk in clients.items():
            authnr.addIdr(idr, vk)
        if c["kind"] == "authenticate":
            res = outcome(lambda: authnr.authenticate(json.loads(json.dumps(c["req"])), **c["kw"]))
        else:
            res = outcome(lambda: authnr.authenticate_multi(json.loads(json.dumps(c["req"])), **c["kw"]))
        out.append(dict(c, out=res))
    return {"clients": clients, "state_nyms": state_nyms, "cases": out}


def gen_reqauth():
    signers = [DidSigner(seed=("rasigner%024d" % i).encode()) for i in range(3)]
    clients = {s.identifier: s.verkey for s in signers}
    seqs = []
    good = signed_request(signers[0], 1)
    bad = dict(good, reqId=good["reqId"] + 1)
    other = signed_request(signers[1], 2)
    query = signed_request(signers[2], 3, op={"type": "105", "dest": signers[2].identifier})
    unknown_type = signed_request(signers[2], 4, op={"type": "999"})
    resigned = signed_request(signers[0], 1)  # same digest key, same signature
    alt_sig = dict(good, signature=other["signature"])  # same key, different signature
    seqs.append([(good, "k1"), (good, "k1"), (bad, "k2"), (other, "k3"), (query, "k4"), (unknown_type, "k5"),
                 (resigned, "k1"), (alt_sig, "k1"), (good, None), (bad, None)])
    seqs.append([(bad, "kb"), (bad, "kb"), (good, "kb"), (bad, "kb")])
    out = []
    for seq in seqs:
        ra = ReqAuthenticator()
        core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=RefState({}))
        for idr, vk in clients.items():
            core.addIdr(idr, vk)
        ra.register_authenticator(core)
        res = [outcome(lambda: ra.authenticate(json.loads(json.dumps(req)), key)) for req, key in seq]
        out.append({"items": [[req, key] for req, key in seq], "out": res})
    # no authenticator registered / core_authenticator error
    ra = ReqAuthenticator()
    out.append({"items": [[good, "k"]], "out": [outcome(lambda: ra.authenticate(good, "k"))]})
    return {"clients": clients, "seqs": out}


def gen_verdicts():
    ls, o = LibSodium(), Oracle()
    g = VectorGen(ls, o, seed=2024)
    out = []
    for cls in VectorGen.CLASSES:
        for _ in range(12 if cls != "mixed_order_A" else 40):
            sm, pk = g.make(cls)
            out.append({"cls": cls, "sm": sm.hex(), "pk": pk.hex(), "ok": ls.sign_open_ok(sm, pk)})
    return out


# ----------------------------------------------------------------------------- Request (wire path)
def request_texts():
    """JSON texts of client requests in the shapes the ingress sees (generated here, data only)."""
    did, did2 = "V4SGRU86Z58d6TV7PBUe6f", "CzkavE58zgX7rUMrzSinLr"
    nym = {"type": "1", "dest": did2, "verkey": "~CoRER63DVYnWZtK8uAzNbx", "alias": "u00000001"}
    taa = {"taaDigest": "ab" * 32, "mechanism": "service_agreement", "time": 1700000000}
    docs = [
        {"identifier": did, "reqId": 1700000000000001, "protocolVersion": 2, "operation": nym,
         "taaAcceptance": taa, "signature": "3v5Xk"},
        {"identifier": did, "reqId": 1, "operation": nym, "signatures": {did: "s1", did2: "s2"}},
        {"reqId": 2, "operation": nym, "signatures": {did2: "s2", did: "s1"}},
        {"identifier": "", "reqId": 3, "operation": nym, "signatures": {did2: "a", "Abc": "b"}},
        {"identifier": None, "reqId": 4, "operation": nym, "signature": "x"},
        {"identifier": did, "reqId": 5, "operation": nym, "signature": "x", "endorser": did2, "fees": [1, 2],
         "unknownField": {"z": 1}, "protocolVersion": None, "taaAcceptance": None},
        {"identifier": did, "reqId": 6, "operation": {"type": "101", "data": {"nested": [1, None, True, False],
                                                                            "u": "\u00fcn\u00efc\u00f6d\u00e9 \u20ac"}},
         "signature": "x"},
        {"identifier": did, "reqId": -0, "operation": {"type": "1", "k": [[], {}, [[1]], {"a": {"b": {}}}]},
         "signature": "x"},
        {"identifier": 0, "reqId": None, "operation": None, "signatures": {}},
        {"identifier": did, "reqId": 7, "operation": nym, "signature": None, "signatures": None},
        {"identifier": did, "reqId": 10 ** 30, "operation": {"type": "1", "big": -10 ** 25}, "signature": "x"},
        {"identifier": did, "reqId": 8, "operation": {"type": "1", "esc": "tab\t nl\n quote\" bs\\ slash/"},
         "signature": "x"},
        {"identifier": did, "reqId": 9, "operation": {"type": "1", "astral": "\ud83d\ude00"}, "signature": "x"},
    ]
    texts = [json.dumps(d) for d in docs]
    texts += [
        '{"identifier": "%s", "reqId": 11, "operation": {"type": "1", "a": 1, "a": 2}, "signature": "x"}' % did,
        '{"reqId": 12, "reqId": 13, "operation": {"type": "1"}, "identifier": "%s", "signature": "y"}' % did,
        '{ "identifier" : "%s" ,\n "reqId":14,"operation":{"type":"1","escaped\\u0041key":"\\u0041"},'
        '"signature":"z" }' % did,
        '{"identifier": "%s", "reqId": 15, "operation": {"type": "1", "e": "\\u00e9", "raw": "é中"},'
        ' "signature": "x"}' % did,
        '{"identifier": "%s", "reqId": -0, "operation": {"type": "1", "neg": -12, "zero": 0}}' % did,
    ]
    return texts


def gen_request():
    out = []
    excluded = {"signature", "signatures", "fees"}
    for text in request_texts():
        def run():
            req = Request(**json.loads(text))
            view = {k: v for k, v in req.as_dict.items() if k not in excluded}
            return {"signing": serialize_msg_for_signing(view).hex(), "digest": req.digest,
                    "payload_digest": req.payload_digest}
        out.append({"text": text, "out": outcome(run)})
    return out


# ----------------------------------------------------------------------------- feed points
def _node_methods():
    """Node's feed-point methods, compiled from the reference's source text and bound to a stub:
    handleOneClientMsg, validateClientMsg, handleInvalidClientMsg, _specific_invalid_client_msg_handling,
    handleOneNodeMsg, validateNodeMsg, verifySignature, authNr (plenum/server/node.py)."""
    import ast
    import contextlib
    from collections.abc import Mapping
    from plenum.common import exceptions as E
    from plenum.common.constants import LEDGER_STATUS, OP_FIELD_NAME
    from plenum.common.messages.internal_messages import PreSigVerification
    from plenum.common.messages.node_message_factory import node_message_factory
    from plenum.common.messages.node_messages import Batch, CatchupReq, LedgerStatus, Propagate
    from plenum.common.txn_util import TxnUtilConfig, idr_from_req_data
    from plenum.common.types import OPERATION, f
    from plenum.common.util import friendlyEx, reasonForClientFromException
    with open(os.path.join(REF, "plenum", "server", "node.py")) as fh:
        tree = ast.parse(fh.read())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Node")
    want = {"handleOneClientMsg", "validateClientMsg", "handleInvalidClientMsg",
            "_specific_invalid_client_msg_handling", "handleOneNodeMsg", "validateNodeMsg", "verifySignature",
            "authNr", "white_list_init"}
    funcs = [fn for fn in cls.body if isinstance(fn, ast.FunctionDef) and fn.name in want]
    assert {fn.name for fn in funcs} == want
    for fn in funcs:
        fn.decorator_list = []  # metrics decorators

    class _Log:
        def __getattr__(self, name):
            return lambda *a, **k: None

    class _Metrics:
        def measure_time(self, *a):
            return contextlib.nullcontext()

    class _MN:
        def __getattr__(self, name):
            return name

    from plenum.common.messages import node_messages as NM
    ns = {n: getattr(NM, n) for n in dir(NM) if not n.startswith("_")}  # white_list_init's classes
    ns.update(f=f, OPERATION=OPERATION, OP_FIELD_NAME=OP_FIELD_NAME, LEDGER_STATUS=LEDGER_STATUS, Batch=Batch,
              LedgerStatus=LedgerStatus, CatchupReq=CatchupReq, Propagate=Propagate,
              node_message_factory=node_message_factory, PreSigVerification=PreSigVerification,
              TxnUtilConfig=TxnUtilConfig, idr_from_req_data=idr_from_req_data, friendlyEx=friendlyEx,
              reasonForClientFromException=reasonForClientFromException, Request=Request, Mapping=Mapping,
              MetricsName=_MN(), logger=_Log(), **{n: getattr(E, n) for n in dir(E) if not n.startswith("_")})
    exec(compile(ast.Module(body=funcs, type_ignores=[]), "reference:plenum/server/node.py", "exec"), ns)
    return {fn.name: ns[fn.name] for fn in funcs}, _Metrics, Batch


class _StubNode:
    """What the feed-point methods touch on a Node; records the side effects."""

    def __init__(self, methods, metrics_cls, req_authnr):
        import types
        for name, fn in methods.items():
            setattr(self, name, types.MethodType(fn, self))
        self.metrics = metrics_cls()
        self.white_list_init()  # the node's own authnWhitelist (node.py:405-431)
        self.clientAuthNr = req_authnr
        self.client_request_class = Request
        self.events = []

        class _Replicas:
            def send_to_internal_bus(self, *a):
                pass

        class _Replica:
            instId = 0

        class _Stack:
            name = "NodeC"
        self.replicas, self.master_replica, self.clientstack = _Replicas(), _Replica(), _Stack()

    def isClientBlacklisted(self, frm):
        return False

    def isNodeBlacklisted(self, frm):
        return False

    def doStaticValidation(self, msg):
        pass

    def unpackClientMsg(self, msg, frm):
        self.events.append({"ev": "accepted", "frm": frm, "type": type(msg).__name__})

    def send_nack_to_client(self, idr_reqid, reason, frm):
        self.events.append({"ev": "nack", "frm": frm, "identifier": idr_reqid[0], "reqId": idr_reqid[1],
                            "reason": reason})

    def discard(self, msg, reason, logMethod=None, cliOutput=False):
        self.events.append({"ev": "discard", "reason": str(reason), "exc": type(reason).__name__})

    def reportSuspiciousClient(self, frm, friendly):
        self.events.append({"ev": "suspicious_client", "frm": frm})

    def reportSuspiciousNodeEx(self, ex):
        self.events.append({"ev": "suspicious_node", "node": ex.node, "code": ex.code, "reason": ex.reason,
                            "cause": type(ex.__cause__).__name__, "cause_str": str(ex.__cause__)})

    def unpackNodeMsg(self, msg, frm):
        self.events.append({"ev": "accepted", "frm": frm, "type": type(msg).__name__})

    def _invalid_client_ledger_status_handling(self, ex, msg, frm):
        pass


def gen_feed():
    methods, metrics_cls, Batch = _node_methods()
    signers = [DidSigner(seed=("feedsigner%022d" % i).encode()) for i in range(4)]
    clients = {s.identifier: s.verkey for s in signers[:3]}
    bad_vk = DidSigner(seed=b"v" * 32)
    clients[bad_vk.identifier] = "~" + "1" * 5  # abbreviated verkey too short -> InvalidKey
    unknown = DidSigner(seed=b"n" * 32)

    def fresh_authnr():
        core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=RefState({}))
        for idr, vk in clients.items():
            core.addIdr(idr, vk)
        ra = ReqAuthenticator()
        ra.register_authenticator(core)
        spy = {"calls": 0, "ids": []}
        orig = ra.authenticate

        def authenticate(req_data, key=None):
            spy["calls"] += 1
            r = orig(req_data, key)
            spy["ids"].append(sorted(r))
            return r
        ra.authenticate = authenticate
        return ra, core, spy

    reqs = []
    for i, s in enumerate(signers[:3]):
        reqs.append(("valid", signed_request(s, 100 + i)))
    reqs.append(("duplicate", json.loads(json.dumps(reqs[0][1]))))  # verified-request cache hit
    r = signed_request(signers[0], 110)
    r["reqId"] += 1
    reqs.append(("tampered", r))
    r = signed_request(signers[1], 111)
    r["signature"] = "0OIl" + r["signature"][4:]
    reqs.append(("bad_base58", r))
    r = signed_request(signers[1], 112)
    del r["signature"]
    reqs.append(("missing_signature", r))
    reqs.append(("unknown_did", signed_request(unknown, 113, op={"type": "101", "dest": unknown.identifier})))
    reqs.append(("invalid_verkey", signed_request(bad_vk, 114, op={"type": "101", "x": 1})))
    reqs.append(("query", signed_request(signers[2], 115, op={"type": "105", "dest": signers[0].identifier})))
    reqs.append(("no_authenticator", signed_request(signers[2], 116, op={"type": "999"})))
    reqs.append(("multisig_ok", multi_signed(signers[:3], 117)))
    reqs.append(("multisig_bad", multi_signed(signers[:3], 118, bad=(1,))))
    r = signed_request(signers[0], 119)
    del r["reqId"]
    reqs.append(("no_reqid", r))
    r = signed_request(signers[0], 120)
    r["self"] = 1
    reqs.append(("bad_kwarg", r))
    reqs.append(("not_a_dict", [1, 2, 3]))
    # messages carrying "op" (validateClientMsg's second branch, node.py:1634-1638)
    ls = {"op": "LEDGER_STATUS", "ledgerId": 1, "txnSeqNo": 10, "viewNo": None, "ppSeqNo": None,
          "merkleRoot": base58.b58encode(bytes(range(32))).decode(), "protocolVersion": 2}
    reqs.append(("op_ledger_status", ls))
    reqs.append(("op_ledger_status_bad", {"op": "LEDGER_STATUS", "ledgerId": "x", "reqId": 77}))
    reqs.append(("op_catchup_req", {"op": "CATCHUP_REQ", "ledgerId": 1, "seqNoStart": 1, "seqNoEnd": 5,
                                    "catchupTill": 5}))
    reqs.append(("op_batch", {"op": "BATCH", "messages": [], "signature": None}))
    reqs.append(("op_propagate", {"op": "PROPAGATE", "request": signed_request(signers[0], 121),
                                  "senderClient": "cli0"}))
    reqs.append(("op_prepare", {"op": "PREPARE", "instId": 0, "viewNo": 0, "ppSeqNo": 1, "ppTime": 1,
                                "digest": "d", "stateRootHash": None, "txnRootHash": None, "reqId": 9}))
    reqs.append(("op_unknown", {"op": "FOO", "reqId": 5, "identifier": signers[0].identifier}))
    reqs.append(("op_unhashable", {"op": ["x"], "identifier": signers[1].identifier}))
    reqs.append(("op_none", {"op": None}))
    frms = ["cli%d" % (i % 3) for i in range(len(reqs))]

    # client quota: handleOneClientMsg per message, in order, one node
    ra, core, spy = fresh_authnr()
    node = _StubNode(methods, metrics_cls, ra)
    client = []
    for (label, msg), frm in zip(reqs, frms):
        node.events.clear()
        before = spy["calls"]
        try:
            node.handleOneClientMsg((json.loads(json.dumps(msg)), frm))
            raised = None
        except Exception as ex:
            raised = {"exc": type(ex).__name__, "msg": str(ex)}
        client.append({"label": label, "msg": msg, "frm": frm, "events": list(node.events), "raised": raised,
                       "ids": spy["ids"][-1] if spy["calls"] > before and node.events and
                       node.events[-1]["ev"] == "accepted" else None,
                       "authenticate_calls": spy["calls"] - before})
    # PROPAGATEs of a node Batch: handleOneNodeMsg per message
    ra, core, spy = fresh_authnr()
    node = _StubNode(methods, metrics_cls, ra)
    props = []
    nodemsgs = []
    for j, (label, msg) in enumerate(reqs):
        if label in ("not_a_dict", "no_reqid", "bad_kwarg") or label.startswith("op_"):
            continue
        nodemsgs.append((label, {"op": "PROPAGATE", "request": msg, "senderClient": "client%d" % j}))
    good = signed_request(signers[1], 130)
    # node messages that are not well-formed PROPAGATEs (validateNodeMsg, node.py:1492-1498)
    nodemsgs += [("prop_missing_request", {"op": "PROPAGATE", "senderClient": "c1"}),
                 ("prop_missing_sender", {"op": "PROPAGATE", "request": good}),
                 ("prop_sender_none", {"op": "PROPAGATE", "request": good, "senderClient": None}),
                 ("prop_sender_int", {"op": "PROPAGATE", "request": good, "senderClient": 5}),
                 ("prop_sender_empty", {"op": "PROPAGATE", "request": good, "senderClient": ""}),
                 ("prop_sender_long", {"op": "PROPAGATE", "request": good, "senderClient": "x" * 300}),
                 ("prop_request_list", {"op": "PROPAGATE", "request": [1, 2], "senderClient": "c1"}),
                 ("prop_extra_field", {"op": "PROPAGATE", "request": good, "senderClient": "c1", "extra": 1}),
                 ("prop_unknown_op", {"op": "PROPAGATEX", "request": good, "senderClient": "c1"}),
                 ("prop_missing_op", {"request": good, "senderClient": "c1"}),
                 ("prop_none_op", {"op": None, "request": good, "senderClient": "c1"}),
                 ("prop_unhashable_op", {"op": {"a": 1}, "request": good, "senderClient": "c1"}),
                 ("node_prepare", {"op": "PREPARE", "instId": 0, "viewNo": 0, "ppSeqNo": 1, "ppTime": 1,
                                   "digest": "d", "stateRootHash": None, "txnRootHash": None}),
                 ("node_not_a_dict", [1, 2])]
    for j, (label, pm) in enumerate(nodemsgs):
        frm = ["Node2", "Node3:9702", "Node4"][j % 3]
        node.events.clear()
        try:
            node.handleOneNodeMsg((json.loads(json.dumps(pm)), frm))
            raised = None
        except Exception as ex:
            raised = {"exc": type(ex).__name__, "msg": str(ex)}
        props.append({"label": label, "msg": pm, "frm": frm, "events": list(node.events), "raised": raised})
    from plenum.common.messages.node_message_factory import node_message_factory
    registry = {k: repr(v) for k, v in node_message_factory._MessageFactory__classes.items()}
    return {"clients": clients, "client_quota": client, "propagates": props, "node_message_registry": registry}


GENERATORS = {"serializer.json": lambda: gen_serializer(), "didverifier.json": lambda: gen_didverifier(),
              "authn.json": lambda: gen_authn(), "reqauth.json": lambda: gen_reqauth(),
              "verdicts.json": lambda: gen_verdicts(), "request.json": lambda: gen_request(),
              "feed.json": lambda: gen_feed()}

if __name__ == "__main__":
    for name in sys.argv[1:] or list(GENERATORS):
        dump(name, GENERATORS[name]())
