"""GPU parity of the ingress batch path (plenum_amd.wire.authenticate_wire_batch):
for received JSON requests it must return exactly what the reference's per-request ingress returns,
    req = Request(**json.loads(raw)); req_authnr.authenticate(req.as_dict, key=req.key)
(plenum/server/node.py:1643, 2636-2650) — same identifier sets, same exception classes and
messages, same verified-request cache — on every kind of request the authenticator meets. The
sequential side runs the drop-in classes (golden-pinned against the reference in
test_host_logic.py) one request at a time."""
import json

import numpy as np
import pytest

from oracle.base58_ref import b58encode as ref_b58encode
from plenum_amd.client_authn import CoreAuthNr
from plenum_amd.req_authenticator import ReqAuthenticator
from plenum_amd.state_utils import DictState
from plenum_amd.wire import Request, authenticate_wire_batch, signing_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from plenum_amd import _native
    _native.ensure_device()
    return _native


class Signer:
    def __init__(self, sodium, seed, cryptonym=False):
        self.pk, self.sk = sodium.seed_keypair(seed)
        self.sodium = sodium
        if cryptonym:
            self.did, self.verkey = ref_b58encode(self.pk).decode(), None
        else:
            self.did = ref_b58encode(self.pk[:16]).decode()
            self.verkey = "~" + ref_b58encode(self.pk[16:]).decode()

    def sign(self, doc):
        return ref_b58encode(self.sodium.sign_detached(signing_bytes(Request(**doc)), self.sk)).decode()


def make_ra(clients, state_nyms):
    core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=DictState(state_nyms))
    for s in clients:
        core.addIdr(s.did, s.verkey)
    ra = ReqAuthenticator()
    ra.register_authenticator(core)
    return ra


def sequential(ra, raws):
    out = []
    for raw in raws:
        msg = None
        try:
            msg = json.loads(raw.decode())
            req = Request(**msg)
            out.append((msg, ra.authenticate(req.as_dict, req.key)))
        except Exception as ex:
            out.append((msg, ex))
    return out


def norm(result):
    msg, r = result
    if isinstance(r, Exception):
        return msg, ("exc", type(r).__name__, str(r))
    return msg, ("ok", sorted(r))


def nym(i, dest=None, verkey=None):
    op = {"type": "1", "dest": dest or "Xx%dYyZz" % i, "alias": "u%08d" % i}
    if verkey:
        op["verkey"] = verkey
    return op


def corpus(sodium):
    rng = np.random.default_rng(9)
    S = [Signer(sodium, rng.bytes(32)) for _ in range(6)] + [Signer(sodium, rng.bytes(32), cryptonym=True)]
    clients, in_state, self_nym = S[:3] + [S[6]], S[3:5], S[5]
    state = {s.did: {"verkey": s.verkey} for s in in_state}
    docs = []

    def single(signer, i, **extra):
        d = {"identifier": signer.did, "reqId": 1000 + i, "protocolVersion": 2, "operation": nym(i)}
        d.update(extra)
        d["signature"] = signer.sign(d)
        return d

    for i, s in enumerate(clients + in_state):
        docs.append(single(s, i))                                     # valid, fast path
    d = single(S[0], 20)
    d["operation"]["alias"] = "changed"                               # message altered after signing
    docs.append(d)
    d = single(S[1], 21)
    d["signature"] = d["signature"][:-1] + "0"                        # not base58
    docs.append(d)
    d = single(S[1], 22)
    d["signature"] = d["signature"] + " \t"                           # trailing whitespace: still valid
    docs.append(d)
    d = single(S[2], 23)
    d["signature"] = ref_b58encode(b"\0" + bytes(63)).decode()        # decodes, verifies False
    docs.append(d)
    d = {"identifier": self_nym.did, "reqId": 24, "operation": nym(24, dest=self_nym.did, verkey=self_nym.verkey)}
    d["signature"] = self_nym.sign(d)                                 # unknown DID creating itself
    docs.append(d)
    d = {"identifier": "UnknownDid1111111111", "reqId": 25, "operation": nym(25)}
    d["signature"] = S[0].sign(d)                                     # no verkey anywhere
    docs.append(d)
    multi = {"reqId": 26, "operation": nym(26), "protocolVersion": 2}
    multi["signatures"] = {s.did: s.sign(multi) for s in (S[0], S[3], S[6])}
    docs.append(multi)                                                # three endorsers, all valid
    bad_multi = {"reqId": 27, "operation": nym(27)}
    sigs = {s.did: s.sign(bad_multi) for s in (S[1], S[2], S[4])}
    sigs[S[2].did] = sigs[S[1].did]                                   # one wrong signature
    bad_multi["signatures"] = sigs
    docs.append(bad_multi)
    docs.append({"identifier": S[0].did, "reqId": 28, "operation": {"type": "105", "dest": "x"}, "signature": "z"})
    docs.append(single(S[0], 29, operation={"type": "999"}))          # no authenticator for the type
    docs.append({"identifier": S[0].did, "reqId": 30, "operation": nym(30)})  # no signature at all
    docs.append(single(S[1], 31, operation={"type": "action", "x": [1, None, True]}))
    docs.append(single(S[2], 32, operation={"type": "101", "ratio": 0.25, "n": 1e3}))  # floats: Python path
    docs.append(single(S[3], 33, endorser=S[0].did, taaAcceptance={"taaDigest": "ab", "time": 1, "mechanism": "m"}))
    docs.append({"identifier": "", "reqId": 34, "operation": nym(34), "signatures": {}})
    docs.append(single(S[0], 35, fees=[[1, 2]], extraField="ignored by Request"))
    raws = [json.dumps(d).encode() for d in docs]
    raws.append(raws[0])                                              # same request again: cache hit
    raws.append(json.dumps(dict(docs[1], signature=docs[2]["signature"])).encode())  # cached key, new sig
    raws += [b'{"identifier": "x", "reqId": 1,', b"[1, 2]", b'"text"', b'{"reqId": 1, "operation": null}']
    return raws, clients, state


def test_wire_batch_matches_sequential(native, sodium):
    raws, clients, state = corpus(sodium)
    ra_seq, ra_wire = make_ra(clients, state), make_ra(clients, state)
    want = [norm(r) for r in sequential(ra_seq, raws)]
    timings = {}
    got = [norm(r) for r in authenticate_wire_batch(ra_wire, raws, timings=timings)]
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, raws[i][:120], g[1], w[1])
    assert ra_wire._verified_reqs == ra_seq._verified_reqs
    kinds = {w[1][0] for w in want}
    assert kinds == {"ok", "exc"} and sum(w[1][0] == "ok" for w in want) >= 10
    assert timings["verifications"] >= 10 and timings["slow"] >= 5


def test_wire_batch_many_valid_requests(native, sodium):
    """4,096 requests from 64 signers (every verification on the fast path) + every 97th altered."""
    rng = np.random.default_rng(12)
    signers = [Signer(sodium, rng.bytes(32)) for _ in range(64)]
    ra = make_ra(signers, {})
    raws, altered = [], []
    for i in range(4096):
        s = signers[i % 64]
        d = {"identifier": s.did, "reqId": 5000 + i, "protocolVersion": 2, "operation": nym(i)}
        d["signature"] = s.sign(d)
        if i % 97 == 5:
            d["reqId"] += 1
        altered.append(i % 97 == 5)
        raws.append(json.dumps(d).encode())
    timings = {}
    res = authenticate_wire_batch(ra, raws, timings=timings)
    for (msg, r), a, i in zip(res, altered, range(len(raws))):
        if a:
            assert type(r).__name__ == "InsufficientCorrectSignatures", (i, r)
        else:
            assert r == {signers[i % 64].did}, (i, r)
    assert timings["slow"] == sum(altered)
    assert len(ra._verified_reqs) == len(raws) - sum(altered)


def check_request_dependent_verkeys(sodium):
    """A DID with no registry or state record creating itself: its verkey comes from each
    request's own operation (NYM self-verkey rule), so it must not be shared across the batch —
    the same DID sends NYMs carrying its right key, another signer's key, and no key; a state DID
    signs many requests (one state read per batch)."""
    rng = np.random.default_rng(21)
    me, other, st = (Signer(sodium, rng.bytes(32)) for _ in range(3))
    ra_seq, ra_wire = make_ra([], {st.did: {"verkey": st.verkey}}), make_ra([], {st.did: {"verkey": st.verkey}})
    docs = []
    for i, vk in enumerate([me.verkey, other.verkey, None, me.verkey, other.verkey]):
        d = {"identifier": me.did, "reqId": 100 + i, "operation": nym(100 + i, dest=me.did, verkey=vk)}
        d["signature"] = me.sign(d)
        docs.append(d)
    for i in range(20):
        d = {"identifier": st.did, "reqId": 200 + i, "operation": nym(200 + i)}
        d["signature"] = st.sign(d)
        docs.append(d)
    raws = [json.dumps(x).encode() for x in docs]
    want = [norm(r) for r in sequential(ra_seq, raws)]
    got = [norm(r) for r in authenticate_wire_batch(ra_wire, raws)]
    assert got == want
    assert [w[1][0] for w in want[:5]] == ["ok", "exc", "exc", "ok", "exc"]
    assert ra_wire._verified_reqs == ra_seq._verified_reqs


def test_wire_batch_request_dependent_verkeys(native, sodium):
    check_request_dependent_verkeys(sodium)
