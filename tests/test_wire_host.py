"""CPU tests of the ingress batch path's host logic (plenum_amd.wire.authenticate_wire_batch) and of
the batch-scoped verkey resolver. The device launches are replaced by a checker
that does what pv_ingress_verify / pv_verify_batch compute — base58 decode, DidVerifier key
resolution, crypto_sign_open — with the host base58 mirror and libsodium 1.0.18 (test
infrastructure only); tests/test_gpu_wire.py runs the same corpus through the HIP library."""
import json

import numpy as np
import pytest

from plenum_amd import _native, batch
from plenum_amd.base58 import b58decode
from plenum_amd.client_authn import CoreAuthNr, VerkeyResolver
from plenum_amd.state_utils import DictState
from plenum_amd.verifier import DidVerifier
from test_gpu_wire import Signer, check_request_dependent_verkeys, corpus, make_ra, nym, norm, sequential

from plenum_amd import wire


@pytest.fixture
def cpu_engine(sodium, monkeypatch):
    calls = {"ingress": 0, "sm": 0, "one": 0}

    def ingress(sb, so, mblob, moff, msg_idx, signer_idx, ib, io, vb, vo, vp):
        calls["ingress"] += 1
        n = len(so) - 1
        status, verdict = np.zeros(n, np.uint8), np.zeros(n, bool)
        for j in range(n):
            sig = bytes(sb[int(so[j]):int(so[j + 1])])
            s, m = int(signer_idx[j]), int(msg_idx[j])
            idr = bytes(ib[int(io[s]):int(io[s + 1])]).decode()
            vk = bytes(vb[int(vo[s]):int(vo[s + 1])]).decode() if vp[s] else None
            try:
                raw_sig = b58decode(sig)
                pk = DidVerifier(vk, identifier=idr).raw_key
            except Exception:
                status[j] = 1
                continue
            msg = bytes(mblob[int(moff[m]):int(moff[m + 1])])
            verdict[j] = sodium.sign_open_ok(raw_sig + msg, pk)
        return status, verdict

    def sm_batch(blob, off, pks):
        calls["sm"] += 1
        return np.array([sodium.sign_open_ok(bytes(blob[int(off[i]):int(off[i + 1])]), bytes(pks[i]))
                         for i in range(len(off) - 1)], bool)

    monkeypatch.setattr(_native, "ingress_verify_arrays", ingress)
    monkeypatch.setattr(_native, "verify_sm_batch", sm_batch)
    # the unbatched per-call path (batch.verdict without a batch context) of the sequential reference
    def one(pk, sm):
        calls["one"] += 1
        return bool(sodium.sign_open_ok(bytes(sm), bytes(pk)))

    monkeypatch.setattr(_native, "verify_one", one)
    return calls


def test_wire_batch_matches_sequential_cpu(cpu_engine, sodium):
    raws, clients, state = corpus(sodium)
    ra_seq, ra_wire = make_ra(clients, state), make_ra(clients, state)
    want = [norm(r) for r in sequential(ra_seq, raws)]
    timings = {}
    got = [norm(r) for r in wire.authenticate_wire_batch(ra_wire, raws, timings=timings)]
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, raws[i][:120], g[1], w[1])
    assert ra_wire._verified_reqs == ra_seq._verified_reqs
    assert timings["verifications"] >= 10 and timings["slow"] >= 5
    assert cpu_engine["ingress"] == 1


def test_wire_batch_edge_requests_cpu(cpu_engine, sodium):
    """JSON the fast view must hand to Request(**msg) itself, unhashable txn types, non-str
    identifiers, and a batch whose requests repeat a key."""
    rng = np.random.default_rng(3)
    s = Signer(sodium, rng.bytes(32))
    ra_seq, ra_wire = make_ra([s], {}), make_ra([s], {})
    docs = []
    d = {"identifier": s.did, "reqId": 1, "operation": nym(1)}
    d["signature"] = s.sign(d)
    docs.append(d)
    docs.append(dict(d, self=1))                                          # Request(**msg) raises TypeError
    docs.append(dict(d, operation={"type": ["1"]}))                       # unhashable type
    docs.append(dict(d, operation={"type": {"a": 1}}))
    docs.append(dict(d, identifier=[s.did]))                              # non-str identifier
    docs.append(dict(d, identifier=7))
    docs.append({"reqId": 2, "operation": nym(2), "signatures": {s.did: 5}})  # non-str signature
    docs.append(dict(d, protocolVersion=None, endorser=None, taaAcceptance=None))
    raws = [json.dumps(x).encode() for x in docs] + [json.dumps(docs[0]).encode()] * 3
    want = [norm(r) for r in sequential(ra_seq, raws)]
    got = [norm(r) for r in wire.authenticate_wire_batch(ra_wire, raws)]
    assert got == want
    assert ra_wire._verified_reqs == ra_seq._verified_reqs


def test_wire_batch_request_dependent_verkeys_cpu(cpu_engine, sodium):
    check_request_dependent_verkeys(sodium)


def test_request_view_matches_request_as_dict():
    docs = [{"identifier": "a", "reqId": 1, "operation": {"type": "1"}, "signature": "s"},
            {"reqId": 1, "operation": None, "signatures": {"a": "x"}, "protocolVersion": 2, "endorser": "e",
             "taaAcceptance": {"t": 1}, "fees": [1], "extra": 3},
            {"taaAcceptance": 0, "protocolVersion": 0, "identifier": "", "signature": ""},
            {}]
    for d in docs:
        v = wire._request_view(d)
        r = wire.Request(**d).as_dict
        assert v == r and list(v) == list(r)
    assert wire._request_view([1]) is None and wire._request_view({"self": 1}) is None


def test_verkey_resolver_reads_each_did_once():
    """VerkeyResolver.get == getVerkey for registry DIDs, state DIDs, self-creating NYMs, DIDs with
    no key anywhere, and a state without `get` (getVerkey raises -> LookupError)."""
    class CountingState(DictState):
        reads = 0

        def get(self, key, isCommitted=True):
            CountingState.reads += 1
            return super().get(key, isCommitted)

    st = CountingState({"StateDid": {"verkey": "~abc"}, "NoKey": {"role": "0"}})
    core = CoreAuthNr(["1"], [], [], state=st)
    core.addIdr("Client", "~xyz")
    reqs = [{"identifier": "Self", "reqId": i, "operation": {"type": "1", "dest": "Self", "verkey": "~v%d" % i}}
            for i in range(3)]
    reqs.append({"identifier": "Other", "reqId": 9, "operation": {"type": "1", "dest": "Nobody"}})
    res = VerkeyResolver(core)
    for _ in range(4):
        for idr in ("Client", "StateDid", "NoKey", "Self", "Other"):
            for r in reqs:
                assert res.get(idr, r) == core.getVerkey(idr, r)
    CountingState.reads = 0
    res = VerkeyResolver(core)
    for _ in range(10):
        for r in reqs:
            res.get("StateDid", r)
            res.get("Self", r)
    assert CountingState.reads == 2 and res.reads == 2
    broken = CoreAuthNr(["1"], [], [], state=None)
    with pytest.raises(AttributeError):
        broken.getVerkey("x", reqs[0])
    with pytest.raises(LookupError):
        VerkeyResolver(broken).get("x", reqs[0])


def test_config1_sequential_and_wire_batch_agree(cpu_engine, sodium):
    """BASELINE configs[0]: 10k signed NYM requests (the bench template, 1,024 signers) through the
    per-request path (json.loads -> Request -> ReqAuthenticator.authenticate, one crypto_sign_open
    per signature) and through authenticate_wire_batch: every request accepted with its signer's
    DID, identical results and verified-request caches; one engine launch for the batch."""
    import nym_workload
    from plenum_amd import batch
    from plenum_amd.req_authenticator import ReqAuthenticator
    k = 10000
    _, _, _, wblob, woff, _, _ = nym_workload.generate_wire(0, k)
    pool = nym_workload._pool()

    def make():
        core = CoreAuthNr(["1"], ["105"], [], state=None)
        for p in pool:
            core.addIdr(p["did"], p["abbr"])
        ra = ReqAuthenticator()
        ra.register_authenticator(core)
        return ra

    raws = [wblob[int(woff[i]):int(woff[i + 1])].tobytes() for i in range(k)]
    ra_seq, ra_wire = make(), make()
    with batch.active(batch.VerdictCache()):
        want = sequential(ra_seq, raws)
    assert all(r == {pool[i % len(pool)]["did"]} for i, (_, r) in enumerate(want))
    # one unbatched verify per signature (batch.verdict -> _native.verify_one), no array launch
    assert cpu_engine["one"] == k and cpu_engine["sm"] == 0 and cpu_engine["ingress"] == 0
    got = wire.authenticate_wire_batch(ra_wire, raws)
    assert [norm(r) for r in got] == [norm(r) for r in want]
    assert ra_wire._verified_reqs == ra_seq._verified_reqs
    assert cpu_engine["ingress"] == 1 and cpu_engine["sm"] == 0 and cpu_engine["one"] == k


@pytest.mark.parametrize("raw", [b'{"a": 1}', b' {"a": 1}', b'{"a": 1} ', b'{"a": 1}\n', b'\xef\xbb\xbf{"a": 1}',
                                 b'{"a": NaN, "b": -Infinity}', b'[1, 2]', b'"text"', b'12', b'12 34', b'{"a": 1}{}',
                                 b'{"a": "\\u00e9\\ud83d\\ude00"}', b'{"a": "\x01"}', b'\xff\xfe', b'', b'   ',
                                 b'{"a": 1,}', b'{"a": [' * 3 + b']}' * 3, '{"é": 1}'.encode()])
def test_loads_matches_json_loads(raw):
    """wire._loads is json.loads(raw.decode()): same object or same exception class and message."""
    def outcome(fn):
        try:
            return ("ok", fn(raw))
        except Exception as ex:
            return ("exc", type(ex).__name__, str(ex))
    a = outcome(wire._loads)
    b = outcome(lambda r: json.loads(r.decode()))
    if a[0] == "ok" and b[0] == "ok":
        assert json.dumps(a[1]) == json.dumps(b[1])
    else:
        assert a == b


def test_wire_batch_one_call_per_request_cpu(cpu_engine, sodium, monkeypatch):
    """one_call_per_request=True: the reference's call pattern (ReqAuthenticator.authenticate ->
    CoreAuthNr.authenticate once per request that is not a verified-cache hit; test_no_reauth's
    spy), identical results, every signature check in one launch."""
    raws, clients, state = corpus(sodium)
    ra_seq, ra_wire = make_ra(clients, state), make_ra(clients, state)
    counts = {"seq": 0, "wire": 0}

    def spy(ra, tag):
        core = ra._authenticators[0]
        orig = core.authenticate

        def counted(*a, **kw):
            counts[tag] += 1
            return orig(*a, **kw)
        core.authenticate = counted

    spy(ra_seq, "seq")
    spy(ra_wire, "wire")
    want = [norm(r) for r in sequential(ra_seq, raws)]
    cpu_engine["sm"] = 0
    answered = []
    orig_answer = batch.answer

    def answer_spy(authnr, req_data):
        a = orig_answer(authnr, req_data)
        answered.append(a is not None)
        return a
    monkeypatch.setattr(batch, "answer", answer_spy)
    got = [norm(r) for r in wire.authenticate_wire_batch(ra_wire, raws, one_call_per_request=True)]
    assert got == want
    assert ra_wire._verified_reqs == ra_seq._verified_reqs
    assert counts["wire"] == counts["seq"] > 10
    assert cpu_engine["sm"] == 1  # the plan's one launch; nothing verified one by one
    # device-finished requests were answered from the plan inside the one authenticate call
    assert sum(answered) > 10 and not all(answered)


def test_c_finisher_matches_python_finish(cpu_engine, sodium):
    """_fastcall.finish_single (the C finish of device-verified single-signature requests) leaves
    the same results and verified-request cache as the Python finish: new keys, a key repeated in
    the batch, keys already cached with the same signature (the cached identifier set is returned)
    and with another signature (overwritten), and a second pass over the whole batch."""
    import nym_workload
    fc = _native._fastcall()
    if not fc or not hasattr(fc, "finish_single"):
        pytest.skip("_fastcall not built (make -C indy-plenum_amd)")
    k = 3000
    _, _, _, wblob, woff, _, _ = nym_workload.generate_wire(0, k)
    pool = nym_workload._pool()
    raws = [wblob[int(woff[i]):int(woff[i + 1])].tobytes() for i in range(k)]
    raws[10] = raws[5]   # a key repeated inside the batch
    raws[2000] = raws[7]

    def make():
        core = CoreAuthNr(["1"], ["105"], [], state=None)
        for p in pool:
            core.addIdr(p["did"], p["abbr"])
        from plenum_amd.req_authenticator import ReqAuthenticator
        ra = ReqAuthenticator()
        ra.register_authenticator(core)
        return ra

    def run(use_c):
        calls = []
        with pytest.MonkeyPatch.context() as mp:
            if use_c:
                orig = fc.finish_single
                mp.setattr(fc, "finish_single", lambda *a: (calls.append(a[2:4]), orig(*a))[1])
            else:
                mp.setattr(_native, "_fast", False)
            ra = make()
            first = wire.authenticate_wire_batch(ra, raws[:1500])
            keys = list(ra._verified_reqs)
            ra._verified_reqs[keys[3]] = {"signature": "other", "identifiers": {"x"}}  # overwritten
            cached = ra._verified_reqs[keys[4]]["identifiers"]
            out = wire.authenticate_wire_batch(ra, raws)
            again = wire.authenticate_wire_batch(ra, raws)
        return first, out, again, ra._verified_reqs, out[4][1] is cached, calls

    c = run(True)
    py = run(False)
    assert c[5] and not py[5]
    for a, b in zip(c[:3], py[:3]):
        assert [norm(r) for r in a] == [norm(r) for r in b]
    assert c[3] == py[3] and list(c[3]) == list(py[3])
    assert c[4] and py[4]
    assert all(r == {pool[i % len(pool)]["did"]} for i, (_, r) in enumerate(c[1]) if i not in (10, 2000))
