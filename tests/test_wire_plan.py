"""CPU tests of pv_wire_plan (the fused C++ ingress planner behind plenum_amd.wire.authenticate_wire_packed):
for every request its plan must be what the reference's Python planning gives for
Request(**json.loads(text)).as_dict — CoreAuthMixin._select_signatures (plenum/server/client_authn.py:
240-264), operation["type"] — or PV_PLAN_PY (the Python path decides); its signing message, digest and
status must be pv_signing_serialize_json's. The batch-level results are checked against the sequential
path with the host checker engine (test_wire_host.py's cpu_engine)."""
import json

import numpy as np
import pytest

from plenum_amd import wire
from plenum_amd.client_authn import CoreAuthNr
from test_gpu_wire import Signer, make_ra, nym, norm, sequential
from test_wire_host import cpu_engine  # noqa: F401  (fixture)


def _docs():
    d = {"identifier": "Did1111", "reqId": 1, "operation": {"type": "1", "dest": "x"}, "signature": "Sig1111"}
    m = {"reqId": 2, "operation": {"type": "1"}, "signatures": {"DidB": "SigB", "DidA": "SigA"}}
    return [
        d,                                                              # SINGLE
        m,                                                              # MULTI, dict order kept
        dict(d, identifier=""),                                         # no identifier: signatures absent -> PY
        dict(m, identifier="DidZ"),                                     # identifier but no signature: MULTI
        dict(m, identifier="DidZ", signature=""),                       # falsy non-None signature: PY
        dict(d, signatures={"DidQ": "SigQ"}),                           # signature wins: SINGLE
        dict(d, signature="Sig 1111"),                                  # space inside: PY
        dict(d, signature="Sig1111 "),                                  # trailing whitespace: PY
        dict(d, identifier="Dïd"),                                      # non-ASCII: PY
        dict(d, identifier=7),                                          # non-str identifier: PY
        dict(d, operation={"type": 1}),                                 # non-str type: PY
        dict(d, operation={"type": "1", "x": 0.5}),                     # float: serializer defers -> PY
        dict(d, operation=["1"]),                                       # operation not a dict: PY
        dict(d, self=1),                                                # Request(**msg) raises: PY
        dict(m, signatures={}),                                         # empty signatures: PY
        dict(m, signatures={"DidA": 5}),                                # non-str signature value: PY
        {"reqId": 3, "operation": {"type": "1"}},                       # no signature at all: PY
        dict(d, operation={"type": "été"}),                   # non-ASCII type: SINGLE, decoded
        dict(d, protocolVersion=2, taaAcceptance={"a": 1}, endorser="E", fees=[1]),
    ]


def _texts():
    texts = [json.dumps(x).encode() for x in _docs()]
    texts += [b'{"identifier": "A", "identifier": "B", "reqId": 1, "operation": {"type": "1"}, "signature": "S"}',
              b'{"reqId": 1, "operation": {"type": "1"}, "signatures": {"A": "x", "A": "y"}}',   # dup names: PY
              b'{"identifier": "A\\u0042", "reqId": 1, "operation": {"type": "1"}, "signature": "S"}',  # escapes
              b'[1]', b'{"a": 1,}', b'', b'{"identifier": "A", "reqId": 1, "operation": {"type": "1"}, "signature": "S"} ']
    return texts


def _expect(text):
    """(kind, [(identifier, signature)], type) from the reference's Python planning."""
    try:
        msg = json.loads(text.decode())
        view = wire.Request(**msg).as_dict
        core = CoreAuthNr([], [], [])
        sigmap = core._select_signatures(view, None, None)
    except Exception:
        return None
    return view, sigmap


def test_plan_matches_python_selection():
    texts = _texts()
    blob, off = wire._native._blob(texts)
    P = wire.WirePlan(blob, off, threads=3)
    st, mb, mo, dg = wire.signing_serialize_packed(blob, off, wire.PV_SER_REQUEST, 3)
    assert np.array_equal(P.status, st) and np.array_equal(P.digests, dg)
    assert np.array_equal(P.moff, mo) and bytes(P.msg[:int(mo[-1])]) == bytes(mb[:int(mo[-1])])
    kinds = P.kind.tolist()
    sigs = P.signatures()
    assert len(sigs) == P.n_pairs
    assert sigs == [bytes(P.sig_blob[int(P.sig_off[p]):int(P.sig_off[p + 1])]).decode() for p in range(P.n_pairs)]
    assert P.keys() == [bytes(x).hex() for x in P.digests]
    for i, text in enumerate(texts):
        k = kinds[i]
        if k == wire.PV_PLAN_PY:
            continue
        exp = _expect(text)
        assert exp is not None, (i, text)
        view, sigmap = exp
        lo, hi = int(P.pair_off[i]), int(P.pair_off[i + 1])
        pairs = [(P.names[int(P.pair_name[p])], sigs[p]) for p in range(lo, hi)]
        assert pairs == list(sigmap.items()), (i, text)
        assert P.types[int(P.type_id[i])] == view["operation"]["type"]
        if k == wire.PV_PLAN_SINGLE:
            assert pairs == [(view["identifier"], view["signature"])]
        else:
            assert view.get("signature") is None
    want = [1, 2, 0, 2, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 0, 1]
    assert kinds == want
    assert P.names[int(P.pair_name[int(P.pair_off[19])])] == "B"   # the last duplicate wins
    assert P.names[int(P.pair_name[int(P.pair_off[21])])] == "AB"  # escapes decoded


def test_plan_many_threads_dedups_names_and_types():
    rng = np.random.default_rng(4)
    texts = []
    for i in range(3000):
        d = {"identifier": "Did%d" % rng.integers(0, 50), "reqId": i, "operation": {"type": str(rng.integers(0, 3))},
             "signature": "S%d" % i}
        if i % 7 == 0:
            d = {"reqId": i, "operation": {"type": "1"}, "signatures": {"Did%d" % j: "S%d_%d" % (i, j) for j in range(3)}}
        texts.append(json.dumps(d).encode())
    blob, off = wire._native._blob(texts)
    P1, P8 = wire.WirePlan(blob, off, threads=1), wire.WirePlan(blob, off, threads=8)
    for P in (P1, P8):
        assert len(set(P.names)) == len(P.names) and len(set(P.types)) == len(P.types)
        sigs = P.signatures()
        got = [[(P.names[int(P.pair_name[p])], sigs[p]) for p in range(int(P.pair_off[i]), int(P.pair_off[i + 1]))]
               for i in range(len(texts))]
        assert P.keys() == [bytes(x).hex() for x in P.digests]
        want = [list(_expect(t)[1].items()) for t in texts]
        assert got == want
        assert [P.types[int(t)] for t in P.type_id] == [json.loads(t)["operation"]["type"] for t in texts]
    assert P1.names == P8.names  # first-appearance order, whatever the thread split


def test_packed_results_and_lazy_messages(cpu_engine, sodium):  # noqa: F811
    rng = np.random.default_rng(5)
    signers = [Signer(sodium, rng.bytes(32)) for _ in range(8)]
    docs = []
    for i in range(300):
        s = signers[i % 8]
        d = {"identifier": s.did, "reqId": 10 + i, "operation": nym(i)}
        d["signature"] = s.sign(d)
        if i % 37 == 3:
            d["reqId"] += 1  # altered after signing
        docs.append(d)
    raws = [json.dumps(d).encode() for d in docs]
    raws += raws[:5]  # repeated requests: cache hits inside the batch
    ra_seq, ra_wire = make_ra(signers, {}), make_ra(signers, {})
    want = [norm(r) for r in sequential(ra_seq, raws)]
    blob, off = wire._native._blob(raws)
    res = wire.authenticate_wire_packed(ra_wire, blob, off, threads=4)
    assert len(res) == len(raws)
    assert [norm(res[i]) for i in range(len(res))] == want
    assert ra_wire._verified_reqs == ra_seq._verified_reqs
    assert list(ra_wire._verified_reqs) == list(ra_seq._verified_reqs)  # insertion order too
    assert [m for m, _ in res] == [json.loads(r) for r in raws]
    # a second batch of the same requests: every one is a cache hit
    res2 = wire.authenticate_wire_packed(ra_wire, blob, off, threads=4)
    want2 = [norm(r) for r in sequential(ra_seq, raws)]
    assert [norm(x) for x in res2] == want2
    assert ra_wire._verified_reqs == ra_seq._verified_reqs


@pytest.mark.parametrize("n", [0, 1])
def test_plan_tiny_batches(n):
    texts = [json.dumps({"identifier": "A", "reqId": 1, "operation": {"type": "1"}, "signature": "S"}).encode()] * n
    blob, off = wire._native._blob(texts)
    P = wire.WirePlan(blob, off)
    assert P.n == n and P.n_pairs == n and len(P.kind) == n
