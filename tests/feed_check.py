"""Shared checks of plenum_amd.feed against tests/golden/feed.json (the reference node's own
handleOneClientMsg / handleOneNodeMsg run on the same messages by tests/golden/make_golden.py).
TEST INFRASTRUCTURE: used by test_feed_host.py (C oracle as the engine) and test_gpu_feed.py (HIP)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "golden", "feed.json")) as f:
        return json.load(f)


def authenticator(clients):
    from plenum_amd.client_authn import CoreAuthNr
    from plenum_amd.req_authenticator import ReqAuthenticator
    from plenum_amd.state_utils import DictState
    core = CoreAuthNr(["1", "101"], ["105"], ["action"], state=DictState({}))
    for idr, vk in clients.items():
        core.addIdr(idr, vk)
    ra = ReqAuthenticator()
    ra.register_authenticator(core)
    spy = {"calls": 0}
    orig = ra.authenticate

    def authenticate(req_data, key=None):  # the test_no_reauth.py:11-23 spy
        spy["calls"] += 1
        return orig(req_data, key)
    ra.authenticate = authenticate
    return ra, spy


def check_client_quota(engine=None):
    from plenum_amd import feed
    d = load()
    ra, spy = authenticator(d["clients"])
    cases = d["client_quota"]
    wrapped = [(json.loads(json.dumps(c["msg"])), c["frm"]) for c in cases]
    out = feed.authenticate_client_quota(ra, wrapped, engine=engine)
    assert len(out) == len(cases)
    for c, o in zip(cases, out):
        if c["raised"]:
            assert isinstance(o, feed.ClientError), (c["label"], o)
            assert (type(o.exc).__name__, str(o.exc)) == (c["raised"]["exc"], c["raised"]["msg"]), c["label"]
            continue
        ev = c["events"][0]
        if ev["ev"] == "accepted":
            assert isinstance(o, feed.ClientAccepted), (c["label"], o)
            assert sorted(o.identifiers) == c["ids"], c["label"]
            assert o.frm == c["frm"]
        else:
            assert ev["ev"] == "nack"
            assert isinstance(o, feed.ClientNack), (c["label"], o)
            assert (o.frm, o.identifier, o.req_id, o.reason) == (ev["frm"], ev["identifier"], ev["reqId"],
                                                                 ev["reason"]), c["label"]
    # one authenticate() call per request that reached the signature check, as the reference
    assert spy["calls"] == sum(c["authenticate_calls"] for c in cases)


def check_propagates(engine=None):
    from plenum_amd import feed
    d = load()
    ra, spy = authenticator(d["clients"])
    cases = d["propagates"]
    wrapped = [(json.loads(json.dumps(c["msg"])), c["frm"]) for c in cases]
    out = feed.authenticate_propagates(ra, wrapped, engine=engine)
    for c, o in zip(cases, out):
        assert c["raised"] is None
        ev = c["events"][0]
        if ev["ev"] == "accepted":
            assert isinstance(o, feed.PropagateAccepted), (c["label"], o)
            assert o.frm == c["frm"]
        elif ev["ev"] == "suspicious_node":
            assert isinstance(o, feed.SuspiciousNode), (c["label"], o)
            assert (o.node, o.code, o.reason) == (ev["node"], ev["code"], ev["reason"]), c["label"]
            assert (type(o.__cause__).__name__, str(o.__cause__)) == (ev["cause"], ev["cause_str"]), c["label"]
            assert repr(o) == "Error code: {}. {}".format(ev["code"], ev["reason"])
        else:
            assert ev["ev"] == "discard"
            assert isinstance(o, feed.PropagateDiscarded), (c["label"], o)
            assert (type(o.exc).__name__, str(o.exc)) == (ev["exc"], ev["reason"]), c["label"]
