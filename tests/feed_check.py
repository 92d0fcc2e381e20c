"""Shared checks of plenum_amd.feed against tests/golden/feed.json (the reference node's own
handleOneClientMsg / handleOneNodeMsg run on the same messages by tests/golden/make_golden.py).
TEST INFRASTRUCTURE: used by test_feed_host.py (C oracle as the engine) and test_gpu_feed.py (HIP)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


# client messages whose op is Batch / LedgerStatus / CatchupReq, and node messages of other ops
CLIENT_OP_LABELS = ("op_ledger_status", "op_ledger_status_bad", "op_catchup_req", "op_batch")
NODE_OTHER_OP_LABELS = ("node_prepare",)


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
        if c["label"] in CLIENT_OP_LABELS:
            # Batch / LedgerStatus / CatchupReq: the node's own validateClientMsg branch handles them
            # (the reference accepted or NACKed them there); the adapter hands them back untouched
            assert isinstance(o, feed.NotARequest), (c["label"], o)
            assert o.msg == wrapped[cases.index(c)][0] and o.frm == c["frm"]
            continue
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
    assert len(out) == len(cases)
    for c, o in zip(cases, out):
        assert c["raised"] is None
        ev = c["events"][0]
        if c["label"] in NODE_OTHER_OP_LABELS:
            # a registered op other than PROPAGATE: the node's own handleOneNodeMsg takes it
            assert isinstance(o, feed.NotAPropagate), (c["label"], o)
            continue
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


def check_registry():
    """The restated op registry equals the reference's node_message_factory classes (names and reprs)."""
    from plenum_amd.node_messages import TYPES
    reg = load()["node_message_registry"]
    assert {k: repr(v) for k, v in TYPES.items()} == reg
