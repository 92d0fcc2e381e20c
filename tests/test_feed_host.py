"""plenum_amd.feed (SURVEY.md §8f-2 feed points) on the CPU: the reference node's outcomes for a
client quota and a batch of PROPAGATEs (tests/golden/feed.json), with the C oracle standing in for
the engine (one launch per quota / batch). tests/test_gpu_feed.py runs the same on the HIP engine."""
import feed_check
from feed_check import check_client_quota, check_propagates
from test_host_logic import CountingEngine


def test_client_quota_matches_reference(oracle):
    eng = CountingEngine(oracle)
    check_client_quota(engine=eng)
    assert eng.launches == 1


def test_propagates_match_reference(oracle):
    eng = CountingEngine(oracle)
    check_propagates(engine=eng)
    assert eng.launches == 1


def test_node_message_registry_matches_reference():
    feed_check.check_registry()


def test_client_op_routing():
    """validateClientMsg's second branch on its own (node.py:1634-1638): the three non-request ops
    come back as NotARequest, other registered ops are InvalidClientMsgType NACKs, unknown or
    unhashable ops NACK with InvalidNodeOp / TypeError -- no engine launch for any of them."""
    from plenum_amd import feed
    ra, spy = feed_check.authenticator({})
    msgs = [({"op": "BATCH", "messages": []}, "c"), ({"op": "REPLY", "reqId": 3}, "c"), ({"op": 7}, "c"),
            ({"op": ["l"]}, "c")]
    out = feed.authenticate_client_quota(ra, msgs, engine=lambda *a: (_ for _ in ()).throw(AssertionError))
    assert isinstance(out[0], feed.NotARequest)
    assert out[1].reason == ("client request invalid: InvalidClientMsgType(<class "
                             "'plenum.common.messages.node_messages.Reply'>, 3)") and out[1].req_id == 3
    assert out[2].reason == "client request invalid: InvalidNodeOp(7,)"
    assert out[3].reason == "client request invalid: unhashable type: 'list'"
    assert spy["calls"] == 0
