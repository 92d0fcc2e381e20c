"""plenum_amd.feed (SURVEY.md §8f-2 feed points) on the CPU: the reference node's outcomes for a
client quota and a batch of PROPAGATEs (tests/golden/feed.json), with the C oracle standing in for
the engine (one launch per quota / batch). tests/test_gpu_feed.py runs the same on the HIP engine."""
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
