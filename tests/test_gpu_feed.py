"""GPU: plenum_amd.feed on the HIP engine against the reference node's outcomes
(tests/golden/feed.json): NACK reasons, SuspiciousNode codes / reasons / causes, discards, accepted
identifier sets, and one authenticate() call per request."""
import pytest

from feed_check import check_client_quota, check_propagates

pytestmark = pytest.mark.gpu


def test_client_quota_on_gpu():
    from plenum_amd import _native
    _native.ensure_device()
    check_client_quota()


def test_propagates_on_gpu():
    from plenum_amd import _native
    _native.ensure_device()
    check_propagates()
