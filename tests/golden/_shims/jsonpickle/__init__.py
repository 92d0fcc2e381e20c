"""TEST-ONLY stub for importing the reference (plenum/common/jsonpickle_util.py; off the hot path)."""
from . import tags, unpickler, handlers  # noqa


def encode(o, *a, **k):
    raise NotImplementedError("jsonpickle stub")


def decode(s, *a, **k):
    raise NotImplementedError("jsonpickle stub")
