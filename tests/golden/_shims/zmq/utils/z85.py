"""TEST-ONLY stub (CurveZMQ key encoding, off path)."""
def encode(data):
    raise NotImplementedError


def decode(data):
    raise NotImplementedError
