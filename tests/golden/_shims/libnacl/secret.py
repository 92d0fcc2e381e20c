"""TEST-ONLY stub (secret boxes are off the verification path)."""
class SecretBox:
    def __init__(self, key=None):
        raise NotImplementedError("libnacl.secret stub")
