"""TEST-ONLY stub (the transport is out of scope; imported transitively by the reference)."""
class _Any:
    def __getattr__(self, name):
        return _Any()
    def __call__(self, *a, **k):
        return _Any()
def __getattr__(name):
    return _Any()
