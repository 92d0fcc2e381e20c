class BaseHandler:
    def __init__(self, context=None):
        self.context = context


def register(cls, handler=None, base=False):
    return None
