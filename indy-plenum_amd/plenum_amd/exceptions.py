"""Exception types raised on the request-authentication path.

Same class names, codes, reasons and ``str()`` forms as the reference's
``plenum/common/exceptions.py:16-20`` (ReqInfo), ``:40-47`` (BaseExc, SigningException),
``:50-153`` (the signing exceptions) and ``:161-163`` (InvalidKey), so callers that catch or
format them (node.py handleInvalidClientMsg / SuspiciousNode paths) behave identically.
"""


class ReqInfo:
    def __init__(self, identifier=None, reqId=None):
        self.identifier = identifier
        self.reqId = reqId


class BaseExc(Exception):
    def __str__(self):
        return "{}{}".format(type(self).__name__, self.args)


class SigningException(BaseExc):
    pass


class _ReasonExc:
    """Mixin for exceptions whose str() is their formatted reason."""

    def __str__(self):
        return self.reason


class CouldNotAuthenticate(_ReasonExc, SigningException, ReqInfo):
    code = 110
    reason = 'could not authenticate, verkey for {} cannot be found'

    def __init__(self, identifier, *args, **kwargs):
        self.reason = type(self).reason.format(identifier)
        ReqInfo.__init__(self, *args, **kwargs)


class MissingSignature(SigningException):
    code = 120
    reason = 'missing signature'


class EmptySignature(SigningException, ReqInfo):
    code = 121
    reason = 'empty signature'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidSignatureFormat(SigningException, ReqInfo):
    code = 123
    reason = 'invalid signature format'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidSignature(SigningException, ReqInfo):
    code = 125
    reason = 'invalid signature'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InsufficientSignatures(_ReasonExc, SigningException, ReqInfo):
    code = 126
    reason = 'insufficient signatures, {} provided but {} required'

    def __init__(self, provided, required, *args, **kwargs):
        self.reason = type(self).reason.format(provided, required)
        ReqInfo.__init__(self, *args, **kwargs)


class InsufficientCorrectSignatures(_ReasonExc, SigningException, ReqInfo):
    code = 127
    reason = ('insufficient number of valid signatures, {} is required but {} valid and {} invalid have been '
              'provided. The following signatures are invalid: {}')

    def __init__(self, required_sig_cnt, valid_sig_cnt, invalid_sigs, *args, **kwargs):
        listing = '; '.join('did={}, signature={}'.format(d, s) for d, s in invalid_sigs.items())
        self.reason = type(self).reason.format(required_sig_cnt, valid_sig_cnt, len(invalid_sigs), listing)
        ReqInfo.__init__(self, *args, **kwargs)


class MissingIdentifier(SigningException):
    code = 130
    reason = 'missing identifier'


class EmptyIdentifier(SigningException):
    code = 131
    reason = 'empty identifier'


class UnknownIdentifier(SigningException, ReqInfo):
    code = 133
    reason = 'unknown identifier'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidIdentifier(SigningException, ReqInfo):
    code = 135
    reason = 'invalid identifier'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class UnregisteredIdentifier(SigningException):
    code = 136
    reason = 'provided owner identifier not registered with agent'


class NoAuthenticatorFound(SigningException):
    code = 137


class InvalidKey(Exception):
    code = 142
    reason = 'invalid key'


# plenum/common/exceptions.py:184-235: the message-validation exceptions the feed points raise
class InvalidMessageException(BaseExc):
    pass


class InvalidNodeMessageException(InvalidMessageException):
    pass


class InvalidClientMessageException(InvalidMessageException):
    def __init__(self, identifier, reqId, reason=None, code=None):
        self.code = code
        self.identifier = identifier
        self.reqId = reqId
        self.reason = reason


class InvalidNodeMsg(InvalidNodeMessageException):
    pass


class InvalidClientRequest(InvalidClientMessageException):
    pass



class MissingNodeOp(InvalidNodeMsg):
    pass


class InvalidNodeOp(InvalidNodeMsg):
    pass


class InvalidClientMsgType(InvalidClientRequest):
    pass
