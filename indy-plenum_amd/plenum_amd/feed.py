"""The node's authentication feed points, batched.

The reference verifies one signature per message, as each message is dispatched:

  client stack  ZStack.processReceived (stp_zmq/zstack.py:606-646) hands the node up to one quota of
                messages per prod (100 client messages, stp_core/config.py:32). Each goes through
                Node.handleOneClientMsg (plenum/server/node.py:1557-1572) -> validateClientMsg
                (:1617-1659) -> verifySignature (:2624-2655). Any exception ends in
                handleInvalidClientMsg (:1574-1591): a NACK to `frm` for (identifier, reqId) with the
                reason "client request invalid: <friendlyEx(ex)>" (plenum/common/util.py:364-381).
  node stack    the messages of a node Batch (node.py:1518-1527) go through handleOneNodeMsg
                (:1456-1476) -> validateNodeMsg (:1479-1505) -> verifySignature, which for a
                PROPAGATE authenticates Request(**msg.request) (:2634-2650). A BaseExc becomes
                SuspiciousNode(frm, ex, message) (:1500-1503), reported by the caller (:1472-1473);
                any other exception discards the message (:1474-1476).

Here a whole quota / batch is authenticated in ONE engine launch (ReqAuthenticator.authenticate_batch:
every signature of every request planned, verified together, then the unchanged per-request
authenticate() answering from those verdicts, once per request as test_no_reauth.py:11-23 spies).
The functions return one outcome per message, in order, with the reference's mapping, and leave the
side effects to the caller (sending the NACK, reporting the node, queueing the message):

  authenticate_client_quota(req_authnr, wrapped) -> [ClientAccepted | ClientNack | NotARequest | ClientError]
  authenticate_propagates(req_authnr, wrapped)   -> [PropagateAccepted | SuspiciousNode | PropagateDiscarded]

Static validation of client requests (Node.doStaticValidation, node.py:1651-1652: request handlers,
out of scope here) is the caller's `static_validation(request)` hook, run where the reference runs
it (after the Request is built, before the signature check). A client message carrying "op" is
routed as validateClientMsg routes it (node.py:1634-1638): Batch / LedgerStatus / CatchupReq are
NotARequest (the node's own handler takes them), any other registered op is NACKed with
InvalidClientMsgType(cls, reqId), an unknown op with InvalidNodeOp. A node message goes through
validateNodeMsg's construction step (node.py:1492-1498) with node_messages.MessageFactory: the
registry (MissingNodeOp / InvalidNodeOp) and Propagate's own schema (missing fields, the request
body's type, senderClient), the reference's exception texts wrapped into InvalidNodeMsg as the
node does; the request body's full schema (ClientMessageValidator) is the factory's
`request_schema` hook, or the whole factory is replaced through `message_factory(msg)` (e.g. the
reference's node_message_factory.get_instance). A message of another registered op is
NotAPropagate (the node's own handleOneNodeMsg takes it).
"""
import re
from collections import namedtuple

from .constants import IDENTIFIER, OPERATION, REQ_ID, SIGNATURES
from .exceptions import BaseExc, InvalidClientMsgType, InvalidClientRequest
from .node_messages import CLIENT_OPS, OP_FIELD_NAME, MessageFactory, NodeMessageType, validate_node_message  # noqa: F401
from .wire import Request

PROPAGATE = "PROPAGATE"       # plenum/common/constants.py PROPAGATE
NODE_MESSAGE_FACTORY = MessageFactory()

# a request that passed: what handleOneClientMsg hands to unpackClientMsg (node.py:1566-1567)
ClientAccepted = namedtuple("ClientAccepted", "request frm identifiers")
# what handleInvalidClientMsg sends: send_nack_to_client((identifier, reqId), reason, frm)
ClientNack = namedtuple("ClientNack", "frm identifier req_id reason exc")
# a client message whose 'op' is Batch / LedgerStatus / CatchupReq: not a request, the node's other
# branch of validateClientMsg (node.py:1634-1638) handles it
NotARequest = namedtuple("NotARequest", "msg frm")
# a node message of a registered op other than PROPAGATE: the node's own handleOneNodeMsg takes it
NotAPropagate = namedtuple("NotAPropagate", "msg frm")
# handleOneClientMsg itself raised (a non-dict message: handleInvalidClientMsg's msg.get fails)
ClientError = namedtuple("ClientError", "msg frm exc")
PropagateAccepted = namedtuple("PropagateAccepted", "message frm request identifiers")
PropagateDiscarded = namedtuple("PropagateDiscarded", "message frm exc")


class SuspiciousNode(BaseExc):
    """plenum/common/exceptions.py:166-177: node name without the ':port' suffix, the suspicion's
    code and reason (the signing exception's), the offending message."""

    def __init__(self, node, suspicion, offendingMsg):
        node = node.decode() if isinstance(node, bytes) else node
        self.code = suspicion.code if suspicion else None
        self.reason = suspicion.reason if suspicion else None
        m = re.compile(r'(\b\w+)(:(\d+))?').match(node)
        self.node = m.groups()[0] if m else node
        self.offendingMsg = offendingMsg

    def __repr__(self):
        return "Error code: {}. {}".format(self.code, self.reason)


def friendly_ex(ex):
    """plenum/common/util.py:364-375 friendlyEx: the exception and its __cause__ chain."""
    cur, friendly, end = ex, "", ""
    while cur:
        if len(friendly):
            friendly += " [caused by "
            end += "]"
        friendly += "{}".format(cur)
        cur = cur.__cause__
    return friendly + end


def reason_for_client(ex):
    """plenum/common/util.py:378-381 reasonForClientFromException."""
    return "client request invalid: {}".format(friendly_ex(ex))


def idr_from_req_data(data):
    """plenum/common/txn_util.py:59-63."""
    if data.get(IDENTIFIER):
        return data[IDENTIFIER]
    return Request.gen_idr_from_sigs(data.get(SIGNATURES, {}))


def _client_request(msg, cls, static_validation):
    """Node.validateClientMsg (node.py:1617-1659) up to the signature check: the Request, None for a
    non-request message, or the exception the node raises."""
    if all([msg.get(OPERATION), msg.get(REQ_ID), idr_from_req_data(msg)]):
        need_static = True
    elif OP_FIELD_NAME in msg:
        cls = NODE_MESSAGE_FACTORY.get_type(msg[OP_FIELD_NAME])  # InvalidNodeOp / TypeError propagate
        if cls not in CLIENT_OPS:
            raise InvalidClientMsgType(cls, msg.get(REQ_ID))
        return None
    else:
        raise InvalidClientRequest(msg.get(IDENTIFIER), msg.get(REQ_ID))
    try:
        req = cls(**msg)
    except TypeError as ex:
        raise InvalidClientRequest(msg.get(IDENTIFIER), msg.get(REQ_ID), str(ex))
    except Exception as ex:
        raise InvalidClientRequest(msg.get(IDENTIFIER), msg.get(REQ_ID)) from ex
    if need_static and static_validation is not None:
        static_validation(req)
    return req


def _nack(msg, frm, ex):
    """Node.handleInvalidClientMsg (node.py:1574-1591): the NACK tuple, or the exception it raises."""
    try:
        if isinstance(msg, Request):
            msg = msg.as_dict
        identifier = idr_from_req_data(msg)
        req_id = msg.get(REQ_ID) or 1
    except Exception as ex2:
        ex2.__context__ = ex
        return ClientError(msg, frm, ex2)
    return ClientNack(frm, identifier, req_id, reason_for_client(ex), ex)


def authenticate_client_quota(req_authnr, wrapped, static_validation=None, request_class=Request, engine=None):
    """One ZStack quota of client messages [(msg dict, frm)] -> one outcome per message, all
    signatures in one engine launch. Side effects on req_authnr (the verified-request cache) are the
    sequential ones."""
    outcomes = [None] * len(wrapped)
    todo = []  # (index, request)
    for i, (msg, frm) in enumerate(wrapped):
        try:
            req = _client_request(msg, request_class, static_validation)
        except Exception as ex:
            outcomes[i] = _nack(msg, frm, ex)
            continue
        if req is None:
            outcomes[i] = NotARequest(msg, frm)
        else:
            todo.append((i, req))
    items = []
    for i, req in todo:
        try:
            items.append((req.as_dict, req.key))  # Node.verifySignature (node.py:2641-2647)
        except Exception as ex:
            outcomes[i] = _nack(wrapped[i][0], wrapped[i][1], ex)
            items.append(None)
    live = [(i, req, it) for (i, req), it in zip(todo, items) if it is not None]
    results = req_authnr.authenticate_batch([it for _, _, it in live], engine) if live else []
    for (i, req, _), res in zip(live, results):
        msg, frm = wrapped[i]
        if isinstance(res, Exception):
            outcomes[i] = _nack(msg, frm, res)
        else:
            outcomes[i] = ClientAccepted(req, frm, res)
    return outcomes


def _suspicious(frm, ex, message):
    """`raise SuspiciousNode(frm, ex, message) from ex` (node.py:1502-1503). Building it reads
    ex.code and ex.reason; an exception without them (NoAuthenticatorFound has no reason) makes the
    constructor raise AttributeError instead, which handleOneNodeMsg discards (node.py:1474-1476)."""
    try:
        s = SuspiciousNode(frm, ex, message)
    except Exception as err:
        err.__context__ = ex
        return PropagateDiscarded(message, frm, err)
    s.__cause__ = ex
    return s


def _default_propagate(msg):
    return validate_node_message(NODE_MESSAGE_FACTORY, msg)


def _is_propagate(message):
    if isinstance(message, NodeMessageType):
        return False
    return isinstance(message, dict) or getattr(message, "typename", PROPAGATE) == PROPAGATE


def authenticate_propagates(req_authnr, wrapped, message_factory=_default_propagate, request_class=Request,
                            engine=None):
    """The messages of a node Batch [(msg dict, frm)] -> one outcome per message, all PROPAGATE
    signatures in one engine launch: PropagateAccepted, the SuspiciousNode the node reports,
    PropagateDiscarded with the exception the node discards the message for, or NotAPropagate for a
    message of another registered op."""
    outcomes = [None] * len(wrapped)
    live = []  # (index, message, request, (req_dict, key))
    for i, (msg, frm) in enumerate(wrapped):
        try:
            message = message_factory(msg)
        except Exception as ex:  # validateNodeMsg: InvalidNodeMsg and friends propagate (node.py:1493-1498)
            outcomes[i] = PropagateDiscarded(msg, frm, ex)
            continue
        if not _is_propagate(message):
            outcomes[i] = NotAPropagate(msg, frm)
            continue
        try:
            request = message["request"] if isinstance(message, dict) else message.request
            req = request_class(**request)  # node.py:2636
            item = (req.as_dict, req.key)
        except BaseExc as ex:
            outcomes[i] = _suspicious(frm, ex, message)
            continue
        except Exception as ex:
            outcomes[i] = PropagateDiscarded(message, frm, ex)
            continue
        live.append((i, message, req, item))
    results = req_authnr.authenticate_batch([it for *_, it in live], engine) if live else []
    for (i, message, req, _), res in zip(live, results):
        frm = wrapped[i][1]
        if isinstance(res, BaseExc):
            outcomes[i] = _suspicious(frm, res, message)
        elif isinstance(res, Exception):
            outcomes[i] = PropagateDiscarded(message, frm, res)
        else:
            outcomes[i] = PropagateAccepted(message, frm, req, res)
    return outcomes
