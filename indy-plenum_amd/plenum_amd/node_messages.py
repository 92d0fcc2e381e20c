"""The node-message type registry and the PROPAGATE schema check the feed points need
(plenum/common/messages/node_message_factory.py, node_messages.py:109-115, message_base.py:12-75,
fields.py:42-144; restated, not imported: the reference's message classes pull in its whole
messaging stack).

Only what decides the feed points' outcomes is restated:
  * the registry of op names (32 typenames, node_message_factory's classes) -- Node.validateClientMsg
    routes a client message carrying "op" by it (node.py:1634-1638), and validateNodeMsg raises
    MissingNodeOp / InvalidNodeOp / InvalidNodeMsg from it (node.py:1493-1498);
  * the Propagate message's own schema: the two required fields, the `request` body's type check
    and the senderClient field (LimitedLengthStringField(256, nullable=True)), with the reference's
    error texts. SCHEMA_IS_STRICT is False there (constants.py:282), so unknown fields pass.
The request body's full schema (ClientMessageValidator, client_request.py:181-230) is NOT restated:
it is the `request_schema` hook of MessageFactory (a node binds the reference's own validator;
INTEGRATION.md §2). Messages of any other registered op are not PROPAGATEs: the feed point returns
them for the node's own handler.
"""
from collections.abc import Mapping

from .exceptions import InvalidNodeMsg, InvalidNodeOp, MissingNodeOp

OP_FIELD_NAME = "op"
NODE_MESSAGES_MODULE = "plenum.common.messages.node_messages"
SENDER_CLIENT_FIELD_LIMIT = 256  # plenum/config.py:313

# typename -> class name in plenum.common.messages.node_messages (node_message_factory's registry)
NODE_MESSAGE_CLASSES = {
    "BACKUP_INSTANCE_FAULTY": "BackupInstanceFaulty", "BATCH": "Batch", "BATCH_COMMITTED": "BatchCommitted",
    "BLACKLIST": "BlacklistMsg", "CATCHUP_REP": "CatchupRep", "CATCHUP_REQ": "CatchupReq",
    "CHECKPOINT": "Checkpoint", "COMMIT": "Commit", "CONSISTENCY_PROOF": "ConsistencyProof",
    "CURRENT_STATE": "CurrentState", "INSTANCE_CHANGE": "InstanceChange", "LEDGER_STATUS": "LedgerStatus",
    "MESSAGE_REQUEST": "MessageReq", "MESSAGE_RESPONSE": "MessageRep", "NEW_VIEW": "NewView",
    "OBSERVED_DATA": "ObservedData", "OLD_VIEW_PREPREPARE_REP": "OldViewPrePrepareReply",
    "OLD_VIEW_PREPREPARE_REQ": "OldViewPrePrepareRequest", "ORDERED": "Ordered",
    "POOL_LEDGER_TXNS": "PoolLedgerTxns", "PREPARE": "Prepare", "PREPREPARE": "PrePrepare",
    "PROPAGATE": "Propagate", "REJECT": "Reject", "REPLY": "Reply", "REQACK": "RequestAck",
    "REQNACK": "RequestNack", "VIEW_CHANGE": "ViewChange", "VIEW_CHANGE_ACK": "ViewChangeAck",
    "VIEW_CHANGE_DONE": "ViewChangeDone", "ViewChangeContinue": "ViewChangeContinueMessage",
    "ViewChangeStart": "ViewChangeStartMessage",
}


class NodeMessageType:
    """Stands for a message class of the registry; repr() is the class's own
    ("<class 'plenum.common.messages.node_messages.Propagate'>"), which is what
    InvalidClientMsgType(cls, reqId) prints."""

    def __init__(self, typename, name):
        self.typename, self.__name__ = typename, name

    def __repr__(self):
        return "<class '{}.{}'>".format(NODE_MESSAGES_MODULE, self.__name__)


TYPES = {op: NodeMessageType(op, name) for op, name in NODE_MESSAGE_CLASSES.items()}
BATCH, LEDGER_STATUS, CATCHUP_REQ, PROPAGATE = (TYPES[k] for k in ("BATCH", "LEDGER_STATUS", "CATCHUP_REQ",
                                                                   "PROPAGATE"))
CLIENT_OPS = (BATCH, LEDGER_STATUS, CATCHUP_REQ)  # validateClientMsg's non-request messages


def _sender_client_error(val):
    """LimitedLengthStringField(max_length=256, nullable=True).validate (fields.py:54-144)."""
    if val is None:
        return None
    if not isinstance(val, str):
        return "expected types 'str', got '{}'".format(type(val).__name__)
    if not val:
        return "empty string"
    if len(val) > SENDER_CLIENT_FIELD_LIMIT:
        val = val[:100] + ("..." if len(val) > 100 else "")
        return "{} is longer than {} symbols".format(val, SENDER_CLIENT_FIELD_LIMIT)
    return None


class MessageFactory:
    """node_message_factory, restricted to what the feed points decide: get_type() over the
    registry, get_instance() building a PROPAGATE (its schema check) and returning any other
    registered message's type unbuilt (the node's own handler validates those)."""

    def __init__(self, request_schema=None):
        self.request_schema = request_schema  # ClientMessageValidator(...).validate, or None

    def get_type(self, message_op):
        message_cls = TYPES.get(message_op, None)  # an unhashable op raises TypeError, as dict.get does
        if message_cls is None:
            raise InvalidNodeOp(message_op)
        return message_cls

    def get_instance(self, **message_raw):
        message_op = message_raw.get(OP_FIELD_NAME, None)
        if message_op is None:
            raise MissingNodeOp
        cls = self.get_type(message_op)
        msg = {k: v for k, v in message_raw.items() if k != OP_FIELD_NAME}
        if cls is not PROPAGATE:
            return cls
        self._validate_propagate(msg)
        return msg

    def _validate_propagate(self, dct):
        """MessageValidator._validate_fields_with_schema (message_base.py:26-43) for Propagate's
        schema ((request, ClientMessageValidator), (senderClient, LimitedLengthStringField))."""
        prefix = "validation error [Propagate]:"
        missed = set(("request", "senderClient")) - set(dct)
        if missed:
            raise TypeError("{} missed fields - {}. ".format(prefix, ', '.join(map(str, missed))))
        for k, v in dct.items():
            if k == "request":
                if not isinstance(v, dict):
                    raise TypeError("validation error [ClientMessageValidator]: invalid type {}, dict expected"
                                    .format(type(v)))
                if self.request_schema is not None:
                    self.request_schema(v)
            elif k == "senderClient":
                err = _sender_client_error(v)
                if err:
                    raise TypeError("{} {} ({}={})".format(prefix, err, k, v))


def validate_node_message(factory, msg):
    """Node.validateNodeMsg's construction step (node.py:1492-1498): the factory's exceptions, with
    everything but MissingNodeOp / InvalidNodeOp wrapped into InvalidNodeMsg(str(ex)). A message that
    is not a mapping fails the reference's `get_instance(**msg)` call itself; its TypeError text
    names the reference's function."""
    if not isinstance(msg, Mapping):
        raise InvalidNodeMsg("plenum.common.messages.node_message_factory.MessageFactory.get_instance() "
                             "argument after ** must be a mapping, not {}".format(type(msg).__name__))
    try:
        return factory.get_instance(**msg)
    except (MissingNodeOp, InvalidNodeOp) as ex:
        raise ex
    except Exception as ex:
        raise InvalidNodeMsg(str(ex))
