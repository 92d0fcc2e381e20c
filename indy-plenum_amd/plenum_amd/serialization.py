"""Signing serialization of request dicts — produces the message M that every signer signs.

Behaviour of the reference's ``SigningSerializer.serialize`` /
``serialize_msg_for_signing`` (common/serializers/signing_serializer.py:35-92,
common/serializers/serialization.py:27-36), including its known ambiguity for nested dicts
(INDY-1469, common/test/test_signing_serializer.py:41-140 — nested keys are NOT prefixed with the
parent path), which must be preserved for signature compatibility:
  str -> itself; dict -> sorted keys, "k:v" joined by "|" (top-level ignore list applied at
  level 0 only); other iterables -> items joined by ","; None -> ""; anything else -> str(obj);
  a value outside (str, int, float, list, dict, None) -> Exception("invalid type found ...").
"""
from collections.abc import Iterable

_ACCEPTED = (str, int, float, list, dict, type(None))


def _raise(msg, exc_type=Exception):
    raise exc_type(msg)


class SigningSerializer:
    def serialize(self, obj, level=0, objname=None, topLevelKeysToIgnore=None, toBytes=True):
        text = self._render(obj, level, objname, topLevelKeysToIgnore)
        return text.encode('utf-8') if toBytes else text

    def _render(self, obj, level, objname, ignore):
        if not isinstance(obj, _ACCEPTED):
            _raise("invalid type found {}: {}".format(objname, obj))
        if isinstance(obj, str):
            return obj
        if isinstance(obj, dict):
            if level > 0:
                keys = list(obj.keys())
            else:
                skip = ignore or []
                keys = [k for k in obj.keys() if k not in skip]
            keys.sort()
            parts = []
            for k in keys:
                child = ".".join([str(objname), str(k)]) if objname else k
                parts.append(str(k) + ":" + self._render(obj[k], level + 1, child, None))
            return "|".join(parts)
        if isinstance(obj, Iterable):
            return ",".join(self._render(item, level + 1, objname, None) for item in obj)
        if obj is None:
            return ""
        return str(obj)


signing_serializer = SigningSerializer()


def serialize_msg_for_signing(msg, topLevelKeysToIgnore=None):
    """UTF-8 bytes of ``msg`` in signing form (serialization.py:27-36)."""
    return signing_serializer.serialize(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)
