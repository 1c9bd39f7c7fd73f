"""JS value semantics needed by the host compiler / encoder.

Policy stores and requests arrive as JSON-shaped Python values (the form
``JSON.parse`` gives the reference after ``unmarshallContext``): ``None`` is
JS null and a missing key is JS undefined (``MISSING``).  The compiler and the
encoder evaluate every request-only or rule-only sub-expression of the
reference on the host with these helpers; only request x rule work runs on
the GPU.
"""
from __future__ import annotations


class _Missing:
    __slots__ = ()

    def __repr__(self):
        return "undefined"

    def __bool__(self):
        return False


MISSING = _Missing()


class Unsupported(Exception):
    """Input shape outside what the packed evaluator encodes (routed to the host)."""


def nullish(v):
    return v is MISSING or v is None


def get(obj, key):
    """``obj?.[key]``"""
    if isinstance(obj, dict):
        return obj.get(key, MISSING)
    if isinstance(obj, list) and isinstance(key, int):
        return obj[key] if 0 <= key < len(obj) else MISSING
    return MISSING


def truthy(v):
    if v is MISSING or v is None or v is False:
        return False
    if isinstance(v, bool):
        return True
    if isinstance(v, (int, float)):
        return v == v and v != 0
    if isinstance(v, str):
        return v != ""
    return True


def strict_eq(a, b):
    if a is MISSING or b is MISSING or a is None or b is None:
        return a is b
    if isinstance(a, bool) or isinstance(b, bool):
        return type(a) is type(b) and a == b
    if isinstance(a, str) or isinstance(b, str):
        return isinstance(a, str) and isinstance(b, str) and a == b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return a == b
    return a is b


def loose_eq_nullish(a, b):
    """``a == b`` for string-or-nullish operands."""
    if nullish(a) or nullish(b):
        return nullish(a) and nullish(b)
    return strict_eq(a, b)


def is_empty(v):
    """lodash ``isEmpty`` for JSON values."""
    if nullish(v):
        return True
    if isinstance(v, (list, str, dict)):
        return len(v) == 0
    return True


def or_list(v):
    """``v || []`` where v must be an array when truthy."""
    if not truthy(v):
        return []
    if not isinstance(v, list):
        raise Unsupported("non-array list value")
    return v


def _path_get(obj, path):
    cur = obj
    for k in path:
        if not isinstance(cur, dict):
            return MISSING
        cur = cur.get(k, MISSING)
    return cur


def _path_has(obj, path):
    cur = obj
    for k in path:
        if not isinstance(cur, dict) or k not in cur:
            return False
        cur = cur[k]
    return True


def find_by(coll, path, value):
    """lodash ``_.find(coll, [path, value])`` for primitive ``value``."""
    if isinstance(value, (dict, list)):
        raise Unsupported("object-valued lookup key")
    keys = path.split(".")
    for obj in coll:
        ov = _path_get(obj, keys)
        if ov is MISSING and value is MISSING:
            if _path_has(obj, keys):
                return obj
            continue
        if isinstance(ov, (dict, list)):
            continue
        if strict_eq(ov, value) or (isinstance(ov, float) and ov != ov and isinstance(value, float) and value != value):
            return obj
    return MISSING


def check_scalar(v):
    """Attribute ids / values must be strings or nullish for exact id equality."""
    if v is MISSING or v is None or isinstance(v, str):
        return v
    raise Unsupported(f"non-string attribute scalar {v!r}")


OBJECT_PROTO_KEYS = frozenset([
    "constructor", "__proto__", "toString", "toLocaleString", "valueOf", "hasOwnProperty",
    "isPrototypeOf", "propertyIsEnumerable", "__defineGetter__", "__defineSetter__",
    "__lookupGetter__", "__lookupSetter__"])
