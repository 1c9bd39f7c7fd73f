"""JS value-semantics helpers for the CPU oracle (TEST INFRASTRUCTURE ONLY).

The reference (restorecommerce/access-control-srv, TypeScript on Node) manipulates
plain JSON-shaped objects.  The oracle models them as Python values:

    JS undefined      -> UNDEF (also: a missing dict key)
    JS null           -> None
    JS string/number  -> str / int / float
    JS boolean        -> bool
    JS array / object -> list / dict

Only the operators the decision path actually uses are restated here:
strict (===) and loose (==) equality, truthiness, lodash ``isEmpty``/``find``
(matchesProperty form), optional chaining and ``String.prototype`` helpers.
Nothing in this module may be imported by the product package.
"""
from __future__ import annotations

import math
import re


class _Undefined:
    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def __repr__(self):
        return "undefined"

    def __bool__(self):
        return False


UNDEF = _Undefined()


class JSError(Exception):
    """A JS exception that would reject the reference's promise."""

    kind = "Error"


class JSTypeError(JSError):
    kind = "TypeError"


class JSSyntaxError(JSError):
    kind = "SyntaxError"


class InvalidCombiningAlgorithm(JSError):
    """reference: src/core/errors.ts:15-20, thrown by decide (accessController.ts:837)."""

    kind = "InvalidCombiningAlgorithm"


class OracleUnsupported(Exception):
    """Input outside what the oracle restates exactly (e.g. a non-trivial JS regex)."""


def nullish(v) -> bool:
    return v is UNDEF or v is None


def is_num(v) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def truthy(v) -> bool:
    if v is UNDEF or v is None or v is False:
        return False
    if v is True:
        return True
    if is_num(v):
        return not (v == 0 or (isinstance(v, float) and math.isnan(v)))
    if isinstance(v, str):
        return len(v) > 0
    return True  # objects, arrays, functions


def strict_eq(a, b) -> bool:
    """JS ``===``."""
    if a is UNDEF or b is UNDEF:
        return a is b
    if a is None or b is None:
        return a is b
    if isinstance(a, bool) or isinstance(b, bool):
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    if is_num(a) or is_num(b):
        return is_num(a) and is_num(b) and a == b
    if isinstance(a, str) or isinstance(b, str):
        return isinstance(a, str) and isinstance(b, str) and a == b
    return a is b


def _to_number(v):
    if is_num(v):
        return float(v)
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, str):
        s = v.strip()
        if s == "":
            return 0.0
        try:
            if s.lower().startswith("0x"):
                return float(int(s, 16))
            return float(s)
        except ValueError:
            return float("nan")
    raise OracleUnsupported("ToNumber on object")


def loose_eq(a, b) -> bool:
    """JS ``==`` for the primitive cases the decision path meets."""
    if nullish(a) or nullish(b):
        return nullish(a) and nullish(b)
    if isinstance(a, (list, dict)) or isinstance(b, (list, dict)):
        if isinstance(a, (list, dict)) and isinstance(b, (list, dict)):
            return a is b
        raise OracleUnsupported("loose == between object and primitive")
    if type(a) is type(b) or (is_num(a) and is_num(b)):
        return strict_eq(a, b)
    return _to_number(a) == _to_number(b)


def same_value_zero(a, b) -> bool:
    """``Array.prototype.includes`` comparison."""
    if is_num(a) and is_num(b) and math.isnan(a) and math.isnan(b):
        return True
    return strict_eq(a, b)


def js_includes(arr, v) -> bool:
    return any(same_value_zero(x, v) for x in arr)


def get(obj, key):
    """``obj?.key``: UNDEF when obj is nullish or the key is absent."""
    if nullish(obj):
        return UNDEF
    if isinstance(obj, dict):
        return obj.get(key, UNDEF)
    if isinstance(obj, list):
        if key == "length":
            return len(obj)
        if isinstance(key, int):
            return obj[key] if 0 <= key < len(obj) else UNDEF
        return UNDEF
    if isinstance(obj, str):
        if key == "length":
            return len(obj)
        return UNDEF
    return UNDEF


def prop(obj, key):
    """``obj.key`` without optional chaining: TypeError on nullish obj."""
    if nullish(obj):
        raise JSTypeError(f"Cannot read properties of {obj!r} (reading '{key}')")
    return get(obj, key)


def iterate(v):
    """``for (const x of v)``: TypeError when v is not iterable."""
    if isinstance(v, list):
        return list(v)
    if isinstance(v, str):
        return list(v)
    raise JSTypeError(f"{v!r} is not iterable")


def or_empty(v):
    """``v || []``"""
    return v if truthy(v) else []


def length_gt0(v) -> bool:
    """``v?.length > 0``"""
    n = get(v, "length")
    if n is UNDEF or n is None:
        return False
    return n > 0


def lodash_is_empty(v) -> bool:
    """lodash ``isEmpty`` for JSON values."""
    if nullish(v):
        return True
    if isinstance(v, (list, str)):
        return len(v) == 0
    if isinstance(v, dict):
        return len(v) == 0
    return True  # numbers, booleans


def _lodash_get_path(obj, path):
    cur = obj
    for k in path.split("."):
        if nullish(cur):
            return UNDEF
        cur = get(cur, k)
    return cur


def _lodash_has_in(obj, path):
    cur = obj
    for k in path.split("."):
        if nullish(cur) or not isinstance(cur, dict) or k not in cur:
            return False
        cur = cur[k]
    return True


def _lodash_base_is_equal(a, b):
    if is_num(a) and is_num(b) and math.isnan(a) and math.isnan(b):
        return True
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_lodash_base_is_equal(a[k], b[k]) for k in a)
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(_lodash_base_is_equal(x, y) for x, y in zip(a, b))
    return strict_eq(a, b)


def lodash_find_matches_property(coll, path, src_value):
    """lodash ``_.find(coll, [path, srcValue])`` (baseMatchesProperty)."""
    items = coll if isinstance(coll, list) else (list(coll.values()) if isinstance(coll, dict) else [])
    for obj in items:
        ov = _lodash_get_path(obj, path)
        if ov is UNDEF and src_value is UNDEF:
            if _lodash_has_in(obj, path):
                return obj
            continue
        if _lodash_base_is_equal(src_value, ov):
            return obj
    return UNDEF


# --- String.prototype helpers (on JS strings only; callers guard nullish) ---

def js_str(v) -> str:
    """``String(v)`` coercion for indexOf arguments."""
    if v is UNDEF:
        return "undefined"
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if is_num(v):
        if isinstance(v, float) and v.is_integer():
            return str(int(v))
        return str(v)
    if isinstance(v, str):
        return v
    raise OracleUnsupported("String() of object")


def last_index_of(s: str, ch: str) -> int:
    return s.rfind(ch)


def substring(s: str, start: int, end: int | None = None) -> str:
    n = len(s)
    start = min(max(start, 0), n)
    if end is None:
        end = n
    end = min(max(end, 0), n)
    if start > end:
        start, end = end, start
    return s[start:end]


def opt_method(v, name, *args):
    """``v?.name(...args)`` for string methods: UNDEF on nullish receiver."""
    if nullish(v):
        return UNDEF
    if not isinstance(v, str):
        raise OracleUnsupported(f"string method {name} on non-string")
    if name == "lastIndexOf":
        return last_index_of(v, args[0])
    if name == "substring":
        return substring(v, *args)
    if name == "split":
        return v.split(args[0])
    if name == "toUpperCase":
        return v.upper()
    if name == "indexOf":
        return v.find(js_str(args[0]))
    raise OracleUnsupported(name)


# A JS RegExp literal pattern that behaves identically under Python ``re``.
_SIMPLE_LITERAL = re.compile(r"^[A-Za-z0-9_\-\s#@%&=,;'\"<>~`!]*$")
_SAFE_REGEX = re.compile(r"^[A-Za-z0-9_\-*+?|()\[\]^$]*$")


def _v8_dollar(pattern: str) -> str:
    """V8's ``$`` (no multiline flag) asserts end of input; Python's ``$`` also matches
    before a trailing newline.  Outside character classes it becomes ``\\Z``."""
    out, in_class = [], False
    for ch in pattern:
        if in_class:
            in_class = ch != "]"
            out.append(ch)
        elif ch == "[":
            in_class = True
            out.append(ch)
        else:
            out.append("\\Z" if ch == "$" else ch)
    return "".join(out)


def js_regex_search(pattern: str, subject: str) -> bool:
    """``subject.match(new RegExp(pattern)) != null`` for patterns in a safe subset.

    Raises JSSyntaxError where V8 rejects the pattern; OracleUnsupported when
    the oracle cannot guarantee V8-identical semantics.  Pinned against V8 by
    tests/golden/regex_cells.json (tests/golden/gen_regex_cells.js, run under node).
    """
    if _SIMPLE_LITERAL.match(pattern):
        return pattern in subject
    if not _SAFE_REGEX.match(pattern) or "(?" in pattern or "[]" in pattern or "[^]" in pattern:
        raise OracleUnsupported(f"regex pattern outside the restated subset: {pattern!r}")
    try:
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            rx = re.compile(_v8_dollar(pattern))
    except re.error as e:  # V8 rejects the same malformed forms in this subset
        raise JSSyntaxError(f"Invalid regular expression: /{pattern}/: {e}")
    return rx.search(subject) is not None
