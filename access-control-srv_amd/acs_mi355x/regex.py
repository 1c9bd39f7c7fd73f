r"""Entity namespace / RegExp test of the reference, precomputed on the host.

For a rule entity value ``v_r`` and a request entity value ``v_q`` the
reference (accessController.ts:528-566 and hierarchicalScope.ts:64-101)
computes a namespace-reset bit and a ``new RegExp(lastSegment(v_r))`` match.
Both depend only on the two strings, so they are tabulated once per
(row value, column value) pair and the kernel reads one byte per pair.

JS RegExp semantics are reproduced exactly for literal patterns (substring
search) and for a conservative metacharacter subset, translated to Python ``re``
where the two engines differ (``$`` is end of input in V8 but also matches before
a trailing newline in Python, so it becomes ``\Z``); any other pattern is marked
RX_HOST so the kernel reports the request to the host instead of guessing.  The
subset is pinned against V8 itself: tests/golden/regex_cells.json (written by
tests/golden/gen_regex_cells.js under node) holds ~10k (rule value, request value)
cells and tests/test_regex_v8.py requires every non-host cell to equal V8's.
"""
from __future__ import annotations

import re
import warnings

from .jsops import nullish
from .layout import RX_HIT, RX_RESET, RX_THROW_TYPE, RX_THROW_SYNTAX, RX_HOST

_LITERAL = re.compile(r"^[A-Za-z0-9_\-\s#@%&=,;'\"<>~`!]*$")
_SAFE = re.compile(r"^[A-Za-z0-9_\-*+?|()\[\]^$]*$")


def _split_entity(v: str):
    """(namespace prefix, first dot segment, last dot segment) of an entity URN."""
    c = v.rfind(":")
    prefix = v[:c] if c >= 0 else ""
    segs = v[c + 1:].split(".")
    return prefix, segs[0], segs[-1]


def _to_python(pattern: str) -> str:
    r"""The safe-subset JS pattern as a Python ``re`` pattern with the same matches: an
    unescaped ``$`` outside a character class asserts end of input (V8, no multiline flag)
    -> ``\Z``.  ``[]`` / ``[^]`` (JS: empty / any-char classes) never reach here, so a
    ``]`` inside a class always closes it, in both engines."""
    out, in_class = [], False
    for ch in pattern:
        if in_class:
            in_class = ch != "]"
            out.append(ch)
        elif ch == "[":
            in_class = True
            out.append(ch)
        else:
            out.append(r"\Z" if ch == "$" else ch)
    return "".join(out)


def _regex_hit(pattern: str, subject: str):
    if _LITERAL.match(pattern):
        return RX_HIT if pattern in subject else 0
    if not _SAFE.match(pattern) or "(?" in pattern or "[]" in pattern or "[^]" in pattern:
        return RX_HOST
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # "possible nested set" for '[[' (a literal '[' in both engines)
            rx = re.compile(_to_python(pattern))
    except re.error:
        return RX_THROW_SYNTAX
    return RX_HIT if rx.search(subject) else 0


def cell(rule_value, req_value) -> int:
    """Bits for one (rule entity value, request entity value) pair."""
    if nullish(rule_value) or nullish(req_value):
        return RX_THROW_TYPE  # nsEntityArray[0] / reqNSEntityArray[0] of undefined
    if not (rule_value.isascii() and req_value.isascii()):
        return RX_HOST  # toUpperCase / RegExp over non-ASCII text: the host decides (Unicode-version exact)
    r_prefix, r_first, r_last = _split_entity(rule_value)
    q_prefix, q_first, q_last = _split_entity(req_value)
    bits = RX_RESET if r_prefix != q_prefix else 0
    rule_ns = r_first.upper() if r_first.upper() != r_last.upper() else None
    req_ns = q_first.upper() if q_first.upper() != q_last.upper() else None
    # ''.toUpperCase() is falsy: treat as absent, exactly like the reference's truthiness test
    rule_ns = rule_ns or None
    req_ns = req_ns or None
    if (req_ns and rule_ns and req_ns == rule_ns) or (not req_ns and not rule_ns):
        bits |= _regex_hit(r_last, q_last)
    return bits
