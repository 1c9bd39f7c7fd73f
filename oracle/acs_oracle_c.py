"""ctypes wrapper of the C++ oracle (oracle/acs_oracle.cpp) — TEST INFRASTRUCTURE ONLY.

The multi-threaded C++ restatement of the reference's isAllowed, used by the tests
(against the golden vectors and the Python oracle), by ``bench.py``'s
``cpu_baseline`` leg (timed on the host cores) and as the full-batch checker of the
GPU results.  The product package never imports it.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "acs_oracle.cpp")
LIB = os.path.join(HERE, "lib", "libacs_oracle.so")

DECISIONS = {2: "PERMIT", 3: "DENY", 4: "NOT_APPLICABLE", 5: "INDETERMINATE", 6: "UNRECOGNIZED"}
EC = {0: "undefined", 1: None, 2: False, 3: True}
ERR_KINDS = {1: "TypeError", 2: "InvalidCombiningAlgorithm", 3: "SyntaxError"}


def build(force=False):
    """g++ -O2 build of the oracle (skipped when the .so is newer than the source)."""
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-Wall", "-o", LIB + ".tmp", SRC],
                       check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB):
            build()
        _LIB = C.CDLL(LIB)
        _LIB.acs_oracle_create.restype = C.c_void_p
        _LIB.acs_oracle_create.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
        _LIB.acs_oracle_free.argtypes = [C.c_void_p]
        _LIB.acs_oracle_is_allowed.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int, C.c_void_p,
                                               C.POINTER(C.c_double)]
        _LIB.acs_oracle_is_allowed_shared.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_int,
                                                      C.c_void_p, C.POINTER(C.c_double)]
        _LIB.acs_oracle_what_is_allowed_shared.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_int,
                                                           C.POINTER(C.c_void_p), C.POINTER(C.c_double)]
        _LIB.acs_oracle_free_text.argtypes = [C.c_void_p]
        _LIB.acs_oracle_free_text.restype = None
        _LIB.acs_oracle_last_error.restype = C.c_char_p
        _LIB.acs_oracle_regex_cell.argtypes = [C.c_char_p, C.c_char_p]
    return _LIB


def _json(v):
    from .acs_oracle import _to_json
    try:  # plain JSON values (no UNDEF inside): serialised directly (a 1M-rule store: seconds)
        return json.dumps(v, separators=(",", ":")).encode()
    except TypeError:
        return json.dumps(_to_json(v), separators=(",", ":")).encode()


class COracle:
    """isAllowed / whatIsAllowed of the reference on one policy store, evaluated by the C++
    restatement."""

    def __init__(self, urns: dict, combining_algorithms: list, doc: dict):
        self.h = lib().acs_oracle_create(_json(urns), _json(combining_algorithms), _json(doc))
        if not self.h:
            raise RuntimeError(f"acs_oracle_create: {lib().acs_oracle_last_error().decode()}")

    def close(self):
        if self.h:
            lib().acs_oracle_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def raw(self, requests, threads=1, shared=None):
        """(int32 [n, 4] outcome records, evaluation seconds): kind (0 ok, 1 rejects, 2
        unsupported), decision code, evaluation_cacheable code, status / error kind.
        ``shared``: values that {"$shared": k} objects inside the requests stand for (parsed
        once; see SynthBatch.decode(i, shared=...))."""
        n = len(requests)
        out = np.zeros((n, 4), np.int32)
        sec = C.c_double(0.0)
        text = b"[" + b",".join(_json(r) for r in requests) + b"]"
        stext = None if shared is None else b"[" + b",".join(_json(v) for v in shared) + b"]"
        rc = lib().acs_oracle_is_allowed_shared(self.h, stext, text, n, int(threads), out.ctypes.data,
                                                C.byref(sec))
        if rc != 0:
            raise RuntimeError(f"acs_oracle_is_allowed: {lib().acs_oracle_last_error().decode()}")
        return out, sec.value

    def what_is_allowed(self, requests, threads=1, shared=None):
        """(results, evaluation seconds) of whatIsAllowed (accessController.ts:326-427) per
        request: {"k": 0, "s": [set idx], "p": [policy idx], "r": [rule idx], "o": [[entity,
        mask], ...]} (global node indices of the compiled image; the maskedProperty pushes in
        order, undefined as {"$undef": 1}), {"k": 1, "e": kind} (the reference rejects) or
        {"k": 2} (outside the restatement)."""
        n = len(requests)
        text = b"[" + b",".join(_json(r) for r in requests) + b"]"
        stext = None if shared is None else b"[" + b",".join(_json(v) for v in shared) + b"]"
        out = C.c_void_p()
        sec = C.c_double(0.0)
        rc = lib().acs_oracle_what_is_allowed_shared(self.h, stext, text, n, int(threads), C.byref(out), C.byref(sec))
        if rc != 0:
            raise RuntimeError(f"acs_oracle_what_is_allowed: {lib().acs_oracle_last_error().decode()}")
        try:
            res = json.loads(C.string_at(out.value).decode("utf-8", "surrogatepass"))
        finally:
            lib().acs_oracle_free_text(out)
        return res, sec.value

    def outcomes(self, requests, threads=1):
        """Normalised outcomes as tests/diff_utils.oracle_outcome builds them:
        ('OK', decision, ec, status) / ('ERR', kind) / ('UNSUPPORTED',)."""
        out, _ = self.raw(requests, threads)
        return [outcome(r) for r in out]


def regex_cell(rule_value, req_value) -> int:
    """One entity namespace / RegExp step of the C++ oracle (None = null): bits as in
    tests/golden/regex_cells.json, -1 when the pattern is outside its restated subset."""
    enc = (lambda v: None if v is None else v.encode())
    return int(lib().acs_oracle_regex_cell(enc(rule_value), enc(req_value)))


def outcome(r):
    kind, dec, ec, code = (int(x) for x in r)
    if kind == 1:
        return ("ERR", ERR_KINDS.get(code, "Error"))
    if kind == 2:
        return ("UNSUPPORTED",)
    return ("OK", DECISIONS[dec], EC.get(ec, "other"), code)
