"""TEST INFRASTRUCTURE: drive the evaluator core on the CPU (tests/native/libacs_core_host.so)
over the same packed tables / batches the GPU kernels consume."""
import ctypes as C
import os

import numpy as np

from acs_mi355x import layout as L
from acs_mi355x.build import build_host_core
from acs_mi355x.compiler import store_blob
from acs_mi355x.native import ReqBatchC, batch_struct

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build_host_core())
        vp = C.c_void_p
        _LIB.acs_host_is_allowed.argtypes = [vp, C.c_size_t, C.POINTER(ReqBatchC), vp]
        _LIB.acs_host_what_is_allowed.argtypes = [vp, C.c_size_t, C.POINTER(ReqBatchC), vp, vp, vp, vp]
    return _LIB


def is_allowed(cs, batch):
    blob = store_blob(cs)
    out = np.zeros(batch.n, L.DECISION_DT)
    s = batch_struct(batch)
    assert lib().acs_host_is_allowed(blob, len(blob), C.byref(s), out.ctypes.data) == 0
    return out


def what_is_allowed(cs, batch):
    blob = store_blob(cs)
    words = (cs.n_sets + cs.n_pols + cs.n_rules + 31) // 32
    n = batch.n
    bits = np.zeros((n, max(words, 1)), np.uint32)
    obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
    obl_n = np.zeros(n, np.uint32)
    out = np.zeros(n, L.DECISION_DT)
    s = batch_struct(batch)
    assert lib().acs_host_what_is_allowed(blob, len(blob), C.byref(s), bits.ctypes.data, obl.ctypes.data,
                                          obl_n.ctypes.data, out.ctypes.data) == 0
    return bits, obl, obl_n, out


class Tables:
    """Same interface as acs_mi355x.native.Tables, backed by the CPU build of the core
    (lets host-side logic such as the AccessController mirror be tested without a GPU)."""

    def __init__(self, blob: bytes):
        self.blob = bytes(blob)

    def _call(self, fn, batch, *bufs):
        s = batch_struct(batch)
        assert fn(self.blob, len(self.blob), C.byref(s), *[b.ctypes.data for b in bufs]) == 0

    def is_allowed(self, batch):
        out = np.zeros(batch.n, L.DECISION_DT)
        self._call(lib().acs_host_is_allowed, batch, out)
        return out

    def what_is_allowed(self, batch):
        h = np.frombuffer(self.blob[:64], np.uint32)
        words = max((int(h[2]) + int(h[3]) + int(h[4]) + 31) // 32, 1)
        n = batch.n
        bits = np.zeros((n, words), np.uint32)
        obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
        obl_n = np.zeros(n, np.uint32)
        out = np.zeros(n, L.DECISION_DT)
        self._call(lib().acs_host_what_is_allowed, batch, bits, obl, obl_n, out)
        return bits, obl, obl_n, out

    def close(self):
        pass
