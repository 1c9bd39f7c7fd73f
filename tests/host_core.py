"""TEST INFRASTRUCTURE: drive the evaluator core on the CPU (tests/native/libacs_core_host.so)
over the same packed tables / batches the GPU kernels consume."""
import ctypes as C
import os

import numpy as np

from acs_mi355x import layout as L
from acs_mi355x.build import build_host_core
from acs_mi355x.compiler import store_blob
from acs_mi355x.native import ReqBatchC, ShardC, batch_struct, host_struct

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build_host_core())
        vp = C.c_void_p
        _LIB.acs_host_is_allowed.argtypes = [vp, C.c_size_t, C.POINTER(ReqBatchC), vp]
        _LIB.acs_host_what_is_allowed.argtypes = [vp, C.c_size_t, C.POINTER(ReqBatchC), vp, vp, vp, vp]
        _LIB.acs_host_shard_keys.argtypes = [vp, C.c_size_t, vp, C.c_size_t, C.POINTER(ShardC), vp]
        _LIB.acs_host_shard_decode.argtypes = [vp, C.c_size_t, vp]
        _LIB.acs_host_shard_decode.restype = None
        _LIB.acs_host_what_is_allowed_obl.argtypes = [vp, C.c_size_t, C.POINTER(ReqBatchC), vp, C.c_size_t,
                                                      C.c_uint32, C.c_uint32, vp, vp]
    return _LIB


def shard_keys(cs, dec, base):
    """Local decision records -> rule-sharded reduction keys (int64 view of the u64 keys)."""
    blob = store_blob(cs)
    dec = np.ascontiguousarray(dec)
    keys = np.zeros(len(dec), np.int64)
    s = ShardC(*base)
    assert lib().acs_host_shard_keys(blob, len(blob), dec.ctypes.data, len(dec), C.byref(s), keys.ctypes.data) == 0
    return keys


def shard_decode(keys):
    keys = np.ascontiguousarray(keys, np.int64)
    out = np.zeros(len(keys), L.DECISION_DT)
    lib().acs_host_shard_decode(keys.ctypes.data, len(keys), out.ctypes.data)
    return out


def _struct(batch, compact):
    """compact: the batch's compact form (a CodecBatch's own view; a RequestBatch's lines +
    extension records), else its SoA rows (+ lines)."""
    return host_struct(batch, True) if compact else batch_struct(batch)


def is_allowed(cs, batch, compact=False):
    blob = store_blob(cs)
    out = np.zeros(batch.n, L.DECISION_DT)
    s = _struct(batch, compact)
    assert lib().acs_host_is_allowed(blob, len(blob), C.byref(s), out.ctypes.data) == 0
    return out


def what_is_allowed(cs, batch, compact=False):
    from acs_mi355x.results import bits_layout
    blob = store_blob(cs)
    words = bits_layout(cs.n_sets, cs.n_pols, cs.n_rules)[2]
    n = batch.n
    bits = np.zeros((n, max(words, 1)), np.uint32)
    obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
    obl_n = np.zeros(n, np.uint32)
    out = np.zeros(n, L.DECISION_DT)
    s = _struct(batch, compact)
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
        from acs_mi355x.results import bits_layout
        h = np.frombuffer(self.blob[:64], np.uint32)
        words = max(bits_layout(int(h[2]), int(h[3]), int(h[4]))[2], 1)
        n = batch.n
        bits = np.zeros((n, words), np.uint32)
        obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
        obl_n = np.zeros(n, np.uint32)
        out = np.zeros(n, L.DECISION_DT)
        self._call(lib().acs_host_what_is_allowed, batch, bits, obl, obl_n, out)
        return bits, obl, obl_n, out

    def what_is_allowed_obl(self, batch, idx, cap, chunks=8):
        idx = np.ascontiguousarray(idx, np.uint32)
        obl = np.zeros((chunks, len(idx), cap, 2), np.uint32)
        obl_n = np.zeros((chunks, len(idx)), np.uint32)
        if len(idx):
            s = batch_struct(batch)
            assert lib().acs_host_what_is_allowed_obl(self.blob, len(self.blob), C.byref(s), idx.ctypes.data, len(idx),
                                                      chunks, cap, obl.ctypes.data, obl_n.ctypes.data) == 0
        return obl, obl_n

    def resolve_overflow(self, batch, out, cap=1024, chunks=8):
        from acs_mi355x.native import resolve_overflow
        return resolve_overflow(self, batch, out, cap, chunks)

    def close(self):
        pass
