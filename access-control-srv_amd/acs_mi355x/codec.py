"""ctypes binding of the native request codec (include/acs_mi355x.h: acs_codec_*).

JSON request text -> packed batch on host threads (csrc/acs_codec.cpp, the C++ restatement
of encoder.py).  ``NativeCodec(blob).encode(json_bytes)`` returns a ``CodecBatch`` whose
arrays are zero-copy numpy views of the codec's buffers with the attribute names of
encoder.RequestBatch, so native.Tables / device.DeviceBatch / results take either.
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import layout as L
from .jsops import MISSING
from .native import ReqBatchC, last_error, load

_DECLARED = set()


def _lib():
    lib = load()
    if id(lib) not in _DECLARED:
        vp = C.c_void_p
        lib.acs_codec_create.restype = vp
        lib.acs_codec_create.argtypes = [vp, C.c_size_t]
        lib.acs_codec_free.argtypes = [vp]
        lib.acs_codec_free.restype = None
        lib.acs_codec_set_subject_scopes.argtypes = [vp, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        lib.acs_codec_evict_subject.argtypes = [vp, C.c_char_p, C.c_size_t]
        lib.acs_codec_encode.restype = vp
        lib.acs_codec_encode.argtypes = [vp, C.c_char_p, C.c_size_t, C.c_int]
        lib.acs_codec_batch_view.argtypes = [vp, C.POINTER(ReqBatchC)]
        lib.acs_codec_batch_reason.restype = C.c_char_p
        lib.acs_codec_batch_reason.argtypes = [vp, C.c_uint32]
        lib.acs_codec_string.argtypes = [vp, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        lib.acs_codec_batch_stats.argtypes = [vp, C.POINTER(C.c_double), C.c_int]
        lib.acs_codec_batch_free.argtypes = [vp]
        lib.acs_codec_batch_free.restype = None
        lib.acs_codec_batch_expand.argtypes = [vp]
        _DECLARED.add(id(lib))
    return lib


def _view(ptr, dtype, count):
    if count == 0 or not ptr:
        return np.zeros(0, dtype)
    buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=count)


class _Strings:
    """Overlay-compatible id -> string view of one encoded batch."""

    def __init__(self, batch):
        self._b = batch

    def string(self, i):
        s, n = C.c_void_p(), C.c_size_t()
        k = _lib().acs_codec_string(self._b.h, int(i), C.byref(s), C.byref(n))
        if k == 0:
            return MISSING
        if k == 1:
            return None
        if k < 0:
            raise KeyError(i)
        return C.string_at(s.value, n.value).decode("utf-8", "surrogatepass") if n.value else ""


class CodecBatch:
    """One encoded batch (owns the codec's buffers until close()).

    The codec's own form is compact (acs_layout.h): request lines + extension records +
    arena + regex matrix + class rows, which is what ``struct`` describes and what
    native.Tables ships to the device.  The SoA rows (hdr / res / subj / act / roles, the
    attribute names of encoder.RequestBatch) are materialised on first access
    (acs_codec_batch_expand), for the tests and the CPU build of the core."""

    _SOA = ("hdr", "res", "subj", "act", "roles")

    def __init__(self, handle, codec):
        self.h = handle
        self._codec = codec  # the batch reads the codec's dictionary: keep it alive
        s = ReqBatchC()
        if _lib().acs_codec_batch_view(handle, C.byref(s)) != 0:
            raise RuntimeError(last_error())
        self.struct = s
        n = self.n = int(s.n)
        self.arena = _view(s.arena, np.uint32, int(s.arena_words))
        self.rx = _view(s.rx, np.uint8, s.rx_cols * s.rx_rows).reshape(s.rx_cols, s.rx_rows)
        self.rx_rows = int(s.rx_rows)
        W = int(s.cand_words)
        self.cand = _view(s.cand, np.uint32, s.cand_rows * W).reshape(s.cand_rows, W) if s.cand else None
        self.cand_wp, self.cand_wr = int(s.cand_wp), int(s.cand_wr)
        self.cand_wsu, self.cand_wpu = int(s.cand_wsu), int(s.cand_wpu)
        self.cand_wv = int(s.cand_wv)
        self.role_key = _view(s.role_key, np.uint32, n) if s.role_key else None
        self.role_bits = (_view(s.role_rows_bits, np.uint32, s.role_rows * W).reshape(s.role_rows, W)
                          if s.role_key else None)
        self.lines = _view(s.lines, L.REQ_LINE_DT, n) if s.lines else np.zeros(0, L.REQ_LINE_DT)
        self.ext = _view(s.ext, np.uint32, int(s.ext_words)) if s.ext else np.zeros(0, np.uint32)
        self.perm = _view(s.perm, np.uint32, int(s.perm_lanes)) if s.perm else None  # coherence order
        self.hints = int(s.hints)  # ACS_HINT_* (acs_req_batch.hints)
        self.cls2 = self.lines["cls2"]  # 1 + second class (composed class rows; 0: none)
        self.overlay = _Strings(self)
        self.host_reasons = {}
        for i in np.flatnonzero((self.lines["h"]["flags"] & np.uint32(L.RQ_HOST)) != 0):
            r = _lib().acs_codec_batch_reason(handle, int(i))
            self.host_reasons[int(i)] = r.decode() if r else "host path"
        self._soa = None

    def __getattr__(self, name):
        if name in CodecBatch._SOA:  # SoA rows on first use
            return self.expand()[name]
        raise AttributeError(name)

    def expand(self):
        """The SoA rows (acs_codec_batch_expand); the struct keeps the compact form."""
        if self._soa is None:
            if _lib().acs_codec_batch_expand(self.h) != 0:
                raise RuntimeError(last_error())
            s = ReqBatchC()
            _lib().acs_codec_batch_view(self.h, C.byref(s))
            n = self.n
            self._soa = {"hdr": _view(s.hdr, L.REQ_HDR_DT, n),
                         "res": _view(s.res, L.REQ_RES_DT, L.QMAX * n).reshape(L.QMAX, n),
                         "subj": _view(s.subj, L.PAIR_DT, L.SMAX * n).reshape(L.SMAX, n),
                         "act": _view(s.act, L.PAIR_DT, L.AMAX * n).reshape(L.AMAX, n),
                         "roles": _view(s.roles, np.uint32, L.RMAX * n).reshape(L.RMAX, n)}
        return self._soa

    def stats(self):
        out = (C.c_double * 8)()
        _lib().acs_codec_batch_stats(self.h, out, 8)
        return {"encode_s": out[0], "regex_s": out[1], "classes_s": out[2], "total_s": out[3],
                "hr_cache_hits": int(out[4]), "hr_cache_misses": int(out[5]), "classes_new": int(out[6]),
                "classes": int(out[7])}

    def nbytes(self):
        """Bytes of the compact form (what the host-buffer path uploads)."""
        return sum(a.nbytes for a in (self.lines, self.ext, self.arena, self.rx)) + \
            (self.cand.nbytes if self.cand is not None else 0) + \
            (self.role_key.nbytes + self.role_bits.nbytes if self.role_key is not None else 0) + \
            (self.perm.nbytes if self.perm is not None else 0)

    compact_nbytes = nbytes

    def close(self):
        if self.h:
            for k in ("arena", "rx", "cand", "role_key", "role_bits", "lines", "ext", "perm", "cls2"):
                setattr(self, k, None)
            self._soa = None
            _lib().acs_codec_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeCodec:
    """The native encoder of one compiled store image (compiler.store_blob)."""

    def __init__(self, blob: bytes):
        self._blob = blob
        self.h = _lib().acs_codec_create(blob, len(blob))
        if not self.h:
            raise RuntimeError(last_error())

    def set_subject_scopes(self, key: str, scopes) -> None:
        """Register (or replace) a subject's hierarchical_scopes forest; requests name it with
        context.subject["$hrs"] = key (the createHRScope / Redis cache of the reference)."""
        k = key.encode()
        text = scopes if isinstance(scopes, (bytes, bytearray)) else json.dumps(scopes).encode()
        if _lib().acs_codec_set_subject_scopes(self.h, k, len(k), bytes(text), len(text)) != 0:
            raise RuntimeError(last_error())

    def evict_subject(self, key: str) -> bool:
        k = key.encode()
        return _lib().acs_codec_evict_subject(self.h, k, len(k)) == 1

    def encode(self, requests, threads: int = 1) -> CodecBatch:
        """``requests``: JSON text (bytes/str) of an array of requests, or a list to serialise."""
        if isinstance(requests, str):
            text = requests.encode("utf-8", "surrogatepass")
        elif isinstance(requests, (bytes, bytearray, memoryview)):
            text = bytes(requests)
        else:
            text = json.dumps(requests, ensure_ascii=False, separators=(",", ":")).encode("utf-8", "surrogatepass")
        h = _lib().acs_codec_encode(self.h, text, len(text), int(threads))
        if not h:
            raise RuntimeError(last_error())
        return CodecBatch(h, self)

    def close(self):
        if self.h:
            _lib().acs_codec_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PipelineStats(C.Structure):
    _fields_ = [("encode_s", C.c_double), ("wait_s", C.c_double), ("total_s", C.c_double), ("gpu_ms", C.c_double),
                ("upload_bytes", C.c_double), ("requests", C.c_uint64), ("chunks", C.c_uint64),
                ("host_requests", C.c_uint64), ("split_s", C.c_double), ("check_s", C.c_double)]


class Pipeline:
    """acs_pipeline (include/acs_mi355x.h): JSON request text -> decision records, encode of
    chunk k+1 overlapped with the device work of chunk k (two streams, page-locked buffers)."""

    def __init__(self, tables, codec: NativeCodec, threads: int = 16, chunk: int = 131072):
        lib = tables.lib
        lib.acs_pipeline_create.restype = C.c_void_p
        lib.acs_pipeline_create.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint32]
        lib.acs_pipeline_free.argtypes = [C.c_void_p]
        lib.acs_pipeline_free.restype = None
        lib.acs_pipeline_is_allowed.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                C.POINTER(C.c_size_t), C.POINTER(PipelineStats)]
        lib.acs_pipeline_host_reason.restype = C.c_char_p
        lib.acs_pipeline_host_reason.argtypes = [C.c_void_p, C.c_size_t]
        self.lib, self._tables, self._codec = lib, tables, codec  # both must outlive the pipeline
        self.h = lib.acs_pipeline_create(tables.h, codec.h, int(threads), int(chunk))
        if not self.h:
            raise RuntimeError(last_error(lib))

    def is_allowed(self, text: bytes, capacity: int):
        """(records [n] DECISION_DT, stats dict) for the JSON array `text` (at most `capacity`
        requests)."""
        out = np.zeros(capacity, L.DECISION_DT)
        n = C.c_size_t(0)
        st = PipelineStats()
        if self.lib.acs_pipeline_is_allowed(self.h, text, len(text), out.ctypes.data, capacity, C.byref(n),
                                            C.byref(st)) != 0:
            raise RuntimeError(last_error(self.lib))
        stats = {k: getattr(st, k) for k, _ in PipelineStats._fields_}
        out = out[:n.value]
        self.host_reasons = {}
        for i in np.flatnonzero((out["flags"] & np.uint8(L.OF_HOST_REQ)) != 0):
            r = self.lib.acs_pipeline_host_reason(self.h, int(i))
            self.host_reasons[int(i)] = r.decode() if r else None
        return out, stats

    def close(self):
        if self.h:
            self.lib.acs_pipeline_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
