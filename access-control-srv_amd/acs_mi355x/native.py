"""ctypes binding of the C ABI (include/acs_mi355x.h) — the product's only compute path.

``load()`` raises if ``lib/libacs_mi355x.so`` is missing: there is no CPU
fallback in the product package.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import layout as L

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ACS_MI355X_LIB: an alternative build of the same library (A/B experiments only)
LIB_PATH = os.environ.get("ACS_MI355X_LIB") or os.path.join(PKG, "lib", "libacs_mi355x.so")


class ReqBatchC(C.Structure):
    _fields_ = [("n", C.c_uint32), ("hdr", C.c_void_p), ("res", C.c_void_p), ("subj", C.c_void_p),
                ("act", C.c_void_p), ("roles", C.c_void_p), ("arena", C.c_void_p), ("arena_words", C.c_size_t),
                ("rx", C.c_void_p), ("rx_cols", C.c_uint32), ("rx_rows", C.c_uint32),
                ("cand", C.c_void_p), ("cand_words", C.c_uint32), ("cand_wp", C.c_uint32), ("cand_wr", C.c_uint32),
                ("cand_rows", C.c_uint32), ("cand_wsu", C.c_uint32), ("cand_wpu", C.c_uint32),
                ("cand_wv", C.c_uint32),
                ("role_key", C.c_void_p), ("role_rows_bits", C.c_void_p),
                ("role_rows", C.c_uint32), ("lines", C.c_void_p), ("ext", C.c_void_p), ("ext_words", C.c_size_t),
                ("perm", C.c_void_p), ("perm_lanes", C.c_size_t), ("hints", C.c_uint32)]


EXPORTS = ["acs_compile", "acs_free", "acs_is_allowed", "acs_is_allowed_device", "acs_wia_words_per_request",
           "acs_what_is_allowed", "acs_what_is_allowed_device", "acs_last_kernel_ms", "acs_last_error",
           "acs_layout_sizes", "acs_device_count", "acs_set_option", "acs_kernel_times",
           "acs_shard_keys_device", "acs_shard_decode_device", "acs_what_is_allowed_obl",
           "acs_what_is_allowed_obl_device", "acs_store_compile", "acs_blob_free", "acs_store_builder_create",
           "acs_store_builder_stage", "acs_store_builder_compile", "acs_store_builder_free", "acs_codec_create",
           "acs_codec_free", "acs_codec_set_subject_scopes", "acs_codec_evict_subject", "acs_codec_encode",
           "acs_codec_batch_view", "acs_codec_batch_reason", "acs_codec_string", "acs_codec_ec_values",
           "acs_codec_batch_stats", "acs_codec_batch_free", "acs_codec_batch_expand", "acs_pipeline_create",
           "acs_pipeline_free", "acs_pipeline_is_allowed", "acs_compile_multi", "acs_compile_sharded", "acs_device_list",
           "acs_pipeline_host_reason", "acs_overflow_index_device", "acs_overflow_repass_device",
           "acs_compile_update", "acs_image_upload_bytes"]


class ShardC(C.Structure):
    _fields_ = [("set_base", C.c_uint32), ("pol_base", C.c_uint32), ("rule_base", C.c_uint32)]


def _declare(lib):
    vp, u32 = C.c_void_p, C.c_uint32
    pb = C.POINTER(ReqBatchC)
    lib.acs_compile.restype = vp
    lib.acs_compile.argtypes = [vp, C.c_size_t, C.c_int]
    lib.acs_compile_multi.restype = vp
    lib.acs_compile_multi.argtypes = [vp, C.c_size_t, C.POINTER(C.c_int), C.c_int]
    if hasattr(lib, "acs_compile_update"):  # (A/B builds of earlier sources lack it)
        lib.acs_compile_update.restype = vp
        lib.acs_compile_update.argtypes = [vp, vp, C.c_size_t]
        lib.acs_image_upload_bytes.restype = C.c_size_t
        lib.acs_image_upload_bytes.argtypes = [vp]
    lib.acs_compile_sharded.restype = vp
    lib.acs_compile_sharded.argtypes = [vp, C.c_size_t, C.POINTER(C.c_int), C.c_int]
    lib.acs_device_list.argtypes = [vp, C.POINTER(C.c_int), C.c_int]
    lib.acs_free.argtypes = [vp]
    lib.acs_free.restype = None
    lib.acs_is_allowed.argtypes = [vp, pb, vp]
    lib.acs_is_allowed_device.argtypes = [vp, pb, vp, vp]
    lib.acs_wia_words_per_request.argtypes = [vp]
    lib.acs_wia_words_per_request.restype = u32
    lib.acs_what_is_allowed.argtypes = [vp, pb, vp, vp, vp, vp]
    lib.acs_what_is_allowed_device.argtypes = [vp, pb, vp, vp, vp, vp, vp]
    lib.acs_what_is_allowed_obl.argtypes = [vp, pb, vp, C.c_size_t, u32, u32, vp, vp]
    lib.acs_what_is_allowed_obl_device.argtypes = [vp, pb, vp, C.c_size_t, u32, u32, vp, vp, vp]
    lib.acs_last_kernel_ms.argtypes = [vp]
    lib.acs_last_kernel_ms.restype = C.c_float
    lib.acs_last_error.restype = C.c_char_p
    lib.acs_layout_sizes.argtypes = [C.POINTER(u32), C.c_int]
    lib.acs_set_option.argtypes = [vp, C.c_int, C.c_int]
    lib.acs_kernel_times.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
    lib.acs_overflow_index_device.argtypes = [vp, pb, vp, vp, C.POINTER(C.c_size_t), vp]
    lib.acs_overflow_repass_device.argtypes = [vp, vp, vp, C.c_size_t, u32, u32, vp, C.POINTER(C.c_size_t),
                                               C.POINTER(u32), vp]
    lib.acs_shard_keys_device.argtypes = [vp, vp, C.c_size_t, C.POINTER(ShardC), vp, vp]
    lib.acs_shard_decode_device.argtypes = [vp, C.c_size_t, vp, vp]
    return lib


_LIB = None


def load(path: str | None = None):
    """Load the HIP library (fails loudly when it has not been built)."""
    global _LIB
    if _LIB is None or path:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(f"MI355X evaluator library missing: {p} (run __graft_entry__.build())")
        _LIB = _declare(C.CDLL(p))
    return _LIB


def last_error(lib=None):
    return (lib or load()).acs_last_error().decode()


def batch_struct(b, ptrs=None, compact=False) -> ReqBatchC:
    """acs_req_batch over host numpy arrays (ptrs=None) or a dict of device pointers.
    compact: lines + extension records only, no SoA rows (acs_layout.h; the form the host
    path uploads)."""
    s = ReqBatchC()
    s.n = b.n
    if compact and (getattr(b, "lines", None) is None or getattr(b, "ext", None) is None):
        raise ValueError("a compact batch needs its lines and extension records (encoder.pack_ext)")
    if ptrs is None:
        if not compact:
            s.hdr = b.hdr.ctypes.data
            s.res = b.res.ctypes.data
            s.subj = b.subj.ctypes.data
            s.act = b.act.ctypes.data
            s.roles = b.roles.ctypes.data
        s.arena = b.arena.ctypes.data if b.arena.size else b.lines.ctypes.data if compact else b.hdr.ctypes.data
        s.rx = b.rx.ctypes.data
        s.cand = b.cand.ctypes.data if b.cand is not None else None
        if b.role_key is not None:
            s.role_key, s.role_rows_bits = b.role_key.ctypes.data, b.role_bits.ctypes.data
        if getattr(b, "lines", None) is not None:
            s.lines = b.lines.ctypes.data
        if compact and b.ext.size:
            s.ext = b.ext.ctypes.data
        if getattr(b, "perm", None) is not None and b.perm.size:
            s.perm = b.perm.ctypes.data
    else:
        for k in ("hdr", "res", "subj", "act", "roles"):
            if not compact:
                setattr(s, k, ptrs[k])
        s.arena, s.rx = ptrs["arena"], ptrs["rx"]
        s.cand = ptrs.get("cand")
        s.role_key, s.role_rows_bits = ptrs.get("role_key"), ptrs.get("role_bits")
        s.lines = ptrs.get("lines")
        s.ext = ptrs.get("ext") if compact else None
        s.perm = ptrs.get("perm")
    if s.perm:
        s.perm_lanes = int(b.perm.size)
    s.hints = int(getattr(b, "hints", 0) or 0)
    if compact:
        s.ext_words = int(b.ext.size)
    s.arena_words = int(b.arena.size)
    s.rx_cols = int(b.rx.shape[0])
    s.rx_rows = int(b.rx.shape[1])
    if b.cand is not None:
        s.cand_words, s.cand_wp, s.cand_wr = b.cand.shape[1], b.cand_wp, b.cand_wr
        s.cand_rows = b.cand.shape[0]
        s.cand_wsu, s.cand_wpu = getattr(b, "cand_wsu", 0), getattr(b, "cand_wpu", 0)
        s.cand_wv = getattr(b, "cand_wv", 0)
    if b.role_key is not None:
        s.role_rows = b.role_bits.shape[0]
    return s


def host_struct(batch, compact=False) -> ReqBatchC:
    """The acs_req_batch a host-buffer entry point gets for `batch`: a CodecBatch's own view
    (compact, plus SoA rows once expanded), else batch_struct over the numpy arrays."""
    s = getattr(batch, "struct", None)
    if s is not None:
        return s
    return batch_struct(batch, compact=compact)


OVERFLOW_CAP = 1024  # first obligation-only pass: log entries per overflowed request and set range
OVERFLOW_CHUNKS = 8  # policy-set ranges per request in the obligation-only pass


def join_chunk_logs(obl, obl_n, cap):
    """Per request j: the concatenation over set ranges c of obl[c, j, :obl_n[c, j]], or None
    when some range's log was truncated (obl_n > cap)."""
    out = []
    for j in range(obl.shape[1]):
        n = obl_n[:, j]
        out.append(None if (n > cap).any() else
                   np.concatenate([obl[c, j, :n[c]] for c in range(obl.shape[0])]).reshape(-1, 2))
    return out


def resolve_overflow(tables, batch, out, cap: int = OVERFLOW_CAP, chunks: int = OVERFLOW_CHUNKS) -> dict:
    """Full maskedProperty logs of the requests whose K2 log overflowed (OF_OBL_OVERFLOW):
    {request index: [k][2] pairs}, from the obligation-only pass (``cap`` entries per set range
    first, then each still-truncated request once more at its exact count).  Clears the flag
    in ``out``."""
    idx = np.flatnonzero((out["flags"] & L.OF_OBL_OVERFLOW) != 0).astype(np.uint32)
    logs = {}
    while len(idx):
        obl, obl_n = tables.what_is_allowed_obl(batch, idx, cap, chunks)
        joined = join_chunk_logs(obl, obl_n, cap)
        for j, lg in enumerate(joined):
            if lg is not None:
                logs[int(idx[j])] = lg
        left = np.array([lg is None for lg in joined])
        idx, cap = idx[left], (int(obl_n[:, left].max()) if left.any() else cap)
    if logs:
        flags = out["flags"]
        flags[np.fromiter(logs, np.int64, len(logs))] &= np.uint8(~L.OF_OBL_OVERFLOW & 0xFF)
    return logs


class Tables:
    """Device-resident compiled store (wraps an acs_tables handle): on one GPU, or with
    ``devices=[d0, d1, ...]`` replicated over several (acs_compile_multi) so that large
    compact host batches and the pipeline split across them; the *_device entry points and
    ``device`` name d0."""

    def __init__(self, blob: bytes, device: int = 0, lib=None, devices=None, sharded: bool = False):
        """sharded: devices=[...] each hold a run of the store's policy sets (acs_compile_sharded,
        rule sharding in one process: is_allowed only) instead of a replica."""
        self.lib = lib or load()
        self._blob = blob
        if devices:
            arr = (C.c_int * len(devices))(*devices)
            compile_fn = self.lib.acs_compile_sharded if sharded else self.lib.acs_compile_multi
            self.h = compile_fn(blob, len(blob), arr, len(devices))
            device = int(devices[0])
        else:
            self.h = self.lib.acs_compile(blob, len(blob), device)
        if not self.h:
            raise RuntimeError(f"acs_compile failed: {last_error(self.lib)}")
        self.device = device
        self.words = int(self.lib.acs_wia_words_per_request(self.h))

    def updated(self, blob: bytes) -> "Tables":
        """A new handle for the changed store's blob (acs_compile_update: a device-side copy of this
        image with only the differing blocks uploaded when the shape is unchanged); this handle
        stays valid.  .upload_bytes: what the compile uploaded."""
        t = Tables.__new__(Tables)
        t.lib, t._blob, t.device = self.lib, blob, self.device
        t.h = self.lib.acs_compile_update(self.h, blob, len(blob))
        if not t.h:
            raise RuntimeError(f"acs_compile_update failed: {last_error(self.lib)}")
        t.words = int(self.lib.acs_wia_words_per_request(t.h))
        return t

    @property
    def upload_bytes(self) -> int:
        return int(self.lib.acs_image_upload_bytes(self.h))

    def devices(self):
        """The handle's devices (acs_device_list), primary first."""
        arr = (C.c_int * 64)()
        m = self.lib.acs_device_list(self.h, arr, 64)
        if m < 0:
            raise RuntimeError(last_error(self.lib))
        return list(arr[:m])

    def close(self):
        if self.h:
            self.lib.acs_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def is_allowed(self, batch, compact: bool = False, out=None) -> np.ndarray:
        """acs_is_allowed on host buffers: a CodecBatch ships its own (compact) form; a
        RequestBatch its SoA rows + lines, or with compact=True its lines + extension records.
        out: the caller's record array (e.g. page-locked), else a new one."""
        if out is None:
            out = np.zeros(batch.n, L.DECISION_DT)
        assert out.dtype == L.DECISION_DT and len(out) >= batch.n and out.flags["C_CONTIGUOUS"]
        if batch.n:
            s = host_struct(batch, compact)
            if self.lib.acs_is_allowed(self.h, C.byref(s), out.ctypes.data) != 0:
                raise RuntimeError(f"acs_is_allowed: {last_error(self.lib)}")
        return out

    def what_is_allowed(self, batch, compact: bool = False):
        n = batch.n
        bits = np.zeros((n, self.words), np.uint32)
        obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
        obl_n = np.zeros(n, np.uint32)
        out = np.zeros(n, L.DECISION_DT)
        if n:
            s = host_struct(batch, compact)
            rc = self.lib.acs_what_is_allowed(self.h, C.byref(s), bits.ctypes.data, obl.ctypes.data,
                                              obl_n.ctypes.data, out.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"acs_what_is_allowed: {last_error(self.lib)}")
        return bits, obl, obl_n, out

    def what_is_allowed_obl(self, batch, idx, cap: int, chunks: int = OVERFLOW_CHUNKS, compact: bool = False):
        """Obligation-only pass over requests ``idx`` of ``batch``, the policy sets cut into
        ``chunks`` ranges: (obl [chunks][m][cap][2], obl_n [chunks][m] = pushes per range)."""
        idx = np.ascontiguousarray(idx, np.uint32)
        m = len(idx)
        obl = np.zeros((chunks, m, cap, 2), np.uint32)
        obl_n = np.zeros((chunks, m), np.uint32)
        if m:
            s = host_struct(batch, compact)
            rc = self.lib.acs_what_is_allowed_obl(self.h, C.byref(s), idx.ctypes.data, m, chunks, cap,
                                                  obl.ctypes.data, obl_n.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"acs_what_is_allowed_obl: {last_error(self.lib)}")
        return obl, obl_n

    def resolve_overflow(self, batch, out, cap: int = OVERFLOW_CAP, chunks: int = OVERFLOW_CHUNKS) -> dict:
        return resolve_overflow(self, batch, out, cap, chunks)

    def set_sort(self, enable: bool):
        if self.lib.acs_set_option(self.h, 1, int(bool(enable))) != 0:
            raise RuntimeError(last_error(self.lib))

    def set_chunk(self, requests: int):
        """ACS_OPT_CHUNK: requests per overlapped chunk of the host-buffer isAllowed (0: off)."""
        if self.lib.acs_set_option(self.h, 3, int(requests)) != 0:
            raise RuntimeError(last_error(self.lib))

    def set_timing(self, enable: bool):
        if self.lib.acs_set_option(self.h, 2, int(bool(enable))) != 0:
            raise RuntimeError(last_error(self.lib))

    def kernel_times(self, n: int):
        buf = (C.c_float * n)()
        m = self.lib.acs_kernel_times(self.h, buf, n)
        if m < 0:
            raise RuntimeError(last_error(self.lib))
        return list(buf)[:m]

    def last_kernel_ms(self):
        return float(self.lib.acs_last_kernel_ms(self.h))
