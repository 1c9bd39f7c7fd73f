"""Device-resident request batches (torch is only the HBM allocator / stream provider).

``DeviceBatch`` copies a packed RequestBatch to one GPU once; the ``*_device``
C-ABI entry points then evaluate it in place on a caller-chosen HIP stream,
which is how the benchmark measures throughput with inputs already in HBM.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import layout as L
from .native import batch_struct, last_error


def _to_dev(a: np.ndarray, dev):
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1))
    return t.to(dev, non_blocking=False)


class DeviceBatch:
    """compact=True (default for a native-codec batch): request lines + extension records +
    arena + regex matrix + class rows, the product's device form (acs_layout.h); False: the
    SoA rows as well (the kernels then read them instead of the extension records)."""

    def __init__(self, batch, device: int = 0, compact: bool | None = None):
        self.batch = batch
        self.dev = torch.device("cuda", device)
        if compact is None:
            compact = hasattr(batch, "struct")
        self.compact = compact
        keys = ("arena", "rx") if compact else ("hdr", "res", "subj", "act", "roles", "arena", "rx")
        self.t = {k: _to_dev(getattr(batch, k) if getattr(batch, k).size else np.zeros(4, np.uint32), self.dev)
                  for k in keys}
        if batch.cand is not None:
            self.t["cand"] = _to_dev(batch.cand, self.dev)
        if batch.role_key is not None:
            self.t["role_key"] = _to_dev(batch.role_key, self.dev)
            self.t["role_bits"] = _to_dev(batch.role_bits, self.dev)
        if getattr(batch, "lines", None) is not None and batch.n:
            self.t["lines"] = _to_dev(batch.lines, self.dev)
        if compact:
            ext = getattr(batch, "ext", None)
            self.t["ext"] = _to_dev(ext if ext is not None and ext.size else np.zeros(4, np.uint32), self.dev)
        perm = getattr(batch, "perm", None)
        if perm is not None and perm.size:  # the encoder's coherence order (no device sort)
            self.t["perm"] = _to_dev(perm, self.dev)
        self.ptrs = {k: v.data_ptr() for k, v in self.t.items()}
        self.struct = batch_struct(batch, self.ptrs, compact=compact)
        self.nbytes = sum(v.numel() for v in self.t.values())


def is_allowed_device(tables, db: DeviceBatch, out: torch.Tensor | None = None, stream=None):
    """Enqueue K1 on ``stream`` (torch stream or None = current); returns the uint8 [n, 8] output tensor."""
    n = db.batch.n
    if out is None:
        out = torch.empty((n, 8), dtype=torch.uint8, device=db.dev)
    s = (stream or torch.cuda.current_stream(db.dev)).cuda_stream
    rc = tables.lib.acs_is_allowed_device(tables.h, C.byref(db.struct), out.data_ptr(), C.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"acs_is_allowed_device: {last_error(tables.lib)}")
    return out


def what_is_allowed_device(tables, db: DeviceBatch, bufs=None, stream=None):
    n = db.batch.n
    if bufs is None:
        bufs = (torch.empty((n, tables.words), dtype=torch.int32, device=db.dev),
                torch.empty((n, L.OBL_MAX, 2), dtype=torch.int32, device=db.dev),
                torch.empty((n,), dtype=torch.int32, device=db.dev),
                torch.empty((n, 8), dtype=torch.uint8, device=db.dev))
    s = (stream or torch.cuda.current_stream(db.dev)).cuda_stream
    rc = tables.lib.acs_what_is_allowed_device(tables.h, C.byref(db.struct), bufs[0].data_ptr(), bufs[1].data_ptr(),
                                               bufs[2].data_ptr(), bufs[3].data_ptr(), C.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"acs_what_is_allowed_device: {last_error(tables.lib)}")
    return bufs


# lanes of one obligation pass that keep the GPU busy (256 CUs x 16 waves x 64 lanes)
OBL_PASS_LANES = 1 << 18


def resolve_overflow_device(tables, db: DeviceBatch, bufs, cap: int | None = None, chunks: int | None = None,
                            stream=None):
    """Obligation-only passes for the requests whose K2 log overflowed (record flag
    OF_OBL_OVERFLOW in ``bufs[3]``): the policy sets cut into ``chunks`` ranges with ``cap``
    entries each, then the still-truncated requests once more at their exact count.  By
    default the ranges are as many (8..64, a power of two) as keep about OBL_PASS_LANES lanes
    busy, so a few overflowed requests take 1/64 of a traversal, not 1/8.  The index lists
    come from the library's selection kernels (acs_overflow_index_device: K2's coherence
    order; acs_overflow_repass_device), each syncing the stream once to size its pass.
    Returns [(idx [m], cap, obl [chunks][m][cap][2], obl_n [chunks][m])] per pass (int32
    tensors; later passes supersede earlier ones)."""
    st = stream or torch.cuda.current_stream(db.dev)
    s = C.c_void_p(st.cuda_stream)
    lib, n = tables.lib, db.batch.n
    with torch.cuda.stream(st):
        idx = torch.empty(max(n, 1), dtype=torch.int32, device=db.dev)
        m = C.c_size_t(0)
        if lib.acs_overflow_index_device(tables.h, C.byref(db.struct), bufs[3].data_ptr(), idx.data_ptr(), C.byref(m),
                                         s) != 0:
            raise RuntimeError(f"acs_overflow_index_device: {last_error(lib)}")
        m = int(m.value)
        if chunks is None:
            chunks = 8
            while chunks < 64 and chunks * 2 * max(m, 1) <= OBL_PASS_LANES:
                chunks *= 2
        if cap is None:
            cap = max(128, 8192 // chunks)
        idx = idx[:m]
        passes = []
        while m:
            obl = torch.empty((chunks, m, cap, 2), dtype=torch.int32, device=db.dev)
            obl_n = torch.empty((chunks, m), dtype=torch.int32, device=db.dev)
            rc = lib.acs_what_is_allowed_obl_device(tables.h, C.byref(db.struct), idx.data_ptr(), m, chunks, cap,
                                                    obl.data_ptr(), obl_n.data_ptr(), s)
            if rc != 0:
                raise RuntimeError(f"acs_what_is_allowed_obl_device: {last_error(lib)}")
            passes.append((idx, cap, obl, obl_n))
            nxt = torch.empty(m, dtype=torch.int32, device=db.dev)
            m2, cap2 = C.c_size_t(0), C.c_uint32(0)
            if lib.acs_overflow_repass_device(tables.h, obl_n.data_ptr(), idx.data_ptr(), m, chunks, cap,
                                              nxt.data_ptr(), C.byref(m2), C.byref(cap2), s) != 0:
                raise RuntimeError(f"acs_overflow_repass_device: {last_error(lib)}")
            m, cap, idx = int(m2.value), int(cap2.value), nxt[:int(m2.value)]
    return passes


def overflow_logs(passes) -> dict:
    """{request index: [k][2] uint32 pairs} from resolve_overflow_device's passes."""
    from .native import join_chunk_logs
    logs = {}
    for idx, cap, obl, obl_n in passes:
        idx = idx.cpu().numpy()
        joined = join_chunk_logs(obl.cpu().numpy().view(np.uint32), obl_n.cpu().numpy().view(np.uint32), cap)
        for j, lg in enumerate(joined):
            if lg is not None:
                logs[int(idx[j])] = lg
    return logs


def decisions_from_tensor(out: torch.Tensor) -> np.ndarray:
    return out.cpu().numpy().reshape(-1).view(L.DECISION_DT)
