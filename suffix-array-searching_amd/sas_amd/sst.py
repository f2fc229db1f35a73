"""Host-side mirror of the reference's u32 search API (sst/lib.rs SearchIndex / SearchScheme).

    SortedVec.new(vals)                       <- sst/binary_search.rs:19-27
    Eytzinger.new(vals)                       <- sst/eytzinger.rs:66-70
    STree16.new(vals) / STree15.new(vals)     <- sst/s_tree.rs:47-50  (new_params(false,false,false))
    STree16.new_params(vals, left_max, reverse, full)   <- sst/s_tree.rs:72-176
    index.size(), index.layers()              <- sst/lib.rs:35-39
    index.query(qs), index.query_one(q)       <- sst/lib.rs:41-47, SearchScheme::query :55-57

Queries run on the GPU (libsas_amd.so); there is no CPU fallback.  Build-time
assertions of the reference (sorted input, keys <= i32::MAX) raise SasError.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import SasError, check, lib

MAX = 0x7FFFFFFF  # sst/node.rs:5


def _is_cuda(x) -> bool:
    return hasattr(x, "is_cuda") and bool(x.is_cuda)


class _Index:
    LAYOUT = None

    def __init__(self, handle, n):
        self._h = handle
        self.n = n

    @classmethod
    def _build(cls, vals, layout, flags=0):
        vals = np.ascontiguousarray(vals, np.uint32)
        h = C.c_void_p()
        check(lib().sst_build(vals.ctypes.data if len(vals) else None, len(vals), layout, flags, C.byref(h)))
        return cls(h, len(vals))

    @classmethod
    def new(cls, vals):
        return cls._build(vals, cls.LAYOUT)

    def free(self):
        if self._h:
            lib().sst_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def size(self) -> int:
        return int(lib().sst_size(self._h))

    def layers(self) -> int:
        return int(lib().sst_layers(self._h))

    def nodes(self) -> np.ndarray:
        words = self.size() // 4
        out = np.zeros(max(words, 1), np.uint32)
        check(lib().sst_copy_nodes(self._h, out.ctypes.data, words))
        return out[:words]

    def query(self, qs, want_rank: bool = False, stream=None, flags: int = 0, out=None):
        """out: (device queries only) a caller-owned 4-byte result tensor of at least qs.numel()
        elements, contiguous, on qs's device; host queries refuse it (they return a new array)."""
        if _is_cuda(qs):
            import torch
            if out is None:
                out = torch.empty(qs.numel(), dtype=torch.int32, device=qs.device)
            elif not (_is_cuda(out) and out.device == qs.device and out.element_size() == 4 and
                      out.is_contiguous() and out.numel() >= qs.numel()):
                raise SasError(22, "sst query: out must be a contiguous 4-byte tensor on the queries' device "
                                   f"with >= {qs.numel()} elements")
            rank = torch.empty(qs.numel(), dtype=torch.int64, device=qs.device) if want_rank else None
            st = stream if stream is not None else torch.cuda.current_stream(qs.device).cuda_stream
            check(lib().sst_query(self._h, qs.data_ptr(), qs.numel(), out.data_ptr(),
                                  rank.data_ptr() if want_rank else None, st, flags | _lib.SST_DEVICE_PTRS))
            return (out, rank) if want_rank else out
        if out is not None:
            raise SasError(22, "sst query: out= is for device queries; host queries return a new array")
        qs = np.ascontiguousarray(qs, np.uint32)
        out = np.zeros(max(len(qs), 1), np.uint32)
        rank = np.zeros(max(len(qs), 1), np.uint64) if want_rank else None
        check(lib().sst_query(self._h, qs.ctypes.data, len(qs), out.ctypes.data,
                              rank.ctypes.data if want_rank else None, stream, flags))
        return (out[: len(qs)], rank[: len(qs)]) if want_rank else out[: len(qs)]

    def query_one(self, q: int) -> int:
        return int(self.query(np.array([q], np.uint32))[0])

    def time_query(self, d_qs, d_out, reps=1, stream=None, flags=0) -> float:
        kn = C.c_double(0)
        check(lib().sst_time_query(self._h, d_qs.data_ptr(), d_qs.numel(), d_out.data_ptr(), reps, stream, flags,
                                   C.byref(kn)))
        return kn.value


class SortedVec(_Index):
    LAYOUT = _lib.SST_SORTED


class Eytzinger(_Index):
    LAYOUT = _lib.SST_EYTZINGER


class _STree(_Index):
    @classmethod
    def new_params(cls, vals, left_max: bool, reverse_storage: bool, full_array: bool):
        flags = (_lib.SST_LEFT_MAX if left_max else 0) | (_lib.SST_REVERSE if reverse_storage else 0)
        flags |= _lib.SST_FULL if full_array else 0
        return cls._build(vals, cls.LAYOUT, flags)


class STree16(_STree):
    LAYOUT = _lib.SST_STREE16


class STree15(_STree):
    LAYOUT = _lib.SST_STREE15


class PartitionedSTree16M(_Index):
    """PartitionedSTree<16,16,Map> (sst/partitioned_s_tree.rs): prefix map on the
    top b key bits + S-tree.  new(vals, b) as in the reference (test.rs uses
    b in {0, 4, 8, 16, 20})."""
    LAYOUT = _lib.SST_PARTITIONED_MAP

    @classmethod
    def new(cls, vals, b: int = 16):
        return cls._build(vals, cls.LAYOUT, (b & 0xFF) << 16)


class _Partitioned(_Index):
    """PartitionedSTree<16,16,Tp>::new(vals, b) (sst/partitioned_s_tree.rs:111-648) for the
    markers the reference's differential test runs beside Map (sst/test.rs:222-246).  The
    leaves are padded per part: query() returns values only."""

    @classmethod
    def new(cls, vals, b: int = 16):
        return cls._build(vals, cls.LAYOUT, (b & 0xFF) << 16)


class PartitionedSTree16(_Partitioned):
    """Simple: every part a full (B+1)^h tree, layer by layer."""
    LAYOUT = _lib.SST_PARTITIONED


class PartitionedSTree16C(_Partitioned):
    """Compact: each part's tree packed on its own (bpp nodes per part)."""
    LAYOUT = _lib.SST_PARTITIONED_COMPACT


class PartitionedSTree16L(_Partitioned):
    """L1: the root's fan-out reduced to what the largest part needs."""
    LAYOUT = _lib.SST_PARTITIONED_L1


class PartitionedSTree16O(_Partitioned):
    """Overlapping: consecutive parts share root windows (16 - overlap new subtrees each)."""
    LAYOUT = _lib.SST_PARTITIONED_OVERLAP


class DirectMap(_Index):
    """SST_DIRECT_MAP: the prefix map of PartitionedSTree16M taken to its limit, a
    direct-address table on the top b of the 31 key bits whose 16-B entries inline
    the first three keys at or after each bucket start (b = 0: ceil(log2 n) + 1).
    Same answers as every other layout: the first key >= q and its index."""
    LAYOUT = _lib.SST_DIRECT_MAP

    @classmethod
    def new(cls, vals, b: int = 0):
        return cls._build(vals, cls.LAYOUT, (b & 0xFF) << 16)
