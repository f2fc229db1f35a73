"""Host-side mirror of the reference's suffix-array query API (sas/sa_search.rs).

    SaNaive.build(t)                      <- SaNaive::build            sas/sa_search.rs:30-57
    binary_search(sa, q, cnt)             <- binary_search (type F1)    sas/sa_search.rs:98-112, :453
    binary_search_batch(sa, qs, cnt)      <- binary_search_batch<B>     sas/sa_search.rs:157-196, :454
    SaNaive.search_batch(queries, algo)   <- bench_batch driver         sas/sa_search.rs:437-451
    random_string / random_queries        <- sas/util.rs:9-26 (ChaCha8Rng::seed_from_u64, sas/main.rs:38)

Every call runs on the GPU through libsas_amd.so.  `cnt` is the reference's
`&mut usize` probe counter: pass a `Counter` and it is incremented by the number
of suffix comparisons the query made.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib


@dataclass
class Counter:
    """Stands in for the reference's `cnt: &mut usize` argument."""
    value: int = 0


def _is_cuda(x) -> bool:
    return hasattr(x, "is_cuda") and bool(x.is_cuda)


def _ptr(x):
    if x is None:
        return None
    if _is_cuda(x) or hasattr(x, "data_ptr"):
        return x.data_ptr()
    return x.ctypes.data


def _as_u8(x):
    if _is_cuda(x):
        return x
    return np.ascontiguousarray(np.frombuffer(x, np.uint8) if isinstance(x, (bytes, bytearray)) else x, np.uint8)


def _prefix_flags(prefix, quad, n: int, inline: bool = False) -> int:
    """prefix=None: build the prefix table (SAS_BUILD_PREFIX, p chosen by the library)
    whenever a quad tree is built and n < 2^32 - 1; False: never; an int: that p.
    inline: 1 (or True): 16-B entries inlining each range's first suffix
    (SAS_BUILD_PREFIX_INLINE); 2 / 4: 32-B / 64-B entries with its first two / four
    (_INLINE2 / _INLINE4)."""
    if prefix is None:
        prefix = bool(quad) and n < 0xFFFFFFFF
    if prefix is False:
        return 0
    f = _lib.SAS_BUILD_PREFIX | ({1: _lib.SAS_BUILD_PREFIX_INLINE, 2: _lib.SAS_BUILD_PREFIX_INLINE2,
                                    4: _lib.SAS_BUILD_PREFIX_INLINE4}.get(int(inline), 0))
    if prefix is True:
        return f
    return f | _lib.SAS_BUILD_PREFIX_P(int(prefix))


def _quad_flags(quad) -> int:
    """True: fused leaves; "compact": key-only leaves.  The inner-node layout is picked
    by the library (SAS_BUILD_QUAD_ABS / _REL in sas.h) unless a suffix forces it:
    "abs" / "rel" (fused) or "compact-abs" / "compact-rel"."""
    if quad is False:
        return 0
    if quad is True:
        quad = "fused"
    if not isinstance(quad, str):
        raise ValueError(f"quad must be a bool or a string, not {quad!r}")
    leaves, _, layout = quad.partition("-") if quad.startswith("compact") else ("fused", "", quad)
    if layout == "fused":
        layout = ""
    flags = {"fused": _lib.SAS_BUILD_QUAD, "compact": _lib.SAS_BUILD_QUAD_COMPACT}.get(leaves)
    lay = {"": 0, "abs": _lib.SAS_BUILD_QUAD_ABS, "rel": _lib.SAS_BUILD_QUAD_REL}.get(layout)
    if flags is None or lay is None:
        raise ValueError(f"quad must be True, False, 'compact', 'abs', 'rel', 'compact-abs' or "
                         f"'compact-rel', not {quad!r}")
    return flags | lay


class SaNaive:
    """GPU-resident suffix-array index: 2-bit packed text, u32 SA, optional LCP
    array and S-tree over 16-char SA keys, all in HBM."""

    def __init__(self, handle, n):
        self._h = handle
        self.n = n  # text length
        self.sa_n = self.stats()["sa_entries"]  # SA entries held (n, or a shard's rank range)
        self.rank_lo = self.stats()["rank_lo"]
        self.next_pos = self.stats()["next_pos"]  # SA value of the rank after this index's range

    @classmethod
    def build(cls, t, sa=None, lcp: bool = True, stree: bool | None = None, verify: bool = False,
              rank_range: tuple[int, int] | None = None, flags: int = 0, sector: bool | None = None,
              sa40: bool = False, quad: bool | str | None = None, llcp: bool | None = None,
              prefix: bool | int | None = None, prefix_inline: bool | int = False,
              tagged: bool | int = False, top2_levels: int = 0, tag_lines: bool = False) -> "SaNaive":
        """Index over t.  rank_range=(lo, hi): sharded-text mode, hold only global SA
        ranks [lo, hi) (sas_build_shard); `sa` is then the FULL suffix array or None
        (u32 or u64 array).  sa40: store a packed 40-bit SA and use the bucketed
        builder even when n < 2^32 (automatic above).  quad="compact": key-only quad
        leaves (8 B per suffix, SA values read from the SA array; SAS_BUILD_QUAD_COMPACT).
        llcp: the Manber-Myers Llcp/Rlcp entries for algo="llcp" (SAS_BUILD_LLCP, 16 B
        per suffix, implies the LCP array); None = only while n < 2^31 (<= 32 GiB).  prefix: the prefix table for algo="prefix"
        (SAS_BUILD_PREFIX; None = whenever quad is built and n < 2^32 - 1, an int = its
        p chars); prefix_inline: 16-B entries that inline each range's first suffix
        (True / 1: SAS_BUILD_PREFIX_INLINE) or 32-B ones with its first two (2:
        SAS_BUILD_PREFIX_INLINE2); fused quad leaves, u32 SA.  tagged: the SA as 8-B tagged
        entries + a bucket table over the first p chars (SAS_BUILD_TAGGED; True = p chosen by
        the library, an int = that p) for algo="tagged"; it replaces the SA and leaves out the
        trees, LLCP and the prefix tables (their defaults turn off).  top2_levels: depth of
        the binary-search pivots (SAS_BUILD_TOP2_LEVELS, rounded up to 4-level prefix-relative
        blocks past the 15 LDS levels; 0 = the library default, 27 levels, 273 MiB; 30 -> all
        31 levels of n = 2^30, 4.3 GiB).
        tag_lines (with tagged): the tagged entries as 128-B bucket lines + an overflow array
        (SAS_BUILD_TAG_LINES; p = ceil(log4 n) - 2 unless tagged gives it): one request gives a
        lookup its bucket and first 20 entries; algo="tagged" only, no SA array."""
        t = _as_u8(t)
        n = int(t.numel() if _is_cuda(t) else len(t))
        if tagged is not False:
            stree, sector, quad, prefix = bool(stree), bool(sector), quad or False, prefix or False
            llcp = bool(llcp)
            flags |= _lib.SAS_BUILD_TAGGED | (0 if tagged is True else _lib.SAS_BUILD_PREFIX_P(int(tagged)))
            flags |= _lib.SAS_BUILD_TAG_LINES if tag_lines else 0
            lcp = lcp and not tag_lines  # a bucket-line index serves TAGGED only: no LCP array
        stree = True if stree is None else stree
        sector = True if sector is None else sector
        quad = True if quad is None else quad
        flags |= (_lib.SAS_BUILD_LCP if lcp else 0) | (_lib.SAS_BUILD_STREE if stree else 0)
        if llcp is None:
            llcp = n < (1 << 31)
        flags |= _lib.SAS_BUILD_LLCP if llcp else 0
        flags |= (_lib.SAS_BUILD_VERIFY if verify else 0) | (_lib.SAS_BUILD_SECTOR if sector else 0)
        flags |= _lib.SAS_BUILD_SA40 if sa40 else 0
        flags |= _lib.SAS_BUILD_TOP2_LEVELS(top2_levels)
        flags |= _quad_flags(quad) | _prefix_flags(prefix, quad, n if rank_range is None else rank_range[1] - rank_range[0],
                                                   prefix_inline)
        sa_ptr, sa_w = None, 4
        if sa is not None:
            if _is_cuda(t) != _is_cuda(sa):
                raise ValueError("text and sa must both be host or both be device arrays")
            if not _is_cuda(sa):
                sa = np.asarray(sa)
                sa = np.ascontiguousarray(sa, np.uint64 if sa.dtype.itemsize == 8 else np.uint32)
                sa_w = sa.dtype.itemsize
            else:
                sa_w = sa.element_size()
            sa_ptr = _ptr(sa)
        if _is_cuda(t):
            flags |= _lib.SAS_DEVICE_PTRS
        h = C.c_void_p()
        if rank_range is None:
            check(lib().sas_build(_ptr(t), n, sa_ptr, sa_w, flags, C.byref(h)))
        else:
            check(lib().sas_build_shard(_ptr(t), n, sa_ptr, sa_w, int(rank_range[0]), int(rank_range[1]), flags,
                                        C.byref(h)))
        return cls(h, n)

    @classmethod
    def build_part(cls, t, part: int, parts: int, lcp: bool = True, stree: bool = True, verify: bool = False,
                   flags: int = 0, sector: bool = True, quad: bool | str = True, llcp: bool | None = None,
                   prefix: bool | int | None = None, prefix_inline: bool | int = False,
                   top2_levels: int = 0) -> "SaNaive":
        """Sharded-text index that builds ONLY its own SA rank range (sas_build_part):
        part `part` of `parts` contiguous 7-char-prefix bin ranges.  The range is
        chosen by the library (stats: rank_lo, sa_entries, next_pos).  prefix_inline as in
        build (inline tables need n < 2^32 beside the part's 40-bit SA)."""
        t = _as_u8(t)
        n = int(t.numel() if _is_cuda(t) else len(t))
        flags |= (_lib.SAS_BUILD_LCP if lcp else 0) | (_lib.SAS_BUILD_STREE if stree else 0)
        flags |= (_lib.SAS_BUILD_VERIFY if verify else 0) | (_lib.SAS_BUILD_SECTOR if sector else 0)
        llcp = (n < (1 << 31)) if llcp is None else llcp
        flags |= _quad_flags(quad) | (_lib.SAS_BUILD_LLCP if llcp else 0) | _prefix_flags(prefix, quad, n, prefix_inline)
        flags |= _lib.SAS_BUILD_TOP2_LEVELS(top2_levels)
        if _is_cuda(t):
            flags |= _lib.SAS_DEVICE_PTRS
        h = C.c_void_p()
        check(lib().sas_build_part(_ptr(t), n, int(part), int(parts), flags, C.byref(h)))
        return cls(h, n)

    @classmethod
    def build_gen(cls, n: int, seed: int = 31415, part: int | None = None, parts: int | None = None,
                  flags: int = 0, **kw) -> "SaNaive":
        """The index over random_string(n, seed) (sas/util.rs:9-15) generated on the GPU
        straight into the packed text (sas_build_gen / sas_build_part_gen): no n-byte text
        exists anywhere.  part/parts: a build_part index; the keyword flags are build's
        (lcp, stree, sector, quad, llcp, prefix, prefix_inline, top2_levels, verify)."""
        lcp, stree = kw.pop("lcp", True), kw.pop("stree", True)
        sector, quad = kw.pop("sector", True), kw.pop("quad", True)
        verify, top2 = kw.pop("verify", False), kw.pop("top2_levels", 0)
        prefix, inline = kw.pop("prefix", None), kw.pop("prefix_inline", False)
        llcp = kw.pop("llcp", None)
        if kw:
            raise TypeError(f"build_gen: unexpected {sorted(kw)}")
        llcp = (n < (1 << 31)) if llcp is None else llcp
        flags |= (_lib.SAS_BUILD_LCP if lcp else 0) | (_lib.SAS_BUILD_STREE if stree else 0)
        flags |= (_lib.SAS_BUILD_VERIFY if verify else 0) | (_lib.SAS_BUILD_SECTOR if sector else 0)
        flags |= _quad_flags(quad) | (_lib.SAS_BUILD_LLCP if llcp else 0) | _prefix_flags(prefix, quad, n, inline)
        flags |= _lib.SAS_BUILD_TOP2_LEVELS(top2)
        h = C.c_void_p()
        if part is None:
            check(lib().sas_build_gen(seed, n, flags, C.byref(h)))
        else:
            check(lib().sas_build_part_gen(seed, n, int(part), int(parts), flags, C.byref(h)))
        return cls(h, n)

    @classmethod
    def build_part_gen(cls, n: int, seed: int = 31415, part: int = 0, parts: int = 1, **kw) -> "SaNaive":
        """build_part over random_string(n, seed) generated on the GPU (sas_build_part_gen)."""
        return cls.build_gen(n, seed=seed, part=part, parts=parts, **kw)

    def free(self):
        if self._h:
            lib().sas_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    # -- introspection (Index<usize> for SaNaive, sas/sa_search.rs:21-27)
    def stats(self) -> dict:
        s = _lib.SasStats()
        check(lib().sas_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    def suffix_array(self, count: int | None = None, start: int = 0) -> np.ndarray:
        """Local SA entries [start, start+count): u32 for a u32 index, u64 for a 40-bit one."""
        count = self.sa_n - start if count is None else count
        if self.stats()["sa_width"] == 4 and start == 0:
            out = np.zeros(max(count, 1), np.uint32)
            check(lib().sas_copy_sa(self._h, out.ctypes.data, count, 0))
            return out[:count]
        out = np.zeros(max(count, 1), np.uint64)
        check(lib().sas_copy_sa64(self._h, self.rank_lo + start, count, out.ctypes.data, 0))
        return out[:count]

    def lcp_array(self) -> np.ndarray:
        out = np.zeros(self.sa_n, np.uint32)
        check(lib().sas_copy_lcp(self._h, out.ctypes.data, self.sa_n, 0))
        return out

    def extract(self, pos, lens, out_off, out, stream=None):
        """Text substrings as byte codes from the index's packed text (sas_extract):
        out[out_off[i] : out_off[i] + lens[i]] = text[pos[i] : pos[i] + lens[i]].
        torch CUDA tensors (int64 pos / out_off, int32 lens, uint8 out), async."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        check(lib().sas_extract(self._h, _ptr(pos), _ptr(lens), _ptr(out_off), int(pos.numel()), _ptr(out), st,
                                _lib.SAS_DEVICE_PTRS))
        return out

    @staticmethod
    def pack_queries(qbytes, m: int, stream=None):
        """2-bit packed fixed-length queries (sas_pack_queries; m <= 32): torch CUDA
        uint8 in -> torch CUDA int64 words out (first char in bits 63..62); numpy uint8 in
        -> numpy uint64 out, packed on the host."""
        if not _is_cuda(qbytes):
            qbytes = _as_u8(qbytes)
            nq = len(qbytes) // m if m else 0
            out = np.zeros(max(nq, 1), np.uint64)
            check(lib().sas_pack_queries(_ptr(qbytes), m, nq, _ptr(out), None, 0))
            return out[:nq]
        import torch
        nq = qbytes.numel() // m if m else 0
        out = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
        st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
        check(lib().sas_pack_queries(_ptr(qbytes), m, nq, _ptr(out), st, _lib.SAS_DEVICE_PTRS))
        return out

    def search_packed(self, qwords, m: int, algo: str = "prefix", probes: bool = False, out=None, stream=None):
        """Lookups of packed fixed-length queries (sas_search_packed): numpy uint64 in ->
        numpy out; torch CUDA in -> torch CUDA out (async)."""
        if _is_cuda(qwords):
            import torch
            nq = qwords.numel()
            out = torch.empty(nq, dtype=torch.int64, device=qwords.device) if out is None else out
            pr = torch.empty(nq, dtype=torch.int32, device=qwords.device) if probes else None
            st = stream if stream is not None else torch.cuda.current_stream(qwords.device).cuda_stream
            check(lib().sas_search_packed(self._h, _ptr(qwords), m, nq, _lib.ALGOS[algo], _ptr(out),
                                          _ptr(pr) if probes else None, st, _lib.SAS_DEVICE_PTRS))
            return (out, pr) if probes else out
        qwords = np.ascontiguousarray(qwords, np.uint64)
        nq = len(qwords)
        out = np.zeros(max(nq, 1), np.uint64)
        pr = np.zeros(max(nq, 1), np.uint32) if probes else None
        check(lib().sas_search_packed(self._h, qwords.ctypes.data, m, nq, _lib.ALGOS[algo], out.ctypes.data,
                                      pr.ctypes.data if probes else None, None, 0))
        return (out[:nq], pr[:nq]) if probes else out[:nq]

    def search_buckets(self, queries, m: int, cap: int, counts, algo: str = "prefix", out=None, stream=None):
        """The sharded step's local lookup (sas_search_buckets): `queries` holds
        counts.numel() buckets of `cap` slots (uint8, m bytes a slot, or int64 2-bit words
        for PREFIX with m <= 32), bucket b's first counts[b] slots are queries; only those
        are searched and written into `out` (int64, one per slot).  torch CUDA tensors."""
        import torch
        dev = queries.device
        for name, tns in (("queries", queries), ("counts", counts)) + ((("out", out),) if out is not None else ()):
            if not tns.is_cuda or tns.device != dev:
                raise ValueError(f"search_buckets: {name} must be a CUDA tensor on {dev}, not {tns.device}")
        nb = int(counts.numel())
        packed = queries.dtype == torch.int64
        need = nb * cap * (1 if packed else m)
        if counts.dtype != torch.int64 or not counts.is_contiguous() or queries.numel() < need or \
                not queries.is_contiguous() or (not packed and queries.dtype != torch.uint8):
            raise ValueError("search_buckets: int64 counts, and uint8 bytes or int64 words for every slot")
        if out is None:
            out = torch.empty(nb * cap, dtype=torch.int64, device=queries.device)
        if out.dtype != torch.int64 or out.numel() < nb * cap:
            raise ValueError("search_buckets: int64 out of one entry per slot")
        st = stream if stream is not None else torch.cuda.current_stream(queries.device).cuda_stream
        fl = _lib.SAS_DEVICE_PTRS | (_lib.SAS_ROUTE_PACKED if packed else 0)
        check(lib().sas_search_buckets(self._h, _ptr(queries), m, nb, int(cap), _ptr(counts), _lib.ALGOS[algo],
                                       _ptr(out), st, fl))
        return out

    def route(self, splitter_pos, qbytes, m: int, stream=None):
        """Sharded mode: shard id of each fixed-length query = number of splitter
        suffixes < q (sas_route).  numpy in -> numpy out; CUDA in -> CUDA out."""
        if _is_cuda(qbytes):
            import torch
            nq = qbytes.numel() // m
            out = torch.empty(nq, dtype=torch.int32, device=qbytes.device)
            st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
            check(lib().sas_route(self._h, splitter_pos.data_ptr(), splitter_pos.numel(), qbytes.data_ptr(), m, nq,
                                  out.data_ptr(), st, _lib.SAS_DEVICE_PTRS))
            return out
        qbytes = _as_u8(qbytes)
        sp = np.ascontiguousarray(splitter_pos, np.uint64)
        nq = len(qbytes) // m
        out = np.zeros(max(nq, 1), np.uint32)
        check(lib().sas_route(self._h, sp.ctypes.data if len(sp) else None, len(sp), qbytes.ctypes.data, m, nq,
                              out.ctypes.data, stream, 0))
        return out[:nq]

    def route_pack(self, splitter_pos, qbytes, m: int, stream=None, cap: int | None = None, send=None,
                   packed: bool = False):
        """Send side of one sharded step, fused on the GPU (sas_route_pack): CUDA
        tensors in -> (counts int64 [W], send uint8 [nq*m] grouped by shard,
        slot int64 [nq] = send position of each query).  cap: fixed-capacity buckets
        (sas_route_pack_cap): send holds W*cap slots, bucket w at slots [w*cap, ...), and
        counts > cap on the device marks an overflow.  packed (m <= 32, SAS_ROUTE_PACKED):
        each slot is the query's 8-B 2-bit word (send is int64) instead of its m bytes.
        `send` may be passed in (reused)."""
        import torch
        nq = qbytes.numel() // m
        W = splitter_pos.numel() + 1
        counts = torch.empty(W, dtype=torch.int64, device=qbytes.device)
        slots = W * cap if cap else nq
        size = slots if packed else slots * m
        dt = torch.int64 if packed else torch.uint8
        if send is None or send.numel() < max(size, 1) or send.dtype != dt:
            send = torch.zeros(max(size, 1), dtype=dt, device=qbytes.device)
        slot = torch.empty(max(nq, 1), dtype=torch.int64, device=qbytes.device)
        st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
        sp = splitter_pos.data_ptr() if W > 1 else None
        fl = _lib.SAS_DEVICE_PTRS | (_lib.SAS_ROUTE_PACKED if packed else 0)
        if cap:
            check(lib().sas_route_pack_cap(self._h, sp, W - 1, qbytes.data_ptr(), m, nq, int(cap), counts.data_ptr(),
                                           send.data_ptr(), slot.data_ptr(), st, fl))
        else:
            check(lib().sas_route_pack(self._h, sp, W - 1, qbytes.data_ptr(), m, nq, counts.data_ptr(),
                                       send.data_ptr(), slot.data_ptr(), st, fl))
        return counts, send[:size], slot[:nq]

    def shard_gather(self, back, slot, out=None, counts=None, cap: int = 0, overflow=None, stream=None):
        """Receive side of one sharded step (sas_shard_gather): out[k] = back[slot[k]]; with
        `overflow` (an int32 CUDA tensor of 1, never cleared here) it is set to 1 when some
        counts[w] > cap."""
        import torch
        nq = slot.numel()
        if out is None:
            out = torch.empty(nq, dtype=torch.int64, device=slot.device)
        if out.numel() < nq or out.dtype != torch.int64 or back.dtype != torch.int64 or slot.dtype != torch.int64:
            raise ValueError("shard_gather: int64 back/slot/out, out of at least len(slot)")
        if overflow is not None and (counts is None or overflow.dtype != torch.int32):
            raise ValueError("shard_gather: overflow needs counts and an int32 flag")
        st = stream if stream is not None else torch.cuda.current_stream(slot.device).cuda_stream
        check(lib().sas_shard_gather(self._h, back.data_ptr(), slot.data_ptr(), nq,
                                     counts.data_ptr() if counts is not None else None,
                                     counts.numel() if counts is not None else 0, int(cap), out.data_ptr(),
                                     overflow.data_ptr() if overflow is not None else None, st,
                                     _lib.SAS_DEVICE_PTRS))
        return out[:nq]

    def verify(self):
        check(lib().sas_verify(self._h))

    # -- searching
    def search_fixed(self, qbytes, m: int, algo: str = "plain", probes: bool = False, stream=None,
                     out=None, flags: int = 0):
        """Fixed-length queries, query k = qbytes[k*m:(k+1)*m].  Host numpy in ->
        numpy out (synchronous); torch CUDA in -> CUDA out (async on `stream`)."""
        dev = _is_cuda(qbytes)
        nq = (qbytes.numel() if dev else len(qbytes)) // max(m, 1) if m else 0
        if m == 0:
            raise ValueError("use search_batch for empty queries")
        return self._run(qbytes, None, None, m, nq, algo, probes, stream, out, flags, dev)

    def search_batch(self, qbytes, qoff, qlen, algo: str = "plain", probes: bool = False, stream=None,
                     out=None, flags: int = 0):
        """Ragged queries, query k = qbytes[qoff[k] : qoff[k] + qlen[k]]."""
        dev = _is_cuda(qbytes)
        if not dev:
            qoff = np.ascontiguousarray(qoff, np.uint64)
            qlen = np.ascontiguousarray(qlen, np.uint32)
        nq = int(qoff.numel() if dev else len(qoff))
        return self._run(qbytes, qoff, qlen, 0, nq, algo, probes, stream, out, flags, dev)

    def search_slices(self, qoff, qlen, algo: str = "tagged", probes: bool = False, stream=None, out=None,
                      flags: int = 0):
        """Queries that are slices of the indexed text, t[qoff[k] : qoff[k] + qlen[k]] (the
        reference's borrowed &t[i..i+len] queries; SAS_QUERIES_ARE_SLICES): torch CUDA int64
        offsets / int32 lengths in, no query bytes -> torch CUDA positions out."""
        import torch
        if not (_is_cuda(qoff) and _is_cuda(qlen)):
            raise ValueError("search_slices: torch CUDA qoff / qlen")
        if qoff.dtype != torch.int64 or qlen.dtype != torch.int32 or not qoff.is_contiguous() or \
                not qlen.is_contiguous() or qoff.numel() != qlen.numel():
            raise ValueError("search_slices: contiguous int64 qoff and int32 qlen of the same length")
        nq = int(qoff.numel())
        if out is None:
            out = torch.empty(nq, dtype=torch.int64, device=qoff.device)
        pr = torch.empty(nq, dtype=torch.int32, device=qoff.device) if probes else None
        st = stream if stream is not None else torch.cuda.current_stream(qoff.device).cuda_stream
        check(lib().sas_search_batch(self._h, None, _ptr(qoff), _ptr(qlen), nq, _lib.ALGOS[algo], _ptr(out),
                                     _ptr(pr), st, flags | _lib.SAS_DEVICE_PTRS | _lib.SAS_QUERIES_ARE_SLICES))
        return (out, pr) if probes else out

    def _run(self, qbytes, qoff, qlen, m, nq, algo, probes, stream, out, flags, dev):
        a = _lib.ALGOS[algo]
        if dev:
            import torch
            if out is None:
                out = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
            pr = torch.empty(nq, dtype=torch.int32, device=qbytes.device) if probes else None
            st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
            flags |= _lib.SAS_DEVICE_PTRS
        else:
            qbytes = _as_u8(qbytes)
            if out is None:
                out = np.zeros(max(nq, 1), np.uint64)
            elif not (isinstance(out, np.ndarray) and out.dtype == np.uint64 and out.flags.c_contiguous
                      and len(out) >= nq):
                raise ValueError("out: a C-contiguous numpy uint64 array of at least nq entries")
            pr = np.zeros(max(nq, 1), np.uint32) if probes else None
            st = stream
        if qoff is None:
            rc = lib().sas_search_fixed(self._h, _ptr(qbytes), m, nq, a, _ptr(out), _ptr(pr), st, flags)
        else:
            rc = lib().sas_search_batch(self._h, _ptr(qbytes), _ptr(qoff), _ptr(qlen), nq, a, _ptr(out), _ptr(pr),
                                        st, flags)
        check(rc)
        if not dev:
            out, pr = out[:nq], (pr[:nq] if pr is not None else None)
        return (out, pr) if probes else out

    def search(self, queries, algo: str = "plain", probes: bool = False):
        """List of byte strings / arrays -> positions (host)."""
        qs = [_as_u8(q) for q in queries]
        lens = np.array([len(q) for q in qs], np.uint32)
        off = np.zeros(len(qs), np.uint64)
        if len(qs):
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        buf = np.concatenate(qs + [np.zeros(64, np.uint8)]) if qs else np.zeros(64, np.uint8)
        return self.search_batch(buf, off, lens, algo=algo, probes=probes)

    def search_range(self, qbytes, qoff, qlen, stream=None, flags: int = 0):
        """Occurrence ranges (Search::search_prefix, sas/util.rs:36-40): global SA
        ranks (lo, hi) of the suffixes starting with each query; count = hi - lo."""
        dev = _is_cuda(qbytes)
        if dev:
            import torch
            nq = qoff.numel()
            lo = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
            hi = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
            st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
            flags |= _lib.SAS_DEVICE_PTRS
        else:
            qbytes = _as_u8(qbytes)
            qoff = np.ascontiguousarray(qoff, np.uint64)
            qlen = np.ascontiguousarray(qlen, np.uint32)
            nq = len(qoff)
            lo = np.zeros(max(nq, 1), np.uint64)
            hi = np.zeros(max(nq, 1), np.uint64)
            st = stream
        check(lib().sas_search_range(self._h, _ptr(qbytes), _ptr(qoff), _ptr(qlen), nq, _ptr(lo), _ptr(hi), st,
                                     flags))
        return (lo, hi) if dev else (lo[:nq], hi[:nq])

    def search_range_fixed(self, qbytes, m: int, stream=None, flags: int = 0):
        """search_range for fixed-length queries qbytes[k*m .. (k+1)*m) (sas_search_range_fixed)."""
        dev = _is_cuda(qbytes)
        nq = qbytes.numel() // m if dev else len(qbytes) // m
        if dev:
            import torch
            lo = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
            hi = torch.empty(nq, dtype=torch.int64, device=qbytes.device)
            st = stream if stream is not None else torch.cuda.current_stream(qbytes.device).cuda_stream
            flags |= _lib.SAS_DEVICE_PTRS
        else:
            qbytes = _as_u8(qbytes)
            lo = np.zeros(max(nq, 1), np.uint64)
            hi = np.zeros(max(nq, 1), np.uint64)
            st = stream
        check(lib().sas_search_range_fixed(self._h, _ptr(qbytes), m, nq, _ptr(lo), _ptr(hi), st, flags))
        return (lo, hi) if dev else (lo[:nq], hi[:nq])

    def search_prefix(self, q) -> np.ndarray:
        """All text positions where q occurs (Search::search_prefix, sas/util.rs:36-40)."""
        q = _as_u8(q)
        buf = np.concatenate([q, np.zeros(64, np.uint8)])
        lo, hi = self.search_range(buf, np.zeros(1, np.uint64), np.array([len(q)], np.uint32))
        cnt = int(hi[0] - lo[0])
        if self.stats()["sa_width"] != 4:
            out = np.zeros(max(cnt, 1), np.uint64)
            check(lib().sas_copy_sa64(self._h, int(lo[0]), cnt, out.ctypes.data, 0))
            return out[:cnt]
        out = np.zeros(max(cnt, 1), np.uint32)
        check(lib().sas_copy_sa_range(self._h, int(lo[0]), cnt, out.ctypes.data, 0))
        return out[:cnt]

    def time_fixed(self, d_qbytes, m: int, nq: int, d_out, algo="plain", reps=1, stream=None, flags=0):
        """Average (kernel_ns, call_ns) of `reps` back-to-back searches on device buffers."""
        kn, cn = C.c_double(0), C.c_double(0)
        check(lib().sas_time_fixed(self._h, _ptr(d_qbytes), m, nq, _lib.ALGOS[algo], _ptr(d_out), reps, stream,
                                   flags, C.byref(kn), C.byref(cn)))
        return kn.value, cn.value


def binary_search(sa: SaNaive, q, cnt: Counter | None = None) -> int:
    """sas/sa_search.rs:98-112 -- position of the first suffix >= q (n if none)."""
    pos, pr = sa.search([q], algo="plain", probes=True)
    if cnt is not None:
        cnt.value += int(pr[0])
    return int(pos[0])


def binary_search_batch(sa: SaNaive, qs, cnt: Counter | None = None, algo: str = "plain") -> list[int]:
    """sas/sa_search.rs:157-196 -- B queries at once (any B; no remainder is dropped)."""
    pos, pr = sa.search(list(qs), algo=algo, probes=True)
    if cnt is not None:
        cnt.value += int(pr.sum())
    return [int(p) for p in pos]


# ---------------------------------------------------------------- generators
def random_string(n: int, seed: int = 31415, device=None):
    """sas/util.rs:9-15 with ChaCha8Rng::seed_from_u64(seed): bit-exact stream."""
    if device is not None:
        import torch
        out = torch.empty(n, dtype=torch.uint8, device=device)
        check(lib().sas_gen_text(seed, n, out.data_ptr(), _lib.SAS_DEVICE_PTRS))
        return out
    out = np.zeros(max(n, 1), np.uint8)
    check(lib().sas_gen_text(seed, n, out.ctypes.data, 0))
    return out[:n]


def random_queries(n: int, nq: int, seed: int = 31415, word_pos: int | None = None, margin: int = 200,
                   len_lo: int = 30, len_hi: int = 100):
    """sas/util.rs:18-26 -> (offsets u64, lengths u32, next keystream word).  The
    stream continues after the text's n words unless word_pos is given."""
    off = np.zeros(max(nq, 1), np.uint64)
    ln = np.zeros(max(nq, 1), np.uint32)
    nxt = C.c_uint64(0)
    check(lib().sas_gen_queries(seed, n if word_pos is None else word_pos, n, nq, margin, len_lo, len_hi,
                                off.ctypes.data, ln.ctypes.data, C.byref(nxt)))
    return off[:nq], ln[:nq], nxt.value


# ---------------------------------------------------------------- real data
def read_fasta_file(path: str) -> np.ndarray:
    """sas/util.rs:144-169: concatenated record sequences as codes 0..3 (others -> 0)."""
    n = C.c_uint64(0)
    check(lib().sas_read_fasta(path.encode(), None, 0, C.byref(n)))
    out = np.zeros(max(n.value, 1), np.uint8)
    check(lib().sas_read_fasta(path.encode(), out.ctypes.data, n.value, C.byref(n)))
    return out[: n.value]


def kmer_keys(t, k: int = 16, limit: int | None = None) -> np.ndarray:
    """sst/bin/bench.rs:58-76 (--human): u32 k-mer keys & i32::MAX, vals[0] = MAX."""
    t = _as_u8(t)
    n = len(t)
    limit = n if limit is None else limit
    cnt = C.c_uint64(0)
    check(lib().sas_kmer_keys(t.ctypes.data, n, k, limit, None, C.byref(cnt), 0))
    out = np.zeros(max(cnt.value, 1), np.uint32)
    check(lib().sas_kmer_keys(t.ctypes.data, n, k, limit, out.ctypes.data, C.byref(cnt), 0))
    return out[: cnt.value]
