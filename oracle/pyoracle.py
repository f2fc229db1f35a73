"""ctypes front-end to oracle/liboracle.so (the CPU restatement of the reference).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
`cpu_baseline` leg of bench.py -- never by the product package.  Each wrapper
names the reference function it restates (see sa_oracle.c for file:line).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")

PAD = 256  # zero bytes after the text (reference pads 200, sas/main.rs:56-58)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_chacha_block.argtypes = [u32p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, u32p]
        L.orc_seed_from_u64.argtypes = [C.c_uint64, u32p]
        L.orc_random_string.argtypes = [C.c_uint64, C.c_uint64, u8p]
        L.orc_random_queries.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                         C.c_uint32, C.c_uint32, u64p, u32p]
        L.orc_random_queries.restype = C.c_uint64
        L.orc_build_sa.argtypes = [u8p, C.c_uint64, u32p]
        L.orc_check_sa.argtypes = [u8p, C.c_uint64, u32p]
        L.orc_kasai_lcp.argtypes = [u8p, C.c_uint64, u32p, u32p]
        for f in ("orc_binary_search", "orc_binary_search_cmp", "orc_branchy_search", "orc_branchfree_search"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_uint64, u32p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
            getattr(L, f).restype = C.c_uint64
        L.orc_interpolation_search.argtypes = [C.c_void_p, C.c_uint64, u32p, C.c_void_p, C.c_uint64, C.c_int,
                                               C.POINTER(C.c_uint64)]
        L.orc_interpolation_search.restype = C.c_uint64
        L.orc_lower_bound_rank.argtypes = [C.c_void_p, C.c_uint64, u32p, C.c_void_p, C.c_uint64]
        L.orc_lower_bound_rank.restype = C.c_uint64
        L.orc_prefix_range.argtypes = [C.c_void_p, C.c_uint64, u32p, C.c_void_p, C.c_uint64,
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_search_many.argtypes = [u8p, C.c_uint64, u32p, u8p, u64p, u32p, C.c_uint64, C.c_int, u64p, C.c_int]
        L.orc_search_many.restype = C.c_uint64
        L.orc_node_find.argtypes = [u32p, C.c_uint32, C.c_uint32]
        L.orc_node_find.restype = C.c_uint32
        L.orc_stree_dims.argtypes = [C.c_uint64, C.c_uint32, C.c_int, u64p, C.POINTER(C.c_uint64)]
        L.orc_stree_dims.restype = C.c_uint32
        L.orc_stree_build.argtypes = [u32p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, u32p, u64p]
        L.orc_stree_query.argtypes = [u32p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, u32p, C.c_uint64, u32p, C.c_void_p]
        L.orc_stree_batch_mt.argtypes = [u32p, u64p, C.c_uint32, C.c_uint32, u32p, C.c_uint64, u32p, C.c_uint32]
        L.orc_eytzinger_build.argtypes = [u32p, C.c_uint64, u32p]
        L.orc_eytzinger_query.argtypes = [u32p, C.c_uint64, u32p, C.c_uint64, C.c_int, u32p]
        L.orc_sorted_query.argtypes = [u32p, C.c_uint64, u32p, C.c_uint64, u32p, C.c_void_p]
        _LIB = L
    return _LIB


# --------------------------------------------------------------------------- generators
def chacha_block(key, w12, w13, w14, w15, rounds=20):
    out = np.zeros(16, np.uint32)
    lib().orc_chacha_block(np.ascontiguousarray(key, np.uint32), w12, w13, w14, w15, rounds, out)
    return out


def random_string(n: int, seed: int = 31415) -> np.ndarray:
    """sas/util.rs:9-15 with ChaCha8Rng::seed_from_u64(seed) (sas/main.rs:38)."""
    out = np.zeros(n, np.uint8)
    lib().orc_random_string(seed, n, out)
    return out


def random_queries(n_text: int, nq: int, seed: int = 31415, word_pos: int | None = None,
                   margin: int = 200, len_lo: int = 30, len_hi: int = 100):
    """sas/util.rs:18-26 (offsets, lengths); the RNG stream continues after the text."""
    off = np.zeros(nq, np.uint64)
    ln = np.zeros(nq, np.uint32)
    pos = lib().orc_random_queries(seed, n_text if word_pos is None else word_pos, n_text, nq,
                                   margin, len_lo, len_hi, off, ln)
    return off, ln, pos


# --------------------------------------------------------------------------- suffix array
def padded(text: np.ndarray) -> np.ndarray:
    """Text followed by PAD zero bytes, as sas/main.rs:56-58 does."""
    buf = np.zeros(len(text) + PAD, np.uint8)
    buf[: len(text)] = text
    return buf


def build_sa(text: np.ndarray) -> np.ndarray:
    t = np.ascontiguousarray(text, np.uint8)
    sa = np.zeros(max(len(t), 1), np.uint32)
    rc = lib().orc_build_sa(t if len(t) else np.zeros(1, np.uint8), len(t), sa)
    assert rc == 0
    return sa[: len(t)]


def check_sa(text: np.ndarray, sa: np.ndarray) -> int:
    return lib().orc_check_sa(np.ascontiguousarray(text, np.uint8), len(text), np.ascontiguousarray(sa, np.uint32))


def kasai_lcp(text: np.ndarray, sa: np.ndarray) -> np.ndarray:
    lcp = np.zeros(max(len(sa), 1), np.uint32)
    lib().orc_kasai_lcp(np.ascontiguousarray(text, np.uint8), len(text), np.ascontiguousarray(sa, np.uint32), lcp)
    return lcp[: len(sa)]


_SINGLE = {
    "binary_search": "orc_binary_search",          # sas/sa_search.rs:98-112 (canonical)
    "binary_search_cmp": "orc_binary_search_cmp",  # :121-136
    "branchy_search": "orc_branchy_search",        # :138-155
    "branchfree_search": "orc_branchfree_search",  # :241-252
}


def search_one(tpad: np.ndarray, n: int, sa: np.ndarray, q: np.ndarray, fn: str = "binary_search"):
    """One query through a restated sa_search.rs function; returns (pos, cnt).
    `tpad` must carry >= 16 zero bytes after n (reference padding)."""
    qb = np.zeros(len(q) + 32, np.uint8)
    qb[: len(q)] = q
    cnt = C.c_uint64(0)
    pos = getattr(lib(), _SINGLE[fn])(tpad.ctypes.data, n, sa, qb.ctypes.data, len(q), C.byref(cnt))
    return int(pos), int(cnt.value)


def lower_bound_rank(tpad, n, sa, q) -> int:
    qb = np.zeros(len(q) + 32, np.uint8)
    qb[: len(q)] = q
    return int(lib().orc_lower_bound_rank(tpad.ctypes.data, n, sa, qb.ctypes.data, len(q)))


def prefix_range(tpad, n, sa, q):
    """Ranks [lo, hi) of the suffixes starting with q (Search::search_prefix,
    sas/util.rs:36-40)."""
    qb = np.zeros(len(q) + 32, np.uint8)
    qb[: len(q)] = q
    lo, hi = C.c_uint64(0), C.c_uint64(0)
    lib().orc_prefix_range(tpad.ctypes.data, n, np.ascontiguousarray(sa, np.uint32), qb.ctypes.data, len(q),
                           C.byref(lo), C.byref(hi))
    return lo.value, hi.value


SEARCH_ALGOS = {"binary_search": 0, "binary_search_cmp": 1, "batch_c16": 2, "batch16": 3, "interpolation16": 4}


def interpolation_search(tpad, n, sa, q, K: int = 16):
    """sas/sa_search.rs:376-421 interpolation_search<K> -> (pos, cnt); q zero padded."""
    qb = np.zeros(len(q) + 64, np.uint8)
    qb[: len(q)] = q
    cnt = C.c_uint64(0)
    pos = lib().orc_interpolation_search(tpad.ctypes.data, n, np.ascontiguousarray(sa, np.uint32), qb.ctypes.data,
                                         len(q), K, C.byref(cnt))
    return int(pos), int(cnt.value)


def search_many(tpad, n, sa, qbytes, qoff, qlen, algo="binary_search", threads=1):
    """Contiguous-chunk multi-threaded driver (sst/bin/bench.rs:558-573).
    qbytes must carry >= 16 readable bytes after the last query."""
    nq = len(qoff)
    out = np.zeros(max(nq, 1), np.uint64)
    cnt = lib().orc_search_many(tpad, n, np.ascontiguousarray(sa, np.uint32), qbytes,
                                np.ascontiguousarray(qoff, np.uint64), np.ascontiguousarray(qlen, np.uint32),
                                nq, SEARCH_ALGOS[algo], out, threads)
    return out[:nq], int(cnt)


# --------------------------------------------------------------------------- static search tree
MAX = 0x7FFFFFFF  # sst/node.rs:5


def node_find(node, q) -> int:
    node = np.ascontiguousarray(node, np.uint32)
    return int(lib().orc_node_find(node, len(node), q))


class STree:
    """Restatement of sst/s_tree.rs STree<B,N> (new_params + search)."""

    def __init__(self, vals, B=16, N=16, left_max=False, reverse=False, full=False):
        vals = np.ascontiguousarray(vals, np.uint32)
        ls = np.zeros(64, np.uint64)
        nb = C.c_uint64(0)
        self.height = lib().orc_stree_dims(len(vals), B, int(full), ls, C.byref(nb))
        self.layer_sizes = ls[: self.height].copy()
        self.n_blocks = nb.value
        self.tree = np.zeros(self.n_blocks * N, np.uint32)
        self.offsets = np.zeros(64, np.uint64)
        rc = lib().orc_stree_build(vals, len(vals), B, N, int(left_max), int(reverse), int(full), self.tree, self.offsets)
        assert rc == 0, "STree::new_params assertion failed"
        self.B, self.N = B, N

    def nodes(self):
        return self.tree.reshape(-1, self.N)

    def query_batch(self, qs, threads: int = 1):
        """batch_final::<128> restatement (sst/s_tree.rs:303-326) over contiguous
        per-thread chunks (sst/bin/bench.rs:558-573); same results as query()."""
        assert self.N == 16
        qs = np.ascontiguousarray(qs, np.uint32)
        out = np.zeros(max(len(qs), 1), np.uint32)
        lib().orc_stree_batch_mt(self.tree, self.offsets, self.height, self.B, qs, len(qs), out, threads)
        return out[: len(qs)]

    def query(self, qs, want_rank=False):
        qs = np.ascontiguousarray(qs, np.uint32)
        out = np.zeros(max(len(qs), 1), np.uint32)
        rank = np.zeros(max(len(qs), 1), np.uint64) if want_rank else None
        lib().orc_stree_query(self.tree, self.offsets, self.height, self.B, self.N, qs, len(qs), out,
                              rank.ctypes.data if want_rank else None)
        return (out[: len(qs)], rank[: len(qs)]) if want_rank else out[: len(qs)]


class Eytzinger:
    """Restatement of sst/eytzinger.rs."""

    def __init__(self, vals):
        vals = np.ascontiguousarray(vals, np.uint32)
        self.n = len(vals)
        self.vals = np.zeros(self.n + 1, np.uint32)
        lib().orc_eytzinger_build(vals, self.n, self.vals)

    def query(self, qs, branchless=False):
        qs = np.ascontiguousarray(qs, np.uint32)
        out = np.zeros(max(len(qs), 1), np.uint32)
        lib().orc_eytzinger_query(self.vals, self.n, qs, len(qs), int(branchless), out)
        return out[: len(qs)]


class SortedVec:
    """Restatement of sst/binary_search.rs SortedVec::binary_search (the test oracle)."""

    def __init__(self, vals):
        self.vals = np.ascontiguousarray(vals, np.uint32)

    def query(self, qs, want_rank=False):
        qs = np.ascontiguousarray(qs, np.uint32)
        out = np.zeros(max(len(qs), 1), np.uint32)
        rank = np.zeros(max(len(qs), 1), np.uint64) if want_rank else None
        lib().orc_sorted_query(self.vals, len(self.vals), qs, len(qs), out,
                               rank.ctypes.data if want_rank else None)
        return (out[: len(qs)], rank[: len(qs)]) if want_rank else out[: len(qs)]
