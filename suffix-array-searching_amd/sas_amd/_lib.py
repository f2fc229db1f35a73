"""ctypes binding of libsas_amd.so (the C ABI declared in include/sas.h and include/sst.h).

The product path has no fallback: if the HIP library is missing this module raises,
so nothing silently runs on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # suffix-array-searching_amd/
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libsas_amd.so")
HEADERS = [os.path.join(REPO_DIR, "include", "sas.h"), os.path.join(REPO_DIR, "include", "sst.h")]

# flags / enums mirrored from include/sas.h and include/sst.h
SAS_DEVICE_PTRS = 1 << 0
SAS_BUILD_LCP = 1 << 1
SAS_BUILD_STREE = 1 << 2
SAS_BUILD_VERIFY = 1 << 3
SAS_NO_LDS_TOP = 1 << 4
SAS_VALIDATE = 1 << 5
SAS_PREFIX_RANGE = 1 << 24
SAS_NO_PREFIX_TABLE = 1 << 25
SAS_RANGE_NO_INLINE = 1 << 27
SAS_QUERIES_ARE_SLICES = 1 << 28
SAS_ROUTE_PACKED = 1 << 26
SAS_BUILD_WIDE = 1 << 6
SAS_BUILD_SECTOR = 1 << 7
SAS_BUILD_SA40 = 1 << 8
SAS_BUILD_QUAD = 1 << 9
SAS_BUILD_QUAD_COMPACT = 1 << 10
SAS_BUILD_QUAD_ABS = 1 << 11
SAS_BUILD_QUAD_REL = 1 << 12
SAS_BUILD_LLCP = 1 << 13
SAS_BUILD_PREFIX = 1 << 14
SAS_BUILD_PREFIX_INLINE = 1 << 15
SAS_BUILD_PREFIX_INLINE2 = 1 << 21
SAS_BUILD_PREFIX_INLINE4 = 1 << 22
SAS_BUILD_TAGGED = 1 << 23
SAS_BUILD_TAG_LINES = 1 << 24


def SAS_BUILD_TOP2_LEVELS(levels: int) -> int:
    """Depth of the binary-search pivot array (sas.h SAS_BUILD_TOP2_LEVELS; 0 = default 23)."""
    if not 0 <= int(levels) <= 31:
        raise ValueError(f"top2_levels must be in 0..31, not {levels}")
    return int(levels) << 27


def SAS_BUILD_PREFIX_P(p: int) -> int:
    return (int(p) & 31) << 16


SAS_MULTI_REPLICATE, SAS_MULTI_SHARD = 0, 1
ALGOS = {"plain": 0, "lcp": 1, "stree": 2, "sector": 3, "quad": 4, "inline": 5, "llcp": 6, "prefix": 7,
         "interp": 8, "tagged": 9, "stree_llcp": 10, "quad_llcp": 11}

SST_SORTED, SST_EYTZINGER, SST_STREE16, SST_STREE15, SST_PARTITIONED_MAP, SST_DIRECT_MAP = 0, 1, 2, 3, 4, 5
SST_PARTITIONED, SST_PARTITIONED_COMPACT, SST_PARTITIONED_L1, SST_PARTITIONED_OVERLAP = 6, 7, 8, 9
SST_LEFT_MAX = 1 << 0
SST_REVERSE = 1 << 1
SST_FULL = 1 << 2
SST_DEVICE_PTRS = 1 << 8
SST_NO_LDS_TOP = 1 << 9


class SasStats(C.Structure):
    _fields_ = [
        ("n", C.c_uint64), ("text_bytes", C.c_uint64), ("sa_bytes", C.c_uint64), ("lcp_bytes", C.c_uint64),
        ("stree_bytes", C.c_uint64), ("stree_layers", C.c_uint32), ("stree_lds_layers", C.c_uint32),
        ("top_levels", C.c_uint32), ("iterations", C.c_uint32), ("build_sa_ns", C.c_uint64),
        ("build_total_ns", C.c_uint64), ("sa_rounds", C.c_uint32), ("sa_width", C.c_uint32),
        ("rank_lo", C.c_uint64), ("sa_entries", C.c_uint64), ("next_pos", C.c_uint64),
        ("sector_bytes", C.c_uint64), ("sector_layers", C.c_uint32), ("sector_lds_layers", C.c_uint32),
        ("quad_bytes", C.c_uint64), ("quad_layers", C.c_uint32), ("quad_lds_layers", C.c_uint32),
        ("quad_entry_bytes", C.c_uint32),
        ("quad_fan", C.c_uint32), ("top2_levels", C.c_uint32), ("llcp_bytes", C.c_uint64),
        ("prefix_bytes", C.c_uint64), ("prefix_chars", C.c_uint32), ("tag_chars", C.c_uint32),
        ("tag_table_bytes", C.c_uint64), ("index_bytes", C.c_uint64),
        ("tag_line_slots", C.c_uint32), ("tag_line_tag_bits", C.c_uint32), ("tag_overflow_entries", C.c_uint64),
        ("text2_bytes", C.c_uint64), ("top2_bytes", C.c_uint64),
        ("rel_levels", C.c_uint32), ("rel_pad", C.c_uint32), ("rel_bytes", C.c_uint64),
        ("prefix_key_lo", C.c_uint64), ("prefix_entries", C.c_uint64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class SasError(RuntimeError):
    """A non-zero status from the C ABI (the reference panics in these cases)."""

    def __init__(self, code, msg):
        super().__init__(f"{msg} (errno {code})")
        self.code = code


_LIB = None


def build_library() -> str:
    subprocess.check_call(["make", "-s", "-C", PKG_DIR])
    return LIB_PATH


def declared_symbols() -> list[str]:
    """Every function the public headers declare."""
    names = []
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*\b((?:sas|sst)_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP extension {LIB_PATH} is missing: run __graft_entry__.build() "
                          f"(there is no CPU fallback)")
    # PyTorch-ROCm bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1.  Load it
    # first so the dynamic linker resolves our NEEDED entries to the same runtime:
    # two HIP runtimes in one process cannot share device pointers or streams.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    L.sas_last_error.restype = C.c_char_p
    L.sas_build.argtypes = [vp, u64, vp, i32, u32, C.POINTER(vp)]
    L.sas_free.argtypes = [vp]
    L.sas_build_shard.argtypes = [vp, u64, vp, i32, u64, u64, u32, C.POINTER(vp)]
    L.sas_build_part.argtypes = [vp, u64, u32, u32, u32, C.POINTER(vp)]
    L.sas_build_gen.argtypes = [u64, u64, u32, C.POINTER(vp)]
    L.sas_build_part_gen.argtypes = [u64, u64, u32, u32, u32, C.POINTER(vp)]
    L.sas_route.argtypes = [vp, vp, u32, vp, u32, u64, vp, vp, u32]
    L.sas_route_pack.argtypes = [vp, vp, u32, vp, u32, u64, vp, vp, vp, vp, u32]
    L.sas_route_pack_cap.argtypes = [vp, vp, u32, vp, u32, u64, u64, vp, vp, vp, vp, u32]
    L.sas_shard_gather.argtypes = [vp, vp, vp, u64, vp, u32, u64, vp, vp, vp, u32]
    L.sas_search_buckets.argtypes = [vp, vp, u32, u32, u64, vp, i32, vp, vp, u32]
    L.sas_source_hash.restype = C.c_char_p
    L.sas_route_batch.argtypes = [vp, vp, u32, vp, vp, vp, u64, vp, vp, u32]
    L.sas_build_multi.argtypes = [vp, u64, vp, i32, i32, u32, C.POINTER(vp)]
    L.sas_extract.argtypes = [vp, vp, vp, vp, u64, vp, vp, u32]
    L.sas_pack_queries.argtypes = [vp, u32, u64, vp, vp, u32]
    L.sas_search_packed.argtypes = [vp, vp, u32, u64, i32, vp, vp, vp, u32]
    L.sas_multi_free.argtypes = [vp]
    L.sas_multi_parts.argtypes = [vp]
    L.sas_multi_get_stats.argtypes = [vp, i32, C.POINTER(SasStats)]
    L.sas_search_multi.argtypes = [vp, vp, vp, vp, u64, i32, vp, u32]
    L.sas_get_stats.argtypes = [vp, C.POINTER(SasStats)]
    L.sas_copy_sa.argtypes = [vp, vp, u64, u32]
    L.sas_copy_lcp.argtypes = [vp, vp, u64, u32]
    L.sas_search_range.argtypes = [vp, vp, vp, vp, u64, vp, vp, vp, u32]
    L.sas_search_range_fixed.argtypes = [vp, vp, u32, u64, vp, vp, vp, u32]
    L.sas_copy_sa_range.argtypes = [vp, u64, u64, vp, u32]
    L.sas_copy_sa64.argtypes = [vp, u64, u64, vp, u32]
    L.sas_read_fasta.argtypes = [C.c_char_p, vp, u64, C.POINTER(u64)]
    L.sas_kmer_keys.argtypes = [vp, u64, u32, u64, vp, C.POINTER(u64), u32]
    L.sas_verify.argtypes = [vp]
    L.sas_search_batch.argtypes = [vp, vp, vp, vp, u64, i32, vp, vp, vp, u32]
    L.sas_search_fixed.argtypes = [vp, vp, u32, u64, i32, vp, vp, vp, u32]
    L.sas_time_fixed.argtypes = [vp, vp, u32, u64, i32, vp, i32, vp, u32, C.POINTER(C.c_double),
                                 C.POINTER(C.c_double)]
    L.sas_gen_text.argtypes = [u64, u64, vp, u32]
    L.sas_gen_queries.argtypes = [u64, u64, u64, u64, u64, u32, u32, vp, vp, C.POINTER(u64)]
    L.sst_build.argtypes = [vp, u64, i32, u32, C.POINTER(vp)]
    L.sst_free.argtypes = [vp]
    L.sst_size.argtypes = [vp]
    L.sst_size.restype = u64
    L.sst_layers.argtypes = [vp]
    L.sst_layers.restype = u64
    L.sst_query.argtypes = [vp, vp, u64, vp, vp, vp, u32]
    L.sst_copy_nodes.argtypes = [vp, vp, u64]
    L.sst_time_query.argtypes = [vp, vp, u64, vp, i32, vp, u32, C.POINTER(C.c_double)]
    _LIB = L
    return L


def check(rc: int):
    if rc != 0:
        raise SasError(rc, lib().sas_last_error().decode())


def source_hash() -> str:
    """The source hash compiled into the loaded libsas_amd.so (sas_source_hash)."""
    return lib().sas_source_hash().decode()
