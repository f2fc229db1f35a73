"""CPU checks of the drop-in boundary: libsas_amd.so loads, exports exactly what
include/*.h declares, and its host-only entry points agree with the oracle.
(No kernel is launched here: this container has no GPU.)"""
import ctypes as C
import os

import numpy as np
import pytest

import sas_amd
from sas_amd import _lib
from oracle import pyoracle as O


def test_library_exports_every_declared_symbol():
    names = _lib.declared_symbols()
    assert len(names) >= 19
    L = C.CDLL(_lib.LIB_PATH)
    missing = [s for s in names if not hasattr(L, s)]
    assert not missing, missing
    for must in ("sas_build", "sas_search_batch", "sas_search_fixed", "sst_build", "sst_query", "sst_size",
                 "sst_layers", "sas_last_error"):
        assert must in names


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_gen_queries_matches_oracle():
    n = 1 << 20
    off, ln, nxt = sas_amd.random_queries(n, 5000)
    o_off, o_ln, o_nxt = O.random_queries(n, 5000)
    assert np.array_equal(off, o_off) and np.array_equal(ln, o_ln) and nxt == o_nxt
    off, ln, nxt = sas_amd.random_queries(n, 777, word_pos=12345, margin=256, len_lo=8, len_hi=257)
    o_off, o_ln, o_nxt = O.random_queries(n, 777, word_pos=12345, margin=256, len_lo=8, len_hi=257)
    assert np.array_equal(off, o_off) and np.array_equal(ln, o_ln) and nxt == o_nxt


def test_error_paths_set_last_error():
    L = _lib.lib()
    off = np.zeros(4, np.uint64)
    ln = np.zeros(4, np.uint32)
    rc = L.sas_gen_queries(1, 0, 100, 4, 200, 30, 100, off.ctypes.data, ln.ctypes.data, None)
    assert rc == 22  # EINVAL: gen_range(0..n-200) empty
    assert b"margin" in L.sas_last_error()
    with pytest.raises(sas_amd.SasError):
        sas_amd.random_queries(100, 4)
    # null out pointers are rejected before any device call
    assert L.sas_build(None, 10, None, 4, 0, None) == 22
    assert L.sst_build(None, 0, 0, 0, None) == 22


def _fasta_restated(text: str) -> list:
    # sas/util.rs:144-169: map[A,C,G,T,a,c,g,t] = 0..3, every other byte 0; records concatenated
    m = {c: i for i, c in enumerate("ACGT")}
    m.update({c: i for i, c in enumerate("acgt")})
    out = []
    for line in text.splitlines():
        if line.startswith(">"):
            continue
        out += [m.get(ch, 0) for ch in line.strip("\r")]
    return out


def test_read_fasta(tmp_path):
    text = ">chr1 test\nACGTNNacgt\nRYKM\n>chr2\n\nTTTTGGGGCCCCAAAA\r\nacg\n"
    p = tmp_path / "x.fa"
    p.write_text(text)
    got = sas_amd.read_fasta_file(str(p))
    assert got.tolist() == _fasta_restated(text)
    q = tmp_path / "x.fq"
    q.write_text("@r1\nACGTN\n+\nIIIII\n@r2\ngggt\n+\n!!!!\n")
    assert sas_amd.read_fasta_file(str(q)).tolist() == [0, 1, 2, 3, 0, 2, 2, 2, 3]
    import gzip
    g = tmp_path / "x.fa.gz"
    g.write_bytes(gzip.compress(text.encode()))
    with pytest.raises(sas_amd.SasError):
        sas_amd.read_fasta_file(str(g))
    with pytest.raises(sas_amd.SasError):
        sas_amd.read_fasta_file(str(tmp_path / "missing.fa"))


def test_quad_layout_flags():
    """Python mirror of the quad build flags (include/sas.h): leaves and inner layout."""
    from sas_amd.sa import _quad_flags
    assert _quad_flags(False) == 0
    assert _quad_flags(True) == _lib.SAS_BUILD_QUAD
    assert _quad_flags("compact") == _lib.SAS_BUILD_QUAD_COMPACT
    assert _quad_flags("abs") == _lib.SAS_BUILD_QUAD | _lib.SAS_BUILD_QUAD_ABS
    assert _quad_flags("rel") == _lib.SAS_BUILD_QUAD | _lib.SAS_BUILD_QUAD_REL
    assert _quad_flags("compact-rel") == _lib.SAS_BUILD_QUAD_COMPACT | _lib.SAS_BUILD_QUAD_REL
    for bad in ("wide", "compact-x", 1, None):
        with pytest.raises(ValueError):
            _quad_flags(bad)
    hdr = open(os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "include", "sas.h")).read()
    for name in ("SAS_BUILD_QUAD_ABS", "SAS_BUILD_QUAD_REL"):
        assert f"#define {name} (1u << {getattr(_lib, name).bit_length() - 1})" in hdr


def test_flag_and_algo_mirror_matches_header():
    """Every single-bit #define in include/sas.h has its _lib mirror with the same value,
    and the algorithm names map to the sas_algo enum."""
    import re
    hdr = open(os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "include", "sas.h")).read()
    defs = dict(re.findall(r"^#define (SAS_[A-Z0-9_]+)\s+\(1u << (\d+)\)", hdr, re.M))
    assert len(defs) >= 15
    for name, bit in defs.items():
        assert getattr(_lib, name) == 1 << int(bit), name
    enum = dict(re.findall(r"SAS_ALGO_([A-Z_]+)\s*=\s*(\d+)", hdr))
    assert {k.lower(): int(v) for k, v in enum.items()} == _lib.ALGOS
    assert _lib.SAS_BUILD_PREFIX_P(17) == 17 << 16


def test_stats_struct_matches_header():
    """ctypes SasStats lists the fields of sas_stats in include/sas.h, in order."""
    import re
    hdr = open(os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "include", "sas.h")).read()
    body = hdr[hdr.index("typedef struct sas_stats {"):hdr.index("} sas_stats;")]
    fields = re.findall(r"^\s*uint(?:32|64)_t\s+(\w+);", body, re.M)
    assert fields == [f for f, _ in _lib.SasStats._fields_]


def test_rust_stats_mirror_matches_header():
    """INTEGRATION.md's Rust `SasStats` declares the fields of sas_stats, in order and with
    their widths (u32 / u64), so a binding built from it reads the struct the library fills."""
    import re
    root = os.path.join(os.path.dirname(_lib.LIB_PATH), "..")
    hdr = open(os.path.join(root, "include", "sas.h")).read()
    body = hdr[hdr.index("typedef struct sas_stats {"):hdr.index("} sas_stats;")]
    c_fields = re.findall(r"^\s*uint(32|64)_t\s+(\w+);", body, re.M)
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    rs = doc[doc.index("pub struct SasStats {"):]
    rs = rs[:rs.index("\n}")]
    rust_fields = re.findall(r"pub (\w+): u(32|64)", rs)
    assert [(w, f) for f, w in rust_fields] == c_fields


def test_pmc_summaries_match_the_built_library():
    """Every committed PMC summary the bench attaches (profiles/pmc_*.json) was collected on the
    library this tree builds: a kernel edit after the PMC sweep would leave the line's traffic
    and request fractions stale (the bench reports them as `stale` and drops them)."""
    import glob
    import json
    root = os.path.join(os.path.dirname(_lib.LIB_PATH), "..")
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libsas_amd.so not built")
    import sas_amd
    h = sas_amd.source_hash()
    files = glob.glob(os.path.join(root, "profiles", "pmc_*.json"))
    assert files
    stale = [os.path.basename(f) for f in files if json.load(open(f)).get("source_hash") != h]
    assert not stale, (h, stale)
