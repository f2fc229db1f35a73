"""GPU parity of the u32 static-search-tree path (sst_* C ABI) -- a port of the
reference's differential test (sst/test.rs:142-260) plus its KATs, with the
node arrays compared word for word against the oracle's restatement of
STree::new_params."""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sas():
    import sas_amd
    return sas_amd


def gen_vals(n, rng):
    v = rng.integers(0, O.MAX, n, dtype=np.uint64).astype(np.uint32)
    v[0] = O.MAX  # sst/util.rs:37
    return np.sort(v)


def test_kats(sas, golden_dir):
    k = json.load(open(os.path.join(golden_dir, "reference_kats.json")))
    for c in k["eytzinger_layout"]:
        e = sas.Eytzinger.new(c["input"])
        assert e.nodes().tolist() == c["vals"]
    for c in k["eytzinger_search"]:
        assert sas.Eytzinger.new(c["input"]).query_one(c["q"]) == c["expect"]
    for c in k["sorted_search"]:
        inp = list(range(1, 2000)) + [O.MAX] if c["input"] == "range(1,2000) + [MAX]" else c["input"]
        assert sas.SortedVec.new(inp).query(c["qs"]).tolist() == c["expect"], c["cite"]
        if inp[-1] != O.MAX:
            inp = inp + [O.MAX]
        for cls in (sas.STree16, sas.STree15, sas.Eytzinger, sas.PartitionedSTree16M):
            assert cls.new(inp).query(c["qs"]).tolist() == c["expect"], (cls.__name__, c["cite"])
    vals = list(range(1, 2000)) + [O.MAX]
    for cls in (sas.STree16, sas.STree15, sas.SortedVec, sas.Eytzinger):
        idx = cls.new(vals)
        for c in k["stree_search"]:
            assert idx.query_one(c["q"]) == c["expect"], cls.__name__


SIZES = [s for p in range(6, 23) for s in ((1 << p), (1 << p) * 5 // 4, (1 << p) * 6 // 4, (1 << p) * 7 // 4)]


@pytest.mark.parametrize("size", SIZES[::3] + [SIZES[-1]])
def test_differential(sas, size):
    """sst/test.rs:143-196: every index/scheme returns the same Vec<u32>."""
    rng = np.random.default_rng(size)
    vals = gen_vals(size // 4, rng)
    qs = rng.integers(0, O.MAX, 1024, dtype=np.uint64).astype(np.uint32)  # 1000.next_multiple_of(128)
    ref, ref_rank = O.SortedVec(vals).query(qs, want_rank=True)
    got, rank = sas.SortedVec.new(vals).query(qs, want_rank=True)
    assert np.array_equal(got, ref) and np.array_equal(rank, ref_rank)
    assert np.array_equal(sas.Eytzinger.new(vals).query(qs), ref)
    for cls, B in ((sas.STree16, 16), (sas.STree15, 15)):
        for lm, rev, full in ((False, False, False), (True, False, False), (True, False, True), (False, True, False)):
            idx = cls.new_params(vals, lm, rev, full)
            o = O.STree(vals, B=B, left_max=lm, reverse=rev, full=full)
            assert np.array_equal(idx.nodes(), o.tree), (B, lm, rev, full)  # layout bit-exact
            assert idx.layers() == o.height and idx.size() == o.n_blocks * 64
            v, r = idx.query(qs, want_rank=True)
            assert np.array_equal(v, ref), (B, lm, rev, full)
            _, orank = o.query(qs, want_rank=True)
            assert np.array_equal(r, orank)
    # PartitionedSTree16M::new(vals, b) for the b of sst/test.rs:249-254
    for b in (0, 4, 8, 16, 20):
        pm = sas.PartitionedSTree16M.new(vals, b)
        v, r = pm.query(qs, want_rank=True)
        assert np.array_equal(v, ref), (size, b)
        assert np.array_equal(vals[np.minimum(r, len(vals) - 1)], ref)
        assert pm.layers() >= 1 and pm.size() >= len(vals) * 4
    # the other PartitionedSTree16 markers of sst/test.rs:222-246 (Simple, Compact, L1,
    # Overlapping), each for b in {0, 4, 8, 16, 20}: values equal SortedVec's
    for cls in (sas.PartitionedSTree16, sas.PartitionedSTree16C, sas.PartitionedSTree16L, sas.PartitionedSTree16O):
        for b in (0, 4, 8, 16, 20):
            idx = cls.new(vals, b)
            assert np.array_equal(idx.query(qs), ref), (cls.__name__, size, b)
            assert idx.layers() >= 1 and idx.size() >= len(vals) * 4
            idx.free()
    # SST_DIRECT_MAP: same values and ranks as SortedVec, for the automatic and forced b
    for b in (0, 1, 5, 12, 24):
        dm = sas.DirectMap.new(vals, b)
        v, r = dm.query(qs, want_rank=True)
        assert np.array_equal(v, ref) and np.array_equal(r, ref_rank), (size, b)


@pytest.mark.parametrize("size", [(1 << 23) * 7 // 4, 1 << 24, (1 << 25) * 5 // 4, (1 << 26) * 3 // 2, 1 << 26])
def test_differential_to_reference_max_size(sas, size):
    """The reference's sweep runs to 2^26 bytes (sst/test.rs:146-153); past the sizes whose
    layouts are compared word for word with the oracle above, every GPU layout of the lineup
    (SortedVec, Eytzinger, STree16/15 with left_max, PartitionedSTree16M at the test's largest b,
    every other PartitionedSTree16 marker, DirectMap) returns SortedVec::binary_search's values
    (ranks for SortedVec / DirectMap) on 1024 uniform and 1024 positive queries."""
    rng = np.random.default_rng(size)
    vals = gen_vals(size // 4, rng)
    qs = np.concatenate([rng.integers(0, O.MAX, 1024, dtype=np.uint64).astype(np.uint32),
                         vals[rng.integers(0, len(vals), 1024)]])
    ref_rank = np.searchsorted(vals, qs, "left")
    ref = np.where(ref_rank < len(vals), vals[np.minimum(ref_rank, len(vals) - 1)], np.uint32(O.MAX))
    v, r = sas.SortedVec.new(vals).query(qs, want_rank=True)
    assert np.array_equal(v, ref) and np.array_equal(r, ref_rank)
    builders = [sas.Eytzinger.new, sas.STree16.new, sas.STree15.new,
                lambda v_: sas.STree16.new_params(v_, True, False, False),
                lambda v_: sas.STree15.new_params(v_, True, False, True),
                lambda v_: sas.PartitionedSTree16M.new(v_, 20)]
    builders += [lambda v_, c=c: c.new(v_, 16) for c in (sas.PartitionedSTree16, sas.PartitionedSTree16C,
                                                          sas.PartitionedSTree16L, sas.PartitionedSTree16O)]
    for mk in builders:
        idx = mk(vals)
        assert np.array_equal(idx.query(qs), ref), (size, idx.__class__.__name__)
        idx.free()
    dm = sas.DirectMap.new(vals)
    v, r = dm.query(qs, want_rank=True)
    assert np.array_equal(v, ref) and np.array_equal(r, ref_rank), size


def test_direct_map_edges(sas):
    """SST_DIRECT_MAP on clustered keys (huge empty bucket runs: the gap list), runs of
    equal keys longer than the three inlined ones (the fallback search), queries above
    every key and above i32::MAX, against SortedVec."""
    rng = np.random.default_rng(9)
    vals = np.sort(np.concatenate([np.full(50, 7), np.full(9, 1 << 30), rng.integers(0, 1000, 300),
                                   rng.integers((1 << 31) - 5000, (1 << 31) - 1, 300)]).astype(np.uint32))
    qs = np.concatenate([rng.integers(0, 1 << 32, 3000, dtype=np.uint64),
                         np.array([0, 6, 7, 8, 999, 1000, (1 << 30) - 1, 1 << 30, (1 << 30) + 1,
                                   (1 << 31) - 1, 1 << 31, (1 << 32) - 1], np.uint64)]).astype(np.uint32)
    ref, ref_rank = O.SortedVec(vals).query(qs, want_rank=True)
    for b in (0, 2, 16, 30):
        v, r = sas.DirectMap.new(vals, b).query(qs, want_rank=True)
        assert np.array_equal(v, ref) and np.array_equal(r, ref_rank), b
    with pytest.raises(sas.SasError):
        sas.DirectMap.new([1, 2, 0x80000000])


def test_no_lds_and_device_path(sas):
    import torch
    from sas_amd import _lib
    rng = np.random.default_rng(1)
    vals = gen_vals(1 << 20, rng)
    qs = rng.integers(0, O.MAX, 1 << 16, dtype=np.uint64).astype(np.uint32)
    ref = O.SortedVec(vals).query(qs)
    idx = sas.STree16.new_params(vals, True, False, False)
    assert np.array_equal(idx.query(qs, flags=_lib.SST_NO_LDS_TOP), ref)
    dq = torch.from_numpy(qs.view(np.int32)).cuda()
    out = idx.query(dq)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref)


def test_partitioned_variants_edges(sas):
    """The four partitioned markers on skewed keys (one part holding most keys, empty
    parts, runs of equal keys across part boundaries), a single key, and queries at every
    part boundary and above every key: values equal SortedVec's; no rank output."""
    rng = np.random.default_rng(12)
    skew = np.sort(np.concatenate([rng.integers(0, 1 << 12, 30_000), rng.integers(1 << 30, (1 << 30) + 5, 500),
                                   np.full(3000, 1 << 25), [O.MAX]]).astype(np.uint32))
    for vals in (skew, np.array([O.MAX], np.uint32), np.array([5, 5, 5, O.MAX], np.uint32)):
        qs = np.concatenate([rng.integers(0, O.MAX, 4096, dtype=np.uint64).astype(np.uint32),
                             vals[:: max(1, len(vals) // 512)], vals[:: max(1, len(vals) // 512)] + 1,
                             np.array([0, 1, 1 << 25, (1 << 25) + 1, O.MAX - 1, O.MAX], np.uint32)])
        qs = np.minimum(qs, O.MAX)  # the trees compare signed: queries live in [0, i32::MAX] (sst/node.rs:5)
        ref = O.SortedVec(vals).query(qs)
        for cls in (sas.PartitionedSTree16, sas.PartitionedSTree16C, sas.PartitionedSTree16L,
                    sas.PartitionedSTree16O):
            for b in (0, 4, 8, 16, 20):
                idx = cls.new(vals, b)
                assert np.array_equal(idx.query(qs), ref), (cls.__name__, len(vals), b)
                with pytest.raises(sas.SasError):
                    idx.query(qs[:4], want_rank=True)
                idx.free()


def test_build_assertions(sas):
    with pytest.raises(sas.SasError):
        sas.STree16.new([3, 2, 1])  # unsorted
    with pytest.raises(sas.SasError):
        sas.STree16.new([1, 2, 0x80000000])  # > i32::MAX (sst/node.rs:5)
    with pytest.raises(sas.SasError):
        sas.STree16.new([])
    with pytest.raises(sas.SasError):
        sas.STree16.new_params([1, 2, 3], False, True, True)  # full + reverse


def test_query_counts_around_the_grid(sas):
    """Every layout at batch sizes that stop inside a group, a wave, the first grid pass and
    a later one (each lane loads its next query one pass ahead, SST_QPREFETCH): values and
    ranks equal SortedVec's."""
    rng = np.random.default_rng(17)
    vals = gen_vals(1 << 16, rng)
    allq = rng.integers(0, O.MAX, 3_000_003, dtype=np.uint64).astype(np.uint32)
    ref, ref_rank = O.SortedVec(vals).query(allq, want_rank=True)
    layouts = [sas.SortedVec.new(vals), sas.Eytzinger.new(vals), sas.STree16.new(vals), sas.STree15.new(vals),
               sas.PartitionedSTree16M.new(vals, 16), sas.PartitionedSTree16.new(vals, 8), sas.DirectMap.new(vals)]
    for nq in (1, 2, 3, 5, 63, 65, 1023, 1025, 600_001, 3_000_003):
        for idx in layouts:
            v = idx.query(allq[:nq])
            assert np.array_equal(v, ref[:nq]), (type(idx).__name__, nq)
        v, r = layouts[-1].query(allq[:nq], want_rank=True)
        assert np.array_equal(r, ref_rank[:nq]), nq
    for idx in layouts:
        idx.free()


def test_query_out_tensor_checked(sas):
    """sst query(out=...): a caller-owned result tensor must hold >= nq 4-byte elements,
    contiguously, on the queries' device (the kernel writes out.data_ptr() directly); host
    queries refuse out=."""
    import torch
    rng = np.random.default_rng(3)
    vals = gen_vals(1 << 12, rng)
    idx = sas.STree16.new(vals)
    qs = torch.from_numpy(rng.integers(0, O.MAX, 1000, dtype=np.uint64).astype(np.uint32).view(np.int32)).cuda()
    ok = torch.empty(1000, dtype=torch.int32, device="cuda")
    ref = idx.query(qs.cpu().numpy().view(np.uint32))
    assert np.array_equal(idx.query(qs, out=ok).cpu().numpy().view(np.uint32), ref)
    bad = [torch.empty(999, dtype=torch.int32, device="cuda"),            # short
           torch.empty(1000, dtype=torch.int64, device="cuda"),           # 8-byte elements
           torch.empty(2000, dtype=torch.int32, device="cuda")[::2],      # not contiguous
           torch.empty(1000, dtype=torch.int32)]                          # host
    for o in bad:
        with pytest.raises(sas.SasError):
            idx.query(qs, out=o)
    with pytest.raises(sas.SasError):
        idx.query(qs.cpu().numpy().view(np.uint32), out=ok)
    idx.free()
