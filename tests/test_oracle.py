"""CPU tests of the oracle itself: pinned against the reference's own known-answer
tests and against the definition oracle (tests/golden/), before anything is
compared with the GPU."""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O


@pytest.fixture(scope="module")
def kats(golden_dir):
    return json.load(open(os.path.join(golden_dir, "reference_kats.json")))


@pytest.fixture(scope="module")
def sadef(golden_dir):
    return json.load(open(os.path.join(golden_dir, "sa_definition.json")))


def test_chacha20_rfc7539_block():
    # RFC 7539 §2.3.2 test vector pins the ChaCha core shared by ChaCha8Rng.
    key = np.array([int.from_bytes(bytes(range(4 * i, 4 * i + 4)), "little") for i in range(8)], np.uint32)
    out = O.chacha_block(key, 1, 0x09000000, 0x4A000000, 0, rounds=20)
    expect = [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
              0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]
    assert [int(x) for x in out] == expect


def test_random_string_is_chacha8_keystream():
    # random_string char i == keystream word i >> 30 (rand 0.8.5 UniformInt<u8>, range 4)
    t = O.random_string(100)
    key = np.zeros(8, np.uint32)
    O.lib().orc_seed_from_u64(31415, key)
    words = np.concatenate([O.chacha_block(key, b, 0, 0, 0, rounds=8) for b in range(7)])
    assert np.array_equal(t, (words[:100] >> 30).astype(np.uint8))
    assert set(np.unique(O.random_string(10000))) == {0, 1, 2, 3}


def test_random_queries_shape():
    n = 5000
    off, ln, pos = O.random_queries(n, 1000)
    assert off.max() < n - 200 and ln.min() >= 30 and ln.max() < 100
    off2, ln2, pos2 = O.random_queries(n, 1000, len_lo=32, len_hi=33)
    assert (ln2 == 32).all() and pos2 < pos  # fixed length draws no length word


# ------------------------------------------------------------------ reference KATs
def test_kat_eytzinger_layout(kats):
    for k in kats["eytzinger_layout"]:
        assert O.Eytzinger(k["input"]).vals.tolist() == k["vals"], k["cite"]


def test_kat_eytzinger_search(kats):
    for k in kats["eytzinger_search"]:
        e = O.Eytzinger(k["input"])
        assert int(e.query([k["q"]])[0]) == k["expect"], k["cite"]
        assert int(e.query([k["q"]], branchless=True)[0]) == k["expect"], k["cite"]


def test_kat_stree_search(kats):
    vals = list(range(1, 2000)) + [O.MAX]
    t = O.STree(vals)
    for k in kats["stree_search"]:
        assert int(t.query([k["q"]])[0]) == k["expect"] == int(O.SortedVec(vals).query([k["q"]])[0]), k["cite"]


def _kat_input(k):
    return list(range(1, 2000)) + [O.MAX] if k["input"] == "range(1,2000) + [MAX]" else k["input"]


def test_kat_sorted_search(kats):
    for k in kats["sorted_search"]:
        got = O.SortedVec(_kat_input(k)).query(k["qs"])
        assert got.tolist() == k["expect"], k["cite"]
        assert O.STree(_kat_input(k) if _kat_input(k)[-1] == O.MAX else _kat_input(k) + [O.MAX]).query(
            k["qs"]).tolist() == k["expect"], k["cite"]


def test_kat_node_find(kats):
    for k in kats["node_find"]:
        assert O.node_find(k["node"], k["q"]) == k["expect"]


# ------------------------------------------------------------------ definition oracle (SA)
def test_sa_construction_matches_definition(sadef):
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        sa = O.build_sa(t)
        assert sa.tolist() == c["sa"], c["name"]
        assert O.check_sa(t, sa) == 0


def test_check_sa_rejects_bad():
    t = np.array([0, 1, 2, 3, 0, 1], np.uint8)
    sa = O.build_sa(t)
    bad = sa.copy()
    bad[[1, 2]] = bad[[2, 1]]
    assert O.check_sa(t, bad) == 2
    bad = sa.copy()
    bad[0] = bad[1]
    assert O.check_sa(t, bad) == 1


def test_kasai_lcp_bruteforce(sadef):
    for c in sadef["cases"]:
        t = c["text"]
        sa = np.array(c["sa"], np.uint32)
        lcp = O.kasai_lcp(np.array(t, np.uint8), sa)
        for r in range(1, len(t)):
            a, b = t[sa[r - 1]:], t[sa[r]:]
            k = 0
            while k < min(len(a), len(b)) and a[k] == b[k]:
                k += 1
            assert lcp[r] == k


def test_binary_search_matches_definition(sadef):
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        n = len(t)
        sa = np.array(c["sa"], np.uint32)
        tp = O.padded(t)
        for qd in c["queries"]:
            q = np.array(qd["q"], np.uint8)
            pos, cnt = O.search_one(tp, n, sa, q, "binary_search")
            assert pos == qd["pos"], (c["name"], qd)
            assert O.lower_bound_rank(tp, n, sa, q) == qd["rank"]
            assert cnt <= int(np.log2(max(n, 1))) + 1


def test_interpolation_search_matches_definition(sadef):
    """interpolation_search<16> (sas/sa_search.rs:376-421) returns binary_search's position
    on every definition-fixture query (its mids are clamped inside (l, r), so only the
    probe count differs); the count is at least 1 for a non-empty range.  The count
    itself has no reference-held vector (parity unpinned beyond this restatement)."""
    for c in sadef["cases"]:
        t = np.array(c["text"], np.uint8)
        n = len(t)
        sa = np.array(c["sa"], np.uint32)
        tp = O.padded(t)
        for qd in c["queries"]:
            pos, cnt = O.interpolation_search(tp, n, sa, np.array(qd["q"], np.uint8))
            assert pos == qd["pos"], (c["name"], qd)
            assert 1 <= cnt <= n
    t = O.random_string(1 << 16)
    sa = O.build_sa(t)
    tp = O.padded(t)
    off, _, _ = O.random_queries(1 << 16, 500, len_lo=16, len_hi=17)
    cnts = [O.interpolation_search(tp, 1 << 16, sa, t[o:o + 16])[1] for o in off.astype(np.int64)]
    assert np.mean(cnts) < 17  # fewer probes than binary search's 17 on uniform keys


def test_batch_and_threads_match_canonical(sadef):
    c = [c for c in sadef["cases"] if c["name"] == "random_4096"][0]
    t = np.array(c["text"], np.uint8)
    n = len(t)
    sa = np.array(c["sa"], np.uint32)
    tp = O.padded(t)
    qs = [np.array(q["q"], np.uint8) for q in c["queries"]]
    lens = np.array([len(q) for q in qs], np.uint32)
    off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    buf = np.concatenate(qs + [np.zeros(64, np.uint8)])
    expect = np.array([q["pos"] for q in c["queries"]], np.uint64)
    for algo in ("binary_search", "batch16"):
        for th in (1, 3):
            got, cnt = O.search_many(tp, n, sa, buf, off, lens, algo, th)
            assert np.array_equal(got, expect), (algo, th)
    # batch16 counts B per lockstep iteration (sas/sa_search.rs:178)
    _, cnt = O.search_many(tp, n, sa, buf, off[:16], lens[:16], "batch16", 1)
    assert cnt == 16 * (int(np.log2(n)) + 1)


def test_reference_variant_disagreements(sadef):
    """Pin SURVEY §8a: A8 (`cmp`) differs from A6 only on padded text-end
    suffixes; A10 returns a rank on full-suffix equality; A11 is a predecessor
    search.  These are documented exclusions from parity."""
    c = [c for c in sadef["cases"] if c["name"] == "ends_with_A_run"][0]
    t = np.array(c["text"], np.uint8)
    n = len(t)
    sa = np.array(c["sa"], np.uint32)
    tp = O.padded(t)
    n_cmp_diff = n_branchy_rank = 0
    for qd in c["queries"]:
        q = np.array(qd["q"], np.uint8)
        a6, _ = O.search_one(tp, n, sa, q, "binary_search")
        a8, _ = O.search_one(tp, n, sa, q, "binary_search_cmp")
        a10, _ = O.search_one(tp, n, sa, q, "branchy_search")
        if a8 != a6:
            n_cmp_diff += 1
            # the zero-padded suffix compares equal where slice order says "shorter = less"
            assert qd["rank"] > 0
        full_suffix = any(list(t[i:]) == qd["q"] for i in range(n))
        if full_suffix and a10 != a6:
            n_branchy_rank += 1
            assert a10 == qd["rank"]
    assert n_cmp_diff > 0 and n_branchy_rank > 0
    # branchfree = predecessor: position of rank lb-1 for a positive query with lb > 0
    q = t[100:130]
    lb = O.lower_bound_rank(tp, n, sa, q)
    bf, _ = O.search_one(tp, n, sa, q, "branchfree_search")
    assert lb > 0 and bf == int(sa[lb - 1])


# ------------------------------------------------------------------ u32 differential (sst/test.rs port)
def gen_vals(n, rng):
    v = rng.integers(0, O.MAX, n, dtype=np.uint64).astype(np.uint32)
    v[0] = O.MAX  # sst/util.rs:37
    return np.sort(v)


@pytest.mark.parametrize("p", range(6, 17, 2))
def test_sst_differential(p):
    rng = np.random.default_rng(p)
    for size in (1 << p, (1 << p) * 5 // 4, (1 << p) * 6 // 4, (1 << p) * 7 // 4):
        vals = gen_vals(size // 4, rng)
        qs = rng.integers(0, O.MAX, 1024, dtype=np.uint64).astype(np.uint32)
        ref, ref_rank = O.SortedVec(vals).query(qs, want_rank=True)
        e = O.Eytzinger(vals)
        assert np.array_equal(e.query(qs), ref)
        assert np.array_equal(e.query(qs, branchless=True), ref)
        for B in (16, 15):
            for lm, full in ((False, False), (True, False), (True, True), (False, True)):
                t = O.STree(vals, B=B, left_max=lm, full=full)
                got, rank = t.query(qs, want_rank=True)
                assert np.array_equal(got, ref), (size, B, lm, full)
                assert np.array_equal(vals[np.minimum(rank, len(vals) - 1)], ref)
            t = O.STree(vals, B=B, reverse=True)
            assert np.array_equal(t.query(qs), ref)


def test_prefix_range_matches_occurrences(sadef):
    """orc_prefix_range: SA[lo:hi] is exactly the set of occurrence positions."""
    for c in sadef["cases"]:
        t = c["text"]
        n = len(t)
        sa = np.array(c["sa"], np.uint32)
        tp = O.padded(np.array(t, np.uint8))
        for qd in c["queries"]:
            q = qd["q"]
            lo, hi = O.prefix_range(tp, n, sa, np.array(q, np.uint8))
            assert lo == qd["rank"]
            occ = sorted(i for i in range(n) if t[i:i + len(q)] == q) if len(q) <= n else []
            assert sorted(sa[lo:hi].tolist()) == occ, (c["name"], q)


def test_stree_batch_final_restatement_matches_search():
    """orc_stree_batch (batch_final::<128>, sst/s_tree.rs:303-326; the u32 CPU
    baseline) returns exactly STree::search's values, single- and multi-threaded."""
    rng = np.random.default_rng(5)
    for size in (17, 1000, 70_001):
        vals = gen_vals(size, rng)
        qs = rng.integers(0, O.MAX, 5000, dtype=np.uint64).astype(np.uint32)
        for B in (16, 15):
            for lm, rev in ((False, False), (True, False), (False, True)):
                t = O.STree(vals, B=B, left_max=lm, reverse=rev)
                ref = t.query(qs)
                assert np.array_equal(t.query_batch(qs), ref), (size, B, lm, rev)
                assert np.array_equal(t.query_batch(qs, threads=3), ref)
