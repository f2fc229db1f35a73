"""bench.py's correctness guard and byte model on the CPU (no GPU): lower_bound_proof accepts
exact lower bounds and rejects any other occurrence of a repeated query, on an
oracle-backed stand-in index; bytes_per_lookup never charges LDS- or cache-served tree
levels to HBM."""
import numpy as np

import bench
from oracle import pyoracle as O


class OracleIndex:
    """The three calls lower_bound_proof makes, on the oracle's SA."""

    def __init__(self, t):
        self.t = t
        self.n = len(t)
        self.sa = O.build_sa(t)
        self.sa_n = self.n
        self.rank_lo = 0
        self.tp = O.padded(t)

    def search_range(self, buf, off, lens):
        lo = np.array([O.prefix_range(self.tp, self.n, self.sa, buf[int(o):int(o) + int(L)])[0]
                       for o, L in zip(off, lens)], np.uint64)
        hi = np.array([O.prefix_range(self.tp, self.n, self.sa, buf[int(o):int(o) + int(L)])[1]
                       for o, L in zip(off, lens)], np.uint64)
        return lo, hi

    def suffix_array(self, count=None, start=0):
        return self.sa[start:start + count].astype(np.uint64)


def test_lower_bound_proof_accepts_and_rejects():
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 4, 50, dtype=np.uint8)
    t = np.concatenate([rng.integers(0, 4, 3000, dtype=np.uint8), blk, rng.integers(0, 4, 500, dtype=np.uint8), blk,
                        rng.integers(0, 4, 700, dtype=np.uint8), blk])
    idx = OracleIndex(t)
    n, m = len(t), 40
    offs = list(rng.integers(0, n - m, 200)) + [3000, 3550, 4300]  # the last three: the repeated block
    qs = [t[o:o + m] for o in offs]
    right = np.array([O.search_one(idx.tp, n, idx.sa, q)[0] for q in qs], np.uint64)
    window = lambda p, L: t[p:p + L]  # noqa: E731
    ids = np.arange(len(qs))
    assert bench.lower_bound_proof(idx, window, lambda i: qs[i], right, ids) == 0
    # another occurrence of a repeated query is an occurrence but not the lower bound
    wrong = right.copy()
    occ = [o for o in (3000, 3550, 4300) if o != int(right[-1])]
    wrong[-1] = occ[0]
    assert np.array_equal(t[int(wrong[-1]):int(wrong[-1]) + m], qs[-1])
    assert bench.lower_bound_proof(idx, window, lambda i: qs[i], wrong, ids) == 1
    # a negative query's lower bound (no occurrence) is proven too; n for a query above all
    neg = [np.full(m, 3, np.uint8), rng.integers(0, 4, m, dtype=np.uint8)]
    ans = np.array([O.search_one(idx.tp, n, idx.sa, q)[0] for q in neg], np.uint64)
    assert int(ans[0]) == n
    assert bench.lower_bound_proof(idx, window, lambda i: neg[i], ans, np.arange(2)) == 0
    assert bench.lower_bound_proof(idx, window, lambda i: neg[i], ans[::-1].copy(), np.arange(2)) >= 1


def test_byte_model_splits_served_levels():
    st = {"sa_width": 4, "prefix_bytes": (4 ** 16 + 1) * 32, "prefix_chars": 16, "quad_entry_bytes": 16,
          "stree_layers": 8, "stree_lds_layers": 2, "sector_layers": 12, "sector_lds_layers": 3, "quad_layers": 8,
          "quad_lds_layers": 3, "quad_fan": 17, "tag_chars": 16, "top_levels": 14, "top2_levels": 21}
    n, m = 1 << 30, 32
    q = bench.bytes_per_lookup("quad", st, n, m, 8.0)
    # quad at 2^30: 3 LDS layers, the 206 KB / 3.5 MB / 59 MB layers in cache, 1 GB + leaves in HBM
    assert q["lds"] == 3 * 64 and q["cache"] == 3 * 64 and q["hbm"] == 2 * 64 + m + 8
    # PLAIN: prefix-relative blocks, levels 1-15 from LDS (3 blocks of 32 B, one of 16 B), 16-27
    # in 3 requests (16-19 and 20-23 cache-resident, 24-27 past the cache's 256 MiB), then the
    # SA run of the last <= 8 ranks (32 B, one request) and a text window per probe
    st27 = dict(st, top2_levels=27, rel_levels=27, rel_bytes=bench.rel_bytes(27))
    p = bench.bytes_per_lookup("plain", st27, n, m, 31.0)
    assert p["lds"] == 3 * 32 + 16 and p["cache"] == 2 * 32 and p["hbm"] == 32 + 4 * (m / 4) + 32 + m + 8
    assert p["requests_model"] == {"cache": 2.0, "hbm": 1 + 4 + 1 + m / 128}
    # mlr LCP has no SA run: SA word + text window per probe
    lc = bench.bytes_per_lookup("lcp", st27, n, m, 31.0)
    assert lc["hbm"] == 32 + 4 * (4 + m / 4) + m + 8 and lc["requests_model"]["hbm"] == 1 + 4 * 2 + m / 128
    # LLCP: the same pivots (exact lcps off the keys), then one 16-B entry per probe
    ll = bench.bytes_per_lookup("llcp", st27, n, m, 31.0)
    assert ll["lds"] == 3 * 32 + 16 and ll["cache"] == 2 * 32 and ll["hbm"] == 32 + 4 * 16 + m + 8
    assert ll["requests_model"] == {"cache": 2.0, "hbm": 1 + 4 + m / 128}
    h = bench.bytes_per_lookup("prefix", st, n, m, 1.0)
    assert h["hbm"] == 32 + m + 8 and h["cache"] == 0 and h["lds"] == 0
    assert bench._tree_layers(n, 4, 64, 17, 64, 8)[-1] == n // 4 * 64


def test_byte_model_hbm_pivot_levels():
    """Deep pivots (SAS_BUILD_TOP2_LEVELS = 30, rounded up to all 31 levels of a 2^30 text):
    levels 1-15 from LDS, blocks of 16-19 and 20-23 cache-resident, 24-27 and 28-31 from HBM;
    the keys decide every level, then SA[r] is one read; requests by tier."""
    assert bench.rel_bytes(27) == 74272 + 32 * ((1 << 15) + (1 << 19) + (1 << 23))
    assert [(d, h) for d, h, _ in bench.rel_groups(27)] == [(0, 4), (4, 4), (8, 4), (12, 3), (15, 4), (19, 4), (23, 4)]
    assert [w for _, _, w in bench.rel_groups(31)] == ["lds"] * 4 + ["cache", "cache", "hbm", "hbm"]
    assert bench.rel_levels(31, 30) == 31 and bench.rel_levels(31, 0 or 27) == 27 and bench.rel_levels(25, 27) == 25
    assert bench.rel_levels(31, 16) == 19 and bench.rel_levels(31, 5) == 5
    st = {"sa_width": 4, "top_levels": 15, "top2_levels": 31, "rel_levels": 31, "rel_bytes": bench.rel_bytes(31)}
    n, m = 1 << 30, 32
    p31 = bench.bytes_per_lookup("plain", st, n, m, 31.0)
    assert p31["lds"] == 3 * 32 + 16 and p31["cache"] == 2 * 32
    assert p31["hbm"] == 2 * 32 + 4 + m + 8
    assert p31["requests_model"] == {"cache": 2.0, "hbm": 2 + 1 + m / 128}
    # fewer probes than the pivot levels (a short range): blocks entered only, SA[r] at the end
    p20 = bench.bytes_per_lookup("plain", st, n, m, 20.0)
    assert p20["hbm"] == 4 + m + 8 and p20["cache"] == 2 * 32
    assert p20["requests_model"] == {"cache": 2.0, "hbm": 1 + m / 128}
    # INLINE: the same blocks, then its fused entry for SA[r]
    pin = bench.bytes_per_lookup("inline", st, n, m, 31.0)
    assert pin["hbm"] == 2 * 32 + 16 + m + 8 and pin["requests_model"]["hbm"] == 2 + 1 + m / 128
    assert pin["requests_model"]["cache"] == 2.0
    # the split: model HBM requests first, the rest of the PMC count is cache-served
    bpl = bench.bytes_per_lookup("plain", dict(st, top2_levels=23, rel_levels=23, rel_bytes=bench.rel_bytes(23)),
                                 n, m, 31.0)
    assert bpl["requests_model"]["hbm"] == 8 + 1 + m / 128
    nq, kms = 10_000_000, 5.0
    sp = bench.request_split(bpl, {"rdreq_per_launch": 20.0 * nq}, nq, kms)
    assert abs(sp["hbm_per_lookup"] - 9.25) < 1e-9 and abs(sp["cache_per_lookup"] - 10.75) < 1e-9
    floor = max(nq * 9.25 / bench.RANDOM_REQ_CEILING, nq * 20.0 / bench.CACHE_REQ_CEILING)
    assert abs(sp["frac"] - floor / (kms * 1e-3)) < 1e-12 and sp["frac"] < 1
    # round 3's measured PLAIN (23 levels): 22.74 requests at 4.089 ms per 10^7 is under both limits
    sp = bench.request_split(bpl, {"rdreq_per_launch": 22.74 * nq}, nq, 4.089)
    assert sp["frac"] <= 1
    # a tree: QUAD at n = 2^30 (3 LDS layers, 3 cache-resident, the 1 GB layer and the leaves in DRAM)
    st = {"sa_width": 4, "quad_layers": 8, "quad_lds_layers": 3, "quad_fan": 17, "quad_entry_bytes": 16}
    q = bench.bytes_per_lookup("quad", st, n, m, 8.0)
    assert q["requests_model"] == {"cache": 3.0, "hbm": 2.0 + m / 128}
    assert bench.request_split(bench.bytes_per_lookup("prefix", {"sa_width": 4, "prefix_bytes": (4 ** 16 + 1) * 32,
                                                                  "prefix_chars": 16, "quad_entry_bytes": 16},
                                                      n, m, 1.0), {"rdreq_per_launch": 1.0}, nq, kms) is None


def test_pmc_attached_only_for_the_same_source_hash(tmp_path, monkeypatch):
    import json
    import sas_amd
    prof = tmp_path / "profiles"
    prof.mkdir()
    import benchlib.common
    monkeypatch.setattr(benchlib.common, "REPO", str(tmp_path))
    json.dump({"hbm_bytes_per_launch": 1e9, "TCC_EA0_RDREQ": 1e7, "source_hash": sas_amd.source_hash()},
              open(prof / "pmc_same.json", "w"))
    json.dump({"hbm_bytes_per_launch": 1e9, "TCC_EA0_RDREQ": 1e7, "source_hash": "0000000000000000"},
              open(prof / "pmc_other.json", "w"))
    json.dump({"hbm_bytes_per_launch": 1e9, "TCC_EA0_RDREQ": 1e7}, open(prof / "pmc_unstamped.json", "w"))
    assert bench.load_pmc("same")["hbm_bytes_per_launch"] == 1e9
    assert bench.load_pmc("other")["stale"] and bench.load_pmc("unstamped")["stale"]
    assert bench.load_pmc("missing") is None
    bpl = {"hbm": 100.0, "cache": 0.0, "lds": 0.0}
    r = bench.record("x", 10, 1.0, 1.0, bpl, 0, bench.load_pmc("other"), 1.0)
    assert r["pmc"]["stale"] and "fabric_bytes_per_lookup" not in r["pmc"]
    r = bench.record("x", 10, 1.0, 1.0, bpl, 0, bench.load_pmc("same"), 1.0)
    assert r["pmc"]["fabric_bytes_per_lookup"] == 1e8


def test_reference_sweep_sizes():
    """sizes() of sst/bin/bench.rs:453-471: 2^5 .. 2^to bytes, dense adds 5/4, 3/2, 7/4."""
    assert bench.ref_sizes(5, 8) == [32, 64, 128, 256]
    assert bench.ref_sizes(5, 7, dense=True) == [32, 40, 48, 56, 64, 80, 96, 112, 128]
    assert bench.ref_sizes()[-1] == 1 << 30 and len(bench.ref_sizes()) == 26


def _stats_2e30():
    """sas_stats of the default bench index at n = 2^30 (text 2-bit packed + 4 pad words,
    u32 SA, 26 pivot levels, fused quad leaves, p = 16 two-suffix inline table)."""
    n = 1 << 30
    return {"n": n, "sa_entries": n, "text_bytes": (n // 32 + 4) * 8, "sa_bytes": 4 * n, "sa_width": 4,
            "top_levels": 15, "top2_levels": 27, "rel_levels": 27,
            "rel_bytes": 74272 + 32 * ((1 << 15) + (1 << 19) + (1 << 23)), "top2_bytes": 0, "lcp_bytes": 4 * n, "llcp_bytes": 16 * n, "quad_entry_bytes": 16,
            "quad_bytes": 18_325_000_000, "sector_bytes": 19_400_000_000, "stree_bytes": 4_563_402_752,
            "prefix_bytes": (4 ** 16 + 1) * 32, "prefix_chars": 16, "index_bytes": 205_755_777_696}


def test_footprint_per_algorithm():
    """Each config reports the arrays its own algorithm reads (bench.rs:526-527's
    index_size per index), not the combined index the bench build holds."""
    st = _stats_2e30()
    gib = 1 << 30
    text = st["text_bytes"]
    piv = st["rel_bytes"]  # the prefix-relative pivot blocks, 273 MiB
    assert 273 << 20 < piv < 274 << 20
    assert bench.footprint("plain", st) == 4 * gib + text + piv  # ~4.5 GiB
    assert 4.3 * gib < bench.footprint("plain", st) < 4.6 * gib
    st31 = dict(st, top2_levels=31, rel_levels=31, rel_bytes=bench.rel_bytes(31))
    assert bench.footprint("plain", st31) == 4 * gib + text + bench.rel_bytes(31)
    assert bench.footprint("llcp", st) == 16 * gib + text + piv
    assert bench.footprint("quad", st) == st["quad_bytes"] + text  # ~17 GiB
    assert bench.footprint("prefix", st) == 128 * gib + 32 + 16 * gib + text  # table + fused leaves + text
    assert bench.footprint("prefix_packed", st) == bench.footprint("prefix", st)
    assert bench.footprint("plain_range", st) == bench.footprint("plain", st) + st["prefix_bytes"]
    assert bench.footprint("stree", st) == st["stree_bytes"] + 4 * gib + text
    # compact (key-only) leaves need the SA beside them
    cst = dict(st, quad_entry_bytes=8)
    assert bench.footprint("quad", cst) == st["quad_bytes"] + 4 * gib + text
    assert bench.footprint("prefix", cst) == st["prefix_bytes"] + 8 * gib + 4 * gib + text
    assert bench.footprint("tagged", st) == st["index_bytes"]
    for a in ("plain", "lcp", "llcp", "inline", "quad", "sector", "stree", "prefix", "interp"):
        assert bench.footprint(a, st) < st["index_bytes"], a


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def test_result_line_is_compact_and_complete():
    """The stdout line the driver parses stays under LINE_LIMIT (round 3's 20.9 KB line went
    unrecorded) with every contract key, the roofline and CPU baseline, and one flat entry
    per config; the full record is the detail file's."""
    import json
    import os
    full = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_record_r3.json")))
    full["lcp_long"] = {"summary": {"ms": dict({f"{t}_m{m}": [4.1, 4.6, 3.1, 3.3, 2.2] for t in ("random", "repetitive")
                                                for m in (64, 128, 256)}, algos=list(bench.LCP_LONG_ALGOS)),
                                    "skipping_beats_plain": ["llcp@random_m64:1.32x"] * 6,
                                    "quad_llcp_over_min_quad_stree_llcp": {f"{t}_m{m}": 0.987 for t in (
                                        "random", "repetitive") for m in (64, 128, 256)}}}
    full["detail"] = "gpurun_out/bench_detail.json"
    full["configs"]["sst"] = _sst_record()
    full["configs"]["c2"]["lcp_stree"] = dict(full["configs"]["c2"], algo="stree_llcp")
    full["configs"]["c2"]["lcp_quad"] = dict(full["configs"]["c2"], algo="quad_llcp")
    line = bench.compact_line(full)
    text = json.dumps(line)
    assert len(text) <= bench.LINE_LIMIT < 8192, len(text)
    # oversized optional summaries give way first; the contract keys stay
    big = dict(full, lcp_long={"summary": {"x" * 40 + str(i): [1.0, 2.0, 3.0] for i in range(200)}})
    bl = bench.compact_line(big)
    assert len(json.dumps(bl)) <= bench.LINE_LIMIT and "lcp_long" not in bl
    assert all(k in bl for k in REQUIRED) and "configs" in bl
    for k in REQUIRED:
        assert k in line, k
    assert isinstance(line["value"], float) and line["value"] > 0
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    for c in ("c0", "c1", "c2", "c3", "c4", "sst"):
        assert c in line["configs"], c
    assert line["configs"]["c2"]["lcp_stree"]["algo"] == "stree_llcp"
    assert line["configs"]["c2"]["lcp_quad"]["algo"] == "quad_llcp"
    assert len(line["configs"]["c2"]["lcp_quad_long_vs_min"]) == 6
    assert set(line["configs"]["sst"]) >= {"best", "lookups_per_s", "kernel_ms", "frac", "traffic", "cpu"}
    for c in ("c1", "c2"):
        assert set(line["configs"][c]) >= {"lookups_per_s", "kernel_ms", "frac", "index_bytes"}
    assert "variants" not in line and "index" not in line
    assert json.loads(text) == line


def test_every_headline_algo_has_a_workload_label():
    """bench.py --algo X names its workload: PLAIN from the index's pivot depth, the rest from
    WORKLOADS (a missing label ended a PMC pass in round 4)."""
    import re
    src = open(bench.__file__).read()
    choices = re.search(r'"--algo", default=None, choices=\[([^\]]*)\]', src).group(1)
    algos = [a.strip().strip('"') for a in choices.replace("\n", " ").split(",") if a.strip()]
    assert "plain" in algos and len(algos) >= 8
    st = {"top_levels": 15, "rel_levels": 27, "rel_bytes": bench.rel_bytes(27)}
    lab = bench.plain_label(st)
    assert "levels 1-27 from 273 MiB" in lab and "levels 1-15 staged in LDS, levels 16-23 cache-resident, 24-27 from " \
        "HBM; the rest" in lab, lab
    assert "16-27 levels" not in lab
    assert "levels 16-23 cache-resident, 24-31 from HBM" in bench.plain_label(
        {"top_levels": 15, "rel_levels": 31, "rel_bytes": bench.rel_bytes(31)})
    assert "levels 16-19 cache-resident;" in bench.plain_label(
        {"top_levels": 15, "rel_levels": 19, "rel_bytes": bench.rel_bytes(19)})
    assert "staged in LDS; the rest" in bench.plain_label({"top_levels": 15, "rel_levels": 15, "rel_bytes": 74272})
    for a in algos:
        if a != "plain":
            assert a in bench.WORKLOADS, a


def _sst_record():
    """A configs.sst record as bench.sst_record writes it (round 4's 2^28-key figures)."""
    lay = {}
    for name, ms, rq in (("SortedVec", 2.851, 13.0), ("STree16_left_max", 0.4641, 2.5),
                         ("PartitionedSTree16M_b16", 0.4717, 2.4), ("PartitionedSTree16M_b20", 0.4983, 2.3),
                         ("DirectMap", 0.24, 1.3)):
        ks = ms * 1e-3
        lay[name] = {"lookups_per_s": 1e7 / ks, "kernel_ms": ms, "kernel_ms_median": ms, "index_bytes": 1 << 30,
                     "equals_sortedvec": True, "requests_per_lookup": rq, "traffic": rq * 128 + 4,
                     "req_frac": rq * 1e7 / ks / bench.CACHE_REQ_CEILING,
                     "frac_hbm": (rq * 128 + 4) * 1e7 / ks / 1e9 / bench.HBM_PEAK_GBPS}
    return {"best": "DirectMap", "layouts": lay, "keys": 1 << 28, "queries": 10_000_000,
            "cpu_baseline": {"value": 2.48e8, "cores": 16, "unit": "lookups/s", "kind": "port"}}


def test_line_fractions_are_physical():
    """Every roofline fraction the line prints is a fraction of a physical ceiling (0 < frac
    <= 1): the headline's HBM-served bytes over 8 TB/s, each config's PMC request floor (or
    HBM-served bytes without a same-hash PMC pass), the u32 path's request rate over the
    measured random-request ceiling.  SURVEY 8(d)'s worst-case byte model, which passes 1 where
    pivot levels never reach HBM, is printed only as frac_8d_model."""
    import json
    import os
    full = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_record_r3.json")))
    full["configs"]["sst"] = _sst_record()
    # round 4's c1: 8(d) model 1.02 at 1.423 ms, request floor 1.00
    line = bench.compact_line(full)
    assert 0 < line["roofline"]["frac"] <= 1
    for k, c in line["configs"].items():
        if "frac" in c and c["frac"] is not None:
            assert 0 < c["frac"] <= 1, (k, c["frac"])
    for k in ("c1", "c2"):
        c = line["configs"][k]
        assert c["frac_basis"] in ("req", "hbm")
        assert c["frac"] == (c["req_frac"] if c["frac_basis"] == "req" else c["frac_hbm"])
        assert "frac_8d_model" in c
    # a deep-pivot PLAIN whose model passes 1 keeps its model out of `frac`
    rec = dict(full["configs"]["c1"], kernel_lookups_per_s=1e7 / 1.244e-3,
               bytes_per_lookup=dict(full["configs"]["c1"]["bytes_per_lookup"], section_8d=1156.0))
    cs = bench.config_summary(rec)
    assert cs["frac_8d_model"] > 1 and cs["frac"] <= 1
    assert line["configs"]["sst"]["frac"] <= 1 and line["configs"]["sst"]["best"] == "DirectMap"
    assert 0 < line["configs"]["sst"]["stree16_left_max_frac"] <= 1


def test_c1_request_floor_of_round5_plain():
    """Round 5's PLAIN (27 pivot levels, u32 SA): 7.199 PMC requests per lookup at 1.323 ms per
    10^7.  With its SA run in the model (one request for the last <= 8 ranks' SA words) the DRAM
    share is 6.25 requests, under the total, and the request floor stays a fraction (the model
    without the run counted 9.25 DRAM requests and put the floor above the measured time)."""
    st = {"sa_width": 4, "top_levels": 15, "top2_levels": 27, "rel_levels": 27, "rel_bytes": bench.rel_bytes(27)}
    n, m, nq = 1 << 30, 32, 10_000_000
    bpl = bench.bytes_per_lookup("plain", st, n, m, 31.0)
    sp = bench.request_split(bpl, {"rdreq_per_launch": 7.199 * nq}, nq, 1.323)
    assert sp["hbm_per_lookup"] == 6.25 and 0.9 < sp["frac"] <= 1, sp
