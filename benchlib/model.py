"""Algorithmic bytes and requests per lookup by where they are served (HBM / Infinity-Cache
resident / LDS), the prefix-relative pivot groups, each algorithm's own index footprint,
configs[4]'s per-GPU share, and the per-config record built from them."""
from __future__ import annotations

import numpy as np

from .common import (CACHE_BYTES, CACHE_REQ_CEILING, HBM_PEAK_GBPS, RANDOM_REQ_CEILING, SEED,  # noqa: F401
                     TOP_LDS_LEVELS)

# ---------------------------------------------------------------- bytes per lookup
def _tree_layers(n: int, leaf_entries: int, leaf_bytes: int, fan: int, node_bytes: int, layers: int):
    """Footprint in bytes of each layer of a tree over n entries, root first (layers counts
    the leaf layer)."""
    cnt = -(-n // leaf_entries)
    sizes = [cnt * leaf_bytes]
    for _ in range(layers - 1):
        cnt = -(-cnt // fan)
        sizes.append(cnt * node_bytes)
    return sizes[::-1]


def _classify(sizes, node_bytes, lds_layers):
    """(hbm, cache, lds) bytes of one node read per layer"""
    hbm = cache = lds = 0.0
    for h, sz in enumerate(sizes):
        if h < lds_layers:
            lds += node_bytes
        elif sz <= CACHE_BYTES:
            cache += node_bytes
        else:
            hbm += node_bytes
    return hbm, cache, lds


def bytes_per_lookup(algo: str, st: dict, n: int, m: float, probes: float, range_flag: bool = False,
                     packed: bool = False) -> dict:
    """Algorithmic bytes one lookup moves on this index's layout (2-bit packed text: a
    compare window of m chars is m/4 bytes), split by where they are served: `hbm`
    (arrays larger than the 256 MiB Infinity Cache, and the query/position streams),
    `cache` (arrays that fit it) and `lds` (top levels staged per workgroup).  `probes` is
    the measured mean of out_probes (the reference's cnt where it applies).  Also returns
    SURVEY §8(d)'s reference-layout figure for PLAIN (byte text)."""
    io = (8.0 if packed else m) + 8  # query in, position out
    win = m / 4.0  # packed text window of a full compare
    P = int(np.log2(n)) + 1
    hbm = cache = lds = 0.0
    sa_w = st["sa_width"]
    if algo == "prefix" and not range_flag:
        entry = prefix_entry_bytes(st)
        hbm += entry  # the table entry (inline entries hold the range's first suffixes)
        leaf = 16 if st["quad_entry_bytes"] == 16 else 8 + sa_w
        hbm += max(0.0, probes - 1) * leaf
    elif algo == "tagged" and st.get("tag_line_slots"):
        # bucket lines: the 128-B line (header + 20 entries), the entries of a mean bucket past
        # the line (overflow), the text past the bucket's p chars and the tag's whole chars
        known = st["tag_chars"] + st.get("tag_line_tag_bits", 24) // 2
        hbm += 128 + max(0.0, n / 4 ** st["tag_chars"] + 1 - st["tag_line_slots"]) * 8 + \
            max(0.0, m - known) / 4
    elif algo == "tagged":
        hbm += 8 + min(n / 4 ** st["tag_chars"] + 1, 8) * 8 + max(0.0, m - st["tag_chars"] - 12) / 4
    elif range_flag:  # PLAIN / LCP from the prefix table's range: table entry + SA word + window per probe
        entry = prefix_entry_bytes(st)  # (INTERP: a fused 16-B entry per probe)
        per = 16 if (algo == "interp" and st["quad_entry_bytes"] == 16) else sa_w + win
        hbm += entry + max(0.0, probes - 1) * per
    elif algo in ("plain", "lcp", "inline", "llcp"):
        # the prefix-relative blocks (common.hpp RelLayout): one per group entered, from LDS for
        # the first 15 levels, else one request (cache or HBM by where its group's array ends),
        # then per probe: SA word + text window (PLAIN / LCP, two requests) or one 16-B entry
        # (INLINE / LLCP, one request); a lookup decided by keys alone reads SA[r] at the end
        per, rq = (sa_w + win, 2) if algo in ("plain", "lcp") else (16, 1)
        # PLAIN over a u32 SA: once the range holds <= 8 ranks (SAS_PLAIN_SA_RUN) their SA words
        # come in one 32-B run (one request), so each later probe reads its text window only
        run = algo == "plain" and sa_w == 4
        if run:
            per, rq = win, 1
        R = st.get("rel_levels") or 0
        rc = rh = 0.0
        for d0, h, where in rel_groups(R):
            if probes - d0 <= 0:
                continue
            bb = 32 if h == 4 else 16
            if where == "lds":
                lds += bb
            elif where == "cache":
                cache += bb
                rc += 1
            else:
                hbm += bb
                rh += 1
        hbm += max(0.0, probes - R) * per
        srun = 1.0 if run and probes > R else 0.0  # the SA run: 32 B, one request
        hbm += srun * 32
        fin = 1.0 if probes <= R else 0.0
        hbm += fin * (sa_w if algo in ("plain", "lcp") else 16)
        reqs = {"cache": rc, "hbm": rh + max(0.0, probes - R) * rq + srun + fin + (8.0 if packed else m) / 128}
    elif algo == "interp":
        hbm += probes * 16
    elif algo in ("stree", "stree_llcp", "quad", "quad_llcp", "sector"):
        if algo in ("stree", "stree_llcp"):
            H, node, lds_l = st["stree_layers"], 64, st["stree_lds_layers"]
            sizes = _tree_layers(n, 16, 64, 17, 64, H)
            tail = sa_w + win if algo == "stree" else 16  # STREE_LLCP: one 16-B LLCP entry a probe
        elif algo == "sector":
            H, node, lds_l = st["sector_layers"], 32, st["sector_lds_layers"]
            sizes = _tree_layers(n, 2, 32, 9, 32, H)
            tail = 12
        else:
            H, node, lds_l = st["quad_layers"], 64, st["quad_lds_layers"]
            leaf_entries = 4 if st["quad_entry_bytes"] == 16 else 8
            sizes = _tree_layers(n, leaf_entries, 64, st["quad_fan"], 64, H)
            tail = 64 if algo == "quad" else 16  # QUAD_LLCP: a 16-B LLCP entry (or a leaf) a probe
        h, c, l = _classify(sizes, node, lds_l)
        hbm, cache, lds = h + max(0.0, probes - H) * tail + (max(0.0, m - 32) / 4 if not algo.startswith("stree")
                                                             else 0), c, l
        # one request per DRAM-level node (a 64-B node is one cooperative request; a 32-B one
        # too), per extra probe past the leaf, and the query stream
        reqs = {"cache": c / node, "hbm": h / node + max(0.0, probes - H) + (8.0 if packed else m) / 128}
    hbm += io
    out = {"hbm": hbm, "cache": cache, "lds": lds, "section_8d_plain": P * (4 + m) + m + 8}
    # SURVEY §8(d)'s algorithmic bytes of this probe sequence on the reference's byte layout,
    # every level counted wherever it is served (the roofline `achieved` of a config): the
    # binary-search family P (4 + m) + m + 8; trees H node bytes + what the tail reads
    if algo in ("plain", "lcp", "llcp", "inline") and not range_flag:
        out["section_8d"] = P * (4 + m) + m + 8
    elif algo in ("stree", "stree_llcp", "quad", "quad_llcp", "sector"):
        node = 32 if algo == "sector" else 64
        tail = {"stree": 4 + m, "stree_llcp": 4 + m, "quad": 64, "quad_llcp": 16, "sector": 12}[algo]
        out["section_8d"] = H * node + max(0.0, probes - H) * tail + m + 8
    else:
        out["section_8d"] = hbm
    if algo in ("plain", "lcp", "inline", "llcp", "stree", "stree_llcp", "quad", "quad_llcp", "sector") and not range_flag:
        out["requests_model"] = reqs
    return out


def request_split(bpl: dict, pmc, lookups: int, kernel_ms: float):
    """A kernel's measured L2->fabric requests split by where they are served: `hbm` = the
    model's DRAM-level requests (bytes_per_lookup's requests_model), `cache` = the rest of the
    PMC count (L2 misses of arrays the 256 MiB Infinity Cache holds).  Two limits apply: every
    request crosses the fabric (at most the best measured random-request rate, 5.73e10/s, the
    cache-resident one), and the DRAM share also needs DRAM (5.08e10/s); `floor_ms` is the larger
    of the two times and `frac` = floor / kernel time (<= 1).  (Adding the two shares' times
    instead is not a bound: PLAIN's mixed stream ran at 5.56e10 requests/s, above the DRAM rate,
    because its cache hits never reach DRAM.)"""
    if not pmc or not pmc.get("rdreq_per_launch") or "requests_model" not in bpl:
        return None
    total = pmc["rdreq_per_launch"] / lookups
    hbm = min(total, bpl["requests_model"]["hbm"])
    cache = total - hbm
    t_dram = lookups * hbm / RANDOM_REQ_CEILING
    t_fabric = lookups * total / CACHE_REQ_CEILING
    floor_s = max(t_dram, t_fabric)
    return {"per_lookup": total, "hbm_per_lookup": hbm, "cache_per_lookup": cache,
            "hbm_ceiling_per_s": RANDOM_REQ_CEILING, "fabric_ceiling_per_s": CACHE_REQ_CEILING,
            "dram_ms": t_dram * 1e3, "fabric_ms": t_fabric * 1e3, "floor_ms": floor_s * 1e3,
            "frac": floor_s / (kernel_ms * 1e-3),
            "basis": "hbm = model (DRAM-level tree nodes / pivot levels: 1 each; SA probes: SA word + text window; "
                     "the query stream m/128), cache = PMC TCC_EA0_RDREQ minus hbm; floor = max(hbm / DRAM rate, "
                     "all / fabric rate)"}


# ---------------------------------------------------------------- the pivot array
def rel_groups(R: int, lds_levels: int = TOP_LDS_LEVELS, G: int = 4):
    """common.hpp rel_layout: the prefix-relative pivot blocks of R levels, groups of up to G
    levels rooted at 0, 4, 8, 12 (3 levels) in LDS, then at 15, 19, ...; one block per root
    node (32 B at 4 levels, else 16 B).  (d0, h, where) per group: "lds", or "cache" while the
    array past the LDS groups fits the 256 MiB Infinity Cache, else "hbm"."""
    out, tot, d0 = [], 0, 0
    while d0 < R:
        h = G
        if d0 < lds_levels < d0 + h:
            h = lds_levels - d0
        h = min(h, R - d0)
        if d0 + h <= lds_levels:
            where = "lds"
        else:
            tot += (32 if h == G else 16) << d0
            where = "cache" if tot <= CACHE_BYTES else "hbm"
        out.append((d0, h, where))
        d0 += h
    return out


def rel_levels(iters: int, L: int, lds_levels: int = TOP_LDS_LEVELS, G: int = 4) -> int:
    """the depth rel_layout gives a requested L (clamped; rounded up to whole groups past LDS)"""
    R = min(L, iters)
    if R > lds_levels:
        R = lds_levels + -(-(R - lds_levels) // G) * G
    return min(R, iters)


def rel_bytes(R: int) -> int:
    return sum((32 if h == 4 else 16) << d0 for d0, h, _ in rel_groups(R))


# ---------------------------------------------------------------- index footprints
def prefix_entry_bytes(st: dict) -> int:
    """Bytes per prefix-table entry (4, 5, 16, 32, 64): a part's table covers only its own key
    interval (sas_stats.prefix_entries), a whole index's all 4^p + 1 keys."""
    ents = st.get("prefix_entries") or (4 ** st["prefix_chars"] + 1)
    return st["prefix_bytes"] // ents if ents else 0


C4_SHARE_TARGET = 1 << 33  # n = 2^33 chars per GPU


def c4_part_bytes(share: int, ws: int, p: int = 16, entry: int = 32) -> int:
    """HBM of one configs[4] rank's part index (sas_build_part_gen, PREFIX): the whole text
    packed (ws x share / 4), its SA range 40-bit (5 B a suffix), the fused quad leaves (16 B)
    and inner nodes (<= 1 B a suffix), the two-suffix inline table over the part's share of
    the 4^p keys (a whole index: all of them; + 5% for an uneven key split), the 72.5 KiB of
    LDS pivot groups."""
    keys = 4 ** p + 1 if ws == 1 else int(4 ** p / ws * 1.05) + 3
    return ws * share // 4 + 5 * share + 17 * share + keys * entry + (1 << 20)


def c4_share_for(ws: int, hbm_bytes: int, reserve: int = 12 << 30) -> int:
    """The largest power-of-two share <= 2^33 chars per GPU whose part index fits one GPU's HBM
    with `reserve` left for the step's buffers and the runtime (N = 1: 2^32, the whole
    4^16-key table; N >= 2: 2^33)."""
    share = C4_SHARE_TARGET
    while share > (1 << 20) and c4_part_bytes(share, ws) > hbm_bytes - reserve:
        share //= 2
    return share


def _quad_leaf_bytes(st: dict) -> int:
    """The quad tree's leaf layer: 64-B leaves of 4 fused {key64, SA} entries (16 B) or 8
    key-only entries (compact, 8 B)."""
    e = st.get("quad_entry_bytes", 0)
    return -(-st["sa_entries"] * e // 64) * 64 if e else 0


def footprint(algo: str, st: dict) -> int:
    """HBM bytes of the arrays one algorithm reads on this index (sas_stats fields), not the
    combined index a bench build holds (bench.rs:526-527 records index_size per index):
    PLAIN / LCP = SA + packed text + the pivot levels it reads (+ nothing else: mlr
    skipping keeps its lcps in registers); LLCP = its 16-B entries + pivots + text; INLINE =
    the fused quad leaves + pivots + text; QUAD = the quad tree (+ SA with compact leaves) +
    text; SECTOR = the sector tree + text; STREE = the S-tree + SA + text; STREE_LLCP = the
    S-tree + the LLCP entries + text; QUAD_LLCP = the quad tree + the LLCP entries + text; PREFIX = the prefix
    table + the quad leaves (+ SA with compact leaves) + text; *_range = + the prefix table;
    TAGGED = the tagged index (it holds nothing else)."""
    base = algo[:-6] if algo.endswith("_range") else ("prefix" if algo == "prefix_packed" else algo)
    text = st["text_bytes"] + st.get("text2_bytes", 0)
    sa = st["sa_bytes"]
    compact_sa = sa if st.get("quad_entry_bytes") == 8 else 0
    # the pivots: the LDS levels' entries and 16-char keys, then the prefix-relative blocks
    piv = st.get("rel_bytes", 0)
    if base == "tagged":
        return st["index_bytes"]
    if base in ("plain", "lcp"):
        b = sa + text + piv
    elif base == "llcp":
        b = st["llcp_bytes"] + text + piv
    elif base == "inline":
        b = _quad_leaf_bytes(st) + text + piv
    elif base == "quad":
        b = st["quad_bytes"] + compact_sa + text
    elif base == "sector":
        b = st["sector_bytes"] + text
    elif base == "stree":
        b = st["stree_bytes"] + sa + text
    elif base == "stree_llcp":  # the S-tree + the LLCP entries (SA values included) + text
        b = st["stree_bytes"] + st["llcp_bytes"] + text
    elif base == "quad_llcp":  # the quad tree + the LLCP entries (SA values included) + text
        b = st["quad_bytes"] + st["llcp_bytes"] + text
    elif base == "prefix":
        b = st["prefix_bytes"] + _quad_leaf_bytes(st) + compact_sa + text
    elif base == "interp":
        b = (_quad_leaf_bytes(st) if st.get("quad_entry_bytes") == 16 else sa) + text
    else:
        raise ValueError(f"footprint: unknown algo {algo}")
    if algo.endswith("_range"):
        b += st["prefix_bytes"]
    return int(b)


def rank_query_offsets(n: int, nq: int, m: int, rank: int) -> np.ndarray:
    """This rank's queries: positive len-m substrings t[i..i+m] (sas/util.rs:18-26);
    the ChaCha8 stream continues after the text's n words, rank r starting at word
    n + r*4*nq (a fixed-length query draws 2 words, rejections are rare)."""
    import sas_amd
    off, _, _ = sas_amd.random_queries(n, nq, seed=SEED, word_pos=n + rank * 4 * nq, margin=200,
                                       len_lo=m, len_hi=m + 1)
    return off


# The one JSON line goes to the original stdout; everything else that writes to fd 1
# (RCCL prints its version banner there when a communicator comes up) is sent to
# stderr, so stdout carries exactly the result line.


def record(name, lookups, kernel_ms, wall_s, bpl, idx_bytes, pmc, probes, extra=None):
    """One sub-record for one launch of `lookups` queries: throughput, ns per lookup, bytes
    per lookup split by where they are served, achieved HBM GB/s (HBM bytes only), PMC
    traffic if a pass exists.  wall_s: the host clock over the timed steps (for
    lookups_per_s the caller sets)."""
    r = {"algo": name, "kernel_ms": kernel_ms,
         "kernel_lookups_per_s": lookups / (kernel_ms * 1e-3), "ns_per_lookup": kernel_ms * 1e6 / lookups,
         "mean_probes": probes, "bytes_per_lookup": bpl,
         "achieved_hbm_GBps": bpl["hbm"] * lookups / (kernel_ms * 1e-3) / 1e9,
         "achieved_cache_GBps": bpl["cache"] * lookups / (kernel_ms * 1e-3) / 1e9,
         "index_bytes": idx_bytes}
    if pmc and pmc.get("stale"):
        r["pmc"] = {"stale": True, "note": "the committed counters were collected on another build "
                                           "(source hash differs): not reported", **pmc}
    elif pmc and pmc.get("hbm_bytes_per_launch"):
        r["pmc"] = {"fabric_bytes_per_lookup": pmc["hbm_bytes_per_launch"] / lookups,
                    "fabric_GBps": pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9,
                    "requests_per_lookup": (pmc["rdreq_per_launch"] or 0) / lookups,
                    "source": pmc["source"], "source_hash": pmc["source_hash"]}
        split = request_split(bpl, pmc, lookups, kernel_ms)
        if split:  # mixed cache / HBM requests: each share against its own ceiling
            r["pmc"]["requests_split"] = split
        else:
            r["pmc"]["requests_frac_of_ceiling"] = (pmc["rdreq_per_launch"] or 0) / (kernel_ms * 1e-3) / \
                RANDOM_REQ_CEILING
    if extra:
        r.update(extra)
    return r
