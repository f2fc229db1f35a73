"""Headline benchmark: batched suffix-array pattern lookups on MI355X.

BASELINE.json metric: "pattern lookups/s + achieved HBM GB/s, 2^30-byte text,
10^7 len-32 queries".  One step = one batched lookup of all queries of this
GPU (inputs already resident in HBM), through the C ABI (sas_search_fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--algo prefix|plain|quad|...]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

One JSON line.  `value` is the headline algorithm (PREFIX: a p = 16-char bucket table with
32-B inline entries over fused quad leaves) on the configs[1]/[2] workload; `configs` holds
one sub-record per BASELINE config, each with its own algorithm, index size, bytes per
lookup split by where they are served (HBM / Infinity-Cache-resident arrays / LDS), PMC
traffic where a committed --pmc pass exists, and ns per lookup:
    c0: the reference's CPU plumbing case (1 MiB text, 10^4 x len-16) timed on the host
        (oracle restatement, 1 thread and all cores), and the GPU on the same queries;
    c1: PLAIN binary search (sas/sa_search.rs:98-112) on the same 2^30 index;
    c2: the fastest LCP / S-tree layout with LDS-staged top layers;
    c3: n = 2^34 text (the configs[3] deviation), 10^8 ragged 8..256 queries
        on the tagged index (run after the 2^30 index is freed; N = 1 only).
Every variant's positions must equal the headline's bit for bit, and a sample of each
batch is proven an exact lower bound (SA[lo-1] < q <= SA[lo], SA[lo] = answer) on the GPU
index's own SA; any mismatch exits non-zero.

Multi-GPU: the index is replicated (the text is generated and indexed on every GPU), each
rank searches its own 10^7 queries -> weak scaling, no collective on the data path; only
the timing barrier and a MAX all-reduce of elapsed times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "suffix-array-searching_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "pattern lookups/s + achieved HBM GB/s, 2^30-byte text, 10^7 len-32 queries"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# independent random 4-B loads over a 4 GiB buffer, one 128-B line each: the chip's
# random-request ceiling (tools/randbench.hip, profiles/r1/randbench_calibration.jsonl)
RANDOM_REQ_CEILING = 5.084e10
# the same random 4-B loads over a 64 MiB buffer (Infinity-Cache resident): the ceiling of
# requests the cache-resident arrays serve (profiles/r1/randbench_calibration.jsonl)
CACHE_REQ_CEILING = 5.731e10
CACHE_BYTES = 256 << 20  # Infinity Cache (MALL): arrays at most this large count as cache-served
SEED = 31415  # sas/main.rs:38
# binary-search levels served by the prefix-relative pivot blocks (the index's stats win): the
# library default reaches 27 levels (SAS_TOP2_CACHE_LEVELS: 15 staged in LDS, 273 MiB of blocks);
# deeper ones (SAS_BUILD_TOP2_LEVELS, e.g. 30 -> 31 levels = 4.3 GiB) read HBM blocks
TOP_LDS_LEVELS = 15  # common.hpp SAS_REL_LDS_LEVELS
C1_DEEP_TOP2_LEVELS = 30  # the second configs[1] figure: rounded up to all 31 levels, 28-31 from HBM

KERNELS = {"stree": "k_sa_stree", "stree_llcp": "k_sa_stree", "sector": "k_sa_sector", "quad": "k_sa_quad", "inline": "k_sa_inline",
           "llcp": "k_sa_binary", "plain": "k_sa_binary", "lcp": "k_sa_binary", "interp": "k_sa_interp",
           "tagged": "k_sa_tagged"}


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
    elif algo in ("stree", "stree_llcp", "quad", "sector"):
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
            tail = 64
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
    elif algo in ("stree", "stree_llcp", "quad", "sector"):
        node = 32 if algo == "sector" else 64
        tail = {"stree": 4 + m, "stree_llcp": 4 + m, "quad": 64, "sector": 12}[algo]
        out["section_8d"] = H * node + max(0.0, probes - H) * tail + m + 8
    else:
        out["section_8d"] = hbm
    if algo in ("plain", "lcp", "inline", "llcp", "stree", "stree_llcp", "quad", "sector") and not range_flag:
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


# ---------------------------------------------------------------- harness
def timed_loop(step, steps: int, warmup: int, sync, barrier, reduce_max):
    """W untimed steps, then K steps bracketed by barrier + device sync on both
    sides; returns the MAX over ranks of the elapsed seconds."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    return reduce_max(elapsed)


def launch_times(torch, step, steps: int, warmup: int, stream, sync=None, barrier=None, reduce_max=None):
    """W untimed launches, then K timed ones with a HIP event recorded on `stream` (the
    stream the library launches on) before each and after the last: the per-launch kernel
    times.  Returns {"mean_ms", "median_ms", "wall_s"}: the events' mean (total / K, the
    roofline's kernel time), their median (what rocprofv3's per-dispatch statistics show
    beside it) and the host clock over the K launches (timed_loop: barrier + sync on both
    sides, MAX over ranks when reduce_max is given)."""
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    state = {"i": 0}

    def timed_step():
        i = state["i"] - warmup
        if 0 <= i < steps:
            evs[i].record(stream)
        step()
        state["i"] += 1
        if state["i"] == warmup + steps:
            evs[steps].record(stream)
    el = timed_loop(timed_step, steps, warmup, sync or torch.cuda.synchronize, barrier or (lambda: None),
                    reduce_max or (lambda x: x))
    per = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    return {"mean_ms": evs[0].elapsed_time(evs[steps]) / steps, "median_ms": float(np.median(per)), "wall_s": el}


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
    S-tree + the LLCP entries + text; PREFIX = the prefix
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
_RESULT_OUT = None


def emit(obj) -> None:
    out = _RESULT_OUT or sys.stdout
    print(json.dumps(obj), file=out, flush=True)


def keep_stdout_for_result() -> None:
    global _RESULT_OUT
    if _RESULT_OUT is None:
        sys.stdout.flush()
        _RESULT_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def load_pmc(key: str):
    """The committed rocprofv3 --pmc summary of this exact workload
    (profiles/pmc_<key>.json, written by tools/pmc_to_json.py): HBM bytes and L2->fabric
    read requests per launch, or None.  Counters are attached only when the summary was
    collected on a library of the same source hash as the one loaded now (sas_source_hash);
    a summary of another build comes back as {"stale": ...} and is never reported as
    traffic."""
    import sas_amd
    path = os.path.join(REPO, "profiles", f"pmc_{key}.json")
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    src, lib_hash = d.get("source_hash"), sas_amd.source_hash()
    rel = os.path.relpath(path, REPO)
    if src != lib_hash:
        return {"stale": True, "source": rel, "pmc_source_hash": src, "library_source_hash": lib_hash}
    return {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"), "rdreq_per_launch": d.get("TCC_EA0_RDREQ"),
            "source": rel, "source_hash": src}


def host_cpu() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """The cores this process is allotted: its affinity mask, capped by OMP_NUM_THREADS when
    the host sets it (the GPU box allots 16 cores per GPU and exports OMP_NUM_THREADS=16,
    while its affinity mask shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(share))) if share.isdigit() and int(share) > 0 else n


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


# ---------------------------------------------------------------- correctness guard
def lower_bound_proof(idx, window, qwin, out, sample_ids) -> int:
    """For each sampled query i: lo = its occurrence range's first rank (sas_search_range),
    and the proof that lo is the lower bound on the index's own (verified) SA:
    SA[lo] == out[i], suffix(SA[lo-1]) < q <= suffix(SA[lo]) in Rust slice order.
    window(p, L) -> the text chars [p, min(p+L, n)); qwin(i) -> query i; out[j] = the
    answer of sample_ids[j].  Returns the count of failures."""
    n = idx.n
    bad = 0
    qs = [np.asarray(qwin(int(i)), np.uint8) for i in sample_ids]
    lens = np.array([len(q) for q in qs], np.uint32)
    off = np.zeros(len(qs), np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.concatenate(qs + [np.zeros(64, np.uint8)])
    lo, _ = idx.search_range(buf, off, lens)

    def less(a, q):  # Rust slice order a < q
        k = min(len(a), len(q))
        d = np.nonzero(a[:k] != q[:k])[0]
        if len(d):
            return a[d[0]] < q[d[0]]
        return len(a) < len(q)

    for j in range(len(sample_ids)):
        q, r = qs[j], int(lo[j]) - idx.rank_lo
        if r < idx.sa_n:
            sa2 = idx.suffix_array(count=2 if r > 0 else 1, start=r - 1 if r > 0 else 0).astype(np.int64)
            p0, prev = int(sa2[-1]), (int(sa2[0]) if r > 0 else None)
        else:  # past this index's range: SA[rank_lo + sa_n] (n for a whole index)
            p0 = getattr(idx, "next_pos", n)
            prev = int(idx.suffix_array(count=1, start=r - 1)[0]) if r > 0 else None
        if p0 != int(out[j]):
            bad += 1
            continue
        if p0 < n and less(window(p0, len(q)), q):
            bad += 1
        if prev is not None and not less(window(prev, len(q)), q):
            bad += 1
    return bad


# ---------------------------------------------------------------- CPU baselines
def cpu_baseline(text_dev, idx, qbytes_dev, m, nq, seconds: float):
    """The oracle's restatement of the reference CPU search, timed on all of this host's
    cores (its affinity mask) and on 1 thread, on a bounded sample of the same queries
    (rank 0, N = 1 only).  Its answers are returned for comparison with the GPU's."""
    from oracle import pyoracle as O
    threads = host_threads()
    n = idx.n
    t = O.padded(text_dev.cpu().numpy())
    sa = idx.suffix_array()
    best = None
    for algo in ("binary_search", "batch_c16"):
        sample = min(nq, 100_000)
        while True:
            qb = np.concatenate([qbytes_dev[: sample * m].cpu().numpy(), np.zeros(64, np.uint8)])
            off = np.arange(sample, dtype=np.uint64) * m
            ln = np.full(sample, m, np.uint32)
            t0 = time.perf_counter()
            pos, _ = O.search_many(t, n, sa, qb, off, ln, algo, threads)
            dt = time.perf_counter() - t0
            if dt * 2 > seconds / 2 or sample >= nq:
                break
            sample = min(nq, int(sample * max(2.0, (seconds / 2) / max(dt, 1e-3))))
        # the whole query set takes less than seconds/2: repeat it (still the same queries)
        reps = 1
        while dt < seconds / 2:
            t0 = time.perf_counter()
            O.search_many(t, n, sa, qb, off, ln, algo, threads)
            dt += time.perf_counter() - t0
            reps += 1
        rate = sample * reps / dt
        if best is None or rate > best[0]:
            best = (rate, algo, sample, dt, pos, reps)
    rate, algo, sample, dt, pos, reps = best
    # one thread on a smaller sample of the same queries (1 thread and all cores)
    s1 = min(nq, max(1000, int(rate / threads * seconds / 8)))
    qb = np.concatenate([qbytes_dev[: s1 * m].cpu().numpy(), np.zeros(64, np.uint8)])
    t0 = time.perf_counter()
    O.search_many(t, n, sa, qb, np.arange(s1, dtype=np.uint64) * m, np.full(s1, m, np.uint32), algo, 1)
    one = s1 / (time.perf_counter() - t0)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"value": rate, "unit": "lookups/s", "cores": threads, "kind": "port",
            "single_thread_value": one, "host_cpu": host_cpu(), "host_nproc": os.cpu_count(),
            "affinity_cpus": aff,
            "cores_note": (f"{threads} = this process's CPU share (OMP_NUM_THREADS); the affinity mask shows {aff} "
                           f"hardware threads of the whole machine, shared with the other GPUs' processes")
            if threads < aff else "every CPU of the affinity mask",
            # every affinity CPU is deliberately not used: the GPU box allots each GPU's
            # process a 16-core share (it exports OMP_NUM_THREADS=16) and its operating rules
            # size worker pools to that share, the other CPUs serving the other GPUs' jobs
            "all_affinity_value": None,
            "all_affinity_note": (f"not measured: the box's rules cap this process's worker pools at its "
                                  f"{threads}-core share of the {aff} affinity CPUs" if threads < aff else
                                  "the measured value uses every affinity CPU"),
            "sample": f"oracle/{algo} (restates sas/sa_search.rs "
                      f"{'98-112' if algo == 'binary_search' else '198-239 batch_c<16>'}) on {sample} of the "
                      f"same len-{m} queries over the same 2^{int(np.log2(n))} text/SA ({reps} passes), {dt:.1f} s, "
                      f"{threads} threads (this process's allotted cores), contiguous chunks "
                      f"(sst/bin/bench.rs:558-573)", "_pos": pos}


def c0_record(torch, sas_amd, dev, seconds: float):
    """configs[0]: the reference's CPU run shape (1 MiB ChaCha8 text, 10^4 len-16 queries,
    sas/main.rs:38-61) timed through the oracle restatement on 1 thread and all cores,
    repeated to ~seconds, and the GPU on the same queries; answers compared."""
    from oracle import pyoracle as O
    n, nq, m = 1 << 20, 10_000, 16
    t = O.random_string(n, SEED)
    sa = O.build_sa(t)
    tp = O.padded(t)
    off, _, _ = sas_amd.random_queries(n, nq, seed=SEED, len_lo=m, len_hi=m + 1)
    qb = np.concatenate([t[o:o + m] for o in off.astype(np.int64)] + [np.zeros(64, np.uint8)])
    qoff = np.arange(nq, dtype=np.uint64) * m
    ln = np.full(nq, m, np.uint32)
    res = {}
    allc = host_threads()
    for threads in sorted({1, allc}):
        reps, dt = 0, 0.0
        t0 = time.perf_counter()
        while dt < seconds / 2:
            pos, _ = O.search_many(tp, n, sa, qb, qoff, ln, "binary_search", threads)
            reps += 1
            dt = time.perf_counter() - t0
        res[threads] = (reps * nq / dt, pos)
    idx = sas_amd.SaNaive.build(torch.from_numpy(t).to(dev), lcp=True, prefix=8)
    dq = torch.from_numpy(qb[: nq * m]).to(dev)
    out = idx.search_fixed(dq, m, algo="plain")
    torch.cuda.synchronize()
    gpu_ok = bool(np.array_equal(out.cpu().numpy().astype(np.uint64), res[1][1]))
    if not gpu_ok:
        raise SystemExit("bench c0: GPU positions differ from the CPU restatement")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        idx.search_fixed(dq, m, algo="plain", out=out)
    e1.record()
    torch.cuda.synchronize()
    gms = e0.elapsed_time(e1) / 20
    idx.free()
    return {"workload": "configs[0]: 1 MiB random ACGT text (ChaCha8Rng(31415)), 10^4 len-16 positive queries",
            "cpu_1thread_lookups_per_s": res[1][0], "cpu_all_cores_lookups_per_s": res[allc][0],
            "cpu_cores": allc, "cpu_kind": "port: oracle/binary_search (restates sas/sa_search.rs:98-112)",
            "cpu_ns_per_lookup_1thread": 1e9 / res[1][0], "host_cpu": host_cpu(),
            "gpu_plain_kernel_ms": gms, "gpu_lookups_per_s": nq / (gms * 1e-3),
            "gpu_matches_cpu": gpu_ok,
            "note": "10^4 queries are ~0.1 ms of GPU work: launch-bound, a plumbing check, not a GPU benchmark"}


# ---------------------------------------------------------------- LCP skipping on long queries
LCP_LONG_MS = (64, 128, 256)
LCP_LONG_ALGOS = ("plain", "lcp", "llcp", "stree_llcp", "quad")


def cut_queries(torch, text, off_t, m: int):
    """Fixed-length queries t[off .. off + m) as one uint8 tensor (gathered in chunks)."""
    nq = off_t.numel()
    q = torch.empty(nq * m, dtype=torch.uint8, device=text.device)
    ar = torch.arange(m, device=text.device, dtype=torch.int64)
    step = max(1, (1 << 23) // m)
    for s0 in range(0, nq, step):
        e0 = min(nq, s0 + step)
        q[s0 * m:e0 * m] = text[(off_t[s0:e0, None] + ar[None, :]).reshape(-1)]
    return q


def repetitive_text(torch, n: int, dev, base_log2: int = 24, rate: float = 0.01):
    """A resequencing-shaped text: one random_string base of 2^base_log2 chars (ChaCha8,
    seed 31415 + 2) copied n / 2^base_log2 times, every copy with i.i.d. substitutions at
    `rate` (torch's seeded device generator).  Suffixes of the same locus in two copies
    agree for ~1/(2 rate) chars, the best of 63 other copies for a few hundred: compares
    run long, which is where LCP skipping can pay."""
    import sas_amd
    base = sas_amd.random_string(1 << base_log2, seed=SEED + 2, device=dev)
    t = base.repeat(n >> base_log2)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED)
    chunk = 1 << 26
    for s0 in range(0, n, chunk):
        e0 = min(n, s0 + chunk)
        hit = torch.rand(e0 - s0, generator=g, device=dev) < rate
        sub = torch.randint(1, 4, (e0 - s0,), generator=g, device=dev, dtype=torch.uint8)
        seg = t[s0:e0]
        seg[hit] = (seg[hit] + sub[hit]) & 3  # a different code
    return t


def lcp_long_runs(torch, idx, text, nq: int, steps: int, warmup: int, stream, label: str) -> dict:
    """PLAIN, mlr LCP and Manber-Myers LLCP on the same index over positive queries of
    m = 64, 128, 256 chars: kernel time (events), mean probes, positions identical to
    PLAIN's and every answer an occurrence of its query."""
    n = idx.n
    res = {}
    for m in LCP_LONG_MS:
        import sas_amd
        off = sas_amd.random_queries(n, nq, seed=SEED, word_pos=n, margin=max(256, m), len_lo=m, len_hi=m + 1)[0]
        off_t = torch.from_numpy(off.astype(np.int64)).to(text.device)
        qb = cut_queries(torch, text, off_t, m)
        out = torch.empty(nq, dtype=torch.int64, device=text.device)
        ref = None
        row = {}
        for a in LCP_LONG_ALGOS:
            t = launch_times(torch, lambda: idx.search_fixed(qb, m, algo=a, out=out), steps, warmup, stream)
            if ref is None:
                ref = out.clone()
                occ = cut_queries(torch, text, out.clamp(max=n - m), m)
                if not bool(torch.equal(occ, qb)):
                    raise SystemExit(f"bench lcp_long: {label} m={m} {a} returned a non-occurrence")
                del occ
            elif not bool(torch.equal(out, ref)):
                raise SystemExit(f"bench lcp_long: {label} m={m} {a} differs from plain")
            _, pr = idx.search_fixed(qb, m, algo=a, probes=True)
            row[a] = {"kernel_ms": t["mean_ms"], "kernel_ms_median": t["median_ms"],
                      "lookups_per_s": nq / (t["mean_ms"] * 1e-3), "mean_probes": float(pr.double().mean().item())}
        row["identical"] = True
        res[f"m{m}"] = row
        log(f"lcp_long {label} m={m}: " + ", ".join(f"{a} {row[a]['kernel_ms']:.3f}" for a in LCP_LONG_ALGOS))
        del qb, out, ref, off_t
    return res


def lcp_long_summary(rec: dict) -> dict:
    """{text_m: kernel ms in LCP_LONG_ALGOS order} and which skipping beats PLAIN where."""
    s, wins = {"algos": list(LCP_LONG_ALGOS)}, []
    for tk, rows in rec.items():
        if not isinstance(rows, dict) or tk in ("what", "summary"):
            continue
        for mk, row in rows.items():
            if not isinstance(row, dict) or "plain" not in row:
                continue
            ms = [_r(row[a]["kernel_ms"]) for a in LCP_LONG_ALGOS]
            s[f"{tk}_{mk}"] = ms
            for a in ("lcp", "llcp", "stree_llcp"):
                if row[a]["kernel_ms"] < row["plain"]["kernel_ms"]:
                    wins.append(f"{a}@{tk}_{mk}:{row['plain']['kernel_ms'] / row[a]['kernel_ms']:.2f}x")
    return {"ms": s, "skipping_beats_plain": wins}


# ---------------------------------------------------------------- configs[3]
def c3_record(args, torch, sas_amd, dev, rank, algo="tagged", extra_algos=("plain", "lcp")):
    """configs[3]-shaped run: n = 2^34 chars (16 GiB of byte-coded text; BASELINE's
    "64 GiB" = 2^36 chars cannot hold any SA in 288 GB) and 10^8 positive
    queries of mixed length 8..256 (random_queries with len in [8, 257), sas/util.rs:18-26),
    ragged, through sas_search_batch on device buffers.  TAGGED on bucket lines
    (SAS_BUILD_TAGGED | SAS_BUILD_TAG_LINES, p = 15: a bucket's header and first 20 entries in
    one 128-B line) by default (--c3-layout lines); then, as the cross-check, the rank-ordered
    tagged index (8-B tagged SA entries + a p = 16 bucket table) with TAGGED and the
    extra algorithms, whose positions must be identical.  PREFIX / QUAD: compact key-only quad
    leaves beside the 40-bit SA (+ a p = 16 40-bit rank table for PREFIX).  The indexes are
    built one after the other from a host copy of the text (two do not fit in HBM together,
    nor does a device byte copy beside the bucket-line build)."""
    n = args.c3_n
    nq = args.c3_nq
    t0 = time.perf_counter()
    text = sas_amd.random_string(n, seed=SEED, device=dev)
    htext = text.cpu().numpy()
    del text
    torch.cuda.empty_cache()

    def build(kind):
        # verify: the reference's adjacency assertion (sas/sa_search.rs:36-38) + permutation, on the GPU
        if kind in ("lines", "tagged"):
            return sas_amd.SaNaive.build(htext, lcp=False, verify=True, tagged=True, tag_lines=kind == "lines")
        return sas_amd.SaNaive.build(htext, lcp=False, stree=kind == "stree", sector=False,
                                     quad="compact" if kind in ("quad", "prefix") else False, verify=True,
                                     llcp=False, prefix=16 if kind == "prefix" else False)
    lines = algo == "tagged" and args.c3_layout == "lines"
    phases = [("lines", (algo,)), ("tagged", (algo,) + tuple(x for x in extra_algos if x != algo))] if lines else \
        [(algo, (algo,) + tuple(x for x in extra_algos if x != algo))]
    if args.c3_no_cross:
        phases = phases[:1]
    idx = build(phases[0][0])
    st = idx.stats()
    # queries are cut from, and answers checked against, the index's packed text
    off, ln, _ = sas_amd.random_queries(n, nq, seed=SEED, word_pos=n + rank * 8 * nq, margin=256, len_lo=8,
                                        len_hi=257)
    lens = torch.from_numpy(ln.astype(np.int64)).to(dev)
    qoff = torch.zeros(nq, dtype=torch.int64, device=dev)
    qoff[1:] = torch.cumsum(lens, 0)[:-1]
    total = int(lens.sum().item())
    qbytes = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    src = torch.from_numpy(off.astype(np.int64)).to(dev)
    qlen = lens.to(torch.int32)
    idx.extract(src, qlen, qoff, qbytes)  # t[off .. off + len) from the packed text
    out = torch.empty(nq, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    log(f"c3 setup {setup:.1f} s ({phases[0][0]}, n={n}, nq={nq})")
    mean_m = total / nq
    res, ref, stats_of, slices = {}, None, {}, None
    for pi, (kind, algos) in enumerate(phases):
        if pi > 0:
            idx.free()
            torch.cuda.empty_cache()
            tb = time.perf_counter()
            idx = build(kind)
            log(f"c3 {kind} index built in {time.perf_counter() - tb:.1f} s")
        kst = idx.stats()
        stats_of[kind] = kst
        for a in algos:
            name = "tagged_lines" if kind == "lines" else a

            def step():
                idx.search_batch(qbytes, qoff, qlen, algo=a, out=out)
            steps = args.c3_steps
            ct = launch_times(torch, step, steps, args.warmup, torch.cuda.current_stream(dev))
            el, kms = ct["wall_s"], ct["mean_ms"]
            if ref is None:
                ref = out.clone()
                # guard 1: each answer is an occurrence of its query (positive queries)
                okc = True
                chunk = 1 << 20
                for s in range(0, nq, chunk):
                    e = min(nq, s + chunk)
                    span = int((qoff[e - 1] + lens[e - 1] - qoff[s]).item())
                    got = torch.empty(span, dtype=torch.uint8, device=dev)
                    idx.extract(out[s:e].contiguous(), qlen[s:e].contiguous(), (qoff[s:e] - qoff[s]).contiguous(),
                                got)
                    okc &= bool(torch.equal(got, qbytes[qoff[s]:qoff[s] + span]))
                if not okc:
                    raise SystemExit(f"bench c3: {name} returned a non-occurrence position")
                # guard 2: exact lower bounds on a sample
                rng = np.random.default_rng(7)
                ids = np.sort(rng.choice(nq, size=min(nq, args.proof_sample), replace=False))
                dids = torch.from_numpy(ids).to(dev)
                qo_h = qoff[dids].cpu().numpy()
                hq = {}
                for j, i in enumerate(ids):
                    hq[int(i)] = qbytes[int(qo_h[j]):int(qo_h[j]) + int(ln[i])].cpu().numpy()

                def window(p, L):
                    L = min(L, n - p)
                    if L <= 0:
                        return np.zeros(0, np.uint8)
                    o = torch.empty(L, dtype=torch.uint8, device=dev)
                    idx.extract(torch.tensor([p], dtype=torch.int64, device=dev),
                                torch.tensor([L], dtype=torch.int32, device=dev),
                                torch.zeros(1, dtype=torch.int64, device=dev), o)
                    return o.cpu().numpy()
                nbad = lower_bound_proof(idx, window, lambda i: hq[i], out[dids].cpu().numpy(), ids)
                if nbad:
                    raise SystemExit(f"bench c3: {nbad} of {len(ids)} sampled answers are not exact lower bounds")
                agrees = True
            else:
                agrees = bool(torch.equal(out, ref))
                if not agrees:
                    raise SystemExit(f"bench c3: {name} differs from the first record")
            _, pr = idx.search_batch(qbytes, qoff, qlen, algo=a, probes=True)
            mp = float(pr.double().mean().item())
            bpl = bytes_per_lookup(a, kst, n, mean_m, mp)
            pmc_key = f"c3_{name}_n{n}_q{nq}"
            res[name] = record(name, nq, kms, el, bpl, footprint(a, kst), load_pmc(pmc_key) if a == algo else None,
                               mp, {"identical_to_first": agrees, "lookups_per_s": nq * steps / el,
                                    "kernel_ms_median": ct["median_ms"], "timed_launches": steps,
                                    "index": "bucket lines (SAS_BUILD_TAG_LINES)" if kind == "lines" else
                                    ("rank-ordered tagged entries + bucket table" if kind == "tagged" else kind)})
            log(f"c3 {name}: {kms:.3f} ms per {nq}")
            if pi == 0 and algo == "tagged":
                # the same queries handed over as the slices of the text they are (random_queries
                # returns borrowed &t[i..i+len], sas/util.rs:18-26): offsets + lengths, no query
                # bytes; a lookup whose candidate is the query's own suffix skips its text compare
                sl_t = launch_times(torch, lambda: idx.search_slices(src, qlen, out=out), args.c3_steps, args.warmup,
                                    torch.cuda.current_stream(dev))
                sms = sl_t["mean_ms"]
                same = bool(torch.equal(out, ref))
                if not same:
                    raise SystemExit("bench c3: text-slice queries differ from the byte queries")
                slices = {"what": "the same queries as slices of the indexed text (sas_search_batch with "
                                  "SAS_QUERIES_ARE_SLICES: offsets + lengths, chars from the packed text)",
                          "kernel_ms": sms, "kernel_ms_median": sl_t["median_ms"], "lookups_per_s": nq / (sms * 1e-3),
                          "identical_to_first": same}
                log(f"c3 {name} slices: {sms:.3f} ms per {nq}")
    first = "tagged_lines" if lines else algo
    h = res[first]
    idx.free()
    del qbytes, qoff, qlen, lens, out, ref, src, htext
    torch.cuda.empty_cache()
    kst = stats_of[phases[0][0]]
    ent = (f"48-bit tagged entries ({kst['tag_line_tag_bits']}-bit tags), {kst['tag_line_slots']} per 128-B "
           f"bucket line" if lines else f"{kst['sa_width'] * 8}-bit {'tagged entries' if algo == 'tagged' else 'SA'}")
    return {"workload": f"configs[3]-shaped: n = 2^{int(np.log2(n))} chars ({ent}), {nq} positive queries of length "
                        f"8..256 (mean {mean_m:.1f}), ragged",
            "algo": first, "lookups_per_s": h["lookups_per_s"], "kernel_ms": h["kernel_ms"],
            "ns_per_lookup": h["ns_per_lookup"], "kernel_ms_median": h.get("kernel_ms_median"),
            "index_bytes": kst["index_bytes"], "setup_s": setup,
            "proof_sample": args.proof_sample, "verified": True,
            "roofline": {"bound": "hbm", "achieved": h["achieved_hbm_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": h["achieved_hbm_GBps"] / HBM_PEAK_GBPS,
                         "traffic": (h.get("pmc") or {}).get("fabric_bytes_per_lookup"),
                         "kernel": "k_sa_tagged_lines" if lines else KERNELS.get(algo, "k_sa_prefix")},
            "variants": res, "text_slices": slices,
            "index": {k: kst[k] for k in ("sa_width", "sa_bytes", "quad_bytes", "prefix_chars", "prefix_bytes",
                                          "tag_chars", "tag_table_bytes", "tag_line_slots", "tag_overflow_entries",
                                          "index_bytes", "build_sa_ns", "build_total_ns")}}


def c4_proof(torch, idx, engine, n: int, m: int, ws: int, rank: int, sample: int) -> dict:
    """lower_bound_proof on the slots this rank received in its last sharded step
    (ShardedSearch.last): their queries (bytes, or 2-bit words unpacked), the local
    answers, windows of this rank's packed text."""
    L = getattr(engine, "last", None)
    if L is None:
        return {"checked": 0, "failures": 0}
    cap = int(L["cap"])
    rc = np.minimum(L["rcounts"].cpu().numpy().astype(np.int64), cap)
    filled = np.concatenate([b * cap + np.arange(int(c), dtype=np.int64) for b, c in enumerate(rc)] +
                            [np.zeros(0, np.int64)])
    if len(filled) == 0:
        return {"checked": 0, "failures": 0}
    rng = np.random.default_rng(101 + rank)
    ids = np.sort(rng.choice(filled, size=min(len(filled), sample), replace=False))
    dids = torch.from_numpy(ids).to(L["recv"].device)
    if L["packed"]:
        w = L["recv"][dids].cpu().numpy().view(np.uint64)
        sh = (62 - 2 * np.arange(m, dtype=np.uint64)).astype(np.uint64)
        qs = ((w[:, None] >> sh[None, :]) & np.uint64(3)).astype(np.uint8)
    else:
        qs = L["recv"].view(-1, m)[dids].cpu().numpy()
    ans = L["local"][dids].cpu().numpy()
    qmap = {int(i): qs[j] for j, i in enumerate(ids)}
    dev = L["recv"].device

    def window(p, ln):
        ln = min(ln, n - p)
        if ln <= 0:
            return np.zeros(0, np.uint8)
        o = torch.empty(ln, dtype=torch.uint8, device=dev)
        idx.extract(torch.tensor([p], dtype=torch.int64, device=dev), torch.tensor([ln], dtype=torch.int32, device=dev),
                    torch.zeros(1, dtype=torch.int64, device=dev), o)
        return o.cpu().numpy()
    bad = lower_bound_proof(idx, window, lambda i: qmap[i], ans, ids)
    return {"checked": int(len(ids)), "failures": int(bad)}


def c4_record(args, torch, sas_amd, dev, ws, rank, dist):
    """configs[4]: the text sharded across the GPUs: SA rank ranges, one part
    per rank (sas_build_part, no rank builds the whole SA), queries routed to the owner of
    their lower bound with RCCL all_to_all_single over fixed-capacity buckets, PREFIX
    queries crossing as 8-B packed words, positions back.  Weak scaling at a fixed share
    of args.c4_share chars per GPU (default: the largest share <= 2^33 whose part fits one
    GPU, c4_share_for: 2^33 at N >= 2, 2^32 at N = 1 where the one part holds the whole
    4^16-key table; BASELINE's "512 GiB" cannot hold a full SA even across 8 x 288 GB,
    DESIGN.md §6); each part's inline table covers only its own key interval (1/N of the
    keys); each rank searches its own 10^7 len-32 positive queries.  N = 1 runs the same
    step through a world-1 RCCL group."""
    from sas_amd.shard import ShardedSearch
    share = args.c4_share or c4_share_for(ws, torch.cuda.mem_get_info(dev)[1])
    n = share * ws
    nq, m = args.nq, args.m
    t0 = time.perf_counter()
    own = None
    if dist is None or not dist.is_initialized():
        import socket
        import torch.distributed as tdist
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        dist = own = tdist
    # the local setup may fail on one rank (e.g. HBM): every rank agrees before the first
    # collective of the step, so a failure skips the record instead of hanging the others
    err = None
    try:
        # the text is generated on the GPU straight into this rank's packed text (the whole
        # text, n/4 bytes: compares need any suffix), never as n bytes; the part holds only
        # its own SA rank range (sas_build_part_gen) with the two-suffix inline table
        # (local ranks < 2^32; SA bits 32..39 in slot 1 above 2^32 chars)
        # (the pivot blocks: the LDS levels only, 72.5 KiB -- PREFIX never reads them)
        idx = sas_amd.SaNaive.build_part_gen(n, seed=SEED + 1, part=rank, parts=ws, lcp=False, stree=False,
                                             sector=False, quad=True, llcp=False, prefix=16, prefix_inline=2,
                                             top2_levels=TOP_LDS_LEVELS)
        st = idx.stats()
        off = torch.from_numpy(rank_query_offsets(n, nq, m, rank).astype(np.int64)).to(dev)
        qbytes = torch.empty(nq * m, dtype=torch.uint8, device=dev)
        idx.extract(off, torch.full((nq,), m, dtype=torch.int32, device=dev),
                    torch.arange(nq, device=dev, dtype=torch.int64) * m, qbytes)
        del off
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 -- reported in the record
        err = repr(e)
    okt = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    if not int(okt.item()):
        if own is not None:
            own.destroy_process_group()
        return {"workload": "configs[4]-shaped (sharded text)", "skipped": err or "setup failed on another rank"}
    # the capacity is agreed once for this batch size (max_nq): the steps run no collective
    # beyond the exchanges, and at N = 1 the exchanges are the identity (no collective at all)
    engine = ShardedSearch(idx, dist, ws, rank, dev, algo="prefix", chunks=args.shard_chunks, max_nq=nq)
    out = torch.empty(nq, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0

    def reduce_max(x):
        tt = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())
    el = timed_loop(lambda: engine.search_fixed(qbytes, m, check=False, out=out), args.c4_steps, args.warmup,
                    torch.cuda.synchronize, dist.barrier, reduce_max)
    engine.assert_no_overflow()
    # the other step shape, for the next round's choice at N > 1 (where the exchanges cross
    # xGMI): the batch in 2 pieces (or in 1 if the main run used pieces), exchanges async
    alt_chunks = 2 if args.shard_chunks == 1 else 1
    alt = ShardedSearch(idx, dist, ws, rank, dev, algo="prefix", chunks=alt_chunks, max_nq=nq)
    out2 = torch.empty(nq, dtype=torch.int64, device=dev)
    el2 = timed_loop(lambda: alt.search_fixed(qbytes, m, check=False, out=out2), max(3, args.c4_steps // 2),
                     args.warmup, torch.cuda.synchronize, dist.barrier, reduce_max)
    alt.assert_no_overflow()
    same = torch.tensor([int(bool(torch.equal(out, out2)))], dtype=torch.int32, device=dev)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if not int(same.item()):
        raise SystemExit("bench c4: the pieced step differs from the whole step")
    del out2
    rccl1 = None
    if ws == 1:  # the same step with the world-1 exchanges sent through RCCL (self copies)
        eng1 = ShardedSearch(idx, dist, ws, rank, dev, algo="prefix", max_nq=nq, exchange_self=True)
        out3 = torch.empty(nq, dtype=torch.int64, device=dev)
        el3 = timed_loop(lambda: eng1.search_fixed(qbytes, m, check=False, out=out3), max(3, args.c4_steps // 2),
                         args.warmup, torch.cuda.synchronize, dist.barrier, reduce_max)
        eng1.assert_no_overflow()
        if not bool(torch.equal(out, out3)):
            raise SystemExit("bench c4: the RCCL world-1 exchange differs from the identity exchange")
        rccl1 = {"ms_per_step": el3 / max(3, args.c4_steps // 2) * 1e3,
                 "lookups_per_s": nq * max(3, args.c4_steps // 2) / el3, "identical": True,
                 "what": "exchange_self: the count, query and position exchanges through the world-1 RCCL group"}
        del out3
    # every answer an occurrence of its query (read back from this rank's packed text)
    occ = torch.empty_like(qbytes)
    idx.extract(out.clamp(max=n - m), torch.full((nq,), m, dtype=torch.int32, device=dev),
                torch.arange(nq, device=dev, dtype=torch.int64) * m, occ)
    ok = torch.tensor([int(bool(torch.equal(occ, qbytes)))], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        raise SystemExit("bench c4: a sharded answer is not an occurrence of its query")
    # and a sample of the queries this rank received proven exact lower bounds on its own
    # part: SA[lo] = its answer, suffix(SA[lo-1]) < q <= suffix(SA[lo]) (lo past the part:
    # the next part's first suffix, next_pos)
    proven = c4_proof(torch, idx, engine, n, m, ws, rank, max(1, args.proof_sample // ws))
    bad = torch.tensor([proven["failures"]], dtype=torch.int64, device=dev)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if int(bad.item()):
        raise SystemExit(f"bench c4: {int(bad.item())} sampled sharded answers are not exact lower bounds")
    cap = engine.capacity(-(-nq // max(1, args.shard_chunks)))  # per piece
    rec = {"workload": f"configs[4]-shaped: text of {ws} x {share} chars sharded by SA rank ranges over "
                       f"{ws} GPU(s) (sas_build_part), {nq} len-{m} queries per GPU routed with RCCL "
                       f"all_to_all_single (fixed-capacity buckets, 8-B packed PREFIX queries, per-bucket counts "
                       f"exchanged so only filled slots are searched), positions back"
                       + (" -- at N = 1 every query is local: the exchanges are the identity, no collective "
                          "(rccl_world1 times them through RCCL)" if ws == 1 else ""),
           "n": n, "parts": ws, "lookups_per_s": ws * nq * args.c4_steps / el, "ms_per_step": el / args.c4_steps * 1e3,
           "steps": args.c4_steps, "scaling": "weak", "part_sa_entries": st["sa_entries"],
           "prefix_entry_bytes": prefix_entry_bytes(st), "share": share,
           "prefix_keys": st["prefix_entries"], "prefix_bytes": st["prefix_bytes"],
           "prefix_key_fraction": _r(st["prefix_entries"] / (4 ** st["prefix_chars"] + 1)),
           "bucket_capacity": cap, "pieces": args.shard_chunks,
           "alt_pieces": {"pieces": alt_chunks, "ms_per_step": el2 / max(3, args.c4_steps // 2) * 1e3,
                          "lookups_per_s": ws * nq * max(3, args.c4_steps // 2) / el2, "identical": True},
           "exchange_bytes_per_step_per_rank": 2 * ws * cap * 8 * args.shard_chunks if ws > 1 else 0,
           "rccl_world1": rccl1,
           "index_bytes": st["index_bytes"], "setup_s": setup, "verified": True,
           "proven": proven["checked"], "proof": "each rank: a sample of the queries it received in its last step, "
                                                  "proven exact lower bounds on its own part's SA"}
    idx.free()
    del qbytes, out, occ
    torch.cuda.empty_cache()
    if own is not None:
        own.destroy_process_group()
    return rec


def run_c3(args, torch, sas_amd, dev, ws, rank):
    """--workload c3: the configs[3] record on its own line."""
    algo = args.algo or "tagged"
    rec = c3_record(args, torch, sas_amd, dev, rank, algo=algo, extra_algos=("plain", "lcp"))
    if rank == 0:
        emit({"metric": "pattern lookups/s (configs[3] shape)", "value": rec["lookups_per_s"], "unit": "lookups/s",
              "n_gpus": ws, "steps": args.c3_steps, "warmup": args.warmup,
              "ms_per_step": args.c3_nq / rec["lookups_per_s"] * 1e3, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "u8",
              "data": f"synthetic: random_string(ChaCha8Rng({SEED})) text, positive queries len in [8,257)",
              "config": {"workload": rec["workload"], "n": args.c3_n, "queries_per_gpu": args.c3_nq, "algo": algo},
              "roofline": rec["roofline"], "c3": rec})


# ---------------------------------------------------------------- u32 path
def sst_layouts(sas_amd):
    """Every GPU layout of the u32 path by the reference's names (sst/bin/bench.rs:487-599)."""
    return {
        "SortedVec": lambda v: sas_amd.SortedVec.new(v),
        "Eytzinger": lambda v: sas_amd.Eytzinger.new(v),
        "STree16": lambda v: sas_amd.STree16.new(v),
        "STree16_left_max": lambda v: sas_amd.STree16.new_params(v, True, False, False),
        "STree15": lambda v: sas_amd.STree15.new(v),
        "PartitionedSTree16M_b16": lambda v: sas_amd.PartitionedSTree16M.new(v, 16),
        "PartitionedSTree16M_b20": lambda v: sas_amd.PartitionedSTree16M.new(v, 20),
        "PartitionedSTree16_b16": lambda v: sas_amd.PartitionedSTree16.new(v, 16),
        "PartitionedSTree16C_b16": lambda v: sas_amd.PartitionedSTree16C.new(v, 16),
        "PartitionedSTree16L_b16": lambda v: sas_amd.PartitionedSTree16L.new(v, 16),
        "PartitionedSTree16O_b16": lambda v: sas_amd.PartitionedSTree16O.new(v, 16),
        "DirectMap": lambda v: sas_amd.DirectMap.new(v),
    }


# the default line's u32 lineup: the reference's oracle (SortedVec::binary_search), its bench
# variant (STree16 left_max, sst/bin/bench.rs:96), its best (PartitionedSTree16M, both b of
# its differential test's large end) and the prefix map taken to its limit
SST_LINEUP = ("SortedVec", "STree16_left_max", "PartitionedSTree16M_b16", "PartitionedSTree16M_b20", "DirectMap")
SST_KERNELS = {"SortedVec": "k_sst_sorted", "Eytzinger": "k_sst_eytzinger", "DirectMap": "k_sst_direct",
               "PartitionedSTree16M_b16": "k_sst_pmap4", "PartitionedSTree16M_b20": "k_sst_pmap4"}


def sst_bytes_per_lookup(name: str, layers: int, keys: int) -> float:
    """SURVEY §8(d)-style algorithmic bytes of one u32 lookup: the query word, the answer word,
    and per level what the layout reads (a 64-B node per S-tree layer, a 4-B key per binary /
    Eytzinger probe, one 16-B entry for DirectMap's table)."""
    if name.startswith("SortedVec") or name.startswith("Eytzinger"):
        return 4 * (keys.bit_length()) + 8
    if name == "DirectMap":
        return 16 + 8
    return 64 * layers + 8


def sst_workload(nk: int, nq: int, positive: bool = False):
    """gen_vals (uniform < i32::MAX, vals[0] = MAX, sorted; sst/util.rs:31-42) and 10^7
    gen_queries (:16-21) or gen_positive_queries (:23-28)."""
    from oracle import pyoracle as O
    rng = np.random.default_rng(SEED)
    vals = rng.integers(0, O.MAX, nk, dtype=np.uint64).astype(np.uint32)
    vals[0] = O.MAX
    vals.sort()
    qs = vals[rng.integers(0, nk, nq)] if positive else rng.integers(0, O.MAX, nq, dtype=np.uint64).astype(np.uint32)
    return vals, qs


def sst_record(args, torch, sas_amd, dev, names=SST_LINEUP, nk: int = 1 << 28, cpu: bool = True) -> dict:
    """The u32 static-search-tree path (sst/bin/bench.rs:548-599, "40x faster binary search",
    readme.org:8) at the reference's largest size: 2^28 keys (1 GiB) and 10^7 uniform queries.
    Every layout is timed like the headline (the driver's steps and warmup, one HIP event pair
    per launch) and must return SortedVec::binary_search's value (the oracle) on every query.
    Roofline: these kernels are bound by random 64-B node requests, so `frac` is the measured
    L2->fabric request rate (same-hash PMC summary, profiles/pmc_sst_*.json) over the
    calibrated random-request ceiling; `frac_hbm` the PMC bytes over 8 TB/s.  CPU: the
    oracle's STree16 left_max batch_final::<128> restatement (the reference's bench variant)
    on the allotted threads."""
    from oracle import pyoracle as O
    nq = args.nq
    vals, qs = sst_workload(nk, nq, getattr(args, "positive", False))
    expect = O.SortedVec(vals).query(qs)
    dq = torch.from_numpy(qs.view(np.int32)).to(dev)
    dout = torch.empty(nq, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    mk = sst_layouts(sas_amd)
    res = {}
    for name in names:
        idx = mk[name](vals)
        t = launch_times(torch, lambda: idx.query(dq, stream=stream.cuda_stream, out=dout), args.steps, args.warmup,
                         stream)
        got = dout.cpu().numpy().view(np.uint32)
        if not np.array_equal(got, expect):
            raise SystemExit(f"bench sst: {name} differs from SortedVec::binary_search")
        layers, size = idx.layers(), idx.size()
        idx.free()
        ks = t["mean_ms"] * 1e-3
        bpl = sst_bytes_per_lookup(name, layers, nk)
        r = {"lookups_per_s": nq / ks, "kernel_ms": t["mean_ms"], "kernel_ms_median": t["median_ms"],
             "ns_per_lookup": ks * 1e9 / nq, "layers": layers, "index_bytes": size,
             "bytes_per_lookup_model": bpl, "frac_8d_model": bpl * nq / ks / 1e9 / HBM_PEAK_GBPS,
             "equals_sortedvec": True, "kernel": SST_KERNELS.get(name, "k_sst_stree4")}
        pmc = load_pmc(f"sst_{name}_k{nk}_q{nq}")
        if pmc and not pmc.get("stale") and pmc.get("rdreq_per_launch"):
            r["requests_per_lookup"] = pmc["rdreq_per_launch"] / nq
            r["traffic"] = pmc["hbm_bytes_per_launch"] / nq
            r["req_frac"] = pmc["rdreq_per_launch"] / ks / CACHE_REQ_CEILING
            r["frac_hbm"] = pmc["hbm_bytes_per_launch"] / ks / 1e9 / HBM_PEAK_GBPS
            r["pmc_source"] = pmc["source"]
        elif pmc:
            r["pmc"] = pmc
        res[name] = r
    best = max(res, key=lambda k: res[k]["lookups_per_s"])
    rec = {"workload": f"u32 static-search-tree path: {nk} keys (gen_vals, {nk * 4 >> 20} MiB), {nq} uniform queries "
                       f"(gen_queries), value of the first key >= q; every layout equal to SortedVec::binary_search",
           "keys": nk, "queries": nq, "best": best, "layouts": res,
           "frac_basis": "frac = PMC L2->fabric read requests / kernel time / the measured random-request ceiling "
                         f"({CACHE_REQ_CEILING:.3g}/s); frac_hbm = PMC bytes (requests x 128 B + writes) / time / 8 TB/s"}
    if cpu:
        tree = O.STree(vals, left_max=True)
        threads = host_threads()
        t0 = time.perf_counter()
        cpu_out = tree.query_batch(qs, threads)
        dt = time.perf_counter() - t0
        s1 = min(nq, 2_000_000)
        t1 = time.perf_counter()
        tree.query_batch(qs[:s1], 1)
        one = s1 / (time.perf_counter() - t1)
        rec["cpu_baseline"] = {"value": nq / dt, "unit": "lookups/s", "cores": threads, "kind": "port",
                               "single_thread_value": one, "agrees": bool(np.array_equal(cpu_out, expect)),
                               "sample": f"oracle STree16 left_max + batch_final::<128> restatement "
                                         f"(sst/s_tree.rs:303-326) on all {nq} queries, {threads} threads"}
        if not rec["cpu_baseline"]["agrees"]:
            raise SystemExit("bench sst: the CPU restatement differs from SortedVec")
    return rec


def sst_summary(rec: dict) -> dict:
    """configs.sst of the line: the best layout, the reference's bench variant and oracle."""
    b = rec["best"]
    lay = rec["layouts"]
    L = lay[b]
    out = {"best": b, "lookups_per_s": _r(L["lookups_per_s"]), "kernel_ms": _r(L["kernel_ms"]),
           "kernel_ms_median": _r(L["kernel_ms_median"]),
           "frac": _r(L.get("req_frac"), 3), "frac_hbm": _r(L.get("frac_hbm"), 3), "traffic": _r(L.get("traffic")),
           "index_bytes": L["index_bytes"],
           "ms": {k.replace("PartitionedSTree16M_", "PSTree16M_"): _r(v["kernel_ms"]) for k, v in lay.items()},
           "stree16_left_max_frac": _r(lay.get("STree16_left_max", {}).get("req_frac"), 3),
           "equal_to_sortedvec": all(v["equals_sortedvec"] for v in lay.values())}
    cpu = rec.get("cpu_baseline")
    if cpu:
        out["cpu"] = _r(cpu["value"])
        out["cpu_cores"] = cpu["cores"]
    return out


def run_sst(args, torch, sas_amd, dev, ws, rank):
    """--workload sst: the u32 path on its own line (every layout, or --sst-layouts), with the
    --range mode (sst/bin/bench.rs:84-109) through STree16 left_max."""
    from oracle import pyoracle as O
    nk = args.n if args.n != 1 << 30 else 1 << 28
    names = tuple(args.sst_layouts.split(",")) if args.sst_layouts else tuple(sst_layouts(sas_amd))
    rec = sst_record(args, torch, sas_amd, dev, names, nk=nk, cpu=not args.no_cpu)
    nq = args.nq
    vals, qs = sst_workload(nk, nq, args.positive)
    range_res = None
    if not args.sst_layouts:
        # --range mode: the interleaved [q, q+1] stream through STree16 left_max;
        # rank(q+1) - rank(q) = number of keys equal to q (checked)
        rq = np.stack([qs, np.minimum(qs.astype(np.uint64) + 1, O.MAX).astype(np.uint32)], 1).reshape(-1)
        drq = torch.from_numpy(rq.view(np.int32)).to(dev)
        drout = torch.empty(2 * nq, dtype=torch.int32, device=dev)
        st16 = sas_amd.STree16.new_params(vals, True, False, False)
        for _ in range(args.warmup):
            st16.query(drq)
        rkns = st16.time_query(drq, drout, reps=args.steps, stream=torch.cuda.current_stream(dev).cuda_stream)
        sample = rq[: 2 * min(nq, 100_000)]
        _, rk = st16.query(sample, want_rank=True)
        cnt = rk[1::2].astype(np.int64) - rk[0::2].astype(np.int64)
        expect = np.searchsorted(vals, sample[1::2], "left") - np.searchsorted(vals, sample[0::2], "left")
        range_res = {"queries": 2 * nq, "lookups_per_s": 2 * nq / (rkns * 1e-9), "kernel_ms": rkns * 1e-6,
                     "ranges_per_s": nq / (rkns * 1e-9), "counts_verified": bool(np.array_equal(cnt, expect))}
        st16.free()
    best = rec["best"]
    emit({
        "metric": "u32 static-search-tree lookups/s (2^28 keys = 1 GiB, 10^7 uniform queries)",
        "value": rec["layouts"][best]["lookups_per_s"], "unit": "lookups/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True, "dtype": "u32", "vs_baseline": None,
        "data": "synthetic: gen_vals / gen_queries shapes (sst/util.rs:16-42)",
        "config": {"workload": "sst u32 path", "keys": nk, "queries": nq, "best": best},
        "layouts": rec["layouts"],
        "range_mode": range_res,
        "queries_kind": "positive" if args.positive else "uniform",
        "cpu_baseline": rec.get("cpu_baseline")})


def ref_sizes(frm: int = 5, to: int = 30, dense: bool = False):
    """sizes() of the reference's u32 bench (sst/bin/bench.rs:453-471): bytes 2^from .. 2^to
    (and 5/4, 3/2, 7/4 of each power with --dense)."""
    v = []
    for b in range(frm, to):
        v.append(1 << b)
        if dense:
            v += [(1 << b) * 5 // 4, (1 << b) * 3 // 2, (1 << b) * 7 // 4]
    v.append(1 << to)
    return v


def run_sst_sweep(args, torch, sas_amd, dev):
    """The reference's u32 size sweep (sst/bin/bench.rs:50-110, 453-471): gen_vals of the
    largest size (vals[0] = MAX), each size takes its prefix and sorts it; 10^6 uniform queries
    (gen_queries, next_multiple_of(768)); per size every GPU layout (kernel time, HIP events)
    and the CPU restatements of the reference's two ends of the '40x' claim (readme.org:8):
    SortedVec::binary_search on 1 thread and STree16 left_max batch_final::<128> on 1 and all
    allotted threads (the reference times 1 and 6, :497-498).  Every GPU layout's answers
    must equal SortedVec's on every query."""
    from oracle import pyoracle as O
    sizes = ref_sizes(5, args.sweep_to, args.sweep_dense)
    nmax = sizes[-1] // 4
    rng = np.random.default_rng(SEED)
    allv = rng.integers(0, O.MAX, nmax, dtype=np.uint64).astype(np.uint32)
    allv[0] = O.MAX
    nq = -(-1_000_000 // 768) * 768
    qs = rng.integers(0, O.MAX, nq, dtype=np.uint64).astype(np.uint32)
    dq = torch.from_numpy(qs.view(np.int32)).to(dev)
    dout = torch.empty(nq, dtype=torch.int32, device=dev)
    threads = host_threads()
    layouts = {
        "SortedVec": lambda v: sas_amd.SortedVec.new(v),
        "Eytzinger": lambda v: sas_amd.Eytzinger.new(v),
        "STree16_left_max": lambda v: sas_amd.STree16.new_params(v, True, False, False),
        "PartitionedSTree16M_b16": lambda v: sas_amd.PartitionedSTree16M.new(v, 16),
        "DirectMap": lambda v: sas_amd.DirectMap.new(v),
    }
    rows = []
    for size in sizes:
        vals = np.sort(allv[: max(1, size // 4)])
        ref = O.SortedVec(vals).query(qs)
        row = {"size_bytes": size, "keys": len(vals), "gpu": {}, "cpu": {}}
        for name, mk in layouts.items():
            try:
                idx = mk(vals)
            except Exception as e:  # noqa: BLE001 -- a layout that cannot take this size is skipped
                row["gpu"][name] = {"skipped": repr(e)[:120]}
                continue
            idx.query(dq)
            kns = idx.time_query(dq, dout, reps=args.steps, stream=torch.cuda.current_stream(dev).cuda_stream)
            got = dout.cpu().numpy().view(np.uint32)
            if not np.array_equal(got, ref):
                raise SystemExit(f"bench sst sweep: {name} differs from SortedVec at {size} B")
            row["gpu"][name] = {"lookups_per_s": nq / (kns * 1e-9), "ns_per_lookup": kns / nq,
                                "layers": idx.layers(), "index_bytes": idx.size()}
            idx.free()
        sv = O.SortedVec(vals)
        t0 = time.perf_counter()
        sv.query(qs)
        row["cpu"]["SortedVec_binary_search_1t"] = nq / (time.perf_counter() - t0)
        tree = O.STree(vals, left_max=True)
        for th in sorted({1, threads}):
            t0 = time.perf_counter()
            got = tree.query_batch(qs, th)
            row["cpu"][f"STree16_left_max_batch_final128_{th}t"] = nq / (time.perf_counter() - t0)
            if not np.array_equal(got, ref):
                raise SystemExit(f"bench sst sweep: CPU STree16 differs from SortedVec at {size} B")
        row["cpu_stree_over_binary_search_1t"] = (row["cpu"]["STree16_left_max_batch_final128_1t"] /
                                                  row["cpu"]["SortedVec_binary_search_1t"])
        best = max((k for k in row["gpu"] if "lookups_per_s" in row["gpu"][k]),
                   key=lambda k: row["gpu"][k]["lookups_per_s"])
        row["gpu_best"] = best
        row["gpu_best_over_cpu_binary_search_1t"] = (row["gpu"][best]["lookups_per_s"] /
                                                     row["cpu"]["SortedVec_binary_search_1t"])
        rows.append(row)
        log(f"sweep {size} B: best {best} {row['gpu'][best]['lookups_per_s']:.3g}/s, CPU STree/binary "
            f"{row['cpu_stree_over_binary_search_1t']:.1f}x")
    emit({"metric": "u32 static-search-tree lookups/s across the reference's size sweep (32 B .. 2^%d B)" %
                    args.sweep_to,
          "value": rows[-1]["gpu"][rows[-1]["gpu_best"]]["lookups_per_s"], "unit": "lookups/s", "n_gpus": 1,
          "steps": args.steps, "warmup": 1, "higher_is_better": True, "dtype": "u32", "vs_baseline": None,
          "data": "synthetic: gen_vals / gen_queries shapes (sst/util.rs:16-42), prefixes of one draw",
          "config": {"workload": "sst u32 size sweep (sst/bin/bench.rs:453-471)", "queries": nq,
                     "cpu_threads": threads, "dense": args.sweep_dense},
          "sweep": rows})


# ---------------------------------------------------------------- the result line
LINE_LIMIT = 4096  # bytes: the driver reads the line back from the tail of stdout
DETAIL_PATH = os.path.join("gpurun_out", "bench_detail.json")


def _r(x, d: int = 4):
    """x to d significant digits (the line carries measurements, not float noise)."""
    if isinstance(x, bool) or x is None or not isinstance(x, (int, float)):
        return x
    if isinstance(x, int):
        return x
    return float(f"{x:.{d}g}") if np.isfinite(x) else None


def config_summary(rec: dict) -> dict:
    """One flat per-config entry of the line from a full record(): throughput, kernel time
    (event mean and median), the roofline fraction, the PMC traffic per lookup when a
    same-hash pass exists, and the algorithm's own index footprint.
    frac is a physical fraction (<= 1): the PMC request floor over the kernel time (req_frac:
    these random-access kernels are bound by L2->fabric requests) when a same-hash PMC pass
    exists, else the HBM-served algorithmic bytes over the time and 8 TB/s (frac_hbm).
    SURVEY §8(d)'s worst-case byte model (every level at P(4 + m) bytes, wherever it is
    served: LDS, the Infinity Cache or HBM) is kept as frac_8d_model; it passes 1 where
    pivot levels never reach HBM, so it is not a roofline."""
    pmc = rec.get("pmc") or {}
    req = _r((pmc.get("requests_split") or {}).get("frac"), 3)
    hbm = _r((rec.get("achieved_hbm_GBps") or 0.0) / HBM_PEAK_GBPS, 3)
    return {"algo": rec.get("algo"), "lookups_per_s": _r(rec.get("kernel_lookups_per_s", rec.get("lookups_per_s"))),
            "kernel_ms": _r(rec.get("kernel_ms")), "kernel_ms_median": _r(rec.get("kernel_ms_median")),
            "frac": req if req is not None else hbm, "frac_basis": "req" if req is not None else "hbm",
            "frac_hbm": hbm, "req_frac": req,
            "frac_8d_model": _r((rec.get("bytes_per_lookup") or {}).get("section_8d", 0.0) *
                                rec["kernel_lookups_per_s"] / 1e9 / HBM_PEAK_GBPS, 3)
            if rec.get("kernel_lookups_per_s") else None,
            "traffic": _r(pmc.get("fabric_bytes_per_lookup")), "index_bytes": rec.get("index_bytes")}


def compact_line(full: dict) -> dict:
    """The one stdout line (<= LINE_LIMIT bytes) from the full record: the contract's keys,
    `roofline` and `cpu_baseline` of the headline, and one flat entry per BASELINE config;
    the full record (variants with their PMC blocks, index stats, byte models) goes to the
    detail file named in `detail` (sst/bin/bench.rs:519-545 writes one flat record per run)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: _r(full[k]) if k in ("value", "ms_per_step") else full[k] for k in keep}
    cfg = full["config"]
    line["config"] = {k: cfg[k] for k in ("workload", "algo", "n", "queries_per_gpu", "m", "mode", "parallelism",
                                          "index_bytes", "index_bytes_per_text_char") if k in cfg}
    rf = full.get("roofline")
    if rf:
        req = rf.get("requests") or {}
        line["roofline"] = {"bound": rf["bound"], "achieved": _r(rf["achieved"]), "peak": rf["peak"], "unit": rf["unit"],
                            "frac": _r(rf["frac"], 3), "traffic": _r(rf.get("traffic")),
                            "traffic_unit": "B/lookup" if rf.get("traffic") is not None else None,
                            "algorithmic_bytes_per_lookup": _r(rf["bytes_per_lookup"]["hbm"]),
                            "kernel": rf.get("kernel"), "kernel_ms": _r(rf.get("kernel_ms")),
                            "kernel_ms_median": _r(rf.get("kernel_ms_median")),
                            "requests_per_lookup": _r(req.get("per_lookup")), "requests_frac": _r(req.get("frac"), 3)}
    else:
        line["roofline"] = None
    cpu = full.get("cpu_baseline")
    line["cpu_baseline"] = None if not cpu else {
        "value": _r(cpu["value"]), "unit": cpu["unit"], "cores": cpu["cores"], "kind": cpu["kind"],
        "single_thread_value": _r(cpu.get("single_thread_value")), "agrees_with_gpu": cpu.get("agrees_with_gpu"),
        "sample": cpu["sample"][:160]}
    confs = full.get("configs") or {}
    out = {}
    if "c0" in confs:
        c0 = confs["c0"]
        out["c0"] = {"cpu_1thread_lookups_per_s": _r(c0["cpu_1thread_lookups_per_s"]),
                     "cpu_all_cores_lookups_per_s": _r(c0["cpu_all_cores_lookups_per_s"]), "cpu_cores": c0["cpu_cores"],
                     "gpu_lookups_per_s": _r(c0["gpu_lookups_per_s"]), "gpu_matches_cpu": c0["gpu_matches_cpu"]}
    for k in ("c1", "c2"):
        if k in confs:
            out[k] = config_summary(confs[k])
    if "c2" in confs and confs["c2"].get("lcp_stree"):
        out["c2"]["lcp_stree"] = {kk: vv for kk, vv in config_summary(confs["c2"]["lcp_stree"]).items()
                                  if kk in ("algo", "kernel_ms", "frac", "frac_basis", "traffic")}
    if "c1" in confs and confs["c1"].get("deep_pivots"):
        out["c1_deep_pivots"] = dict(config_summary(confs["c1"]["deep_pivots"]),
                                     pivot_levels=confs["c1"]["deep_pivots"].get("pivot_levels"))
    if "c3" in confs and not confs["c3"].get("skipped"):
        c3 = confs["c3"]
        out["c3"] = {"algo": c3["algo"], "lookups_per_s": _r(c3["lookups_per_s"]), "kernel_ms": _r(c3["kernel_ms"]),
                     "kernel_ms_median": _r(c3.get("kernel_ms_median")), "frac": _r(c3["roofline"]["frac"], 3),
                     "traffic": _r(c3["roofline"].get("traffic")), "index_bytes": c3["index_bytes"],
                     "n": c3.get("n"), "cross_checks": {k: _r(v["kernel_ms"]) for k, v in c3["variants"].items()
                                                        if k != c3["algo"]}}
    if "c4" in confs:
        c4 = confs["c4"]
        out["c4"] = {"skipped": c4["skipped"]} if c4.get("skipped") else {
            "lookups_per_s": _r(c4["lookups_per_s"]), "ms_per_step": _r(c4["ms_per_step"]), "n": c4["n"],
            "share": c4.get("share"), "parts": c4["parts"], "index_bytes": c4["index_bytes"],
            "prefix_key_fraction": c4.get("prefix_key_fraction"), "proven": c4.get("proven")}
    if "sst" in confs:
        out["sst"] = sst_summary(confs["sst"])
    line["configs"] = out
    line["configs_frac_basis"] = ("frac <= 1: req = PMC request floor / kernel time, hbm = HBM-served algorithmic "
                                  "bytes / time / 8 TB/s; frac_8d_model: SURVEY 8(d) bytes wherever served")
    if full.get("variants"):
        line["variants_kernel_ms"] = {k: _r(v["kernel_ms"]) for k, v in full["variants"].items()}
    if full.get("lcp_long"):
        line["lcp_long"] = full["lcp_long"].get("summary")
    if full.get("occurrence_ranges"):
        line["ranges_per_s"] = _r(full["occurrence_ranges"]["ranges_per_s"])
    if full.get("e2e_host"):
        line["e2e_host_lookups_per_s"] = _r(full["e2e_host"]["lookups_per_s"])
    line["verified"] = full.get("verified", False)
    line["detail"] = full.get("detail")
    # the optional summaries give way before the line outgrows LINE_LIMIT (all in the detail file)
    for k in ("e2e_host_lookups_per_s", "ranges_per_s", "lcp_long", "variants_kernel_ms", "configs_frac_basis"):
        if len(json.dumps(line)) <= LINE_LIMIT:
            break
        line.pop(k, None)
    return line


def write_detail(full: dict, path: str) -> str | None:
    """The full record, for the reader who wants every variant, byte model and PMC block."""
    try:
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1, default=float)
        return path
    except OSError as e:
        log(f"detail not written: {e!r}")
        return None


# ---------------------------------------------------------------- configs[1] / [2] (headline)
WORKLOADS = {
    "prefix": "PREFIX: p = {p}-char bucket table (the reference's prefix table, sas/sa_search.rs:59-95, "
              "with p live) of {e}-B inline entries holding each bucket's first {k} suffixes "
              "({tb:.0f} GiB), then binary search over the fused {{32-char key, SA}} quad-leaf entries "
              "of the bucket; 2^30 text in HBM, 10^7 len-32 queries",
    "plain_rel": "configs[1]: PLAIN binary search over the SA (sas/sa_search.rs:98-112): the pivots of levels "
                 "1-{R} from {rb} of prefix-relative blocks (4 levels per 32-B block: the 8 chars after the block "
                 "bounds' common prefix), levels 1-{t1} staged in LDS{where}; the rest read SA[mid] and a text window",
    "lcp": "configs[1] + mlr LCP skipping",
    "llcp": "configs[1] probe sequence + Manber-Myers Llcp/Rlcp skipping (16-B {SA, Llcp, Rlcp, chars} entries)",
    "inline": "configs[1] probe sequence over fused {32-char key, SA} entries",
    "stree": "configs[2]: S-tree of 16-char SA keys (17-ary 64-B nodes, top layers LDS-staged) + LCP-skipping tail",
    "stree_llcp": "configs[2] as named: LCP-accelerated search on the static-search-tree layout, LDS-staged: the "
                  "S-tree of 16-char SA keys (17-ary 64-B nodes, top layers in LDS) gives the run of suffixes sharing "
                  "q's key, Manber-Myers LLCP skipping (16-B {SA, Llcp, Rlcp, chars} entries) finishes inside it",
    "sector": "configs[2]: sector S-tree (9-ary 32-B nodes, fused 32-char key + SA leaves, top layers LDS-staged)",
    "quad": "configs[2]: quad S-tree (17-ary 64-B nodes read by 4-lane groups, 4-entry fused {32-char key, SA} "
            "leaves, top layers LDS-staged)",
    "interp": "interpolation_search<16> (sas/sa_search.rs:376-421) over fused {32-char key, SA} entries",
    "tagged": "tagged SA entries + bucket table",
}


def plain_label(st: dict) -> str:
    """configs[1]'s workload text from the index's own pivot depth (sas_stats.rel_levels)."""
    t1, R = st["top_levels"], st.get("rel_levels", 0)
    rb = st.get("rel_bytes", 0)
    hb = [d0 for d0, _, w in rel_groups(R) if w == "hbm"]
    if R <= t1:
        where = ""
    elif not hb:
        where = f", levels {t1 + 1}-{R} cache-resident"
    elif hb[0] <= t1:
        where = f", levels {t1 + 1}-{R} from HBM"
    else:
        where = f", levels {t1 + 1}-{hb[0]} cache-resident, {hb[0] + 1}-{R} from HBM"
    return WORKLOADS["plain_rel"].format(
        t1=t1, R=R, rb=(f"{rb / 2 ** 30:.2f} GiB" if rb >= 1 << 30 else f"{rb >> 20} MiB"), where=where)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 30, help="text length (chars)")
    ap.add_argument("--nq", type=int, default=10_000_000, help="queries per GPU")
    ap.add_argument("--m", type=int, default=32, help="query length")
    ap.add_argument("--algo", default=None, choices=["stree", "stree_llcp", "plain", "lcp", "sector", "quad", "inline",
                                                     "llcp",
                                                     "prefix", "tagged", "interp"])
    ap.add_argument("--variants",
                    default="plain,plain_range,llcp,stree,stree_llcp,sector,quad,inline,interp,interp_range,"
                            "prefix_packed",
                    help="other algos timed beside the headline one (mlr LCP skipping, 'lcp', lost to PLAIN at every "
                         "m and on both texts of the lcp_long record: it runs there and in configs[3] only)")
    ap.add_argument("--prefix-chars", type=int, default=16,
                    help="p of the prefix table in chars (the reference's main.rs intends -p 20 key BITS)")
    ap.add_argument("--prefix-table", default="inline2", choices=["inline2", "inline4", "inline", "ranks"],
                    help="inline2: 32-B entries holding each range's first two suffixes, read by lane pairs "
                         "(4^16 x 32 B = 128 GiB); inline: 16-B entries with the first suffix (64 GiB); "
                         "ranks: u32 ranks only (sas/sa_search.rs:59-75's table)")
    ap.add_argument("--c1-deep-levels", type=int, default=C1_DEEP_TOP2_LEVELS,
                    help="configs[1]'s second figure: PLAIN with this many pivot-array levels (0: skip)")
    ap.add_argument("--top2-levels", type=int, default=0,
                    help="pivot-array depth of the headline index (SAS_BUILD_TOP2_LEVELS; 0 = library default 27)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="skip the configs[3] sub-record")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer end-to-end pass")
    ap.add_argument("--c3-n", type=int, default=1 << 34)
    ap.add_argument("--c3-nq", type=int, default=100_000_000)
    ap.add_argument("--c3-steps", type=int, default=5)
    ap.add_argument("--c3-no-cross", action="store_true",
                    help="configs[3]: time the first index only (no rank-ordered cross-check index)")
    ap.add_argument("--c3-layout", default="lines", choices=["lines", "tagged"],
                    help="configs[3] index: tagged entries in 128-B bucket lines (SAS_BUILD_TAG_LINES) or "
                         "rank-ordered with a bucket table; with lines the rank-ordered index runs as the cross-check")
    ap.add_argument("--proof-sample", type=int, default=3000, help="queries per batch proven exact lower bounds")
    ap.add_argument("--no-c4", action="store_true", help="skip the configs[4] (sharded text) sub-record")
    ap.add_argument("--c4-share", type=int, default=0,
                    help="configs[4]: text chars per GPU (0: the largest power of two <= 2^33 whose part index fits "
                         "one GPU, bench.c4_share_for: 2^33 at N >= 2, 2^32 at N = 1)")
    ap.add_argument("--shard-chunks", type=int, default=1,
                    help="sharded step in this many pieces, exchanges overlapped with the other pieces' work")
    ap.add_argument("--c4-steps", type=int, default=10)
    ap.add_argument("--workload", default="c1", choices=["c1", "c3", "sst"],
                    help="c1: 2^30 text, 10^7 len-32 queries (BASELINE metric) + every config's sub-record; "
                         "c3: the configs[3] record alone; sst: the u32 static-search-tree path")
    ap.add_argument("--positive", action="store_true", help="sst workload: queries drawn from the keys")
    ap.add_argument("--sst-layouts", default="", help="sst workload: these layouts only (comma-separated names)")
    ap.add_argument("--no-sst", action="store_true", help="skip the u32 static-search-tree sub-record (configs.sst)")
    ap.add_argument("--sweep", action="store_true",
                    help="sst workload: the reference's size sweep (32 B .. 2^--sweep-to B) instead of one size")
    ap.add_argument("--sweep-to", type=int, default=30, help="sst sweep: largest size 2^k bytes")
    ap.add_argument("--sweep-dense", action="store_true", help="sst sweep: also 5/4, 3/2, 7/4 of each power")
    ap.add_argument("--detail", default=DETAIL_PATH,
                    help="file for the full record (every variant, byte model and PMC block); '' = none")
    ap.add_argument("--no-lcp-long", action="store_true", help="skip the long-query LCP-skipping record")
    ap.add_argument("--mode", default="replicated", choices=["replicated", "shard"],
                    help="replicated index (weak scaling, no data-path collective) or sharded SA rank "
                         "ranges with RCCL all-to-all query routing (SURVEY §8e)")
    args = ap.parse_args()
    keep_stdout_for_result()

    import torch
    import sas_amd

    ws, rank, local = dist_env()
    dist = None
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.workload == "c3":
        return run_c3(args, torch, sas_amd, dev, ws, rank)
    if args.workload == "sst":
        if args.sweep:
            return run_sst_sweep(args, torch, sas_amd, dev)
        return run_sst(args, torch, sas_amd, dev, ws, rank)
    if args.algo is None:
        args.algo = "prefix"
    n, nq, m = args.n, args.nq, args.m

    t_build0 = time.perf_counter()
    text = sas_amd.random_string(n, seed=SEED, device=dev)  # sas/util.rs:9-15, identical on every rank
    if args.mode == "shard":
        from sas_amd.shard import ShardedSearch
        # each rank builds ONLY its own SA rank range (sas_build_part: no whole-SA step)
        # a part holds a 40-bit SA; below 2^32 chars it carries the same inline table as the
        # replicated index, and PREFIX queries cross the exchange as 8-B packed words
        idx = sas_amd.SaNaive.build_part(text, rank, ws, lcp=True, stree=True, prefix=args.prefix_chars,
                                         prefix_inline=({"ranks": 0, "inline": 1, "inline2": 2, "inline4": 4}
                                                        [args.prefix_table] if n < (1 << 32) else 0))
        if dist is None:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            dist.init_process_group("nccl", rank=0, world_size=1)
        engine = ShardedSearch(idx, dist, ws, rank, dev, algo=args.algo, chunks=args.shard_chunks, max_nq=nq)
    else:
        idx = sas_amd.SaNaive.build(text, lcp=True, stree=True, prefix=args.prefix_chars,
                                    prefix_inline={"ranks": 0, "inline": 1, "inline2": 2,
                                                   "inline4": 4}[args.prefix_table], top2_levels=args.top2_levels)
    stats = idx.stats()
    off = rank_query_offsets(n, nq, m, rank)
    off_t = torch.from_numpy(off.astype(np.int64)).to(dev)
    qbytes = torch.empty(nq * m, dtype=torch.uint8, device=dev)
    ar = torch.arange(m, device=dev, dtype=torch.int64)
    chunk = 1 << 18  # bounds the gather temporaries
    for s in range(0, nq, chunk):
        e = min(nq, s + chunk)
        qbytes[s * m:e * m] = text[(off_t[s:e, None] + ar[None, :]).reshape(-1)]
    out = torch.empty(nq, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build0
    log(f"c1 index built + queries cut in {build_s:.1f} s")

    def reduce_max(x):
        if dist is None:
            return x
        tt = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    barrier = (lambda: dist.barrier()) if dist is not None else (lambda: None)
    stream = torch.cuda.current_stream(dev)

    def algo_flags(name):
        # "<algo>_range": PLAIN / LCP from the prefix table's range (SAS_PREFIX_RANGE), the
        # reference's binary_search with its prefix table live (sas/sa_search.rs:86-112)
        return (name[:-6], sas_amd._lib.SAS_PREFIX_RANGE) if name.endswith("_range") else (name, 0)

    packed = {}

    def run_algo(algo, steps, warmup, dst):
        base, fl = algo_flags(algo)
        if algo == "prefix_packed" and "w" not in packed:
            # queries handed over 2-bit packed (sas_pack_queries, untimed: the caller's format)
            packed["w"] = sas_amd.SaNaive.pack_queries(qbytes, m)

        def step():
            if args.mode == "shard":
                # fixed-capacity buckets, no host sync inside the step; the overflow flag is
                # checked once after the timed loop (engine.assert_no_overflow)
                engine.search_fixed(qbytes, m, check=False, out=dst)
            elif algo == "prefix_packed":
                idx.search_packed(packed["w"], m, out=dst)
            else:
                idx.search_fixed(qbytes, m, algo=base, out=dst, flags=fl)
        # events bracket each of the K timed launches on the launch stream
        t = launch_times(torch, step, steps, warmup, stream, barrier=barrier, reduce_max=reduce_max)
        return t["wall_s"], t["mean_ms"], t["median_ms"]

    def probes_of(algo):
        base, fl = algo_flags(algo)
        if algo == "prefix_packed":
            _, vp = idx.search_packed(packed["w"], m, probes=True)
        else:
            _, vp = idx.search_fixed(qbytes, m, algo=base, probes=True, flags=fl)
        return float(vp.double().mean().item())

    el, kernel_ms, kernel_med = run_algo(args.algo, args.steps, args.warmup, out)
    if args.mode == "shard":
        engine.assert_no_overflow()
    log(f"headline {args.algo}: {kernel_ms:.3f} ms per {nq}")
    # correctness guard (untimed): every answer is an occurrence of its query, and a sample
    # is proven an exact lower bound on the index's own SA
    occ = text[(out[:, None] + ar[None, :]).reshape(-1).clamp_(max=n - 1)]
    if not bool(torch.equal(occ, qbytes)):
        raise SystemExit(f"bench: {args.algo} returned a non-occurrence position")
    del occ
    whole = args.mode == "replicated" or ws == 1
    proven = 0
    if whole:
        rng = np.random.default_rng(11 + rank)
        ids = np.sort(rng.choice(nq, size=min(nq, args.proof_sample), replace=False))
        dids = torch.from_numpy(ids).to(dev)
        hq = qbytes.view(nq, m)[dids].cpu().numpy()
        qmap = {int(i): hq[j] for j, i in enumerate(ids)}
        htext = text.cpu().numpy()
        nbad = lower_bound_proof(idx, lambda p, L: htext[p:p + L], lambda i: qmap[i], out[dids].cpu().numpy(), ids)
        if nbad:
            raise SystemExit(f"bench: {nbad} of {len(ids)} sampled {args.algo} answers are not exact lower bounds")
        proven = len(ids)
        del htext
    mean_probes = probes_of(args.algo) if whole else float("nan")

    # end to end from host buffers: pageable query bytes in, positions out, as a
    # caller handing host memory through the C ABI sees it (pinned staging, chunked
    # H2D / kernel / D2H over 3 streams, csrc/host_stage.hpp).  Never `value`.
    e2e = None
    if args.mode == "replicated" and not args.no_e2e:
        hq = qbytes.cpu().numpy()
        ref_host = out.cpu().numpy().astype(np.uint64)
        # the caller's result array is allocated and touched once and reused, as a caller
        # running batch after batch would (a fresh np.zeros per call adds its first-touch
        # page faults, ~5 ms per 80 MB on the GPU box, to every call)
        hpos = np.ones(nq, np.uint64)
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            idx.search_fixed(hq, m, algo=args.algo, out=hpos)
            times.append(time.perf_counter() - t0)
        e2e = {"lookups_per_s": nq / min(times), "ms": min(times) * 1e3, "ms_first_call": times[0] * 1e3,
               "matches_device_run": bool(np.array_equal(hpos, ref_host)),
               "path": "pageable host query bytes -> sas_search_fixed -> the caller's (reused) pageable result array: "
                       "reusable pinned staging (the index's slot set), chunked H2D / kernel / D2H overlapped on 3 "
                       "streams, a 16-thread host pool filling and emptying the staging buffers"
                       + ("; PREFIX with m <= 32 packs the queries 2-bit on the host (8 B per query over PCIe)"
                          if args.algo == "prefix" and m <= 32 else "")}
        if not e2e["matches_device_run"]:
            raise SystemExit("bench: the host-buffer path differs from the device run")
        del hq
        log(f"e2e host: {e2e['ms']:.2f} ms")

    headline_pos = out.clone()
    variants = {}
    vout = torch.empty_like(out)
    for v in [x for x in args.variants.split(",") if x and x != args.algo and args.mode == "replicated"]:
        # every variant is timed like the headline: the driver's steps and warmup
        vsteps = args.steps
        vel, vk, vmed = run_algo(v, vsteps, args.warmup, vout)
        same = bool(torch.equal(vout, headline_pos))
        if not same:
            raise SystemExit(f"bench: variant {v} differs from {args.algo}")
        vmean = probes_of(v)
        vbase, vfl = algo_flags(v)
        bpl = bytes_per_lookup("prefix" if v == "prefix_packed" else vbase, stats, n, m, vmean,
                               range_flag=bool(vfl), packed=v == "prefix_packed")
        key = {"plain": "plain", "quad": "quad", "stree": "stree", "sector": "sector", "llcp": "llcp",
               "stree_llcp": "stree_llcp"}.get(v)
        pmc = load_pmc(f"{key}_n{n}_q{nq}_m{m}" + (f"_t{stats['top2_levels']}" if key == "plain" else "")) \
            if key else None
        variants[v] = record(v, nq, vk, vel, bpl, footprint(v, stats), pmc, vmean,
                             {"identical_to_headline": same, "lookups_per_s": ws * nq * vsteps / vel,
                              "kernel_ms_median": vmed, "timed_launches": vsteps})
        log(f"variant {v}: {vk:.3f} ms")

    # configs[1]'s second figure: the same PLAIN probe sequence on an index whose pivots reach
    # C1_DEEP_TOP2_LEVELS levels (SAS_BUILD_TOP2_LEVELS, rounded up to the 4-level grid: every
    # level of a 2^30 text, 4.3 GiB of blocks): the block of levels 28-31 is one HBM request
    # instead of four SA words and text windows
    deep = None
    if args.mode == "replicated" and "plain" in variants and args.c1_deep_levels:
        didx = sas_amd.SaNaive.build(text, lcp=False, stree=False, sector=False, quad=False, llcp=False,
                                     prefix=False, top2_levels=args.c1_deep_levels)
        dst = didx.stats()
        dout = torch.empty_like(out)

        def dstep():
            didx.search_fixed(qbytes, m, algo="plain", out=dout)
        dsteps = args.steps
        dt_ = launch_times(torch, dstep, dsteps, args.warmup, stream)
        del_s, dk = dt_["wall_s"], dt_["mean_ms"]
        if not bool(torch.equal(dout, headline_pos)):
            raise SystemExit("bench: PLAIN on the deep pivot array differs from the headline")
        _, dpr = didx.search_fixed(qbytes, m, algo="plain", probes=True)
        dmean = float(dpr.double().mean().item())
        dbpl = bytes_per_lookup("plain", dst, n, m, dmean)
        deep = record("plain", nq, dk, del_s, dbpl, footprint("plain", dst),
                      load_pmc(f"plain_n{n}_q{nq}_m{m}_t{dst['top2_levels']}"), dmean,
                      {"identical_to_headline": True, "lookups_per_s": ws * nq * dsteps / del_s,
                       "kernel_ms_median": dt_["median_ms"], "timed_launches": dsteps,
                       "workload": plain_label(dst), "pivot_levels": dst["top2_levels"],
                       "pivot_bytes": dst["rel_bytes"]})
        didx.free()
        del dout, dpr
        torch.cuda.empty_cache()
        log(f"c1 plain, {dst['top2_levels']} pivot levels: {dk:.3f} ms")

    # LCP skipping where compares run long (sas/sa_search.rs:344-345's TODO): PLAIN / LCP /
    # LLCP at m = 64..256 on this random text now, on a repetitive text after this index is
    # freed (below); N = 1 only
    lcp_long = None
    if ws == 1 and args.mode == "replicated" and not args.no_lcp_long and stats["llcp_bytes"]:
        lcp_long = {"what": "PLAIN vs mlr LCP vs Manber-Myers LLCP skipping vs the S-tree + LLCP tail (configs[2]'s "
                            "combination) vs QUAD, 10^7 positive len-m queries, kernel ms (HIP events), positions "
                            "identical; random: the headline's 2^30 text; repetitive: 2^24 random chars x 64 copies, "
                            "1% substitutions per copy",
                    "random": lcp_long_runs(torch, idx, text, nq, args.steps, args.warmup, stream, "random")}

    # occurrence ranges (Search::search_prefix / search_range, sas/util.rs:36-46): the rank
    # range [lo, hi) of each query's occurrences from the prefix table (inline slots first,
    # k_sa_prefix2_range; SAS_RANGE_NO_INLINE: both bounds bisected, k_sa_prefix_range);
    # checked: every positive query occurs, SA[lo] is the headline's position, and the
    # two kernels agree
    ranges = None
    if args.mode == "replicated":
        def time_ranges(fl):
            res = {}

            def rstep():
                res["r"] = idx.search_range_fixed(qbytes, m, flags=fl)
            return launch_times(torch, rstep, args.steps, args.warmup, stream)["mean_ms"], res["r"]
        rms, (lo_d, hi_d) = time_ranges(0)
        bms, (lo_b, hi_b) = time_ranges(sas_amd._lib.SAS_RANGE_NO_INLINE)
        if not (torch.equal(lo_d, lo_b) and torch.equal(hi_d, hi_b)):
            raise SystemExit("bench: the inline-slot and bisection range kernels disagree")
        cnt_d = hi_d - lo_d
        if bool((cnt_d < 1).any().item()):
            raise SystemExit("bench: a positive query has an empty occurrence range")
        rng = np.random.default_rng(5)
        sids = rng.choice(nq, size=min(nq, 300), replace=False)
        los = lo_d[torch.from_numpy(sids).to(dev)].cpu().numpy()
        hp = headline_pos[torch.from_numpy(sids).to(dev)].cpu().numpy()
        for j in range(len(sids)):
            if int(idx.suffix_array(count=1, start=int(los[j]))[0]) != int(hp[j]):
                raise SystemExit("bench: SA[lo] of an occurrence range differs from the headline position")
        ranges = {"what": "sas_search_range_fixed: the SA rank range of each query's occurrences (prefix table: "
                          "the inline slots test both bounds, the rest bisected; k_sa_prefix2_range)",
                  "ranges_per_s": nq / (rms * 1e-3), "kernel_ms": rms,
                  "bisect_kernel_ms": bms, "mean_occurrences": float(cnt_d.double().mean().item()),
                  "verified": True}
        del lo_d, hi_d, lo_b, hi_b, cnt_d
        log(f"ranges: {rms:.3f} ms (bisection {bms:.3f} ms)")

    pe = prefix_entry_bytes(stats) if stats["prefix_chars"] else 0
    pkey = str(stats["prefix_chars"]) + {16: "i", 32: "d", 64: "q"}.get(pe, "")
    hpmc = load_pmc(f"{args.algo}{pkey if args.algo == 'prefix' else ''}_n{n}_q{nq}_m{m}")
    hbpl = bytes_per_lookup(args.algo, stats, n, m, mean_probes)
    head = record(args.algo, nq, kernel_ms, el, hbpl, footprint(args.algo, stats), hpmc, mean_probes,
                  {"kernel_ms_median": kernel_med, "timed_launches": args.steps})
    achieved = head["achieved_hbm_GBps"]

    cpu = None
    configs = {}
    if rank == 0 and ws == 1 and not args.no_cpu and args.mode == "replicated":
        cpu = cpu_baseline(text, idx, qbytes, m, nq, args.cpu_seconds)
        cpos = cpu.pop("_pos")
        cpu["agrees_with_gpu"] = bool(np.array_equal(cpos, headline_pos[:len(cpos)].cpu().numpy().astype(np.uint64)))
        if not cpu["agrees_with_gpu"]:
            raise SystemExit("bench: the CPU restatement of the reference differs from the GPU positions")
        log("cpu baseline done")
        configs["c0"] = c0_record(torch, sas_amd, dev, min(10.0, args.cpu_seconds / 2))
        log("c0 done")
    if args.mode == "replicated":
        if "plain" in variants:
            configs["c1"] = dict(variants["plain"], workload=plain_label(stats),
                                 pivot_levels=stats["top2_levels"],
                                 pivot_bytes=stats["rel_bytes"])
            if deep is not None:
                configs["c1"]["deep_pivots"] = deep
        best2 = max((v for v in ("quad", "sector", "stree") if v in variants),
                    key=lambda v: variants[v]["kernel_lookups_per_s"], default=None)
        if best2:
            configs["c2"] = dict(variants[best2], workload=WORKLOADS[best2],
                                 lds_layers={"quad": stats["quad_lds_layers"], "sector": stats["sector_lds_layers"],
                                             "stree": stats["stree_lds_layers"]}[best2])
            # BASELINE's configs[2] names the combination: LCP-accelerated search on the static
            # search tree layout, LDS-staged (the S-tree descent + the LLCP tail); its m > 32
            # shapes are in lcp_long
            if "stree_llcp" in variants:
                configs["c2"]["lcp_stree"] = dict(variants["stree_llcp"], workload=WORKLOADS["stree_llcp"],
                                                  lds_layers=stats["stree_lds_layers"])
    idx_stats = {k: stats[k] for k in ("stree_layers", "stree_lds_layers", "sector_layers", "sector_lds_layers",
                                       "quad_layers", "quad_lds_layers", "quad_fan", "top_levels", "top2_levels", "rel_levels",
                                       "iterations", "prefix_chars", "prefix_bytes", "sa_bytes", "text_bytes",
                                       "quad_bytes", "stree_bytes", "sector_bytes", "lcp_bytes", "llcp_bytes",
                                       "rel_bytes", "index_bytes", "sa_rounds", "build_sa_ns", "build_total_ns")}
    if lcp_long is not None:
        idx.free()
        torch.cuda.empty_cache()
        tb = time.perf_counter()
        rt = repetitive_text(torch, n, dev)
        ridx = sas_amd.SaNaive.build(rt, lcp=True, llcp=True, stree=True, sector=False, quad=True, prefix=False)
        log(f"lcp_long repetitive index built in {time.perf_counter() - tb:.1f} s")
        lcp_long["repetitive"] = lcp_long_runs(torch, ridx, rt, nq, args.steps, args.warmup, stream, "repetitive")
        lc = ridx.lcp_array()
        lcp_long["repetitive_text"] = {"mean_adjacent_lcp": float(lc.mean()), "p99_adjacent_lcp": float(np.percentile(
            lc[:: 97], 99)), "max_adjacent_lcp": int(lc.max()), "build_s": time.perf_counter() - tb}
        del lc
        ridx.free()
        del rt
        torch.cuda.empty_cache()
        lcp_long["summary"] = lcp_long_summary(lcp_long)
        log("lcp_long done")
    # the u32 static-search-tree path (the reference's other crate, sst/bin/bench.rs:548-599): N = 1
    if ws == 1 and not args.no_sst and args.mode == "replicated":
        configs["sst"] = sst_record(args, torch, sas_amd, dev)
        log(f"sst done: best {configs['sst']['best']}")
    # configs[3]: free the 2^30 index first (N = 1 only: the scaling runs time the headline)
    if ws == 1 and not args.no_c3 and args.mode == "replicated":
        idx.free()
        del text, qbytes, out, headline_pos, vout, off_t, packed
        torch.cuda.empty_cache()
        configs["c3"] = c3_record(args, torch, sas_amd, dev, rank)
        log("c3 done")
    # configs[4]: the sharded-text step on every rank (the driver's 1/2/4/8-GPU runs time it)
    if not args.no_c4 and args.mode == "replicated":
        idx.free()  # idempotent: the c3 block may have freed it already
        torch.cuda.empty_cache()
        configs["c4"] = c4_record(args, torch, sas_amd, dev, ws, rank, dist)
        log("c4 done")

    if rank == 0:
        ms = el / args.steps * 1e3
        value = ws * nq * args.steps / el
        wl = plain_label(stats) if args.algo == "plain" else WORKLOADS[args.algo]
        if args.algo == "prefix":
            wl = wl.format(p=stats["prefix_chars"], e=pe, k=max(1, pe // 16), tb=stats["prefix_bytes"] / 2 ** 30)
        line = {
            "metric": METRIC, "value": value, "unit": "lookups/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic: random_string(ChaCha8Rng::seed_from_u64({SEED})) text + positive len-{m} "
                    f"substrings (sas/util.rs:9-26), per-rank query stream",
            "config": {"workload": wl, "algo": args.algo, "n": n, "queries_per_gpu": nq, "m": m,
                       "prefix_chars": stats["prefix_chars"], "prefix_entry_bytes": pe,
                       "index_bytes": footprint(args.algo, stats),
                       "index_bytes_per_text_char": _r(footprint(args.algo, stats) / n),
                       "built_index_bytes": stats["index_bytes"], "prefix_bytes": stats["prefix_bytes"],
                       "ns_per_lookup": head["ns_per_lookup"], "mode": args.mode,
                       "parallelism": (f"replicated index x{ws}, query shards (no data-path collective)"
                                       if args.mode == "replicated" else
                                       f"SA rank ranges over {ws} GPUs, sas_route + RCCL all_to_all_single "
                                       f"(queries out, positions back)")},
            # shard mode: the events bracket route + exchanges + search, not one kernel
            "roofline": None if args.mode != "replicated" else {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": (head.get("pmc") or {}).get("fabric_bytes_per_lookup"),
                "traffic_unit": "bytes per lookup (PMC, L2->fabric, Infinity-Cache hits included)",
                "traffic_bytes_per_launch": (hpmc or {}).get("hbm_bytes_per_launch"),
                "algorithmic_hbm_bytes_per_launch": hbpl["hbm"] * nq,
                "traffic_source": (hpmc or {}).get("source"),
                "kernel": "k_sa_prefix2" if args.algo == "prefix" and pe >= 32 else
                          ("k_sa_prefix" if args.algo == "prefix" else KERNELS.get(args.algo)),
                "kernel_ms": kernel_ms, "kernel_ms_median": kernel_med, "bytes_per_lookup": hbpl,
                "mean_probes": mean_probes,
                # what bounds this path: random 128-B-line requests (PMC L2->fabric reads of this
                # workload, query stream included), against the measured random-request ceiling
                "requests": None if not (head.get("pmc") or {}).get("requests_per_lookup") else {
                    "per_lookup": head["pmc"]["requests_per_lookup"],
                    "ceiling_per_s": RANDOM_REQ_CEILING, "frac": head["pmc"]["requests_frac_of_ceiling"]},
                "pmc_stale": bool((head.get("pmc") or {}).get("stale"))},
            "cpu_baseline": cpu,
            "e2e_host": e2e,
            "occurrence_ranges": ranges,
            "configs": configs,
            "variants": variants,
            "index": idx_stats,
            "setup_s": build_s, "verified": True,
            "verification": f"every answer an occurrence; {proven} sampled answers proven exact lower bounds on the "
                            f"index's SA; every variant bit-identical to the headline"
                            + ("; CPU restatement identical on its sample" if cpu else ""),
        }
        if lcp_long is not None:
            line["lcp_long"] = lcp_long
        line["detail"] = write_detail(line, args.detail) if args.detail else None
        short = compact_line(line)
        log(f"result line {len(json.dumps(short))} B; full record {args.detail}")
        emit(short)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
