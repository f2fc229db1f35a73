"""Headline benchmark: batched suffix-array pattern lookups on MI355X.

BASELINE.json metric: "pattern lookups/s + achieved HBM GB/s, 2^30-byte text,
10^7 len-32 queries".  One step = one batched lookup of all queries of this
GPU (inputs already resident in HBM), through the C ABI (sas_search_fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--algo stree|plain|lcp]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Multi-GPU: the index is replicated (the text is generated and indexed on every
GPU), each rank searches its own 10^7 queries -> weak scaling, no collective on
the data path; only the timing barrier and a MAX all-reduce of elapsed times.
"""
from __future__ import annotations

import argparse
import glob
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
SEED = 31415  # sas/main.rs:38


def algorithmic_bytes(algo: str, n: int, m: int, stree_layers: int, tail_probes: float,
                      sector_layers: int = 0, quad_layers: int = 0, prefix_entry: int = 8) -> float:
    """Bytes a lookup must move: 4 B SA word + m text bytes per
    probe, the query, the 8 B position.  PLAIN/LCP: P = ilog2(n)+1 probes.
    STREE: H 64-B nodes + measured tail probes.  SECTOR: H 32-B nodes (the
    leaf holds the keys and the SA values) + measured extra leaf probes x 12 B.
    QUAD: H 64-B nodes (4-entry leaves) + measured extra leaf probes x 64 B."""
    if algo == "stree":
        return stree_layers * 64 + tail_probes * (4 + m) + m + 8
    if algo == "sector":
        return sector_layers * 32 + tail_probes * 12 + m + 8
    if algo == "quad":
        return quad_layers * 64 + tail_probes * 64 + m + 8
    if algo == "prefix":  # the table entry (two u32, or one 16-B inline entry) + probes of
        # 16-B fused entries; probes = the reference's cnt, which counts the table once
        return prefix_entry + max(0.0, tail_probes - 1) * 16 + m + 8
    if algo == "inline":  # P probes of one 16-B fused (key, SA) entry
        P = int(np.log2(n)) + 1
        return P * 16 + m + 8
    P = int(np.log2(n)) + 1
    return P * (4 + m) + m + 8


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


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def load_traffic(algo: str, n: int, nq: int, m: int, with_requests: bool = False):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass of this exact
    workload (profiles/pmc_<algo>_n<n>_q<nq>_m<m>.json, written by
    tools/pmc_to_json.py), or None; with_requests: also its L2->fabric read
    requests per launch (TCC_EA0_RDREQ)."""
    path = os.path.join(REPO, "profiles", f"pmc_{algo}_n{n}_q{nq}_m{m}.json")
    if not os.path.exists(path):
        return (None, None, None) if with_requests else (None, None)
    d = json.load(open(path))
    if with_requests:
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO), d.get("TCC_EA0_RDREQ")
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO)


def host_cpu() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(text_dev, idx, qbytes_dev, m, nq, seconds: float):
    """The oracle's restatement of the reference CPU search, timed on this host's
    cores on a bounded sample of the same queries (rank 0, N=1 only)."""
    from oracle import pyoracle as O
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    n = idx.n
    t = O.padded(text_dev.cpu().numpy())
    sa = idx.suffix_array()
    best = None
    for algo in ("binary_search", "batch_c16"):
        sample = min(nq, 50_000)
        while True:
            qb = np.concatenate([qbytes_dev[: sample * m].cpu().numpy(), np.zeros(64, np.uint8)])
            off = np.arange(sample, dtype=np.uint64) * m
            ln = np.full(sample, m, np.uint32)
            t0 = time.perf_counter()
            O.search_many(t, n, sa, qb, off, ln, algo, threads)
            dt = time.perf_counter() - t0
            if dt * 2 > seconds / 2 or sample >= nq:
                break
            sample = min(nq, int(sample * max(2.0, (seconds / 2) / max(dt, 1e-3))))
        rate = sample / dt
        if best is None or rate > best[0]:
            best = (rate, algo, sample, dt)
    rate, algo, sample, dt = best
    # one thread on a smaller sample of the same queries (1 thread and all cores)
    s1 = min(nq, max(1000, int(sample * (seconds / 8) / max(dt * threads, 1e-3))))
    qb = np.concatenate([qbytes_dev[: s1 * m].cpu().numpy(), np.zeros(64, np.uint8)])
    t0 = time.perf_counter()
    O.search_many(t, n, sa, qb, np.arange(s1, dtype=np.uint64) * m, np.full(s1, m, np.uint32), algo, 1)
    one = s1 / (time.perf_counter() - t0)
    return {"value": rate, "unit": "lookups/s", "cores": threads, "kind": "port",
            "single_thread_value": one, "host_cpu": host_cpu(), "host_nproc": os.cpu_count(),
            "sample": f"oracle/{algo} (restates sas/sa_search.rs "
                      f"{'98-112' if algo == 'binary_search' else '198-239 batch_c<16>'}) on {sample} of the "
                      f"same len-{m} queries over the same 2^{int(np.log2(n))} text/SA, {dt:.1f} s, "
                      f"{threads} threads, contiguous chunks (sst/bin/bench.rs:558-573)"}


def run_sst(args, torch, sas_amd, dev, ws, rank):
    """The u32 path (static-search-tree crate): the reference's bench sweeps sizes up to
    2^30 bytes (sst/bin/bench.rs:455-472); this runs the largest, 2^28 keys (gen_vals:
    uniform < i32::MAX, vals[0] = MAX, sorted; sst/util.rs:31-42) and 10^7 uniform
    queries (gen_queries, :16-21) on every GPU layout, all checked against each other."""
    from oracle import pyoracle as O
    nk = args.n if args.n != 1 << 30 else 1 << 28
    nq = args.nq
    rng = np.random.default_rng(SEED)
    vals = rng.integers(0, O.MAX, nk, dtype=np.uint64).astype(np.uint32)
    vals[0] = O.MAX
    vals.sort()
    if args.positive:  # gen_positive_queries (sst/util.rs:23-28)
        qs = vals[rng.integers(0, nk, nq)]
    else:  # gen_queries (sst/util.rs:16-21)
        qs = rng.integers(0, O.MAX, nq, dtype=np.uint64).astype(np.uint32)
    dq = torch.from_numpy(qs.view(np.int32)).to(dev)
    dout = torch.empty(nq, dtype=torch.int32, device=dev)
    layouts = {
        "SortedVec": lambda: sas_amd.SortedVec.new(vals),
        "Eytzinger": lambda: sas_amd.Eytzinger.new(vals),
        "STree16": lambda: sas_amd.STree16.new(vals),
        "STree16_left_max": lambda: sas_amd.STree16.new_params(vals, True, False, False),
        "STree15": lambda: sas_amd.STree15.new(vals),
        "PartitionedSTree16M_b16": lambda: sas_amd.PartitionedSTree16M.new(vals, 16),
        "PartitionedSTree16M_b20": lambda: sas_amd.PartitionedSTree16M.new(vals, 20),
        "DirectMap": lambda: sas_amd.DirectMap.new(vals),
    }
    res, ref = {}, None
    for name, mk in layouts.items():
        idx = mk()
        for _ in range(args.warmup):
            idx.query(dq)
        kns = idx.time_query(dq, dout, reps=args.steps, stream=torch.cuda.current_stream(dev).cuda_stream)
        got = dout.cpu().numpy().view(np.uint32).copy()
        if ref is None:
            ref = got
        res[name] = {"lookups_per_s": nq / (kns * 1e-9), "kernel_ms": kns * 1e-6, "layers": idx.layers(),
                     "index_bytes": idx.size(), "agrees": bool(np.array_equal(got, ref))}
        idx.free()
    # --range mode (sst/bin/bench.rs:84-109): the interleaved [q, q+1] stream through
    # STree16 left_max; rank(q+1) - rank(q) = number of keys equal to q (checked)
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
    # CPU: the oracle's restatement of the reference's bench variant, STree16 left_max
    # + batch_final::<128> (sst/bin/bench.rs:96; sst/s_tree.rs:303-326), contiguous
    # per-thread chunks (sst/bin/bench.rs:558-573); 16 threads and 1 thread
    tree = O.STree(vals, left_max=True)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    sample = nq
    t0 = time.perf_counter()
    cpu_out = tree.query_batch(qs[:sample], threads)
    dt = time.perf_counter() - t0
    s1 = min(nq, 2_000_000)
    t1 = time.perf_counter()
    tree.query_batch(qs[:s1], 1)
    one = s1 / (time.perf_counter() - t1)
    cpu_ok = bool(np.array_equal(cpu_out, ref[:sample]))
    best = max(res, key=lambda k: res[k]["lookups_per_s"])
    emit({
        "metric": "u32 static-search-tree lookups/s (2^28 keys = 1 GiB, 10^7 uniform queries)",
        "value": res[best]["lookups_per_s"], "unit": "lookups/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True, "dtype": "u32", "vs_baseline": None,
        "data": "synthetic: gen_vals / gen_queries shapes (sst/util.rs:16-42)",
        "config": {"workload": "sst u32 path", "keys": nk, "queries": nq, "best": best},
        "layouts": res,
        "range_mode": range_res,
        "queries_kind": "positive" if args.positive else "uniform",
        "cpu_baseline": {"value": sample / dt, "unit": "lookups/s", "cores": threads, "kind": "port",
                         "single_thread_value": one, "host_cpu": host_cpu(), "host_nproc": os.cpu_count(),
                         "sample": f"oracle STree16 left_max + batch_final::<128> restatement (sst/s_tree.rs:303-326) "
                                   f"on all {sample} queries, {threads} threads, {dt:.2f} s", "agrees": cpu_ok}})


def run_c3(args, torch, sas_amd, dev, ws, rank, dist):
    """configs[3]-shaped run: n = 2^34 chars (16 GiB of byte-coded text, a 40-bit SA:
    BASELINE's "64 GiB" = 2^36 chars cannot hold any SA in 288 GB) and
    10^8 positive queries of mixed length 8..256 (random_queries with len in
    [8, 257)), ragged, through sas_search_batch on device buffers.  The sector tree
    and the fused quad leaves (16 B per suffix) fit next to the SA only up to n = 2^33;
    above, QUAD / INLINE run on compact key-only quad leaves (8 B per suffix,
    SAS_BUILD_QUAD_COMPACT) and SECTOR falls back to STREE."""
    n = args.n if args.n != 1 << 30 else 1 << 34
    nq = args.nq if args.nq != 10_000_000 else 100_000_000
    fits = n <= (1 << 33)  # 16 B per suffix next to the 40-bit SA
    main_algo = args.algo if (args.algo != "sector" or fits) else "stree"
    quad_mode = (("compact" if (args.quad_compact or not fits) else True) if main_algo in ("quad", "inline", "prefix")
                 else False)
    # prefix table beside a 40-bit SA: packed 40-bit entries, p = 16 (20 GiB); it fits
    # because the 16 GiB byte copy of the text is dropped after the build (queries are
    # cut from, and answers checked against, the index's packed text: sas_extract)
    c3_prefix = min(args.prefix_chars, 16) if main_algo == "prefix" else False
    t0 = time.perf_counter()
    text = sas_amd.random_string(n, seed=SEED, device=dev)
    # verify: the reference's adjacency assertion (sas/sa_search.rs:36-38) + permutation, on the GPU
    idx = sas_amd.SaNaive.build(text, lcp=False, stree=main_algo == "stree", sector=main_algo == "sector",
                                quad=quad_mode, verify=True, llcp=False, prefix=c3_prefix)
    stats = idx.stats()
    del text
    torch.cuda.empty_cache()
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
    del src
    chunk = 1 << 20
    out = torch.empty(nq, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    results = {}
    for algo in [a for a in (main_algo, "plain", "lcp") if a]:
        if algo in results:
            continue
        def step():
            idx.search_batch(qbytes, qoff, qlen, algo=algo, out=out)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        ev0.record()
        tt = time.perf_counter()
        steps = args.steps if algo == main_algo else max(2, args.steps // 4)
        for _ in range(steps):
            step()
        ev1.record()
        torch.cuda.synchronize()
        el = time.perf_counter() - tt
        kms = ev0.elapsed_time(ev1) / steps
        # guard: each answer is an occurrence of its query (positive queries)
        okc = True
        for s in range(0, nq, chunk):
            e = min(nq, s + chunk)
            span = int((qoff[e - 1] + lens[e - 1] - qoff[s]).item())
            got = torch.empty(span, dtype=torch.uint8, device=dev)
            idx.extract(out[s:e].contiguous(), qlen[s:e].contiguous(), (qoff[s:e] - qoff[s]).contiguous(), got)
            okc &= bool(torch.equal(got, qbytes[qoff[s]:qoff[s] + span]))
        _, pr = idx.search_batch(qbytes, qoff, qlen, algo=algo, probes=True)
        mp = float(pr.double().mean().item())
        mean_m = total / nq
        P = int(np.log2(n)) + 1
        if algo == "stree":
            ab = stats["stree_layers"] * 64 + max(0.0, mp - stats["stree_layers"]) * (4 + mean_m) + mean_m + 8
        elif algo in ("sector", "quad"):
            # H nodes (leaf = keys + SA), extra leaf probes, the query, the position, and
            # the packed text window past char 32 for the final compare (+ the 5-B SA
            # entry for compact key-only quad leaves)
            H = stats[f"{algo}_layers"]
            node, extra = (32, 12) if algo == "sector" else (64, 64)
            ab = H * node + max(0.0, mp - H) * extra + mean_m + 8 + max(0.0, mean_m - 32) / 4
            if algo == "quad" and stats["quad_entry_bytes"] == 8:
                ab += stats["sa_width"]
        elif algo == "prefix":
            # the table pair, entry probes (8-B key-only or 16-B fused), the SA entry of
            # key-only leaves, the query, the position, the text window past char 32
            eb = stats["quad_entry_bytes"]
            ab = 2 * stats["sa_width"] + max(0.0, mp - 1) * eb + mean_m + 8 + max(0.0, mean_m - 32) / 4
            if eb == 8:
                ab += stats["sa_width"]
        else:
            ab = P * (4 + mean_m) + mean_m + 8
        results[algo] = {"lookups_per_s": nq * steps / el, "kernel_ms": kms, "mean_probes": mp,
                         "algorithmic_bytes_per_lookup": ab, "achieved_GBps": ab * nq / (kms * 1e-3) / 1e9,
                         "verified": okc}
    if rank == 0:
        h = results[main_algo]
        traffic, tsrc = load_traffic(f"c3_{main_algo}", n, nq, "8-256")
        emit({
            "metric": "pattern lookups/s (configs[3] shape)", "value": h["lookups_per_s"], "unit": "lookups/s",
            "n_gpus": ws, "steps": args.steps, "warmup": args.warmup, "ms_per_step": nq / h["lookups_per_s"] * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic: random_string(ChaCha8Rng({SEED})) text, positive queries len in [8,257)",
            "config": {"workload": f"configs[3]-shaped: n={n} chars, {stats['sa_width'] * 8}-bit SA, "
                                   f"{nq} mixed-length 8..256 queries, ragged", "n": n, "queries_per_gpu": nq,
                       "mean_m": total / nq, "algo": main_algo},
            "roofline": {"bound": "hbm", "achieved": h["achieved_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": h["achieved_GBps"] / HBM_PEAK_GBPS, "traffic": traffic,
                         "traffic_source": tsrc,
                         "kernel": {"stree": "k_sa_stree4x", "sector": "k_sa_sector", "quad": "k_sa_quad4x",
                                    "inline": "k_sa_inline", "prefix": "k_sa_prefix"}.get(main_algo, "k_sa_binary"),
                         "kernel_ms": h["kernel_ms"]},
            "variants": results, "setup_s": setup,
            "index": {k: stats[k] for k in ("stree_layers", "stree_lds_layers", "iterations", "sa_rounds",
                                            "build_sa_ns", "build_total_ns", "sa_width", "sa_bytes",
                                            "stree_bytes", "sector_bytes", "quad_bytes", "quad_fan",
                                            "quad_entry_bytes", "prefix_chars", "prefix_bytes")}})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 30, help="text length (chars)")
    ap.add_argument("--nq", type=int, default=10_000_000, help="queries per GPU")
    ap.add_argument("--m", type=int, default=32, help="query length")
    ap.add_argument("--algo", default=None, choices=["stree", "plain", "lcp", "sector", "quad", "inline", "llcp",
                                                         "prefix"])
    ap.add_argument("--variants", default="plain,plain_range,lcp,llcp,stree,sector,quad,inline,prefix,prefix_packed",
                    help="other algos timed beside the headline one")
    ap.add_argument("--prefix-chars", type=int, default=16,
                    help="p of the prefix table (the reference's main.rs default is -p 20 key bits)")
    ap.add_argument("--prefix-table", default="inline2", choices=["inline2", "inline4", "inline", "ranks"],
                    help="inline2: 32-B entries holding each range's first two suffixes, read by lane pairs "
                         "(4^16 x 32 B = 128 GiB); inline: 16-B entries with the first suffix (64 GiB); "
                         "ranks: u32 ranks only (sas/sa_search.rs:59-75's table)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", default="c1", choices=["c1", "c3", "sst"],
                    help="c1: 2^30 text, 10^7 len-32 queries (BASELINE metric); c3: largest u32-SA text "
                         "(2^32 - 2^20 chars), 10^8 queries of mixed length 8..256")
    ap.add_argument("--quad-compact", action="store_true",
                    help="c3: key-only quad leaves even where the fused ones fit (n <= 2^33)")
    ap.add_argument("--positive", action="store_true", help="sst workload: queries drawn from the keys")
    ap.add_argument("--mode", default="replicated", choices=["replicated", "shard"],
                    help="replicated index (weak scaling, no data-path collective) or sharded SA rank "
                         "ranges with RCCL all-to-all query routing (SURVEY §8e)")
    args = ap.parse_args()
    if args.algo is None:
        # the prefix table: c1 2.77e10 vs QUAD 1.40e10 lookups/s; c3 (n = 2^34, 40-bit SA,
        # ragged 8..256, p = 16 rank table) 24.5 vs 24.9 ms per 10^8 (tools/ab_c3.py: -7%)
        args.algo = "prefix"
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
        return run_c3(args, torch, sas_amd, dev, ws, rank, dist)
    if args.workload == "sst":
        return run_sst(args, torch, sas_amd, dev, ws, rank)
    n, nq, m = args.n, args.nq, args.m

    t_build0 = time.perf_counter()
    text = sas_amd.random_string(n, seed=SEED, device=dev)  # sas/util.rs:9-15, identical on every rank
    if args.mode == "shard":
        from sas_amd.shard import ShardedSearch
        # each rank builds ONLY its own SA rank range (sas_build_part: no whole-SA step)
        idx = sas_amd.SaNaive.build_part(text, rank, ws, lcp=True, stree=True, prefix=args.prefix_chars)  # 40-bit SA
        if dist is None:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            dist.init_process_group("nccl", rank=0, world_size=1)
        engine = ShardedSearch(idx, dist, ws, rank, dev, algo=args.algo)
    else:
        idx = sas_amd.SaNaive.build(text, lcp=True, stree=True, prefix=args.prefix_chars,
                                    prefix_inline={"ranks": 0, "inline": 1, "inline2": 2,
                                                   "inline4": 4}[args.prefix_table])
    stats = idx.stats()
    off = rank_query_offsets(n, nq, m, rank)
    off_t = torch.from_numpy(off.astype(np.int64)).to(dev)
    qbytes = torch.empty(nq * m, dtype=torch.uint8, device=dev)
    ar = torch.arange(m, device=dev, dtype=torch.int64)
    chunk = 1 << 18  # bounds the gather temporaries (HBM is nearly full at n = 2^34)
    for s in range(0, nq, chunk):
        e = min(nq, s + chunk)
        qbytes[s * m:e * m] = text[(off_t[s:e, None] + ar[None, :]).reshape(-1)]
    out = torch.empty(nq, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build0

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

    def run_algo(algo, steps, warmup):
        base, fl = algo_flags(algo)
        if algo == "prefix_packed" and "w" not in packed:
            # queries handed over 2-bit packed (sas_pack_queries, untimed: the caller's format)
            packed["w"] = sas_amd.SaNaive.pack_queries(qbytes, m)

        def step():
            if args.mode == "shard":
                out.copy_(engine.search_fixed(qbytes, m))
            elif algo == "prefix_packed":
                idx.search_packed(packed["w"], m, out=out)
            else:
                idx.search_fixed(qbytes, m, algo=base, out=out, flags=fl)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        holder = {}

        def timed_step_factory():
            # events bracket exactly the K timed launches on the launch stream
            state = {"i": 0}

            def s():
                if state["i"] == warmup:
                    ev0.record(stream)
                step()
                state["i"] += 1
                if state["i"] == warmup + steps:
                    ev1.record(stream)
            return s
        el = timed_loop(timed_step_factory(), steps, warmup, torch.cuda.synchronize, barrier, reduce_max)
        holder["kernel_ms"] = ev0.elapsed_time(ev1) / steps
        # correctness guard (untimed): every answer must be an occurrence of its query
        occ = text[(out[:, None] + ar[None, :]).reshape(-1).clamp_(max=n - 1)]
        ok = bool(torch.equal(occ, qbytes))
        return el, holder["kernel_ms"], ok

    el, kernel_ms, ok = run_algo(args.algo, args.steps, args.warmup)
    if not ok:
        raise SystemExit(f"bench: {args.algo} returned a non-occurrence position")
    # end to end from host buffers: pageable queries H2D, the search, positions
    # D2H, as a caller handing host memory through the C ABI would see it.  Never `value`.
    e2e = None
    if args.mode == "replicated":
        hq = qbytes.cpu().numpy()
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            hpos = idx.search_fixed(hq, m, algo=args.algo)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        e2e = {"lookups_per_s": nq / best, "ms": best * 1e3,
               "matches_device_run": bool(np.array_equal(hpos, out.cpu().numpy().astype(np.uint64))),
               "path": "host query bytes -> sas_search_fixed (staging hipMalloc + H2D, kernel, D2H)"}
    # probes -> tail probes for the algorithmic byte count (untimed pass; a shard of a
    # multi-GPU sharded run only holds part of the SA, so the pass needs the whole index)
    whole = args.mode == "replicated" or ws == 1
    if whole:
        _, probes = idx.search_fixed(qbytes, m, algo=args.algo, probes=True)
        mean_probes = float(probes.double().mean().item())
    else:
        mean_probes = float("nan")
    layers_of = {"stree": stats["stree_layers"], "sector": stats["sector_layers"], "quad": stats["quad_layers"]}
    tail = max(0.0, mean_probes - layers_of[args.algo]) if args.algo in layers_of else mean_probes
    pe = {16: 16, 32: 32, 64: 64}.get(stats["prefix_bytes"] // (4 ** stats["prefix_chars"] + 1), 8)
    algo_bytes = algorithmic_bytes(args.algo, n, m, stats["stree_layers"], tail, stats["sector_layers"],
                                   stats["quad_layers"], pe)
    achieved = algo_bytes * nq / (kernel_ms * 1e-3) / 1e9

    variants = {}
    for v in [x for x in args.variants.split(",") if x and x != args.algo and args.mode == "replicated"]:
        vel, vk, vok = run_algo(v, max(3, args.steps // 4), 1)
        vbase, vfl = algo_flags(v)
        if v == "prefix_packed":
            vbase = "prefix"
            _, vp = idx.search_packed(packed["w"], m, probes=True)
        else:
            _, vp = idx.search_fixed(qbytes, m, algo=vbase, probes=True, flags=vfl)
        vmean = float(vp.double().mean().item())
        vtail = max(0.0, vmean - layers_of[v]) if v in layers_of else vmean
        if vfl:  # the table entry + the reference's per-iteration SA word and text window
            vb = pe + max(0.0, vmean - 1) * (4 + m) + m + 8
        else:
            vb = algorithmic_bytes(vbase, n, 8 if v == "prefix_packed" else m, stats["stree_layers"], vtail,
                                   stats["sector_layers"], stats["quad_layers"], pe)
        variants[v] = {"lookups_per_s": ws * nq * max(3, args.steps // 4) / vel, "kernel_ms": vk,
                       "achieved_GBps": vb * nq / (vk * 1e-3) / 1e9, "algorithmic_bytes_per_lookup": vb,
                       "mean_probes": float(vp.double().mean().item()), "verified": vok}

    pkey = str(stats["prefix_chars"]) + {16: "i", 32: "d", 64: "q"}.get(pe, "")
    traffic, traffic_src, rdreq = load_traffic(args.algo + (pkey if args.algo == "prefix" else ""), n, nq, m,
                                               with_requests=True)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu and args.mode == "replicated":
        cpu = cpu_baseline(text, idx, qbytes, m, nq, args.cpu_seconds)

    if rank == 0:
        ms = el / args.steps * 1e3
        value = ws * nq * args.steps / el
        workload = {"stree": "configs[2]: 2^30 text in HBM, 10^7 len-32 queries, LCP-skipping search over an "
                             "S-tree of 16-char SA keys (top layers LDS-staged)",
                    "plain": "configs[1]: 2^30 text in HBM, 10^7 len-32 queries, plain binary search over SA",
                    "lcp": "configs[1] + mlr LCP skipping",
                    "prefix": "configs[2]: 2^30 text in HBM, 10^7 len-32 queries, the reference's prefix table "
                              "(sas/sa_search.rs:59-95, p = config.prefix_chars: one 8-B read gives the rank range) + binary "
                              "search over the fused 32-char key + SA entries of that range",
                    "llcp": "configs[1] probe sequence + Manber-Myers Llcp/Rlcp skipping (one 8-B {SA, Llcp, Rlcp} "
                            "entry per probe, text only on lcp ties), 2^30 text in HBM, 10^7 len-32 queries",
                    "sector": "configs[2]: 2^30 text in HBM, 10^7 len-32 queries, sector S-tree (32-B nodes, "
                              "fused 32-char key + SA leaves, top layers LDS-staged)",
                    "inline": "configs[1] probe sequence (binary_search_batch) over fused 32-char key + SA "
                              "entries, 2^30 text in HBM, 10^7 len-32 queries",
                    "quad": "configs[2]: 2^30 text in HBM, 10^7 len-32 queries, quad S-tree (17-ary 64-B nodes "
                            "loaded by 4-lane groups in one request each, 4-entry fused 32-char key + SA leaves, "
                            "top layers LDS-staged)"}[args.algo]
        line = {
            "metric": METRIC, "value": value, "unit": "lookups/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic: random_string(ChaCha8Rng::seed_from_u64({SEED})) text + positive len-{m} "
                    f"substrings (sas/util.rs:9-26), per-rank query stream",
            "config": {"workload": workload, "algo": args.algo, "n": n, "queries_per_gpu": nq, "m": m,
                       "prefix_chars": stats["prefix_chars"],
                       "mode": args.mode,
                       "parallelism": (f"replicated index x{ws}, query shards (no data-path collective)"
                                       if args.mode == "replicated" else
                                       f"SA rank ranges over {ws} GPUs, sas_route + RCCL all_to_all_single "
                                       f"(queries out, positions back)")},
            # shard mode: the events bracket route + exchanges + search, not one kernel
            "roofline": None if args.mode != "replicated" else {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": {"stree": "k_sa_stree", "sector": "k_sa_sector", "quad": "k_sa_quad",
                                    "inline": "k_sa_inline",
                                    "prefix": "k_sa_prefix2" if pe >= 32 else "k_sa_prefix"}.get(args.algo,
                                                                                                 "k_sa_binary"),
                         "kernel_ms": kernel_ms, "algorithmic_bytes_per_lookup": algo_bytes,
                         "mean_probes": mean_probes,
                         # what bounds this path: random 128-B-line requests (PMC L2->fabric reads
                         # of this workload, query stream included), against the measured
                         # random-request ceiling
                         "requests": None if rdreq is None else {
                             "per_lookup": rdreq / nq, "achieved_per_s": rdreq / (kernel_ms * 1e-3),
                             "ceiling_per_s": RANDOM_REQ_CEILING,
                             "frac": rdreq / (kernel_ms * 1e-3) / RANDOM_REQ_CEILING, "source": traffic_src}},
            "cpu_baseline": cpu,
            "e2e_host": e2e,
            "variants": variants,
            "index": {k: stats[k] for k in ("stree_layers", "stree_lds_layers", "sector_layers", "sector_lds_layers",
                                            "quad_layers", "quad_lds_layers", "quad_fan", "top_levels", "top2_levels", "iterations", "prefix_chars",
                                            "sa_rounds", "build_sa_ns", "build_total_ns")},
            "setup_s": build_s, "verified": ok,
        }
        emit(line)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
