"""Headline benchmark: batched suffix-array pattern lookups on MI355X.

BASELINE.json metric: "pattern lookups/s + achieved HBM GB/s, 2^30-byte text,
10^7 len-32 queries".  One step = one batched lookup of all queries of this
GPU (inputs already resident in HBM), through the C ABI (sas_search_fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--algo prefix|plain|quad|...]
        (N > 1: bench.py starts N rank processes itself, one per GPU, benchlib/launch.py)
    torchrun --nproc-per-node N bench.py --gpus N ...   (the same N ranks from a launcher)

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

# the pieces live in benchlib/; their names stay importable as bench.<name>
from benchlib.common import *  # noqa: E402,F401,F403
from benchlib.common import _r  # noqa: E402,F401
from benchlib.model import *  # noqa: E402,F401,F403
from benchlib.model import _classify, _quad_leaf_bytes, _tree_layers  # noqa: E402,F401
from benchlib.records import *  # noqa: E402,F401,F403
from benchlib.sst import *  # noqa: E402,F401,F403
from benchlib.line import *  # noqa: E402,F401,F403
from benchlib.launch import needs_spawn, probe_main, resolve_world, spawn_ranks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) on this node: without a launcher, N > 1 starts N rank processes itself "
                         "(benchlib/launch.py); under torchrun it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 30, help="text length (chars)")
    ap.add_argument("--nq", type=int, default=10_000_000, help="queries per GPU")
    ap.add_argument("--m", type=int, default=32, help="query length")
    ap.add_argument("--algo", default=None, choices=["stree", "stree_llcp", "quad_llcp", "plain", "lcp", "sector", "quad", "inline",
                                                     "llcp",
                                                     "prefix", "tagged", "interp"])
    ap.add_argument("--variants",
                    default="plain,plain_range,llcp,stree,stree_llcp,sector,quad,quad_llcp,inline,interp,interp_range,"
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
    ap.add_argument("--workload", default="c1", choices=["c1", "c3", "sst", "launch_probe"],
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
    ap.add_argument("--probe-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    # --gpus N without a launcher: N fresh rank processes, started before this process makes
    # any HIP call; rank 0 prints the line, the job fails if any rank does
    if needs_spawn(args.gpus):
        return spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    ws, rank, local = resolve_world(args.gpus)  # under a launcher: --gpus must equal WORLD_SIZE
    keep_stdout_for_result()
    if args.workload == "launch_probe":
        return probe_main(args, emit, log)

    import torch
    import sas_amd

    dist = None
    # under a launcher (torchrun, or this script's own children) the group comes from its
    # environment, at world size 1 too: torchrun's agent hosts the store, and a group of our
    # own over tcp:// would wait as a client of a store nobody serves (the configs[4] record)
    if ws > 1 or "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        # n_gpus is the group the step ran in, not the environment's claim
        ws = dist.get_world_size()
        rank = dist.get_rank()
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
               "stree_llcp": "stree_llcp", "quad_llcp": "quad_llcp"}.get(v)
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
            # the two joined: QUAD's descent + the LLCP tail where the leaf does not settle q (at
            # m = 32 the 32-char key always does: QUAD's kernel; its long-query shapes in lcp_long)
            if "quad_llcp" in variants:
                configs["c2"]["lcp_quad"] = dict(variants["quad_llcp"], workload=WORKLOADS["quad_llcp"],
                                                 lds_layers=stats["quad_lds_layers"])
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
    sys.exit(main())
