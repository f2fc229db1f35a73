"""The u32 static-search-tree path (the reference's static-search-tree crate): the default line's
configs.sst record, --workload sst, and the reference's size sweep."""
from __future__ import annotations

import os
import time

import numpy as np

from .common import *  # noqa: F401,F403
from .common import _r  # noqa: F401

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
