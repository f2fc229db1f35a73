"""The sub-records beside the headline: the correctness guard (exact lower bounds), the CPU
baselines (configs[0] and the headline's), LCP skipping on long queries, configs[3] and
configs[4]."""
from __future__ import annotations

import os
import time

import numpy as np

from .common import *  # noqa: F401,F403
from .common import _r  # noqa: F401
from .model import *  # noqa: F401,F403
from .model import _quad_leaf_bytes  # noqa: F401

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
LCP_LONG_ALGOS = ("plain", "lcp", "llcp", "stree_llcp", "quad", "quad_llcp")


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
            for a in ("lcp", "llcp", "stree_llcp", "quad_llcp"):
                if row[a]["kernel_ms"] < row["plain"]["kernel_ms"]:
                    wins.append(f"{a}@{tk}_{mk}:{row['plain']['kernel_ms'] / row[a]['kernel_ms']:.2f}x")
    # configs[2]'s one kernel against the best of the two it joins, shape by shape
    best = {}
    for tk, rows in rec.items():
        if not isinstance(rows, dict) or tk in ("what", "summary"):
            continue
        for mk, row in rows.items():
            if isinstance(row, dict) and "quad_llcp" in row:
                ref = min(row["quad"]["kernel_ms"], row["stree_llcp"]["kernel_ms"])
                best[f"{tk}_{mk}"] = _r(row["quad_llcp"]["kernel_ms"] / ref, 3)
    return {"ms": s, "skipping_beats_plain": wins, "quad_llcp_over_min_quad_stree_llcp": best}


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
    rccl1 = routed1 = None
    if ws == 1:  # the routed shape a W > 1 rank runs (route + identity exchange + gather)
        engr = ShardedSearch(idx, dist, ws, rank, dev, algo="prefix", max_nq=nq, routed=True)
        outr = torch.empty(nq, dtype=torch.int64, device=dev)
        elr = timed_loop(lambda: engr.search_fixed(qbytes, m, check=False, out=outr), max(3, args.c4_steps // 2),
                         args.warmup, torch.cuda.synchronize, dist.barrier, reduce_max)
        engr.assert_no_overflow()
        if not bool(torch.equal(out, outr)):
            raise SystemExit("bench c4: the routed world-1 step differs from the identity step")
        routed1 = {"ms_per_step": elr / max(3, args.c4_steps // 2) * 1e3,
                   "lookups_per_s": nq * max(3, args.c4_steps // 2) / elr, "identical": True,
                   "what": "routed=True: sas_route_pack_cap + the identity exchange + sas_shard_gather around the "
                           "bucket lookup (the shape of each rank's step at N > 1)"}
        del outr
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
                       + (" -- at N = 1 every query is local: route, exchanges and gather are the identity, the "
                          "step is the part's lookup (routed_world1 times the routed shape, rccl_world1 its "
                          "exchanges through RCCL)" if ws == 1 else ""),
           "n": n, "parts": ws, "lookups_per_s": ws * nq * args.c4_steps / el, "ms_per_step": el / args.c4_steps * 1e3,
           "steps": args.c4_steps, "scaling": "weak", "part_sa_entries": st["sa_entries"],
           "prefix_entry_bytes": prefix_entry_bytes(st), "share": share,
           "prefix_keys": st["prefix_entries"], "prefix_bytes": st["prefix_bytes"],
           "prefix_key_fraction": _r(st["prefix_entries"] / (4 ** st["prefix_chars"] + 1)),
           "bucket_capacity": cap, "pieces": args.shard_chunks,
           "alt_pieces": {"pieces": alt_chunks, "ms_per_step": el2 / max(3, args.c4_steps // 2) * 1e3,
                          "lookups_per_s": ws * nq * max(3, args.c4_steps // 2) / el2, "identical": True},
           "exchange_bytes_per_step_per_rank": 2 * ws * cap * 8 * args.shard_chunks if ws > 1 else 0,
           "rccl_world1": rccl1, "routed_world1": routed1,
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
