"""The one stdout line (<= 4 KB) the driver parses, the full detail file, and the workload
labels."""
from __future__ import annotations

import json
import os

from .common import *  # noqa: F401,F403
from .common import _r  # noqa: F401
from .model import rel_groups
from .sst import sst_summary

# ---------------------------------------------------------------- the result line
LINE_LIMIT = 4096  # bytes: the driver reads the line back from the tail of stdout
DETAIL_PATH = os.path.join("gpurun_out", "bench_detail.json")


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
    for sk in ("lcp_stree", "lcp_quad"):
        if "c2" in confs and confs["c2"].get(sk):
            out["c2"][sk] = {kk: vv for kk, vv in config_summary(confs["c2"][sk]).items()
                             if kk in ("algo", "kernel_ms", "frac", "frac_basis", "traffic")}
    # configs[2]'s one kernel on the long-query shapes: QUAD_LLCP's time over the better of
    # QUAD and STREE_LLCP, text_m -> ratio (<= 1: at or below both; lcp_long in the detail file)
    qo = ((full.get("lcp_long") or {}).get("summary") or {}).get("quad_llcp_over_min_quad_stree_llcp")
    if "c2" in out and qo:
        out["c2"]["lcp_quad_long_vs_min"] = qo
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
    "quad_llcp": "configs[2] as one kernel: the quad S-tree's descent (17-ary 64-B nodes, top layers LDS-staged, "
                 "fused {32-char key, SA} leaves); where the leaf does not settle q, Manber-Myers LLCP skipping inside "
                 "the run of suffixes sharing q's key (m <= 32: the quad S-tree alone)",
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
