"""Summarise rocprofv3 --pmc counter CSVs for one kernel into a JSON that
bench.py reports as roofline.traffic.

Usage:
  python tools/pmc_to_json.py --kernel k_sa_stree --nq 10000000 \
      --fetch gpurun_out/pmc_fetch/run_counter_collection.csv \
      --write gpurun_out/pmc_write/run_counter_collection.csv \
      [--req gpurun_out/pmc_req/run_counter_collection.csv] \
      --out profiles/pmc_stree_n1073741824_q10000000_m32.json

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
  * counters come from separate passes (FETCH_SIZE and WRITE_SIZE do not fit
    one TCC pass);
  * FETCH_SIZE / WRITE_SIZE are in KiB;
  * gfx950 tallies 128-B read requests at 64 B in FETCH_SIZE, so the read side
    is taken as TCC_EA0_RDREQ x 128 B when the request counters are available
    (--req pass: TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum) and as
    2 x FETCH_SIZE otherwise; both are reported.
  * Infinity-Cache hits are included in these L2 memory-side counters, so the
    figure is an upper bound on DRAM bytes.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict


def per_dispatch(path, kernel):
    """Counter sums per dispatch of `kernel` (the name itself, then its template arguments or
    parameter list: k_sa_prefix2 does not match k_sa_prefix2_range)."""
    pat = re.compile(r"(^|[^\w])" + re.escape(kernel) + r"\s*[<(]")
    vals = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for row in csv.DictReader(f):
            if not pat.search(row.get("Kernel_Name", "")):
                continue
            vals[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    return vals


STAT = "median"


def mean_counter(path, kernel, name):
    """The counter over the kernel's dispatches: their median by default (the bench's one
    out_probes dispatch reads more than the timed ones and would skew a mean), or the mean
    (--stat mean)."""
    d = per_dispatch(path, kernel)
    xs = sorted(v[name] for v in d.values() if name in v)
    if not xs:
        return None, 0
    if STAT == "mean":
        return sum(xs) / len(xs), len(xs)
    k = len(xs) // 2
    return (xs[k] if len(xs) % 2 else (xs[k - 1] + xs[k]) / 2), len(xs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--nq", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--req")
    ap.add_argument("--out", required=True)
    ap.add_argument("--algo-bytes", type=float, default=None, help="algorithmic bytes per lookup")
    ap.add_argument("--source-hash", default=None,
                    help="source hash of the library the counters were collected on (default: the in-tree "
                         "libsas_amd.so's sas_source_hash); bench.py reports the counters only for that build")
    ap.add_argument("--stat", default="median", choices=["median", "mean"], help="over the kernel's dispatches")
    a = ap.parse_args()
    global STAT
    STAT = a.stat
    fetch_kib, nf = mean_counter(a.fetch, a.kernel, "FETCH_SIZE")
    write_kib, nw = mean_counter(a.write, a.kernel, "WRITE_SIZE")
    if a.source_hash is None:
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "suffix-array-searching_amd"))
        import sas_amd
        a.source_hash = sas_amd.source_hash()
    out = {"kernel": a.kernel, "source_hash": a.source_hash, "dispatch_stat": a.stat, "dispatches_fetch": nf,
           "dispatches_write": nw,
           "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib}
    read_bytes = 2 * fetch_kib * 1024 if fetch_kib is not None else None
    out["read_bytes_2xFETCH"] = read_bytes
    if a.req:
        rdreq, _ = mean_counter(a.req, a.kernel, "TCC_EA0_RDREQ_sum")
        rd32, _ = mean_counter(a.req, a.kernel, "TCC_EA0_RDREQ_32B_sum")
        hit, _ = mean_counter(a.req, a.kernel, "TCC_HIT_sum")
        miss, _ = mean_counter(a.req, a.kernel, "TCC_MISS_sum")
        out.update({"TCC_EA0_RDREQ": rdreq, "TCC_EA0_RDREQ_32B": rd32, "TCC_HIT": hit, "TCC_MISS": miss})
        if rdreq is not None:
            wide = rdreq - (rd32 or 0)
            read_bytes = wide * 128 + (rd32 or 0) * 32
            out["read_bytes_from_requests"] = read_bytes
        if hit is not None and miss is not None and hit + miss > 0:
            out["L2_hit_rate"] = hit / (hit + miss)
    write_bytes = write_kib * 1024 if write_kib is not None else 0
    total = (read_bytes or 0) + write_bytes
    out["hbm_bytes_per_launch"] = total
    out["hbm_bytes_per_lookup"] = total / a.nq
    if a.algo_bytes:
        out["algorithmic_bytes_per_lookup"] = a.algo_bytes
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
