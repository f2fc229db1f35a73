"""bench.py's shared pieces: the chip ceilings the roofline is stated against, the timing
harness (W untimed steps, K timed ones bracketed by barrier + device sync, HIP events per
launch), the result stream, the PMC summaries of the same library build, host facts."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
           "tagged": "k_sa_tagged", "quad_llcp": "k_sa_quad"}


# ---------------------------------------------------------------- harness
def timed_loop(step, steps: int, warmup: int, sync, barrier, reduce_max):
    """W untimed steps, then K steps bracketed by barrier + device sync on both sides;
    returns the MAX over ranks of the elapsed seconds.  Each rank's clock runs from the
    common start (the first barrier and sync) to its own device sync after the K steps; the
    closing barrier follows the reading, so the job time is the slowest rank's and no
    rank's time carries the barrier's own cost (an RCCL barrier, ~0.3 ms, would add 6% to
    a 20-step headline at N > 1 and not at N = 1)."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    barrier()
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


def _r(x, d: int = 4):
    """x to d significant digits (the line carries measurements, not float noise)."""
    if isinstance(x, bool) or x is None or not isinstance(x, (int, float)):
        return x
    if isinstance(x, int):
        return x
    return float(f"{x:.{d}g}") if np.isfinite(x) else None
