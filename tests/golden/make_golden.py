"""Generate the committed golden fixtures under tests/golden/.

* reference_kats.json -- the known-answer tests the reference itself carries,
  transcribed as data (inputs + expected outputs):
    sst/eytzinger.rs:200-230, sst/s_tree.rs:861-895, sst/btree.rs:179-187.
* sa_definition.json -- a DEFINITION oracle for the suffix-array path:
  SA = sorted(range(n), key=lambda i: T[i:]) and lower bound by bisect, in
  pure Python (list comparison == Rust slice order: a proper prefix sorts
  first).  Inputs come from Python's own `random` (seeded), independent of
  every line of this repository's C/HIP code.

Run:  python tests/golden/make_golden.py   (deterministic; rewrites both files)
"""
from __future__ import annotations

import bisect
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
U32_MAX = 0xFFFFFFFF
I32_MAX = 0x7FFFFFFF


def reference_kats() -> dict:
    return {
        "source": "RagnarGrootKoerkamp/suffix-array-searching @ 2025-07-11, static-search-tree/src",
        "eytzinger_layout": [
            {"cite": "sst/eytzinger.rs:200-206", "input": list(range(1, 16)),
             "vals": [U32_MAX, 8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15]},
            {"cite": "sst/eytzinger.rs:208-214", "input": list(range(0, 10)),
             "vals": [U32_MAX, 6, 3, 8, 1, 5, 7, 9, 0, 2, 4]},
        ],
        "eytzinger_search": [
            {"cite": "sst/eytzinger.rs:216-222", "input": list(range(0, 10)), "q": 3, "expect": 3},
            {"cite": "sst/eytzinger.rs:224-230", "input": list(range(0, 10)), "q": 12, "expect": U32_MAX},
        ],
        "stree_search": [
            {"cite": "sst/s_tree.rs:861-872 (test_bptree_search_bottom_layer)",
             "input": "range(1,2000) + [MAX]", "q": 452, "expect": 452},
            {"cite": "sst/s_tree.rs:874-885 (test_bptree_search_top_node)",
             "input": "range(1,2000) + [MAX]", "q": 289, "expect": 289},
        ],
        "node_find": [
            {"cite": "sst/s_tree.rs:887-895, sst/btree.rs:179-187", "node": list(range(1, 16)) + [I32_MAX],
             "q": 1, "expect": 0},
        ],
        # SortedVec::binary_search results pinned by the interpolation-search tests
        # (their expected values are binary_search's; q = 9 there reads vals[n], out
        # of bounds, and is left out) and the btree tests (same values as s_tree's)
        "sorted_search": [
            {"cite": "sst/interp_search.rs:258-266 (interppolation_vs_binsearch)",
             "input": list(range(1, 16)), "qs": [5], "expect": [5]},
            {"cite": "sst/interp_search.rs:268-276 (normal_vs_batched, q < 9)",
             "input": list(range(1, 9)), "qs": [0, 1, 2, 3, 4, 5, 6], "expect": [1, 1, 2, 3, 4, 5, 6]},
            {"cite": "sst/btree.rs:153-177 (test_btree_search_bottom_layer / _top_node)",
             "input": "range(1,2000) + [MAX]", "qs": [452, 289], "expect": [452, 289]},
        ],
    }


def sa_of(t):
    return sorted(range(len(t)), key=lambda i: t[i:])


def lower_bound(t, sa, q):
    sufs = [t[i:] for i in sa]
    return bisect.bisect_left(sufs, q)


def case(name, t, rng, extra_queries=()):
    sa = sa_of(t)
    n = len(t)
    qs = []
    for _ in range(24):  # positive substrings (random_queries shape, sas/util.rs:18-26)
        if n == 0:
            break
        i = rng.randrange(n)
        ln = rng.randrange(1, min(48, n - i) + 1)
        qs.append(t[i:i + ln])
    for _ in range(12):  # random (mostly negative) queries
        qs.append([rng.randrange(4) for _ in range(rng.randrange(0, 40))])
    qs.append([])  # empty query -> SA[0]
    qs.append([3] * (n + 5))  # above every suffix -> sentinel n
    if n:
        qs.append(t[:])  # the whole text
        qs.append(t + [0])  # longer than the text
        for k in (1, 2, 5, 17):  # text-end suffix + zero padding: the A7 `cmp` edge case
            s = t[max(0, n - k):]
            qs.append(s + [0] * 8)
            qs.append(s)  # full suffix: branchy_search (A10) returns a RANK here
    qs += [list(q) for q in extra_queries]
    out = []
    for q in qs:
        r = lower_bound(t, sa, q)
        out.append({"q": q, "rank": r, "pos": sa[r] if r < n else n})
    return {"name": name, "text": t, "sa": sa, "queries": out}


def sa_definition() -> dict:
    rng = random.Random(20250711)
    cases = []
    cases.append(case("single", [2], rng))
    cases.append(case("two", [3, 0], rng))
    cases.append(case("all_A_100", [0] * 100, rng, extra_queries=[[0] * 99, [0] * 100, [0] * 101, [0] * 50 + [1]]))
    cases.append(case("all_T_64", [3] * 64, rng))
    cases.append(case("periodic_ACGT_50", [0, 1, 2, 3] * 50, rng))
    cases.append(case("periodic_AC_long", [0, 1] * 300, rng))
    r = [rng.randrange(4) for _ in range(300)]
    cases.append(case("ends_with_A_run", r + [0] * 40, rng))
    cases.append(case("random_1000", [rng.randrange(4) for _ in range(1000)], rng))
    cases.append(case("random_4096", [rng.randrange(4) for _ in range(4096)], rng))
    # repeats longer than 32 / 64 chars: exercises multi-word compares and doubling rounds
    blk = [rng.randrange(4) for _ in range(150)]
    cases.append(case("long_repeats", blk + [rng.randrange(4) for _ in range(20)] + blk + blk[:90], rng,
                      extra_queries=[blk[:100], blk[:100] + [3], blk[10:140]]))
    return {"oracle": "definition: sorted(range(n), key=lambda i: T[i:]) + bisect_left over suffixes",
            "position_of_missing": "n (sentinel)", "cases": cases}


def main():
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(reference_kats(), f, indent=1)
    with open(os.path.join(HERE, "sa_definition.json"), "w") as f:
        json.dump(sa_definition(), f, separators=(",", ":"))


if __name__ == "__main__":
    main()
