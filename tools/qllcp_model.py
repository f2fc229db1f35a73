"""CPU model of k_sa_quad_llcp (SAS_ALGO_QUAD_LLCP, csrc/sas_search.hip) for m > 32: the
quad tree's routing invariants (leaf k = the leaf of the first suffix whose 16-char key is
>= K16; leaf kU = that of the first key16 > K16), the leaf counts, L0 / U / s0 / kappa, and the
LLCP walk with its substituted lcps.  Every tie compare asserts that the chars it skips are
really equal to q's, and every answer is checked against the oracle's binary_search.  A
design check run before the kernel meets the GPU (python tools/qllcp_model.py)."""
import bisect
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pyoracle as O  # noqa: E402

CAP = 4095
NEXT_MODE = int(os.environ.get("QLLCP_NEXT", "2"))  # the kernel's SAS_QLLCP_NEXT


def key_of(t, p, c):
    """zero-padded c-char key of suffix p as an int (2 bits a char)"""
    s = t[p:p + c]
    v = 0
    for j in range(c):
        v = (v << 2) | (int(s[j]) if j < len(s) else 0)
    return v


def lcp_str(a, b):
    k = 0
    n = min(len(a), len(b))
    while k < n and a[k] == b[k]:
        k += 1
    return k


def leaf_keys(t, sa):
    """the fused leaves' 32-char keys in SA order, the last leaf padded with all ones"""
    sa_n = len(sa)
    nl = (sa_n + 3) // 4
    return [key_of(t, int(sa[r]), 32) for r in range(sa_n)] + [(1 << 64) - 1] * (4 * nl - sa_n)


def model(t, sa, lcpa, q, stats, keys=None):
    n = len(t)
    sa_n = n
    m = len(q)
    assert m > 32
    K64 = key_of(q, 0, 32)
    K16 = K64 >> 32
    if keys is None:
        keys = leaf_keys(t, sa)
    nl = (sa_n + 3) // 4
    k16s = [x >> 32 for x in keys[:sa_n]] if "k16s" not in stats else stats["k16s"]
    first16 = bisect.bisect_left(k16s, K16)
    k = min(first16 // 4, nl - 1)
    leaf = keys[4 * k:4 * k + 4]
    c16 = sum((x >> 32) < K16 for x in leaf)
    c64 = sum(x < K64 for x in leaf)
    le64 = sum(x <= K64 for x in leaf)
    kb = 4 * k

    def lam_of(x):
        key = keys[x]
        d = 32 if key == K64 else (64 - (key ^ K64).bit_length()) // 2
        ln = n - int(sa[x]) if x < sa_n else 0
        return min(d, ln)
    x32 = c64 < 4
    x32_u = True
    if le64 < 4:
        U = kb + le64
    elif K16 == 0xFFFFFFFF:
        U = sa_n
        x32 = False
        x32_u = False
    else:
        firstgt = bisect.bisect_right(k16s, K16)
        kU = min(firstgt // 4, nl - 1)
        lf = keys[4 * kU:4 * kU + 4]
        le64U = sum(x <= K64 for x in lf)
        le16U = sum((x >> 32) <= K16 for x in lf)
        f = le64U if le64U else le16U
        x32 = x32 and le64U > 0
        x32_u = le64U > 0
        U = 4 * kU + f
        stats["kU_descents"] += kU != k
    U = min(U, sa_n)
    L0 = kb + c64
    s0 = kb + c16
    kappa = 32 if x32 else 16
    qs = bytes(q)

    def suf(p):
        return bytes(t[p:])
    if L0 >= sa_n:
        return n, 0
    lam0 = None
    next_read = NEXT_MODE == 1 or (NEXT_MODE == 2 and c16 == 3)
    if next_read and c64 == 4 and keys[L0] >= K64:
        # the kernel reads the next entry: its key >= q's makes L0 exact at 32 chars
        c64 = 3  # (as if leaf k had held it)
        x32 = x32_u
        kappa = 32 if x32 else 16
    if c64 < 4:
        # the first suffix not below q's 32-char key: > it, or one compare from char 32
        S0 = suf(int(sa[L0]))
        if keys[L0] != K64 or S0 >= qs:
            stats["one"] += 1
            return int(sa[L0]), 0
        lam0 = lcp_str(S0, qs)
        L0 += 1
    stats["walk"] += 1
    # the walk
    lo, r = 0, sa_n
    llcp = rlcp = 0
    reads = 0
    while True:
        mid = None
        while lo < r:
            mid = (lo + r) >> 1
            if mid < L0:
                lo = mid + 1
            elif mid >= U:
                r = mid
            else:
                break
        if not lo < r:
            break
        # the implicit interval of mid is exactly [lo, r) (a bisection from [0, sa_n))
        p = int(sa[mid])
        x = 0 if lo == 0 else min(int(lcpa[lo:mid + 1].min()), CAP)
        y = 0 if r >= sa_n else min(int(lcpa[mid + 1:r + 1].min()), CAP)
        if lo <= s0:
            llcp = x
        elif lo <= L0:
            llcp = lam0 if (lam0 is not None and lo == L0) else lam_of(lo - 1)
            assert llcp == lcp_str(suf(int(sa[lo - 1])), qs), "lam"
        if r >= U:
            rlcp = y
        reads += 1
        decided = True
        if llcp >= rlcp:
            if x > llcp:
                lt, lc = True, llcp
            elif x < llcp and x < CAP:
                lt, lc = False, x
            else:
                decided, hh = False, x
        else:
            if y > rlcp:
                lt, lc = False, rlcp
            elif y < rlcp and y < CAP:
                lt, lc = True, y
            else:
                decided, hh = False, y
        S = suf(p)
        true_l = lcp_str(S, qs)
        if decided:
            assert lt == (S < qs) and lc == true_l, ("rule", mid, lt, lc, true_l)
        else:
            if n - p < kappa:
                assert S < qs and true_l == n - p, "short"
                lt, lc = True, n - p
            else:
                h = hh if hh + 16 > kappa else kappa
                assert true_l >= h, ("skip", h, true_l, hh, kappa)
                lt, lc = S < qs, true_l
        if lt:
            lo = mid + 1
            llcp = lc
        else:
            r = mid
            rlcp = lc
    stats["reads"] += reads
    return (n if r >= sa_n else int(sa[r])), reads


def run(name, t, nq=400, seed=1):
    rng = np.random.default_rng(seed)
    n = len(t)
    sa = O.build_sa(t)
    lcpa = O.kasai_lcp(t, sa).astype(np.int64)
    qs = []
    for o, L in zip(rng.integers(0, n - 300, nq), rng.integers(33, 300, nq)):
        q = t[o:o + L].copy()
        qs.append(q)
        mq = q.copy()
        k = int(rng.integers(16, len(q)))
        mq[k] = (mq[k] + 1 + rng.integers(0, 3)) % 4
        qs.append(mq)
    qs += [np.concatenate([t[n - k:], np.zeros(j, np.uint8)]) for k in (33, 40, 70) for j in (0, 5)]
    qs += [np.concatenate([t[n - k:], np.full(40, 3, np.uint8)]) for k in (5, 20)]
    st = {"settled": 0, "one": 0, "walk": 0, "reads": 0, "kU_descents": 0}
    keys = leaf_keys(t, sa)
    aux = dict(st, k16s=[x >> 32 for x in keys[:n]])
    tp = O.padded(t)
    for q in qs:
        if len(q) <= 32:
            continue
        qb = np.concatenate([q, np.zeros(64, np.uint8)])
        exp, _ = O.search_many(tp, n, sa, qb, np.zeros(1, np.uint64), np.array([len(q)], np.uint32),
                               "binary_search", 1)
        got, _ = model(t, sa, lcpa, q, aux, keys)
        assert got == int(exp[0]), (name, got, int(exp[0]), q[:40])
    st = {k: aux[k] for k in st}
    print(name, st)
    return st


if __name__ == "__main__":
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 4, 700, dtype=np.uint8)
    run("random", rng.integers(0, 4, 3000, dtype=np.uint8))
    run("all_A", np.zeros(2000, np.uint8), nq=100)
    run("period_7", np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 400), nq=150)
    run("repeats", np.concatenate([blk, rng.integers(0, 4, 30, dtype=np.uint8), blk, blk[:500], blk]))
    sub = np.tile(rng.integers(0, 4, 300, dtype=np.uint8), 8)
    sub[rng.integers(0, len(sub), 25)] = rng.integers(0, 4, 25)
    run("copies_subst", sub)
