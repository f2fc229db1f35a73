"""configs[3] at full size (BASELINE.json configs[3]; the n = 2^34 deviation of DESIGN.md §5):
a 2^34-char ChaCha8 text, 10^6 ragged positive queries of length 8..256 (random_queries,
sas/util.rs:18-26), on the two indexes the bench uses at that size.

* the tagged index (SAS_BUILD_TAGGED: 8-B tagged entries + p = 16 bucket table): TAGGED,
  PLAIN and LCP give identical positions;
* the 40-bit SA index with compact key-only quad leaves and a p = 16 40-bit rank table:
  PREFIX, QUAD and PLAIN give the same positions as the tagged index;
* the bucket-line index (SAS_BUILD_TAG_LINES, p = 15, the bench's configs[3] record; built
  from a host copy of the text): TAGGED, byte queries and text slices, the same positions;
  its ranges and SA values equal the tagged index's;
* every answer is an occurrence of its query (positive queries), and 3000 sampled answers
  are proven exact lower bounds on the index's own SA: SA[lo] = answer and
  suffix(SA[lo-1]) < q, with lo from sas_search_range; the indexes' ranges agree.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 34
NQ = 1_000_000


def less(a, q):
    """Rust slice order a < q"""
    k = min(len(a), len(q))
    d = np.nonzero(a[:k] != q[:k])[0]
    if len(d):
        return a[d[0]] < q[d[0]]
    return len(a) < len(q)


def window(torch, idx, p, L):
    L = min(L, idx.n - p)
    o = torch.empty(max(L, 1), dtype=torch.uint8, device="cuda")
    if L > 0:
        idx.extract(torch.tensor([p], dtype=torch.int64, device="cuda"),
                    torch.tensor([L], dtype=torch.int32, device="cuda"),
                    torch.zeros(1, dtype=torch.int64, device="cuda"), o)
    return o[:L].cpu().numpy()


def test_c3_full_size():
    import torch

    import sas_amd
    t = sas_amd.random_string(N, seed=31415, device="cuda")
    tagged = sas_amd.SaNaive.build(t, lcp=False, verify=True, tagged=True)
    st = tagged.stats()
    assert st["sa_width"] == 8 and st["tag_chars"] == 16 and st["sa_entries"] == N
    off, ln, _ = sas_amd.random_queries(N, NQ, seed=31415, word_pos=N, margin=256, len_lo=8, len_hi=257)
    lens = torch.from_numpy(ln.astype(np.int64)).cuda()
    qoff = torch.zeros(NQ, dtype=torch.int64, device="cuda")
    qoff[1:] = torch.cumsum(lens, 0)[:-1]
    qlen = lens.to(torch.int32)
    total = int(lens.sum().item())
    qb = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(off.astype(np.int64)).cuda()
    qb[:total] = 0
    tagged.extract(src, qlen, qoff, qb)
    # the queries are the text's own substrings (the byte text vs the packed index text)
    pick = np.random.default_rng(1).choice(NQ, 200, replace=False)
    for i in pick:
        o, L, s = int(qoff[i]), int(ln[i]), int(off[i])
        assert torch.equal(qb[o:o + L], t[s:s + L])
    del t
    torch.cuda.empty_cache()

    res = {}
    for algo in ("tagged", "plain", "lcp"):
        res[algo] = tagged.search_batch(qb, qoff, qlen, algo=algo)
        torch.cuda.synchronize()
    for algo in ("plain", "lcp"):
        assert torch.equal(res[algo], res["tagged"]), algo
    pos = res["tagged"]
    # every answer is an occurrence
    got = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    tagged.extract(pos, qlen, qoff, got)
    assert torch.equal(got[:total], qb[:total])
    # exact lower bounds on a sample, from the index's own SA
    ids = np.sort(np.random.default_rng(2).choice(NQ, 3000, replace=False))
    dids = torch.from_numpy(ids).cuda()
    qo = qoff[dids].cpu().numpy()
    qs = [qb[int(qo[j]):int(qo[j]) + int(ln[i])].cpu().numpy() for j, i in enumerate(ids)]
    lens_s = np.array([len(q) for q in qs], np.uint32)
    off_s = np.zeros(len(qs), np.uint64)
    off_s[1:] = np.cumsum(lens_s[:-1], dtype=np.uint64)
    buf = np.concatenate(qs + [np.zeros(64, np.uint8)])
    lo_t, hi_t = tagged.search_range(buf, off_s, lens_s)
    ans = pos[dids].cpu().numpy()
    for j in range(len(ids)):
        r, q = int(lo_t[j]), qs[j]
        sa2 = tagged.suffix_array(count=2, start=r - 1) if r > 0 else tagged.suffix_array(count=1, start=0)
        assert int(sa2[-1]) == int(ans[j]), j
        assert not less(window(torch, tagged, int(sa2[-1]), len(q)), q), j
        if r > 0:
            assert less(window(torch, tagged, int(sa2[0]), len(q)), q), j
        assert int(hi_t[j]) > r  # a positive query occurs at least once
    ref = pos.cpu()
    tagged.free()
    torch.cuda.empty_cache()

    # the 40-bit SA index with compact quad leaves and a p = 16 rank table
    t = sas_amd.random_string(N, seed=31415, device="cuda")
    idx = sas_amd.SaNaive.build(t, lcp=False, stree=False, sector=False, quad="compact", verify=True, llcp=False,
                                prefix=16)
    del t
    torch.cuda.empty_cache()
    assert idx.stats()["sa_width"] == 5
    for algo in ("prefix", "quad", "plain"):
        r = idx.search_batch(qb, qoff, qlen, algo=algo)
        torch.cuda.synchronize()
        assert torch.equal(r.cpu(), ref), algo
    lo_q, hi_q = idx.search_range(buf, off_s, lens_s)
    assert np.array_equal(lo_q, lo_t) and np.array_equal(hi_q, hi_t)
    sa_probe = [int(idx.suffix_array(count=1, start=int(lo_t[j]))[0]) for j in range(0, len(ids), 100)]
    idx.free()
    torch.cuda.empty_cache()

    # the bucket-line index (from a host copy: a device byte text does not fit beside its build)
    ht = sas_amd.random_string(N, seed=31415, device="cuda").cpu().numpy()
    torch.cuda.empty_cache()
    lines = sas_amd.SaNaive.build(ht, lcp=False, verify=True, tagged=True, tag_lines=True)
    del ht
    st = lines.stats()
    assert st["tag_chars"] == 15 and st["tag_line_slots"] == 20 and st["tag_line_tag_bits"] == 13 and st["sa_entries"] == N
    r = lines.search_batch(qb, qoff, qlen, algo="tagged")
    torch.cuda.synchronize()
    assert torch.equal(r.cpu(), ref)
    r = lines.search_slices(src, qlen)
    torch.cuda.synchronize()
    assert torch.equal(r.cpu(), ref)
    lo_l, hi_l = lines.search_range(buf, off_s, lens_s)
    assert np.array_equal(lo_l, lo_t) and np.array_equal(hi_l, hi_t)
    assert sa_probe == [int(lines.suffix_array(count=1, start=int(lo_t[j]))[0]) for j in range(0, len(ids), 100)]
    lines.free()
