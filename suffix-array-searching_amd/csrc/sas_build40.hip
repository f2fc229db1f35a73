// sas_build40.hip -- suffix array of a long text into a packed 40-bit array.
//
// SaNaive::build (sas/sa_search.rs:30-57) keeps a u32 SA, so the reference caps
// n below 2^32 (the `as u32` cast at :35).  BASELINE's C3 config wants a text
// that fills HBM; this builder lifts the cap (n < 2^40, as HBM allows) without
// ever holding all (key, position) pairs at once:
//
//   1. histogram of the first HIST_BITS/2 chars of every suffix (LDS counters),
//   2. consecutive histogram bins are grouped into buckets of at most `cap`
//      suffixes (cap from free HBM); per bucket, in key order:
//        - collect (32-char key, position) of its suffixes in position order
//          (block counts -> scan -> ballot-compacted stores: no atomics),
//        - radix sort the pairs (rocPRIM onesweep, 64-bit keys, 64-bit values),
//        - emit SA ranks off..off+c, the group id (rank of the first suffix with
//          the same 32-char key) of every suffix into the 40-bit rank array, and
//          append the still-tied ranks to one ascending list,
//   3. prefix-doubling rounds over the tied list only (h = 32, 64, ...), the
//      same LSD two-pass scheme as the u32 builder's n >= 2^31 path with
//      40-bit ids: sort by the second key (BIG + rank[p + h], or n - p for a
//      suffix shorter than h: Rust slice order puts a proper prefix first),
//      then stably by the group.
//
// Working memory: text (n/4 B) + SA (5n) + rank (5n) + ~40 B per bucket entry
// + ~60 B per tied suffix.  A single HIST_BITS bin larger than cap (a text
// dominated by one 7-mer) is refused with ENOTSUP rather than overcommitting.
#include "build_util.hpp"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <cstdlib>
#include <vector>

#define HIST_BITS 14
#define HIST_BINS (1u << HIST_BITS)
#define COLLECT_BLOCK 1024
#define COLLECT_ITEMS 16
#define COLLECT_CHUNK (COLLECT_BLOCK * COLLECT_ITEMS)  // positions per block
#define BIG40 (1ull << 40)

__device__ __forceinline__ uint32_t bin_of(uint64_t key) { return (uint32_t)(key >> (64 - HIST_BITS)); }

__global__ __launch_bounds__(1024) void k_hist(const uint64_t* __restrict__ tw, uint64_t n,
                                               unsigned long long* __restrict__ hist) {
    __shared__ uint32_t h[HIST_BINS];
    for (uint32_t i = threadIdx.x; i < HIST_BINS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    GRID_STRIDE(p, n) atomicAdd(&h[bin_of(text_chars32(tw, p))], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < HIST_BINS; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* s_w) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) s_w[wave] = v;
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) t += s_w[w];
    __syncthreads();
    return t;
}

// Chunk k owns positions [k*CHUNK, (k+1)*CHUNK): count those whose bin is in [lo, hi).  The
// workgroups stride over the chunks (a dispatch holds < 2^32 work-items: n = 2^36 is 2^22
// chunks of 1024 threads)
#define COLLECT_GRID (1u << 16)
// debug: SAS_COLLECT_GRID=g caps the grid at g workgroups, so a small text takes the stride loop
// that n = 2^36 needs (tests/test_gpu_sa.py::test_collect_grid_stride)
static uint32_t collect_grid(uint64_t nblk) {
    uint64_t g = nblk < COLLECT_GRID ? nblk : COLLECT_GRID;
    if (const char* e = getenv("SAS_COLLECT_GRID")) {
        const long v = atol(e);
        if (v > 0 && (uint64_t)v < g) g = (uint64_t)v;
    }
    return (uint32_t)g;
}
__global__ __launch_bounds__(COLLECT_BLOCK) void k_bucket_count(const uint64_t* __restrict__ tw, uint64_t n,
                                                                uint32_t lo, uint32_t hi,
                                                                uint64_t* __restrict__ block_cnt) {
    __shared__ uint32_t s_w[COLLECT_BLOCK / 64];
    const uint64_t nblk = (n + COLLECT_CHUNK - 1) / COLLECT_CHUNK;
    for (uint64_t k = blockIdx.x; k < nblk; k += gridDim.x) {
        const uint64_t base = k * COLLECT_CHUNK;
        uint32_t c = 0;
#pragma unroll 4
        for (int it = 0; it < COLLECT_ITEMS; it++) {
            uint64_t p = base + (uint64_t)it * COLLECT_BLOCK + threadIdx.x;
            if (p < n) {
                uint32_t b = bin_of(text_chars32(tw, p));
                c += (b >= lo && b < hi);
            }
        }
        uint32_t t = block_sum(c, s_w);
        if (threadIdx.x == 0) block_cnt[k] = t;
    }
}

// Same walk; matches are stored at block_off[b] + (rank among the block's
// matches in position order): wave ballot + per-wave offsets, no atomics.
__global__ __launch_bounds__(COLLECT_BLOCK) void k_bucket_collect(const uint64_t* __restrict__ tw, uint64_t n,
                                                                  uint32_t lo, uint32_t hi,
                                                                  const uint64_t* __restrict__ block_off,
                                                                  uint64_t* __restrict__ keys,
                                                                  uint64_t* __restrict__ vals) {
    __shared__ uint32_t s_w[COLLECT_BLOCK / 64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t nblk = (n + COLLECT_CHUNK - 1) / COLLECT_CHUNK;
    for (uint64_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    uint64_t run = block_off[k];
    const uint64_t base = k * COLLECT_CHUNK;
    for (int it = 0; it < COLLECT_ITEMS; it++) {
        uint64_t p = base + (uint64_t)it * COLLECT_BLOCK + threadIdx.x;
        uint64_t key = 0;
        bool match = false;
        if (p < n) {
            key = text_chars32(tw, p);
            uint32_t b = bin_of(key);
            match = b >= lo && b < hi;
        }
        uint64_t bal = __ballot(match);
        if (lane == 0) s_w[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < COLLECT_BLOCK / 64; w++) {
            uint32_t cw = s_w[w];
            before += (w < wave) ? cw : 0u;
            total += cw;
        }
        if (match) {
            uint64_t at = run + before + (uint32_t)__popcll(bal & lt_mask);
            keys[at] = key;
            vals[at] = p;
        }
        run += total;
        __syncthreads();
    }
    }  // chunks
}

__global__ void k_b_heads(const uint64_t* __restrict__ keys, uint64_t c, uint64_t off,
                          uint64_t* __restrict__ headpos) {
    GRID_STRIDE(j, c) headpos[j] = (j == 0 || keys[j] != keys[j - 1]) ? off + j : 0ull;
}

__global__ void k_b_emit(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ vals,
                         const uint64_t* __restrict__ group, uint64_t c, uint64_t off, uint8_t* __restrict__ sa5,
                         uint8_t* __restrict__ rank5, uint8_t* __restrict__ tied) {
    GRID_STRIDE(j, c) {
        uint64_t p = vals[j];
        sa_put<5>(sa5, off + j, p);
        if (rank5) sa_put<5>(rank5, p, group[j]);
        bool h0 = (j == 0) || keys[j] != keys[j - 1];
        bool h1 = (j + 1 == c) || keys[j + 1] != keys[j];
        tied[j] = !(h0 && h1);
    }
}

// ---- doubling rounds over the tied ranks (40-bit ids)
__device__ __forceinline__ uint64_t second_key40(SaView<5> rank, uint64_t n, uint64_t p, uint64_t h) {
    return (p + h < n) ? (BIG40 + rank[p + h]) : (n - p);
}

__global__ void k_r40_second(const uint64_t* __restrict__ list, uint64_t cnt, SaView<5> sa, SaView<5> rank,
                             uint64_t n, uint64_t h, uint64_t* __restrict__ keys, uint64_t* __restrict__ vals) {
    GRID_STRIDE(k, cnt) {
        uint64_t p = sa[list[k]];
        keys[k] = second_key40(rank, n, p, h);
        vals[k] = p;
    }
}

__global__ void k_r40_group(const uint64_t* __restrict__ vals, uint64_t cnt, SaView<5> rank,
                            uint64_t* __restrict__ keys) {
    GRID_STRIDE(k, cnt) keys[k] = rank[vals[k]];
}

__global__ void k_r40_heads(const uint64_t* __restrict__ vals, uint64_t cnt, SaView<5> rank, uint64_t n, uint64_t h,
                            const uint64_t* __restrict__ list, uint64_t* __restrict__ headpos,
                            uint8_t* __restrict__ head) {
    GRID_STRIDE(k, cnt) {
        bool hd = true;
        if (k > 0) {
            uint64_t p = vals[k], q = vals[k - 1];
            hd = rank[p] != rank[q] || second_key40(rank, n, p, h) != second_key40(rank, n, q, h);
        }
        head[k] = hd;
        headpos[k] = hd ? list[k] : 0ull;
    }
}

__global__ void k_r40_scatter(const uint64_t* __restrict__ list, uint64_t cnt, const uint64_t* __restrict__ vals,
                              uint8_t* __restrict__ sa5) {
    GRID_STRIDE(k, cnt) sa_put<5>(sa5, list[k], vals[k]);
}

__global__ void k_r40_assign(uint64_t cnt, const uint64_t* __restrict__ vals, const uint64_t* __restrict__ group,
                             const uint8_t* __restrict__ head, uint8_t* __restrict__ rank5,
                             uint8_t* __restrict__ unresolved) {
    GRID_STRIDE(k, cnt) {
        sa_put<5>(rank5, vals[k], group[k]);
        bool h1 = (k + 1 == cnt) || head[k + 1];
        unresolved[k] = !(head[k] && h1);
    }
}

template <class Fn>
static int with_temp(DevBuf& tmp, size_t& have, Fn fn) {
    size_t need = 0;
    HIP_TRY(fn((void*)nullptr, need));
    if (need > have) {
        TRY(tmp.alloc(need, "rocprim temp"));
        have = need;
    }
    HIP_TRY(fn(tmp.p, need));
    return 0;
}

static int histogram(const uint64_t* tw, uint64_t n, std::vector<uint64_t>& h) {
    DevBuf hist;
    TRY(hist.alloc(HIST_BINS * 8, "histogram"));
    HIP_TRY(hipMemset(hist.p, 0, HIST_BINS * 8));
    unsigned g = grid_for(n, 1024);
    hipLaunchKernelGGL(k_hist, dim3(g < 1024 ? g : 1024), dim3(1024), 0, 0, tw, n, hist.as<unsigned long long>());
    HIP_TRY(hipGetLastError());
    h.assign(HIST_BINS, 0);
    HIP_TRY(hipMemcpy(h.data(), hist.p, HIST_BINS * 8, hipMemcpyDeviceToHost));
    return 0;
}

// Tied entries collected while sorting buckets: ascending SA slots + group ids.
struct TiedSink {
    DevBuf list, grp;
    uint64_t cap = 0, cnt = 0;
};

static int append_dev(DevBuf& dst, uint64_t& cap, uint64_t have, const uint64_t* src, uint64_t d, const char* what) {
    if (have + d > cap) {
        uint64_t nc = cap ? cap : 1024;
        while (nc < have + d) nc *= 2;
        DevBuf grown;
        TRY(grown.alloc(nc * 8, what));
        if (have) HIP_TRY(hipMemcpy(grown.p, dst.p, have * 8, hipMemcpyDeviceToDevice));
        dst.alloc(0, "free");
        dst.p = grown.release();
        cap = nc;
    }
    if (d) HIP_TRY(hipMemcpy(dst.as<uint64_t>() + have, src, d * 8, hipMemcpyDeviceToDevice));
    return 0;
}

// Sorted (key, position) pairs of the suffixes in bins [lo, hi) -> SA slots
// off0.. of sa5; entries whose 32-char key repeats go to `ties`.
// rank5 (optional): also write the 40-bit group id of every suffix (the whole-SA
// builder's doubling rounds read it); nbuckets (optional): buckets sorted.
static int sort_bins_into(const uint64_t* tw, uint64_t n, const std::vector<uint64_t>& h, uint32_t lo, uint32_t hi,
                          uint64_t cap, uint8_t* sa5, uint64_t off0, TiedSink& ties, uint8_t* rank5 = nullptr,
                          uint64_t* nbuckets = nullptr) {
    hipStream_t st = 0;
    uint64_t bucket_max = 0, acc = 0;
    std::vector<uint32_t> edges{lo};
    for (uint32_t b = lo; b < hi; b++) {
        if (acc + h[b] > cap && acc) {
            edges.push_back(b);
            bucket_max = acc > bucket_max ? acc : bucket_max;
            acc = 0;
        }
        acc += h[b];
    }
    edges.push_back(hi);
    bucket_max = acc > bucket_max ? acc : bucket_max;
    if (nbuckets) *nbuckets = edges.size() - 1;
    if (bucket_max == 0) return 0;
    DevBuf ka, kb, va, vb, grp, flg, bcnt, cnt_d, tmp;
    size_t tmp_have = 0;
    TRY(ka.alloc(bucket_max * 8, "bucket keys"));
    TRY(kb.alloc(bucket_max * 8, "bucket keys alt"));
    TRY(va.alloc(bucket_max * 8, "bucket positions"));
    TRY(vb.alloc(bucket_max * 8, "bucket positions alt"));
    TRY(grp.alloc(bucket_max * 8, "bucket groups"));
    TRY(flg.alloc(bucket_max, "bucket tied flags"));
    const uint64_t nblk = (n + COLLECT_CHUNK - 1) / COLLECT_CHUNK;
    TRY(bcnt.alloc(nblk * 8, "block counts"));
    TRY(cnt_d.alloc(16, "counter"));
    uint64_t off = off0;
    for (size_t b = 0; b + 1 < edges.size(); b++) {
        uint32_t blo = edges[b], bhi = edges[b + 1];
        uint64_t c = 0;
        for (uint32_t i = blo; i < bhi; i++) c += h[i];
        if (c == 0) continue;
        const dim3 cg(collect_grid(nblk));
        hipLaunchKernelGGL(k_bucket_count, cg, dim3(COLLECT_BLOCK), 0, st, tw, n, blo, bhi,
                           bcnt.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::exclusive_scan(t, sz, bcnt.as<uint64_t>(), bcnt.as<uint64_t>(), (uint64_t)0,
                                           (size_t)nblk, rocprim::plus<uint64_t>(), st);
        }));
        hipLaunchKernelGGL(k_bucket_collect, cg, dim3(COLLECT_BLOCK), 0, st, tw, n, blo, bhi,
                           bcnt.as<uint64_t>(), ka.as<uint64_t>(), va.as<uint64_t>());
        rocprim::double_buffer<uint64_t> kdb(ka.as<uint64_t>(), kb.as<uint64_t>());
        rocprim::double_buffer<uint64_t> vdb(va.as<uint64_t>(), vb.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::radix_sort_pairs(t, sz, kdb, vdb, (size_t)c, 0, 64, st);
        }));
        const uint64_t* sk = kdb.current();
        const uint64_t* sv = vdb.current();
        uint64_t* free_k = (sk == ka.as<uint64_t>()) ? kb.as<uint64_t>() : ka.as<uint64_t>();
        uint64_t* free_v = (sv == va.as<uint64_t>()) ? vb.as<uint64_t>() : va.as<uint64_t>();
        hipLaunchKernelGGL(k_b_heads, dim3(grid_for(c)), dim3(256), 0, st, sk, c, off, grp.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::inclusive_scan(t, sz, grp.as<uint64_t>(), grp.as<uint64_t>(), (size_t)c, MaxOp64(), st);
        }));
        hipLaunchKernelGGL(k_b_emit, dim3(grid_for(c)), dim3(256), 0, st, sk, sv, grp.as<uint64_t>(), c, off, sa5,
                           rank5, flg.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        rocprim::counting_iterator<uint64_t> cit(off);
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::select(t, sz, cit, flg.as<uint8_t>(), free_k, cnt_d.as<uint64_t>(), (size_t)c, st);
        }));
        uint64_t d = 0;
        HIP_TRY(hipMemcpy(&d, cnt_d.p, 8, hipMemcpyDeviceToHost));
        if (d) {
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::select(t, sz, grp.as<uint64_t>(), flg.as<uint8_t>(), free_v, cnt_d.as<uint64_t>(),
                                       (size_t)c, st);
            }));
            uint64_t cap_l = ties.cap, cap_g = ties.cap;
            TRY(append_dev(ties.list, cap_l, ties.cnt, free_k, d, "tied list"));
            TRY(append_dev(ties.grp, cap_g, ties.cnt, free_v, d, "tied groups"));
            ties.cap = cap_l;
            ties.cnt += d;
        }
        off += c;
    }
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int build_sa_gpu40(const uint64_t* tw, uint64_t n, uint8_t* sa5, uint32_t* rounds_out, uint64_t* buckets_out) {
    hipStream_t st = 0;
    DevBuf tmp;
    size_t tmp_have = 0;

    // 1) histogram of the first 7 chars
    std::vector<uint64_t> h;
    TRY(histogram(tw, n, h));

    // rank array, then size the buckets from what HBM has left
    DevBuf rank;
    TRY(rank.alloc(5 * n + SAS_SA40_PAD, "rank (40-bit)"));
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    uint64_t cap = (uint64_t)(free_b * 0.55) / 42;  // keys x2, vals x2, group, flags, sort temp
    if (cap > n) cap = n;
    if (cap > (1ull << 31)) cap = 1ull << 31;       // one radix sort stays below 2^31 pairs
    uint64_t maxbin = 0;
    for (uint64_t c : h) maxbin = c > maxbin ? c : maxbin;
    if (maxbin > cap)
        SAS_FAIL(ENOTSUP, "sas_build (40-bit): " + std::to_string(maxbin) +
                              " suffixes share one 7-char prefix, more than one bucket (" + std::to_string(cap) +
                              ") fits in free HBM");
    if (cap < maxbin) cap = maxbin;

    // 2) buckets in key order: SA, 40-bit group ids, tied ranks
    TiedSink ties;
    TRY(sort_bins_into(tw, n, h, 0, HIST_BINS, cap, sa5, 0, ties, rank.as<uint8_t>(), buckets_out));
    DevBuf& list = ties.list;
    DevBuf list_alt, cnt_d;
    TRY(cnt_d.alloc(16, "counter"));
    const uint64_t tied = ties.cnt;

    // 3) doubling rounds over the tied ranks
    uint32_t rounds = 0;
    uint64_t cnt = tied;
    if (cnt) {
        DevBuf rk, rk2, rv, rv2, hp, hd, uf;
        TRY(list_alt.alloc(cnt * 8, "tied list alt"));
        TRY(rk.alloc(cnt * 8, "round keys"));
        TRY(rk2.alloc(cnt * 8, "round keys alt"));
        TRY(rv.alloc(cnt * 8, "round positions"));
        TRY(rv2.alloc(cnt * 8, "round positions alt"));
        TRY(hp.alloc(cnt * 8, "round groups"));
        TRY(hd.alloc(cnt, "round heads"));
        TRY(uf.alloc(cnt, "round flags"));
        uint64_t* L = list.as<uint64_t>();
        uint64_t* Ln = list_alt.as<uint64_t>();
        SaView<5> sav{sa5}, rkv{rank.as<uint8_t>()};
        for (uint64_t hh = 32; cnt > 0; hh *= 2) {
            if (hh >= 2 * n + 64) SAS_FAIL(EIO, "sa construction (40-bit) did not converge");
            rounds++;
            hipLaunchKernelGGL(k_r40_second, dim3(grid_for(cnt)), dim3(256), 0, st, L, cnt, sav, rkv, n, hh,
                               rk.as<uint64_t>(), rv.as<uint64_t>());
            rocprim::double_buffer<uint64_t> k2(rk.as<uint64_t>(), rk2.as<uint64_t>());
            rocprim::double_buffer<uint64_t> v2(rv.as<uint64_t>(), rv2.as<uint64_t>());
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::radix_sort_pairs(t, sz, k2, v2, (size_t)cnt, 0, 41, st);
            }));
            hipLaunchKernelGGL(k_r40_group, dim3(grid_for(cnt)), dim3(256), 0, st, v2.current(), cnt, rkv,
                               k2.current());
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::radix_sort_pairs(t, sz, k2, v2, (size_t)cnt, 0, 40, st);
            }));
            const uint64_t* sv = v2.current();
            hipLaunchKernelGGL(k_r40_heads, dim3(grid_for(cnt)), dim3(256), 0, st, sv, cnt, rkv, n, hh, L,
                               hp.as<uint64_t>(), hd.as<uint8_t>());
            hipLaunchKernelGGL(k_r40_scatter, dim3(grid_for(cnt)), dim3(256), 0, st, L, cnt, sv, sa5);
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::inclusive_scan(t, sz, hp.as<uint64_t>(), hp.as<uint64_t>(), (size_t)cnt, MaxOp64(),
                                               st);
            }));
            hipLaunchKernelGGL(k_r40_assign, dim3(grid_for(cnt)), dim3(256), 0, st, cnt, sv, hp.as<uint64_t>(),
                               hd.as<uint8_t>(), rank.as<uint8_t>(), uf.as<uint8_t>());
            HIP_TRY(hipGetLastError());
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::select(t, sz, L, uf.as<uint8_t>(), Ln, cnt_d.as<uint64_t>(), (size_t)cnt, st);
            }));
            HIP_TRY(hipMemcpy(&cnt, cnt_d.p, 8, hipMemcpyDeviceToHost));
            uint64_t* t = L; L = Ln; Ln = t;
        }
    }
    HIP_TRY(hipStreamSynchronize(st));
    *rounds_out = rounds;
    return 0;
}

// ======================================================================
// Part builder (sharded text): part g of P builds ONLY its own SA
// rank range.  Every part computes the same histogram from the full text and
// takes the contiguous bins [B_g, B_{g+1}) whose cumulative counts straddle
// g*n/P, so its suffixes are exactly the global ranks [cum(B_g), cum(B_{g+1})).
// Suffixes that tie on their 32-char key share a bin, hence a part, so ties are
// resolved locally, by text windows instead of the global rank array: round w
// stably sorts each tied group by the next 32 chars (zero padded) and then by
// how many of them exist (a proper prefix sorts first, Rust slice order).
// Rounds = longest tied prefix / 32, capped (ENOTSUP past the cap: such a text
// needs the whole-SA builder, sas_build_shard).
// ======================================================================
#define PART_MAX_ROUNDS (1u << 16)

// Window of the tied element k at offset o: key = chars [p+o, p+o+32) (zero
// padded), len = min(n - p, o + 32).  Group members agree on their first o chars
// (zero padded), so ordering by (key, len) is slice order: equal keys with a
// shorter length mean a proper prefix (the padding zeros stand for real zeros in
// the longer suffix); equal keys and len = o + 32 stay tied for the next window.
__global__ void k_w_keys(const uint64_t* __restrict__ list, uint64_t cnt, SaView<5> sa, const uint64_t* tw,
                         uint64_t n, uint64_t o, uint64_t* __restrict__ pos, uint64_t* __restrict__ key,
                         uint64_t* __restrict__ lc, uint64_t* __restrict__ perm) {
    GRID_STRIDE(k, cnt) {
        uint64_t p = sa[list[k]];
        pos[k] = p;
        key[k] = (p + o < n) ? text_chars32(tw, p + o) : 0ull;
        const uint64_t len = n - p;
        lc[k] = len < o + 32 ? len : o + 32;
        perm[k] = k;
    }
}

__global__ void k_gather64(const uint64_t* __restrict__ src, const uint64_t* __restrict__ perm, uint64_t cnt,
                           uint64_t* __restrict__ dst) {
    GRID_STRIDE(k, cnt) dst[k] = src[perm[k]];
}

__global__ void k_w_heads(const uint64_t* __restrict__ perm, uint64_t cnt, const uint64_t* __restrict__ grp,
                          const uint64_t* __restrict__ key, const uint64_t* __restrict__ lc,
                          const uint64_t* __restrict__ list, uint64_t* __restrict__ headpos,
                          uint8_t* __restrict__ head) {
    GRID_STRIDE(k, cnt) {
        bool hd = true;
        if (k > 0) {
            uint64_t a = perm[k], b = perm[k - 1];
            hd = grp[a] != grp[b] || key[a] != key[b] || lc[a] != lc[b];
        }
        head[k] = hd;
        headpos[k] = hd ? list[k] : 0ull;
    }
}

__global__ void k_w_scatter(const uint64_t* __restrict__ list, const uint64_t* __restrict__ perm,
                            const uint64_t* __restrict__ pos, uint64_t cnt, const uint8_t* __restrict__ head,
                            uint8_t* __restrict__ sa5, uint8_t* __restrict__ unresolved) {
    GRID_STRIDE(k, cnt) {
        sa_put<5>(sa5, list[k], pos[perm[k]]);
        bool h1 = (k + 1 == cnt) || head[k + 1];
        unresolved[k] = !(head[k] && h1);
    }
}

// Resolve tied groups in place.  list: ascending SA slots of the tied entries,
// grp: their group ids (slot of the group's first entry), both device, cnt entries;
// sa5: the (local) SA whose slots they index.  Consumes list / grp.
static int resolve_ties_windows(const uint64_t* tw, uint64_t n, uint8_t* sa5, DevBuf& list, DevBuf& grp, uint64_t cnt,
                                uint32_t* rounds_out) {
    hipStream_t st = 0;
    uint32_t rounds = 0;
    if (cnt == 0) {
        *rounds_out = 0;
        return 0;
    }
    DevBuf pos, key, lc, perm, perm2, kbuf, kbuf2, hp, hd, uf, list2, grp2, tmp, cnt_d;
    TRY(pos.alloc(cnt * 8, "tie positions"));
    TRY(key.alloc(cnt * 8, "tie window keys"));
    TRY(lc.alloc(cnt * 8, "tie window lengths"));
    TRY(perm.alloc(cnt * 8, "tie order"));
    TRY(perm2.alloc(cnt * 8, "tie order alt"));
    TRY(kbuf.alloc(cnt * 8, "tie sort keys"));
    TRY(kbuf2.alloc(cnt * 8, "tie sort keys alt"));
    TRY(hp.alloc(cnt * 8, "tie groups"));
    TRY(hd.alloc(cnt, "tie heads"));
    TRY(uf.alloc(cnt, "tie flags"));
    TRY(list2.alloc(cnt * 8, "tie list alt"));
    TRY(grp2.alloc(cnt * 8, "tie group alt"));
    TRY(cnt_d.alloc(16, "counter"));
    size_t tmp_have = 0;
    SaView<5> sav{sa5};
    uint64_t* L = list.as<uint64_t>();
    uint64_t* G = grp.as<uint64_t>();
    uint64_t* Ln = list2.as<uint64_t>();
    uint64_t* Gn = grp2.as<uint64_t>();
    for (uint64_t o = 32; cnt > 0; o += 32) {
        if (++rounds > PART_MAX_ROUNDS)
            SAS_FAIL(ENOTSUP, "sas_build_part: suffixes share prefixes longer than " +
                                  std::to_string(32ull * PART_MAX_ROUNDS) + " chars; use sas_build_shard");
        hipLaunchKernelGGL(k_w_keys, dim3(grid_for(cnt)), dim3(256), 0, st, L, cnt, sav, tw, n, o, pos.as<uint64_t>(),
                           key.as<uint64_t>(), lc.as<uint64_t>(), perm.as<uint64_t>());
        // stable LSD: window length, then window key, then group (outermost)
        const uint64_t* srcs[3] = {lc.as<uint64_t>(), key.as<uint64_t>(), G};
        const int bits[3] = {41, 64, 40};
        uint64_t* pa = perm.as<uint64_t>();
        uint64_t* pb = perm2.as<uint64_t>();
        for (int pass = 0; pass < 3; pass++) {
            hipLaunchKernelGGL(k_gather64, dim3(grid_for(cnt)), dim3(256), 0, st, srcs[pass], pa, cnt,
                               kbuf.as<uint64_t>());
            rocprim::double_buffer<uint64_t> kd(kbuf.as<uint64_t>(), kbuf2.as<uint64_t>());
            rocprim::double_buffer<uint64_t> vd(pa, pb);
            const int nb = bits[pass];
            TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
                return rocprim::radix_sort_pairs(t, sz, kd, vd, (size_t)cnt, 0, nb, st);
            }));
            if (vd.current() != pa) { uint64_t* t = pa; pa = pb; pb = t; }
        }
        hipLaunchKernelGGL(k_w_heads, dim3(grid_for(cnt)), dim3(256), 0, st, pa, cnt, G, key.as<uint64_t>(),
                           lc.as<uint64_t>(), L, hp.as<uint64_t>(), hd.as<uint8_t>());
        hipLaunchKernelGGL(k_w_scatter, dim3(grid_for(cnt)), dim3(256), 0, st, L, pa, pos.as<uint64_t>(), cnt,
                           hd.as<uint8_t>(), sa5, uf.as<uint8_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::inclusive_scan(t, sz, hp.as<uint64_t>(), hp.as<uint64_t>(), (size_t)cnt, MaxOp64(), st);
        }));
        HIP_TRY(hipGetLastError());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::select(t, sz, hp.as<uint64_t>(), uf.as<uint8_t>(), Gn, cnt_d.as<uint64_t>(), (size_t)cnt, st);
        }));
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::select(t, sz, L, uf.as<uint8_t>(), Ln, cnt_d.as<uint64_t>(), (size_t)cnt, st);
        }));
        HIP_TRY(hipMemcpy(&cnt, cnt_d.p, 8, hipMemcpyDeviceToHost));
        uint64_t* t1 = L; L = Ln; Ln = t1;
        uint64_t* t2 = G; G = Gn; Gn = t2;
    }
    HIP_TRY(hipStreamSynchronize(st));
    *rounds_out = rounds;
    return 0;
}

// The smallest suffix among those whose bin is >= b_from (the first suffix of the
// next part): its bin is the first non-empty one; sort that bin and resolve the
// ties of its first key group.
static int min_suffix_from(const uint64_t* tw, uint64_t n, const std::vector<uint64_t>& h, uint32_t b_from,
                           uint64_t cap, uint64_t* out) {
    uint32_t b = b_from;
    while (b < HIST_BINS && h[b] == 0) b++;
    if (b >= HIST_BINS) {
        *out = n;
        return 0;
    }
    const uint64_t c = h[b];
    DevBuf sa;
    TRY(sa.alloc(c * 5 + SAS_SA40_PAD, "next-part bin SA"));
    HIP_TRY(hipMemset(sa.p, 0, c * 5 + SAS_SA40_PAD));
    TiedSink ties;
    TRY(sort_bins_into(tw, n, h, b, b + 1, cap, sa.as<uint8_t>(), 0, ties));
    uint32_t r = 0;
    TRY(resolve_ties_windows(tw, n, sa.as<uint8_t>(), ties.list, ties.grp, ties.cnt, &r));
    uint8_t bytes[8] = {};
    HIP_TRY(hipMemcpy(bytes, sa.p, 5, hipMemcpyDeviceToHost));
    uint64_t v = 0;
    for (int k = 0; k < 5; k++) v |= (uint64_t)bytes[k] << (8 * k);
    *out = v;
    return 0;
}

int build_sa_part40(const uint64_t* tw, uint64_t n, uint32_t part, uint32_t parts, uint8_t** sa5_out,
                    uint64_t* rank_lo, uint64_t* count, uint64_t* next_pos, uint32_t* rounds_out) {
    std::vector<uint64_t> h;
    TRY(histogram(tw, n, h));
    // part boundaries: B_g = first bin whose preceding count reaches g*n/P
    std::vector<uint64_t> cum(HIST_BINS + 1, 0);
    for (uint32_t b = 0; b < HIST_BINS; b++) cum[b + 1] = cum[b] + h[b];
    auto bound = [&](uint32_t g) -> uint32_t {
        if (g == 0) return 0;
        if (g >= parts) return HIST_BINS;
        const uint64_t target = (uint64_t)(((unsigned __int128)n * g) / parts);
        uint32_t b = 0;
        while (b < HIST_BINS && cum[b] < target) b++;
        return b;
    };
    const uint32_t lo = bound(part), hi = bound(part + 1);
    *rank_lo = cum[lo];
    *count = cum[hi] - cum[lo];
    if (*count == 0)
        SAS_FAIL(EINVAL, "sas_build_part: part " + std::to_string(part) + " of " + std::to_string(parts) +
                             " holds no suffixes (too many parts for this text)");
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    uint64_t cap = (uint64_t)(free_b * 0.45) / 42;
    uint64_t maxbin = 0;
    for (uint32_t b = lo; b < hi; b++) maxbin = h[b] > maxbin ? h[b] : maxbin;
    if (cap > (1ull << 31)) cap = 1ull << 31;
    if (maxbin > cap)
        SAS_FAIL(ENOTSUP, "sas_build_part: " + std::to_string(maxbin) + " suffixes share one 7-char prefix");
    if (cap < maxbin) cap = maxbin;
    DevBuf sa;
    TRY(sa.alloc(*count * 5 + SAS_SA40_PAD, "suffix array part"));
    HIP_TRY(hipMemset(sa.p, 0, *count * 5 + SAS_SA40_PAD));
    TiedSink ties;
    TRY(sort_bins_into(tw, n, h, lo, hi, cap, sa.as<uint8_t>(), 0, ties));
    TRY(resolve_ties_windows(tw, n, sa.as<uint8_t>(), ties.list, ties.grp, ties.cnt, rounds_out));
    TRY(min_suffix_from(tw, n, h, hi, cap, next_pos));
    *sa5_out = static_cast<uint8_t*>(sa.release());
    return 0;
}
