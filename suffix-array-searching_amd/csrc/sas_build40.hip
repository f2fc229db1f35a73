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

// Block b owns positions [b*CHUNK, (b+1)*CHUNK): count those whose bin is in [lo, hi).
__global__ __launch_bounds__(COLLECT_BLOCK) void k_bucket_count(const uint64_t* __restrict__ tw, uint64_t n,
                                                                uint32_t lo, uint32_t hi,
                                                                uint64_t* __restrict__ block_cnt) {
    __shared__ uint32_t s_w[COLLECT_BLOCK / 64];
    uint64_t base = (uint64_t)blockIdx.x * COLLECT_CHUNK;
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
    if (threadIdx.x == 0) block_cnt[blockIdx.x] = t;
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
    uint64_t run = block_off[blockIdx.x];
    uint64_t base = (uint64_t)blockIdx.x * COLLECT_CHUNK;
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
        sa_put<5>(rank5, p, group[j]);
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

int build_sa_gpu40(const uint64_t* tw, uint64_t n, uint8_t* sa5, uint32_t* rounds_out, uint64_t* buckets_out) {
    hipStream_t st = 0;
    DevBuf tmp;
    size_t tmp_have = 0;

    // 1) histogram of the first 7 chars
    DevBuf hist;
    TRY(hist.alloc(HIST_BINS * 8, "histogram"));
    HIP_TRY(hipMemsetAsync(hist.p, 0, HIST_BINS * 8, st));
    hipLaunchKernelGGL(k_hist, dim3(grid_for(n, 1024) < 1024 ? grid_for(n, 1024) : 1024), dim3(1024), 0, st, tw, n,
                       hist.as<unsigned long long>());
    HIP_TRY(hipGetLastError());
    std::vector<uint64_t> h(HIST_BINS);
    HIP_TRY(hipMemcpy(h.data(), hist.p, HIST_BINS * 8, hipMemcpyDeviceToHost));

    // rank array, then size the buckets from what HBM has left
    DevBuf rank;
    TRY(rank.alloc(5 * n + SAS_SA40_PAD, "rank (40-bit)"));
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    uint64_t cap = (uint64_t)(free_b * 0.55) / 42;  // keys x2, vals x2, group, flags, sort temp
    if (cap > n) cap = n;
    uint64_t maxbin = 0;
    for (uint64_t c : h) maxbin = c > maxbin ? c : maxbin;
    if (maxbin > cap)
        SAS_FAIL(ENOTSUP, "sas_build (40-bit): " + std::to_string(maxbin) +
                              " suffixes share one 7-char prefix, more than one bucket (" + std::to_string(cap) +
                              ") fits in free HBM");
    if (cap < maxbin) cap = maxbin;
    std::vector<uint32_t> edges{0};  // bucket b = bins [edges[b], edges[b+1])
    uint64_t acc = 0, bucket_max = 0;
    for (uint32_t b = 0; b < HIST_BINS; b++) {
        if (acc + h[b] > cap) {
            edges.push_back(b);
            bucket_max = acc > bucket_max ? acc : bucket_max;
            acc = 0;
        }
        acc += h[b];
    }
    edges.push_back(HIST_BINS);
    bucket_max = acc > bucket_max ? acc : bucket_max;
    *buckets_out = edges.size() - 1;

    DevBuf ka, kb, va, vb, grp, flg, bcnt, cnt_d, list, list_alt;
    TRY(ka.alloc(bucket_max * 8, "bucket keys"));
    TRY(kb.alloc(bucket_max * 8, "bucket keys alt"));
    TRY(va.alloc(bucket_max * 8, "bucket positions"));
    TRY(vb.alloc(bucket_max * 8, "bucket positions alt"));
    TRY(grp.alloc(bucket_max * 8, "bucket groups"));
    TRY(flg.alloc(bucket_max, "bucket tied flags"));
    const uint64_t nblk = (n + COLLECT_CHUNK - 1) / COLLECT_CHUNK;
    TRY(bcnt.alloc(nblk * 8, "block counts"));
    TRY(cnt_d.alloc(16, "counter"));
    uint64_t list_cap = 1 << 20, tied = 0;
    TRY(list.alloc(list_cap * 8, "tied list"));

    // 2) buckets in key order
    uint64_t off = 0;
    for (size_t b = 0; b + 1 < edges.size(); b++) {
        uint32_t lo = edges[b], hi = edges[b + 1];
        uint64_t c = 0;
        for (uint32_t i = lo; i < hi; i++) c += h[i];
        if (c == 0) continue;
        hipLaunchKernelGGL(k_bucket_count, dim3((unsigned)nblk), dim3(COLLECT_BLOCK), 0, st, tw, n, lo, hi,
                           bcnt.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::exclusive_scan(t, sz, bcnt.as<uint64_t>(), bcnt.as<uint64_t>(), (uint64_t)0,
                                           (size_t)nblk, rocprim::plus<uint64_t>(), st);
        }));
        hipLaunchKernelGGL(k_bucket_collect, dim3((unsigned)nblk), dim3(COLLECT_BLOCK), 0, st, tw, n, lo, hi,
                           bcnt.as<uint64_t>(), ka.as<uint64_t>(), va.as<uint64_t>());
        HIP_TRY(hipGetLastError());
        rocprim::double_buffer<uint64_t> kdb(ka.as<uint64_t>(), kb.as<uint64_t>());
        rocprim::double_buffer<uint64_t> vdb(va.as<uint64_t>(), vb.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::radix_sort_pairs(t, sz, kdb, vdb, (size_t)c, 0, 64, st);
        }));
        const uint64_t* sk = kdb.current();
        const uint64_t* sv = vdb.current();
        uint64_t* free_k = (sk == ka.as<uint64_t>()) ? kb.as<uint64_t>() : ka.as<uint64_t>();
        hipLaunchKernelGGL(k_b_heads, dim3(grid_for(c)), dim3(256), 0, st, sk, c, off, grp.as<uint64_t>());
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::inclusive_scan(t, sz, grp.as<uint64_t>(), grp.as<uint64_t>(), (size_t)c, MaxOp64(), st);
        }));
        hipLaunchKernelGGL(k_b_emit, dim3(grid_for(c)), dim3(256), 0, st, sk, sv, grp.as<uint64_t>(), c, off, sa5,
                           rank.as<uint8_t>(), flg.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        rocprim::counting_iterator<uint64_t> cit(off);
        TRY(with_temp(tmp, tmp_have, [&](void* t, size_t& sz) {
            return rocprim::select(t, sz, cit, flg.as<uint8_t>(), free_k, cnt_d.as<uint64_t>(), (size_t)c, st);
        }));
        uint64_t d = 0;
        HIP_TRY(hipMemcpy(&d, cnt_d.p, 8, hipMemcpyDeviceToHost));
        if (d) {
            if (tied + d > list_cap) {
                uint64_t nc = list_cap;
                while (nc < tied + d) nc *= 2;
                DevBuf grown;
                TRY(grown.alloc(nc * 8, "tied list"));
                HIP_TRY(hipMemcpyAsync(grown.p, list.p, tied * 8, hipMemcpyDeviceToDevice, st));
                list.alloc(0, "free");
                list.p = grown.release();
                list_cap = nc;
            }
            HIP_TRY(hipMemcpyAsync(list.as<uint64_t>() + tied, free_k, d * 8, hipMemcpyDeviceToDevice, st));
            tied += d;
        }
        off += c;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (off != n) SAS_FAIL(EIO, "sas_build (40-bit): buckets cover " + std::to_string(off) + " of n suffixes");
    ka.alloc(0, "free"); kb.alloc(0, "free"); va.alloc(0, "free"); vb.alloc(0, "free");
    grp.alloc(0, "free"); flg.alloc(0, "free"); bcnt.alloc(0, "free");

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
