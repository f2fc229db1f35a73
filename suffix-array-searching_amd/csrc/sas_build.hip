// sas_build.hip -- index construction for the MI355X suffix-array engine.
//
// Replaces SaNaive::build (sas/sa_search.rs:30-57): the reference calls
// libsais (sais64::parallel::sais, :33), casts to u32 (:35), asserts adjacent
// suffixes increase (:36-38) and fills a (dead, p = 0) prefix table (:59-74).
// Here everything is built on the GPU into HBM:
//   1. pack the byte-coded text to 2 bits/char (rejects codes > 3),
//   2. suffix array by prefix doubling: one rocPRIM radix sort of
//      (32-char packed key, position) pairs, then doubling rounds over the
//      still-tied groups only (h = 32, 64, ...),
//   3. optional LCP array (direct parallel word compares),
//   4. optional S-tree over 16-char keys (STree<16,16> layout of
//      sst/s_tree.rs:72-176, unsigned keys, MAX padding),
//   5. the LDS "top" of the lockstep binary search (Eytzinger order).
#include "common.hpp"
#include "build_util.hpp"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

// ------------------------------------------------------------------ error state
static thread_local std::string g_err = "ok";

void sas_set_error(int code, const std::string& msg) {
    g_err = "[" + std::to_string(code) + "] " + msg;
}
int sas_errno_of(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return ENOMEM;
    if (e == hipErrorInvalidValue) return EINVAL;
    return EIO;
}
extern "C" const char* sas_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------ text packing
__global__ void k_pack_text(const uint8_t* __restrict__ text, uint64_t n, uint64_t* __restrict__ tw,
                            uint64_t words, uint32_t* __restrict__ bad) {
    uint32_t b = 0;
    GRID_STRIDE(w, words) {
        uint64_t base = w * 32;
        uint64_t v = 0;
        if (base < n) {
            uint32_t m = n - base < 32 ? (uint32_t)(n - base) : 32;
            v = pack_query_word(text + base, m, 0, &b);
        }
        tw[w] = v;
    }
    if (b) atomicOr(bad, 1u);
}

// ------------------------------------------------------------------ ChaCha8 text generator
// random_string (sas/util.rs:9-15) with ChaCha8Rng::seed_from_u64 (sas/main.rs:38):
// char i = keystream word i >> 30 (rand 0.8.5 UniformInt<u8>, range 4, no rejection).
__device__ __forceinline__ uint32_t rotl32d(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define DQR(a, b, c, d)                    \
    a += b; d ^= a; d = rotl32d(d, 16);   \
    c += d; b ^= c; b = rotl32d(b, 12);   \
    a += b; d ^= a; d = rotl32d(d, 8);    \
    c += d; b ^= c; b = rotl32d(b, 7);

struct ChaKey { uint32_t k[8]; };

// keystream block `blk`: x[i] = the state after the 8 rounds, s[i] = the input state (the
// output word is x[i] + s[i])
__device__ __forceinline__ void chacha8_block(const ChaKey& key, uint64_t blk, uint32_t (&s)[16], uint32_t (&x)[16]) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                             key.k[0], key.k[1], key.k[2], key.k[3], key.k[4], key.k[5], key.k[6], key.k[7],
                             (uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = x[i] = in[i];
#pragma unroll
    for (int r = 0; r < 8; r += 2) {
        DQR(x[0], x[4], x[8], x[12]) DQR(x[1], x[5], x[9], x[13])
        DQR(x[2], x[6], x[10], x[14]) DQR(x[3], x[7], x[11], x[15])
        DQR(x[0], x[5], x[10], x[15]) DQR(x[1], x[6], x[11], x[12])
        DQR(x[2], x[7], x[8], x[13]) DQR(x[3], x[4], x[9], x[14])
    }
}

__global__ void k_gen_text(ChaKey key, uint64_t n, uint8_t* __restrict__ out) {
    uint64_t blocks = (n + 15) / 16;
    GRID_STRIDE(blk, blocks) {
        uint32_t s[16], x[16];
        chacha8_block(key, blk, s, x);
        uint64_t base = blk * 16;
        if (base + 16 <= n && (((uintptr_t)(out + base)) & 15) == 0) {
            uint32_t wv[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t v = 0;
#pragma unroll
                for (int i = 0; i < 4; i++) v |= ((x[4 * q + i] + s[4 * q + i]) >> 30) << (8 * i);
                wv[q] = v;
            }
            *reinterpret_cast<uint4*>(out + base) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        } else {
            for (int i = 0; i < 16 && base + i < n; i++) out[base + i] = (uint8_t)((x[i] + s[i]) >> 30);
        }
    }
}

// Host ChaCha8Rng (rand_chacha 0.3.1) + rand_core 0.6 seed_from_u64 (PCG32 expansion).
static void h_seed_from_u64(uint64_t state, uint32_t key[8]) {
    const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
    for (int i = 0; i < 8; i++) {
        state = state * MUL + INC;
        uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
    }
}
static inline uint32_t h_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define HQR(a, b, c, d)                  \
    a += b; d ^= a; d = h_rotl(d, 16);  \
    c += d; b ^= c; b = h_rotl(b, 12);  \
    a += b; d ^= a; d = h_rotl(d, 8);   \
    c += d; b ^= c; b = h_rotl(b, 7);

struct HostRng {
    uint32_t key[8];
    uint64_t blk = UINT64_MAX, pos = 0;
    uint32_t buf[16];
    uint32_t word(uint64_t w) {
        uint64_t b = w >> 4;
        if (b != blk) {
            uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                              key[4], key[5], key[6], key[7], (uint32_t)b, (uint32_t)(b >> 32), 0, 0};
            uint32_t x[16];
            memcpy(x, s, sizeof x);
            for (int r = 0; r < 8; r += 2) {
                HQR(x[0], x[4], x[8], x[12]) HQR(x[1], x[5], x[9], x[13])
                HQR(x[2], x[6], x[10], x[14]) HQR(x[3], x[7], x[11], x[15])
                HQR(x[0], x[5], x[10], x[15]) HQR(x[1], x[6], x[11], x[12])
                HQR(x[2], x[7], x[8], x[13]) HQR(x[3], x[4], x[9], x[14])
            }
            for (int i = 0; i < 16; i++) buf[i] = x[i] + s[i];
            blk = b;
        }
        return buf[w & 15];
    }
    uint64_t next_u64() {  // BlockRng::next_u64: two consecutive words, low first
        uint64_t lo = word(pos), hi = word(pos + 1);
        pos += 2;
        return lo | (hi << 32);
    }
    uint64_t range(uint64_t low, uint64_t high) {  // rand 0.8.5 UniformInt<usize>::sample_single
        uint64_t r = high - low;
        uint64_t zone = (r << __builtin_clzll(r)) - 1;
        for (;;) {
            unsigned __int128 p = (unsigned __int128)next_u64() * r;
            if ((uint64_t)p <= zone) return low + (uint64_t)(p >> 64);
        }
    }
};

extern "C" int sas_gen_text(uint64_t seed, uint64_t n, uint8_t* out, uint32_t flags) {
    if (!out && n) SAS_FAIL(EINVAL, "sas_gen_text: null output");
    if (n == 0) return 0;
    ChaKey key;
    h_seed_from_u64(seed, key.k);
    uint8_t* d = out;
    if (!(flags & SAS_DEVICE_PTRS)) HIP_TRY(hipMalloc(&d, n));
    hipLaunchKernelGGL(k_gen_text, dim3(grid_for((n + 15) / 16)), dim3(256), 0, 0, key, n, d);
    HIP_TRY(hipGetLastError());
    if (!(flags & SAS_DEVICE_PTRS)) {
        HIP_TRY(hipMemcpy(out, d, n, hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(d));
    } else {
        HIP_TRY(hipDeviceSynchronize());
    }
    return 0;
}

extern "C" int sas_gen_queries(uint64_t seed, uint64_t word_pos, uint64_t n, uint64_t nq, uint64_t margin,
                               uint32_t len_lo, uint32_t len_hi, uint64_t* off, uint32_t* len,
                               uint64_t* next_word) {
    if (margin >= n) SAS_FAIL(EINVAL, "sas_gen_queries: margin >= n (gen_range(0..n-margin) is empty)");
    if (len_hi <= len_lo) SAS_FAIL(EINVAL, "sas_gen_queries: empty length range");
    if (nq && (!off || !len)) SAS_FAIL(EINVAL, "sas_gen_queries: null output");
    HostRng r;
    h_seed_from_u64(seed, r.key);
    r.pos = word_pos;
    for (uint64_t k = 0; k < nq; k++) {  // sas/util.rs:20-24
        off[k] = r.range(0, n - margin);
        len[k] = (len_hi == len_lo + 1) ? len_lo : (uint32_t)r.range(len_lo, len_hi);
    }
    if (next_word) *next_word = r.pos;
    return 0;
}

// random_string straight into the index's packed layout (sas_build_gen): text word w holds
// chars [32w, 32w + 32), i.e. keystream blocks 2w and 2w + 1, first char in bits 63..62,
// zero past n (the words k_pack_text would make of k_gen_text's bytes), so a sharded
// rank never holds the n-byte text.
__global__ void k_gen_packed(ChaKey key, uint64_t n, uint64_t* __restrict__ tw, uint64_t words) {
    GRID_STRIDE(w, words) {
        uint64_t v = 0;
        const uint64_t base = w * 32;
        if (base < n) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint32_t s[16], x[16];
                chacha8_block(key, 2 * w + h, s, x);
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const uint32_t c = 16 * h + i;
                    if (base + c < n) v |= (uint64_t)((x[i] + s[i]) >> 30) << (62 - 2 * c);
                }
            }
        }
        tw[w] = v;
    }
}

// ------------------------------------------------------------------ SA construction
__global__ void k_init_pairs(const uint64_t* __restrict__ tw, uint64_t n, uint64_t* __restrict__ keys,
                             uint32_t* __restrict__ vals) {
    GRID_STRIDE(i, n) {
        keys[i] = text_chars32(tw, i);
        vals[i] = (uint32_t)i;
    }
}

// headpos[k] = k if element k starts a new key group (else 0); group id = max-scan.
__global__ void k_heads(const uint64_t* __restrict__ keys, uint64_t cnt, const uint32_t* __restrict__ pos_of,
                        uint32_t* __restrict__ headpos) {
    GRID_STRIDE(k, cnt) {
        bool h = (k == 0) || keys[k] != keys[k - 1];
        headpos[k] = h ? (pos_of ? pos_of[k] : (uint32_t)k) : 0u;
    }
}

// rank[p] = group id; unresolved flag = element's group has size > 1.
__global__ void k_assign(const uint64_t* __restrict__ keys, uint64_t cnt, const uint32_t* __restrict__ list,
                         const uint32_t* __restrict__ sa, const uint32_t* __restrict__ group,
                         uint32_t* __restrict__ rank, uint8_t* __restrict__ unresolved) {
    GRID_STRIDE(k, cnt) {
        uint32_t r = list ? list[k] : (uint32_t)k;
        rank[sa[r]] = group[k];
        bool h0 = (k == 0) || keys[k] != keys[k - 1];
        bool h1 = (k + 1 == cnt) || keys[k + 1] != keys[k];
        unresolved[k] = !(h0 && h1);
    }
}

// Doubling key for the tied element at rank list[k]: (group of p, order of p + h).
// p + h >= n -> the suffix is shorter than h: value n - p (<= h) sorts it
// before every longer one and by length among the short ones (Rust slice order:
// a proper prefix sorts first); otherwise BIG + rank[p + h] with BIG > h.
__device__ __forceinline__ uint64_t second_key(const uint32_t* __restrict__ rank, uint64_t n, uint64_t p,
                                               uint64_t h, uint64_t big) {
    return (p + h < n) ? (big + rank[p + h]) : (n - p);
}

// n < 2^31: one 64-bit key (group << 32 | second) with BIG = 2^31.
__global__ void k_round_keys(const uint32_t* __restrict__ list, uint64_t cnt, const uint32_t* __restrict__ sa,
                             const uint32_t* __restrict__ rank, uint64_t n, uint64_t h,
                             uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    GRID_STRIDE(k, cnt) {
        uint32_t p = sa[list[k]];
        keys[k] = ((uint64_t)rank[p] << 32) | second_key(rank, n, p, h, 0x80000000ull);
        vals[k] = p;
    }
}

// n >= 2^31: LSD two-pass -- sort by the 33-bit second key (BIG = 2^32), then
// stably by the group id gathered from the positions.
__global__ void k_round_second(const uint32_t* __restrict__ list, uint64_t cnt, const uint32_t* __restrict__ sa,
                               const uint32_t* __restrict__ rank, uint64_t n, uint64_t h,
                               uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    GRID_STRIDE(k, cnt) {
        uint32_t p = sa[list[k]];
        keys[k] = second_key(rank, n, p, h, 0x100000000ull);
        vals[k] = p;
    }
}
__global__ void k_round_group(const uint32_t* __restrict__ vals, uint64_t cnt, const uint32_t* __restrict__ rank,
                              uint64_t* __restrict__ keys) {
    GRID_STRIDE(k, cnt) keys[k] = rank[vals[k]];
}

// Group heads of a sorted round, from the (not yet updated) ranks.
__global__ void k_round_heads(const uint32_t* __restrict__ vals, uint64_t cnt, const uint32_t* __restrict__ rank,
                              uint64_t n, uint64_t h, const uint32_t* __restrict__ list,
                              uint32_t* __restrict__ headpos, uint8_t* __restrict__ head) {
    GRID_STRIDE(k, cnt) {
        bool hd = true;
        if (k > 0) {
            uint32_t p = vals[k], q = vals[k - 1];
            hd = rank[p] != rank[q] || second_key(rank, n, p, h, 0x100000000ull) !=
                                           second_key(rank, n, q, h, 0x100000000ull);
        }
        head[k] = hd;
        headpos[k] = hd ? list[k] : 0u;
    }
}

__global__ void k_round_assign(uint64_t cnt, const uint32_t* __restrict__ list, const uint32_t* __restrict__ sa,
                               const uint32_t* __restrict__ group, const uint8_t* __restrict__ head,
                               uint32_t* __restrict__ rank, uint8_t* __restrict__ unresolved) {
    GRID_STRIDE(k, cnt) {
        rank[sa[list[k]]] = group[k];
        bool h1 = (k + 1 == cnt) || head[k + 1];
        unresolved[k] = !(head[k] && h1);
    }
}

__global__ void k_scatter_sa(const uint32_t* __restrict__ list, uint64_t cnt, const uint32_t* __restrict__ vals,
                             uint32_t* __restrict__ sa) {
    GRID_STRIDE(k, cnt) sa[list[k]] = vals[k];
}

// Prefix doubling on the GPU.  sa_out: device u32[n].
static int build_sa_gpu(const uint64_t* tw, uint64_t n, uint32_t* sa_out, uint32_t* rounds_out, bool force_wide) {
    hipStream_t st = 0;
    DevBuf keys_a, keys_b, vals_b, rank, aux, list_a, list_b, flags, tmp, counter;
    TRY(keys_a.alloc(n * 8, "sa keys"));
    TRY(keys_b.alloc(n * 8, "sa keys alt"));
    TRY(vals_b.alloc(n * 4, "sa vals alt"));
    hipLaunchKernelGGL(k_init_pairs, dim3(grid_for(n)), dim3(256), 0, st, tw, n, keys_a.as<uint64_t>(), sa_out);
    HIP_TRY(hipGetLastError());

    // 1) sort all suffixes by their 32-char packed prefix
    rocprim::double_buffer<uint64_t> kdb(keys_a.as<uint64_t>(), keys_b.as<uint64_t>());
    rocprim::double_buffer<uint32_t> vdb(sa_out, vals_b.as<uint32_t>());
    size_t tbytes = 0;
    HIP_TRY(rocprim::radix_sort_pairs(nullptr, tbytes, kdb, vdb, (size_t)n, 0, 64, st));
    TRY(tmp.alloc(tbytes, "radix sort temp"));
    HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tbytes, kdb, vdb, (size_t)n, 0, 64, st));
    if (vdb.current() != sa_out)
        HIP_TRY(hipMemcpyAsync(sa_out, vdb.current(), n * 4, hipMemcpyDeviceToDevice, st));
    const uint64_t* skeys = kdb.current();
    tmp.alloc(0, "free");

    // 2) group ids + first unresolved list
    TRY(rank.alloc(n * 4, "rank"));
    TRY(aux.alloc(n * 4, "group"));
    TRY(flags.alloc(n, "flags"));
    TRY(list_a.alloc(n * 4, "tied list"));
    TRY(list_b.alloc(n * 4, "tied list alt"));
    TRY(counter.alloc(16, "counter"));
    hipLaunchKernelGGL(k_heads, dim3(grid_for(n)), dim3(256), 0, st, skeys, n, (const uint32_t*)nullptr,
                       aux.as<uint32_t>());
    size_t sbytes = 0;
    HIP_TRY(rocprim::inclusive_scan(nullptr, sbytes, aux.as<uint32_t>(), aux.as<uint32_t>(), (size_t)n, MaxOp(), st));
    TRY(tmp.alloc(sbytes, "scan temp"));
    HIP_TRY(rocprim::inclusive_scan(tmp.p, sbytes, aux.as<uint32_t>(), aux.as<uint32_t>(), (size_t)n, MaxOp(), st));
    hipLaunchKernelGGL(k_assign, dim3(grid_for(n)), dim3(256), 0, st, skeys, n, (const uint32_t*)nullptr, sa_out,
                       aux.as<uint32_t>(), rank.as<uint32_t>(), flags.as<uint8_t>());
    HIP_TRY(hipGetLastError());
    rocprim::counting_iterator<uint32_t> cit(0);
    size_t selbytes = 0;
    HIP_TRY(rocprim::select(nullptr, selbytes, cit, flags.as<uint8_t>(), list_a.as<uint32_t>(),
                            counter.as<uint64_t>(), (size_t)n, st));
    TRY(tmp.alloc(selbytes, "select temp"));
    HIP_TRY(rocprim::select(tmp.p, selbytes, cit, flags.as<uint8_t>(), list_a.as<uint32_t>(), counter.as<uint64_t>(),
                            (size_t)n, st));
    uint64_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, counter.p, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));

    // 3) doubling rounds over the tied elements only (keys_a/keys_b, vals_b reused)
    uint32_t rounds = 0;
    uint32_t* list = list_a.as<uint32_t>();
    uint32_t* list_next = list_b.as<uint32_t>();
    const bool wide = force_wide || n >= (1ull << 31);
    DevBuf heads;
    if (cnt) TRY(heads.alloc(n, "round heads"));
    for (uint64_t h = 32; cnt > 0; h *= 2) {
        if (h >= 2 * n + 64) SAS_FAIL(EIO, "sa construction did not converge");
        rounds++;
        uint64_t* rk = keys_a.as<uint64_t>();
        uint64_t* rk2 = keys_b.as<uint64_t>();
        uint32_t* rv = vals_b.as<uint32_t>();
        uint32_t* rv2 = aux.as<uint32_t>();
        const uint32_t* sv;
        size_t b2 = 0;
        if (!wide) {
            hipLaunchKernelGGL(k_round_keys, dim3(grid_for(cnt)), dim3(256), 0, st, list, cnt, sa_out,
                               rank.as<uint32_t>(), n, h, rk, rv);
            rocprim::double_buffer<uint64_t> k2(rk, rk2);
            rocprim::double_buffer<uint32_t> v2(rv, rv2);
            HIP_TRY(rocprim::radix_sort_pairs(nullptr, b2, k2, v2, (size_t)cnt, 0, 64, st));
            TRY(tmp.alloc(b2, "round sort temp"));
            HIP_TRY(rocprim::radix_sort_pairs(tmp.p, b2, k2, v2, (size_t)cnt, 0, 64, st));
            sv = v2.current();
        } else {
            hipLaunchKernelGGL(k_round_second, dim3(grid_for(cnt)), dim3(256), 0, st, list, cnt, sa_out,
                               rank.as<uint32_t>(), n, h, rk, rv);
            rocprim::double_buffer<uint64_t> k2(rk, rk2);
            rocprim::double_buffer<uint32_t> v2(rv, rv2);
            HIP_TRY(rocprim::radix_sort_pairs(nullptr, b2, k2, v2, (size_t)cnt, 0, 33, st));
            TRY(tmp.alloc(b2, "round sort temp"));
            HIP_TRY(rocprim::radix_sort_pairs(tmp.p, b2, k2, v2, (size_t)cnt, 0, 33, st));
            hipLaunchKernelGGL(k_round_group, dim3(grid_for(cnt)), dim3(256), 0, st, v2.current(), cnt,
                               rank.as<uint32_t>(), k2.current());
            size_t b3 = 0;
            HIP_TRY(rocprim::radix_sort_pairs(nullptr, b3, k2, v2, (size_t)cnt, 0, 32, st));
            TRY(tmp.alloc(b3, "round sort temp 2"));
            HIP_TRY(rocprim::radix_sort_pairs(tmp.p, b3, k2, v2, (size_t)cnt, 0, 32, st));
            sv = v2.current();
        }
        uint32_t* gbuf = (sv == rv) ? rv2 : rv;  // the free value buffer holds group ids
        hipLaunchKernelGGL(k_round_heads, dim3(grid_for(cnt)), dim3(256), 0, st, sv, cnt, rank.as<uint32_t>(), n, h,
                           list, gbuf, heads.as<uint8_t>());
        hipLaunchKernelGGL(k_scatter_sa, dim3(grid_for(cnt)), dim3(256), 0, st, list, cnt, sv, sa_out);
        size_t b4 = 0;
        HIP_TRY(rocprim::inclusive_scan(nullptr, b4, gbuf, gbuf, (size_t)cnt, MaxOp(), st));
        TRY(tmp.alloc(b4, "round scan temp"));
        HIP_TRY(rocprim::inclusive_scan(tmp.p, b4, gbuf, gbuf, (size_t)cnt, MaxOp(), st));
        hipLaunchKernelGGL(k_round_assign, dim3(grid_for(cnt)), dim3(256), 0, st, cnt, list, sa_out, gbuf,
                           heads.as<uint8_t>(), rank.as<uint32_t>(), flags.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        size_t b5 = 0;
        HIP_TRY(rocprim::select(nullptr, b5, list, flags.as<uint8_t>(), list_next, counter.as<uint64_t>(),
                                (size_t)cnt, st));
        TRY(tmp.alloc(b5, "round select temp"));
        HIP_TRY(rocprim::select(tmp.p, b5, list, flags.as<uint8_t>(), list_next, counter.as<uint64_t>(),
                                (size_t)cnt, st));
        HIP_TRY(hipMemcpyAsync(&cnt, counter.p, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        uint32_t* t = list; list = list_next; list_next = t;
    }
    *rounds_out = rounds;
    return 0;
}

// ------------------------------------------------------------------ LCP, verify
// Kernels below take the text length n (suffix lengths) and the number of SA
// entries sa_n separately: a shard index holds a rank range of the global SA.
template <int W>
__global__ void k_lcp(const uint64_t* __restrict__ tw, uint64_t n, SaView<W> sa, uint64_t sa_n,
                      uint32_t* __restrict__ lcp) {
    GRID_STRIDE(r, sa_n) {
        if (r == 0) { lcp[0] = 0; continue; }
        uint64_t a = sa[r - 1], b = sa[r];
        uint64_t L = n - (a > b ? a : b);  // min suffix length
        uint64_t l = 0;
        while (l < L) {
            uint64_t x = text_chars32(tw, a + l) ^ text_chars32(tw, b + l);
            if (x) { l += __clzll(x) >> 1; break; }
            l += 32;
        }
        l = l < L ? l : L;
        lcp[r] = l > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)l;
    }
}

// ------------------------------------------------------------------ LLCP / RLCP
// The Manber-Myers accelerant behind SAS_ALGO_LLCP.  binary_search's loop over
// [0, sa_n) (sas/sa_search.rs:98-112) probes rank m in exactly one interval [l, r):
// the one whose mid (l + r) / 2 is m.  Entry m (16 B) holds, for that interval,
//   .x, .y  SA[m] (40 bits) | Llcp << 40 | Rlcp << 52 (12 bits each, capped at
//           SAS_LLCP_CAP): Llcp = lcp(SA[l-1], SA[m]) = min LCP[l..m],
//           Rlcp = lcp(SA[m], SA[r]) = min LCP[m+1..r], LCP[0] = LCP[sa_n] = 0
//           standing for the virtual bounds (no inference there);
//   .z      16 chars of suffix SA[m] from char Llcp,  .w  16 chars from char Rlcp
//           (2-bit packed, first char high, zero past the text end): the chars a
//           tie compares first, so a tie rarely reads text.
// Built bottom-up over the implicit tree, one launch per depth: min LCP[l..m] is the
// smaller of the left child's two values (LCP[m] when that child is empty), and
// likewise on the right; a min of capped values is the capped min.
// Depth of rank m's interval, or maxd + 1 when it is deeper than maxd.
__device__ __forceinline__ uint32_t bs_node(uint64_t sa_n, uint64_t m, uint32_t maxd, uint64_t* l, uint64_t* r) {
    uint64_t lo = 0, hi = sa_n;
    uint32_t d = 0;
    for (;;) {
        const uint64_t mid = (lo + hi) >> 1;
        if (mid == m) break;
        if (d == maxd) return maxd + 1;
        if (m < mid) hi = mid;
        else lo = mid + 1;
        d++;
    }
    *l = lo;
    *r = hi;
    return d;
}

template <int W>
__global__ void k_llcp_level(const uint64_t* __restrict__ tw, SaView<W> sa, const uint32_t* __restrict__ lcp,
                             uint64_t sa_n, uint32_t depth, uint4* __restrict__ e) {
    GRID_STRIDE(m, sa_n) {
        uint64_t l = 0, r = 0;
        if (bs_node(sa_n, m, depth, &l, &r) != depth) continue;
        auto lcp_at = [&](uint64_t i) -> uint64_t {
            return (i == 0 || i >= sa_n) ? 0ull : (lcp[i] < SAS_LLCP_CAP ? lcp[i] : SAS_LLCP_CAP);
        };
        auto child_min = [&](uint64_t c) -> uint64_t {
            const uint4 v = e[c];
            const uint64_t a = (v.y >> 8) & SAS_LLCP_CAP, b = v.y >> 20;
            return a < b ? a : b;
        };
        const uint64_t L = l < m ? child_min((l + m) >> 1) : lcp_at(m);
        const uint64_t R = m + 1 < r ? child_min((m + 1 + r) >> 1) : lcp_at(r);
        const uint64_t p = sa[m];
        const uint64_t lo = p | (L << 40) | (R << 52);
        // L, R <= n - p (an lcp never exceeds the suffix), so these reads stay inside
        // the padded text
        e[m] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)(text_chars32(tw, p + L) >> 32),
                          (uint32_t)(text_chars32(tw, p + R) >> 32));
    }
}

template <int W>
__global__ void k_verify_adj(const uint64_t* __restrict__ tw, uint64_t n, SaView<W> sa,
                             uint64_t sa_n, uint32_t* __restrict__ bitmap, uint32_t* __restrict__ bad) {
    GRID_STRIDE(r, sa_n) {
        uint64_t b = sa[r];
        if (b >= n) { atomicOr(bad, 1u); continue; }
        if (bitmap) atomicOr(&bitmap[b >> 5], 1u << (b & 31));
        if (r == 0) continue;
        uint64_t a = sa[r - 1];
        if (a >= n) continue;
        uint64_t la = n - a, lb = n - b, L = la < lb ? la : lb, l = 0;
        bool lt;
        for (;;) {
            if (l >= L) { lt = la < lb; break; }
            uint64_t c = L - l < 32 ? L - l : 32;
            uint64_t mk = chars_mask((uint32_t)c);
            uint64_t x = text_chars32(tw, a + l) & mk, y = text_chars32(tw, b + l) & mk;
            if (x != y) { lt = x < y; break; }
            l += 32;
        }
        if (!lt) atomicOr(bad, 2u);  // sas/sa_search.rs:36-38 assert!(t[x..] < t[y..])
    }
}

__global__ void k_count_bits(const uint32_t* __restrict__ bitmap, uint64_t words, unsigned long long* cnt) {
    unsigned long long c = 0;
    GRID_STRIDE(w, words) c += __popc(bitmap[w]);
    if (c) atomicAdd(cnt, c);
}

// ------------------------------------------------------------------ S-tree over 16-char keys
template <int W>
__global__ void k_keys16(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n,
                         uint32_t* __restrict__ leaves, uint64_t leaf_words) {
    GRID_STRIDE(r, leaf_words) leaves[r] = r < sa_n ? (uint32_t)(text_chars32(tw, sa[r]) >> 32) : SAS_KEY_MAX;
}

// One internal layer (sst/s_tree.rs:149-172 with left_max = false):
// key j of node i = first key of child subtree j+1, MAX if beyond the keys.
__global__ void k_stree_layer(uint32_t* __restrict__ tree, uint64_t oh, uint64_t layer_nodes, uint64_t ol,
                              uint32_t h, uint32_t height, uint64_t nkeys) {
    const uint64_t B = SAS_STREE_B;
    GRID_STRIDE(i, B * layer_nodes) {
        uint64_t k = (i / B) * (B + 1) + (i % B) + 1;
        for (uint32_t l = h; l + 2 < height; l++) k *= (B + 1);
        tree[(oh + i / B) * 16 + (i % B)] = (k * B < nkeys) ? tree[(ol + k) * 16] : SAS_KEY_MAX;
    }
}

// TreeBase<16> (sst/s_tree.rs:22-45)
static uint64_t tb_blocks(uint64_t n) { return (n + 15) / 16; }
static uint64_t tb_prev(uint64_t n) { return (tb_blocks(n) + 16) / 17 * 16; }
static uint32_t tb_height(uint64_t n) { return n <= 16 ? 1 : tb_height(tb_prev(n)) + 1; }
static uint64_t tb_layer(uint64_t n, uint32_t h, uint32_t height) {
    for (uint32_t i = h; i + 1 < height; i++) n = tb_prev(n);
    return n;
}

// ------------------------------------------------------------------ sector tree
// Leaves: leaf i = 32 B = one HBM sector = entries 2i, 2i+1 as {key lo, key hi} x2
// then {sa, sa, 0, 0}; key = 32-char packed prefix of the suffix (zero padded),
// padding entries key = ~0, sa = ~0.
// The SA values' bits 32..39 (n >= 2^32) ride in the otherwise unused third word.
template <int W>
__global__ void k_sector_leaves(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n,
                                uint4* __restrict__ leaves, uint64_t nleaves) {
    GRID_STRIDE(i, nleaves) {
        uint64_t r0 = 2 * i, r1 = 2 * i + 1;
        uint64_t k0 = ~0ull, k1 = ~0ull;
        uint64_t s0 = 0xFFFFFFFFu, s1 = 0xFFFFFFFFu;
        if (r0 < sa_n) { s0 = sa[r0]; k0 = text_chars32(tw, s0); }
        if (r1 < sa_n) { s1 = sa[r1]; k1 = text_chars32(tw, s1); }
        leaves[2 * i] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
        uint32_t hi = (uint32_t)((s0 >> 32) & 0xFF) | ((uint32_t)((s1 >> 32) & 0xFF) << 8);
        leaves[2 * i + 1] = make_uint4((uint32_t)s0, (uint32_t)s1, (r0 < sa_n ? hi : 0u), 0u);
    }
}

// Internal layer, left_max style (sst/s_tree.rs:163-171 with left_max = true):
// separator j of node i = 16-char key (high word) of the LAST entry of child
// 9i+j's subtree, so count(sep < K16) lands exactly on the child holding the
// first entry with key16 >= K16.  child_span = leaves per child subtree.  The
// globally last child and nonexistent children get 0xFFFFFFFF, which no query
// key exceeds, so routing never leaves the tree.
__global__ void k_sector_layer(uint32_t* __restrict__ inner, uint64_t oh, uint64_t layer_nodes,
                               uint64_t child_span, uint64_t child_layer_nodes, const uint4* __restrict__ leaves,
                               uint64_t sa_n) {
    GRID_STRIDE(i, 8 * layer_nodes) {
        uint64_t node = i / 8, j = i % 8;
        uint64_t child = node * SAS_SECTOR_FAN + j;
        uint32_t sep = 0xFFFFFFFFu;
        if (child + 1 < child_layer_nodes) {
            uint64_t last = 2 * (child + 1) * child_span - 1;  // last entry rank of the subtree
            if (last >= sa_n) last = sa_n - 1;
            uint4 v = leaves[2 * (last >> 1)];
            sep = (last & 1) ? v.w : v.y;
        }
        inner[(oh + node) * 8 + j] = sep;
    }
}

static int build_sector(sas_index* x) {
    uint64_t sa_n = x->sa_n;
    uint64_t nl = (sa_n + 1) / 2;
    uint64_t sizes[SAS_SECTOR_MAX_LAYERS];
    uint32_t H = 0;
    uint64_t c = nl;
    do {
        c = (c + SAS_SECTOR_FAN - 1) / SAS_SECTOR_FAN;
        if (H >= SAS_SECTOR_MAX_LAYERS) SAS_FAIL(ENOTSUP, "sector tree too high");
        sizes[H++] = c;
    } while (c > 1);
    // sizes[] is bottom-up; store top-down
    uint64_t tot = 0;
    for (uint32_t h = 0; h < H; h++) {
        x->sec_off[h] = tot;
        tot += sizes[H - 1 - h];
    }
    DevBuf leaves, inner;
    TRY(leaves.alloc(nl * 32, "sector leaves"));
    TRY(inner.alloc(tot * 32, "sector inner nodes"));
    if (x->sa_w == 5)
        hipLaunchKernelGGL(k_sector_leaves<5>, dim3(grid_for(nl)), dim3(256), 0, 0, x->text_w, SaView<5>{x->sa},
                           sa_n, leaves.as<uint4>(), nl);
    else
        hipLaunchKernelGGL(k_sector_leaves<4>, dim3(grid_for(nl)), dim3(256), 0, 0, x->text_w, SaView<4>{x->sa},
                           sa_n, leaves.as<uint4>(), nl);
    uint64_t span = 1, child_nodes = nl;
    for (int h = (int)H - 1; h >= 0; h--) {
        uint64_t ln = sizes[H - 1 - h];
        hipLaunchKernelGGL(k_sector_layer, dim3(grid_for(8 * ln)), dim3(256), 0, 0, inner.as<uint32_t>(),
                           x->sec_off[h], ln, span, child_nodes, leaves.as<uint4>(), sa_n);
        span *= SAS_SECTOR_FAN;
        child_nodes = ln;
    }
    HIP_TRY(hipGetLastError());
    x->sec_leaves = static_cast<uint4*>(leaves.release());
    x->sec_inner = static_cast<uint32_t*>(inner.release());
    x->sec_leaf_count = nl;
    x->sec_inner_layers = H;
    x->sec_inner_nodes = tot;
    uint32_t L = 0;
    uint64_t ln = 0;
    for (uint32_t h = 0; h < H; h++) {
        uint64_t sz = sizes[H - 1 - h];
        if (ln + sz > SAS_SECTOR_LDS_NODES) break;
        ln += sz;
        L++;
    }
    x->sec_lds_layers = L;
    x->sec_lds_nodes = (uint32_t)ln;
    return 0;
}

// ------------------------------------------------------------------ quad tree
// Leaf entry x (16 B) = {key64 lo, key64 hi, SA lo32, SA bits 32..39} for rank x;
// leaf i = entries 4i..4i+3 = 64 B, so lane j of a 4-lane group loads entry j
// and the group's load is one 64-B request.  Padding entries are all ones.
template <int W>
__global__ void k_quad_leaves(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n,
                              uint4* __restrict__ leaves, uint64_t entries) {
    GRID_STRIDE(x, entries) {
        if (x < sa_n) {
            uint64_t p = sa[x];
            uint64_t k = text_chars32(tw, p);
            leaves[x] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)p, (uint32_t)(p >> 32));
        } else {
            leaves[x] = make_uint4(~0u, ~0u, ~0u, ~0u);
        }
    }
}

// Compact leaves: entry x = key64 of rank x only; leaf i = entries 8i..8i+7 (lane j
// of a group loads keys 2j, 2j+1).  Padding keys are all ones.
template <int W>
__global__ void k_quad_keys(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n,
                            uint64_t* __restrict__ keys, uint64_t entries) {
    GRID_STRIDE(x, entries) keys[x] = x < sa_n ? text_chars32(tw, sa[x]) : ~0ull;
}

// Internal layer, left-max (as k_sector_layer, 17-ary): separator j of node i =
// 16-char key of the last entry of child 17i+j's subtree (child_span leaves of epl
// entries), 0xFFFFFFFF for the globally last child and beyond.  Fused leaves hold
// the key's high word at uint32 4x+1, compact ones at 2x+1.
__global__ void k_quad_layer(uint32_t* __restrict__ inner, uint64_t oh, uint64_t layer_nodes, uint64_t child_span,
                             uint64_t child_layer_nodes, const uint32_t* __restrict__ leaves, uint64_t sa_n,
                             uint32_t epl) {
    GRID_STRIDE(i, 16 * layer_nodes) {
        uint64_t node = i / 16, j = i % 16;
        uint64_t child = node * SAS_QUAD_FAN + j;
        uint32_t sep = 0xFFFFFFFFu;
        if (child + 1 < child_layer_nodes) {
            uint64_t last = epl * (child + 1) * child_span - 1;
            if (last >= sa_n) last = sa_n - 1;
            sep = leaves[(epl == 4 ? 4 : 2) * last + 1];
        }
        inner[(oh + node) * 16 + j] = sep;
    }
}

// Prefix-relative internal layer (quad_fan 31).  A node's whole subtree shares its
// first d chars P (d = LCP of the subtree's first and last 32-char keys, capped at
// SAS_QUAD_RMAXD), so its separators only need the 8 chars after them:
//   word 0   = d << 27 | P (2d bits, right-aligned): u16 slots 0 and 1
//   u16 slot 2 + s (s = 0..29) = chars [d, d+8) of the key of the LAST entry of child
//            31i+s (left-max, as k_quad_layer), 0xFFFF for the globally last child and
//            beyond; stored XOR 0x8000 so that a saturating packed i16 subtract compares
//            two of them at once (quad_rel_child).
// Within the subtree these 16-bit windows are monotone in rank (the keys agree on
// chars [0, d)), so "window < q's window" still implies "suffix < q" for a query
// whose first d chars equal P; the search decides the other two cases from P alone
// ("above P" = every entry < q: the last child).  The LAST node of a layer may have
// fewer than 31 children, so it always gets d = 0 (its windows are the first 8 chars,
// still monotone): "above P" cannot happen there and no child index leaves the layer.
__device__ __forceinline__ uint64_t quad_key_at(const uint32_t* __restrict__ leaves, uint32_t epl, uint64_t x) {
    const uint2 k = reinterpret_cast<const uint2*>(leaves)[epl == 4 ? 2 * x : x];
    return (uint64_t)k.x | ((uint64_t)k.y << 32);
}

__global__ void k_quad_rel_layer(uint32_t* __restrict__ inner, uint64_t oh, uint64_t layer_nodes,
                                 uint64_t child_span, uint64_t child_layer_nodes,
                                 const uint32_t* __restrict__ leaves, uint64_t sa_n, uint32_t epl) {
    GRID_STRIDE(i, 16 * layer_nodes) {
        const uint64_t node = i / 16, w = i % 16;
        const uint64_t span = epl * child_span;  // entries per child
        const uint64_t first = node * SAS_QUAD_RFAN * span;
        uint64_t last = (node + 1) * SAS_QUAD_RFAN * span;
        last = (last < sa_n ? last : sa_n) - 1;
        const uint64_t kf = quad_key_at(leaves, epl, first), kl = quad_key_at(leaves, epl, last);
        uint32_t d = (kf == kl) ? 32u : (uint32_t)__builtin_clzll(kf ^ kl) / 2;
        if (d > SAS_QUAD_RMAXD) d = SAS_QUAD_RMAXD;
        if (node + 1 == layer_nodes) d = 0;
        uint32_t word;
        if (w == 0) {
            word = (d << 27) | (d ? (uint32_t)(kf >> (64 - 2 * d)) : 0u);
        } else {
            uint32_t half[2];
            for (int e = 0; e < 2; e++) {
                const uint64_t child = node * SAS_QUAD_RFAN + (2 * w - 2 + e);
                half[e] = 0xFFFFu;
                if (child + 1 < child_layer_nodes)
                    half[e] = (uint32_t)(quad_key_at(leaves, epl, (child + 1) * span - 1) >> (48 - 2 * d)) & 0xFFFFu;
            }
            word = (half[0] | (half[1] << 16)) ^ 0x80008000u;
        }
        inner[(oh + node) * 16 + w] = word;
    }
}

// Levels (inner layers and the leaf layer) whose 64-B nodes outgrow the 256 MiB
// Infinity Cache: each costs one DRAM-level request per lookup.
static uint32_t quad_dram_levels(uint64_t nl, uint32_t fan) {
    const uint64_t mall_nodes = (256ull << 20) / 64;
    uint32_t cnt = 0;
    for (uint64_t c = nl;; c = (c + fan - 1) / fan) {
        cnt += c > mall_nodes;
        if (c <= 1) break;
    }
    return cnt;
}

// mode: SAS_BUILD_QUAD_ABS / SAS_BUILD_QUAD_REL force a layout; neither = the one
// with fewer levels beyond the Infinity Cache, the absolute layout on a tie
// (measured: at n = 2^30 both have two such levels and the absolute one is ~4%
// faster; at n = 2^34 with compact leaves the relative one saves a level, -8% on
// ragged 8..256 queries; tools/ab_quad_rel.py).
static int build_quad(sas_index* x, bool compact, uint32_t mode) {
    const uint64_t sa_n = x->sa_n;
    const uint32_t epl = compact ? 8 : 4;  // entries per 64-B leaf
    const uint64_t nl = (sa_n + epl - 1) / epl;
    bool absolute = true;
    if (mode & SAS_BUILD_QUAD_REL) absolute = false;
    else if (!(mode & SAS_BUILD_QUAD_ABS))
        absolute = quad_dram_levels(nl, SAS_QUAD_RFAN) >= quad_dram_levels(nl, SAS_QUAD_FAN);
    const uint32_t fan = absolute ? SAS_QUAD_FAN : SAS_QUAD_RFAN;
    uint64_t sizes[SAS_QUAD_MAX_LAYERS];
    uint32_t H = 0;
    uint64_t c = nl;
    do {
        c = (c + fan - 1) / fan;
        if (H >= SAS_QUAD_MAX_LAYERS) SAS_FAIL(ENOTSUP, "quad tree too high");
        sizes[H++] = c;
    } while (c > 1);
    if (H > SAS_QUAD_MAX_INNER || nl > (1ull << 32)) SAS_FAIL(ENOTSUP, "quad tree: more than 2^32 leaves");
    uint64_t tot = 0;
    for (uint32_t h = 0; h < H; h++) {
        x->quad_off[h] = tot;
        tot += sizes[H - 1 - h];
    }
    DevBuf leaves, inner;
    TRY(leaves.alloc(nl * 64, "quad leaves"));
    TRY(inner.alloc(tot * 64, "quad inner nodes"));
    const dim3 lg(grid_for(epl * nl)), lb(256);
    if (compact && x->sa_w == 5)
        hipLaunchKernelGGL(k_quad_keys<5>, lg, lb, 0, 0, x->text_w, SaView<5>{x->sa}, sa_n, leaves.as<uint64_t>(), 8 * nl);
    else if (compact)
        hipLaunchKernelGGL(k_quad_keys<4>, lg, lb, 0, 0, x->text_w, SaView<4>{x->sa}, sa_n, leaves.as<uint64_t>(), 8 * nl);
    else if (x->sa_w == 5)
        hipLaunchKernelGGL(k_quad_leaves<5>, lg, lb, 0, 0, x->text_w, SaView<5>{x->sa}, sa_n, leaves.as<uint4>(), 4 * nl);
    else
        hipLaunchKernelGGL(k_quad_leaves<4>, lg, lb, 0, 0, x->text_w, SaView<4>{x->sa}, sa_n, leaves.as<uint4>(), 4 * nl);
    uint64_t span = 1, child_nodes = nl;
    for (int h = (int)H - 1; h >= 0; h--) {
        uint64_t ln = sizes[H - 1 - h];
        if (absolute)
            hipLaunchKernelGGL(k_quad_layer, dim3(grid_for(16 * ln)), dim3(256), 0, 0, inner.as<uint32_t>(),
                               x->quad_off[h], ln, span, child_nodes, leaves.as<uint32_t>(), sa_n, epl);
        else
            hipLaunchKernelGGL(k_quad_rel_layer, dim3(grid_for(16 * ln)), dim3(256), 0, 0, inner.as<uint32_t>(),
                               x->quad_off[h], ln, span, child_nodes, leaves.as<uint32_t>(), sa_n, epl);
        span *= fan;
        child_nodes = ln;
    }
    HIP_TRY(hipGetLastError());
    x->quad_leaves = static_cast<uint4*>(leaves.release());
    x->quad_inner = static_cast<uint4*>(inner.release());
    x->quad_leaf_count = nl;
    x->quad_compact = compact ? 1 : 0;
    x->quad_fan = fan;
    x->quad_inner_layers = H;
    x->quad_inner_nodes = tot;
    uint32_t L = 0;
    uint64_t ln = 0;
    for (uint32_t h = 0; h < H; h++) {
        uint64_t sz = sizes[H - 1 - h];
        if (ln + sz > SAS_QUAD_LDS_NODES || L == SAS_QUAD_MAX_LDS) break;
        ln += sz;
        L++;
    }
    x->quad_lds_layers = L;
    x->quad_lds_nodes = (uint32_t)ln;
    return 0;
}

// ------------------------------------------------------------------ top of the binary search
// The prefix-relative pivot blocks (common.hpp RelLayout).  Node k (1-based Eytzinger) = the
// state after the path given by k's bits below the leading one (0 = went left: r = mid, 1 =
// right: l = mid + 1); at level d in group g it sits t = d - d0 levels below its block's
// root.  The root's interval [l0, r0) gives P = lcp(SA[l0 - 1], SA[r0]) (whole suffixes:
// never past either one's end; capped), the node's pivot SA[(l + r) / 2] its chars [P, P + 8)
// (zero past the text's end) in slot (1 << t) | (k's low t bits); the root thread writes P to
// slot 0.  Nodes whose interval is empty keep 0 (never read: the search stops probing there).
template <int W>
__global__ void k_rel(const uint64_t* __restrict__ tw, uint64_t n, SaView<W> sa, uint64_t sa_n,
                      uint8_t* __restrict__ rel, uint64_t nodes, const RelLayout lay) {
    GRID_STRIDE(i, nodes) {
        const uint64_t k = 1 + i;
        const int depth = 63 - __clzll(k);
        uint32_t g = 0;
        while (g + 1 < lay.groups && (int)lay.d0[g + 1] <= depth) g++;
        const int d0 = lay.d0[g];
        const uint32_t t = (uint32_t)(depth - d0);
        uint64_t l = 0, r = sa_n, l0 = 0, r0 = sa_n;
        bool live = true;
        for (int b = depth - 1; b >= 0; b--) {
            if (depth - 1 - b == d0) { l0 = l; r0 = r; }
            const uint64_t mid = (l + r) >> 1;
            if (l >= r) { live = false; break; }
            if ((k >> b) & 1) l = mid + 1; else r = mid;
        }
        if (depth == d0) { l0 = l; r0 = r; }
        if (!(l < r)) live = false;
        if (!(l0 < r0)) continue;  // the whole block is empty
        uint32_t P = 0;
        if (l0 > 0 && r0 < sa_n) {
            const uint64_t a = sa[l0 - 1], c = sa[r0];
            const uint64_t x = text_chars32(tw, a) ^ text_chars32(tw, c);
            uint64_t lc = x ? (uint64_t)(__clzll(x) >> 1) : 32;
            if (lc > n - a) lc = n - a;
            if (lc > n - c) lc = n - c;
            P = lc < SAS_REL_PMAX ? (uint32_t)lc : SAS_REL_PMAX;
        }
        const uint64_t k0 = k >> t;
        const uint32_t sh = lay.h[g] == SAS_REL_GROUP ? 5u : 4u;
        uint16_t* blk = reinterpret_cast<uint16_t*>(rel + lay.base[g] + ((k0 - (1ull << d0)) << sh));
        if (t == 0) {
            // bit 15: a pivot of the block ends inside its key (chars [P, P + 8) padded): its
            // first difference with q may lie in the padding, so LCP / LLCP compare the text
            uint32_t flag = 0;
            for (uint32_t j = 1; j < (1u << lay.h[g]) && !flag; j++) {
                uint64_t ll = l0, rr = r0;
                for (int bb = 30 - __clz(j); bb >= 0 && ll < rr; bb--) {
                    const uint64_t mm = (ll + rr) >> 1;
                    if ((j >> bb) & 1) ll = mm + 1; else rr = mm;
                }
                if (ll < rr && n - sa[(ll + rr) >> 1] < (uint64_t)P + 8) flag = 1;
            }
            blk[0] = (uint16_t)(P | (flag << 15));
        }
        if (live) {
            const uint64_t p = sa[(l + r) >> 1];
            blk[(1u << t) | (uint32_t)(k & ((1ull << t) - 1))] = (uint16_t)(text_chars32(tw, p + P) >> 48);
        }
    }
}

// ------------------------------------------------------------------ prefix table
// The reference's prefix table (fill_prefix_table / prefix_range, sas/sa_search.rs:59-95,
// dead there because p = 0 at :31): table[x] = the first SA rank whose p-char key
// (zero padded, so key order is SA order) is >= x, for x in [0, 4^p]; the suffixes
// whose key is x are the ranks [table[x], table[x+1]).  Rank r with a new key fills
// table(key(r-1), key(r)] = r (rank sa_n fills the rest up to 4^p); a gap longer than
// PT_SMALL goes to a list that whole workgroups fill.  Keys come from the quad leaves.
// Entries are u32, or packed 40-bit (SaView<5> / sa_put<5>) beside a 40-bit SA, or
// (SAS_BUILD_PREFIX_INLINE, TW = 16) {key64, rank, SA} of that first suffix, so a lookup
// whose answer is the first suffix of its range needs this one read.
#define PT_SMALL 256
#ifndef SAS_PREFIX_ALLOC_FLAGS
#define SAS_PREFIX_ALLOC_FLAGS 0  // hipExtMallocWithFlags flags for the table (A/B: contiguous, uncached)
#endif
template <bool KO>
__device__ __forceinline__ uint64_t pt_key64(const uint4* leaves, uint64_t r) {
    if (KO) return reinterpret_cast<const uint64_t*>(leaves)[r];
    const uint2 k = reinterpret_cast<const uint2*>(leaves)[2 * r];
    return (uint64_t)k.x | ((uint64_t)k.y << 32);
}

// inline entry for rank r (fused leaves: entry r = {key lo, key hi, SA lo32, SA hi8});
// r = sa_n (nothing >= the key): key MAX, and the kernel answers next_pos
__device__ __forceinline__ uint4 pt_inline_entry(const uint4* leaves, uint64_t sa_n, uint64_t r) {
    if (r >= sa_n) return make_uint4(~0u, ~0u, (uint32_t)sa_n, 0u);
    const uint4 e = leaves[r];
    return make_uint4(e.x, e.y, (uint32_t)r, e.z);
}

// Entry x <- rank r: TW = 4 / 5 bytes of rank, or TW / 16 inline slots (ranks r, r+1, ..)
template <int TW>
__device__ __forceinline__ void pt_fill_range(uint8_t* t, uint64_t lo, uint64_t hi, uint64_t step, uint64_t r,
                                              const uint4* leaves, uint64_t sa_n) {
    if (TW >= 16) {
        constexpr int G = TW >= 16 ? TW / 16 : 1;
        uint4 ev[G];
#pragma unroll
        for (int j = 0; j < G; j++) ev[j] = pt_inline_entry(leaves, sa_n, r + j);
        if (G >= 2) {  // bits 32..39 of every slot's SA value, in slot 1's (unread) rank word
            uint32_t hb = 0;
#pragma unroll
            for (int j = 0; j < G; j++)
                if (r + j < sa_n) hb |= (leaves[r + j].w & 0xFFu) << (8 * j);
            // two slots: bits 32..39 of slot 0's rank too (a part of >= 2^32 suffixes)
            if (G == 2) hb |= (uint32_t)((r < sa_n ? r : sa_n) >> 32 & 0xFFu) << 16;
            ev[G >= 2 ? 1 : 0].z = hb;
        }
        for (uint64_t x = lo; x <= hi; x += step) {
#pragma unroll
            for (int j = 0; j < G; j++) reinterpret_cast<uint4*>(t)[G * x + j] = ev[j];
        }
    } else {
        for (uint64_t x = lo; x <= hi; x += step) sa_put<TW>(t, x, r);
    }
}

// Keys base .. base + entries - 1 (local entries 0 .. entries - 1): the whole key space (base 0,
// 4^p + 1 entries), or a part's key interval (its first key .. its last key + 2, so the two
// entries past its last key hold rank sa_n)
template <bool KO, int TW>
__global__ void k_pt_fill(const uint4* __restrict__ leaves, uint64_t sa_n, uint32_t p, uint64_t base,
                          uint64_t entries, uint8_t* __restrict__ table, uint64_t* __restrict__ big,
                          unsigned long long* __restrict__ nbig, uint64_t big_cap) {
    const uint32_t sh = 64 - 2 * p;
    const uint64_t top = entries - 1;
    GRID_STRIDE(r, sa_n + 1) {
        const uint64_t kr = r < sa_n ? (pt_key64<KO>(leaves, r) >> sh) - base : top;
        const uint64_t lo = r > 0 ? (pt_key64<KO>(leaves, r - 1) >> sh) - base + 1 : 0;
        if (lo > kr) continue;  // same key as rank r - 1
        if (kr - lo < PT_SMALL) {
            pt_fill_range<TW>(table, lo, kr, 1, r, leaves, sa_n);
        } else {
            const unsigned long long slot = atomicAdd(nbig, 1ull);
            if (slot < big_cap) {
                big[3 * slot] = lo;
                big[3 * slot + 1] = kr;
                big[3 * slot + 2] = r;
            }
        }
    }
}

template <int TW>
__global__ void k_pt_big(const uint64_t* __restrict__ big, const unsigned long long* __restrict__ nbig,
                         uint64_t big_cap, uint8_t* __restrict__ table, const uint4* __restrict__ leaves,
                         uint64_t sa_n) {
    const uint64_t nb = *nbig < big_cap ? *nbig : big_cap;  // the host fails the build past the cap
    for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x)
        pt_fill_range<TW>(table, big[3 * b] + threadIdx.x, big[3 * b + 1], blockDim.x, big[3 * b + 2], leaves, sa_n);
}

static int build_prefix(sas_index* x, uint32_t p, uint32_t inl) {
    const uint64_t sa_n = x->sa_n;
    if (!x->quad_leaves) SAS_FAIL(EINVAL, "SAS_BUILD_PREFIX needs SAS_BUILD_QUAD (keys and SA values of the leaves)");
    // inline entries hold a u32 rank and the low 32 bits of each slot's SA value: fused
    // leaves and ranks below 2^32; the one-suffix table also needs positions below 2^32, the
    // two/four-suffix ones carry bits 32..39 in slot 1 (a part index of a 2^33-char text), and
    // the two-suffix one there also bits 32..39 of the rank (a part of >= 2^32 suffixes)
    const bool hi40 = inl >= 2 && x->n > 0xFFFFFFFFull;
    if (inl && (x->quad_compact || (sa_n >= 0xFFFFFFFFull && !(inl == 2 && hi40)) ||
                (inl == 1 && x->n > 0xFFFFFFFFull)))
        SAS_FAIL(ENOTSUP, "SAS_BUILD_PREFIX_INLINE / _INLINE2 / _INLINE4 need fused quad leaves and fewer than "
                          "2^32 - 1 SA entries (SAS_BUILD_PREFIX_INLINE2 on a text of n >= 2^32: any count; "
                          "SAS_BUILD_PREFIX_INLINE also n < 2^32)");
    // u32 entries for a u32 SA, packed 40-bit ones beside a 40-bit SA, 16-B inline ones
    const uint32_t tw = inl ? 16 * inl : (x->sa_w == 5 ? 5 : 4);
    if (tw != 5 && !(tw == 32 && hi40) && sa_n >= 0xFFFFFFFFull)
        SAS_FAIL(ENOTSUP, "SAS_BUILD_PREFIX: u32 ranks need fewer than 2^32 - 1 SA entries");
    if (p == 0) {
        uint32_t l4 = 0;  // ceil(log4(sa_n))
        while (l4 < 32 && (1ull << (2 * l4)) < sa_n) l4++;
        p = l4 + 1 < 16 ? l4 + 1 : 16;
    }
    if (p > 17) SAS_FAIL(EINVAL, "SAS_BUILD_PREFIX_P: p must be 1..17");
    // the keys the table covers: every p-char key for a whole index; for a part (a contiguous
    // SA rank range) the interval from its first suffix's key to its last one's,
    // plus two entries of rank sa_n.  Keys are monotone over the ranks (zero padding), so a
    // part's suffixes are exactly that interval's, and a query outside it clamps to a
    // neighbouring entry whose suffixes are all > q (below) or to rank sa_n (above)
    // (pt_slot, sas_search.hip).  At 8 parts of a random text: 1/8 of the 4^p keys each
    uint64_t base = 0, entries = (1ull << (2 * p)) + 1;
    if (sa_n < x->n) {
        const uint32_t sh = 64 - 2 * p;
        uint64_t k0 = 0, k1 = 0;
        const uint8_t* lv = reinterpret_cast<const uint8_t*>(x->quad_leaves);
        const uint64_t eb = x->quad_compact ? 8 : 16;
        HIP_TRY(hipMemcpy(&k0, lv, 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&k1, lv + (sa_n - 1) * eb, 8, hipMemcpyDeviceToHost));
        base = k0 >> sh;
        entries = (k1 >> sh) - base + 3;
    }
    const uint64_t cap = entries / (PT_SMALL + 1) + 2;
    DevBuf t, big, nbig;
    TRY(t.alloc_flags(entries * tw + 8, "prefix table", SAS_PREFIX_ALLOC_FLAGS));
    TRY(big.alloc(cap * 24, "prefix table gap list"));
    TRY(nbig.alloc(8, "prefix table gap count"));
    HIP_TRY(hipMemset(nbig.p, 0, 8));
    const dim3 g(grid_for(sa_n + 1)), b(256);
    uint8_t* tb = t.as<uint8_t>();
    uint64_t* bl = big.as<uint64_t>();
    unsigned long long* nb_d = nbig.as<unsigned long long>();
    if (tw == 64)
        hipLaunchKernelGGL((k_pt_fill<false, 64>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else if (tw == 32)
        hipLaunchKernelGGL((k_pt_fill<false, 32>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else if (tw == 16)
        hipLaunchKernelGGL((k_pt_fill<false, 16>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else if (x->quad_compact && tw == 5)
        hipLaunchKernelGGL((k_pt_fill<true, 5>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else if (x->quad_compact)
        hipLaunchKernelGGL((k_pt_fill<true, 4>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else if (tw == 5)
        hipLaunchKernelGGL((k_pt_fill<false, 5>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    else
        hipLaunchKernelGGL((k_pt_fill<false, 4>), g, b, 0, 0, x->quad_leaves, sa_n, p, base, entries, tb, bl, nb_d, cap);
    if (tw == 64) hipLaunchKernelGGL(k_pt_big<64>, dim3(4096), dim3(256), 0, 0, bl, nb_d, cap, tb, x->quad_leaves, sa_n);
    else if (tw == 32) hipLaunchKernelGGL(k_pt_big<32>, dim3(4096), dim3(256), 0, 0, bl, nb_d, cap, tb, x->quad_leaves, sa_n);
    else if (tw == 16) hipLaunchKernelGGL(k_pt_big<16>, dim3(4096), dim3(256), 0, 0, bl, nb_d, cap, tb, x->quad_leaves, sa_n);
    else if (tw == 5) hipLaunchKernelGGL(k_pt_big<5>, dim3(4096), dim3(256), 0, 0, bl, nb_d, cap, tb, x->quad_leaves, sa_n);
    else hipLaunchKernelGGL(k_pt_big<4>, dim3(4096), dim3(256), 0, 0, bl, nb_d, cap, tb, x->quad_leaves, sa_n);
    HIP_TRY(hipGetLastError());
    uint64_t nb = 0;
    HIP_TRY(hipMemcpy(&nb, nbig.p, 8, hipMemcpyDeviceToHost));
    if (nb > cap) SAS_FAIL(EFAULT, "prefix table: gap list overflow");  // cannot happen: gaps are disjoint
    x->prefix = t.as<uint8_t>();
    t.release();
    x->prefix_chars = p;
    x->prefix_w = tw;
    x->prefix_key_lo = base;
    x->prefix_entries = entries;
    x->prefix_hi40 = hi40;
    return 0;
}

// ------------------------------------------------------------------ tagged SA + bucket table
// SAS_BUILD_TAGGED: entry r = SA[r] | chars [p, p+12) of suffix SA[r] << 40
// (zero padded past the text end), so the entries of a p-char bucket carry the suffixes'
// (p+12)-char keys next to their positions.  The bucket table is the reference's prefix
// table (sas/sa_search.rs:59-75) with p live, u64 entries {first rank with key >= x |
// min(count, 2^24 - 1) << 40}: one aligned 8-B read gives a bucket's whole rank range.
template <int W>
__global__ void k_tag_entries(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n, uint32_t p,
                              uint64_t* __restrict__ out) {
    GRID_STRIDE(r, sa_n) {
        const uint64_t s = sa[r];
        const uint64_t tag = (text_chars32(tw, s) << (2 * p)) >> 40;
        out[r] = s | (tag << 40);
    }
}

// p-char key of the suffix at rank r (S: SaView<4|5> over an SA, SaView<8> over tagged entries)
template <class S>
__device__ __forceinline__ uint64_t tag_key(const uint64_t* tw, S ent, uint64_t r, uint32_t p) {
    return text_chars32(tw, ent[r]) >> (64 - 2 * p);
}

// Rank r with a new p-char key fills table(key(r-1), key(r)] = r (rank sa_n fills the rest
// up to 4^p); gaps longer than PT_SMALL go to a list that whole workgroups fill.
template <class S>
__global__ void k_tt_fill(const uint64_t* __restrict__ tw, S ent, uint64_t sa_n,
                          uint32_t p, uint64_t* __restrict__ table, uint64_t* __restrict__ big,
                          unsigned long long* __restrict__ nbig, uint64_t big_cap) {
    const uint64_t top = 1ull << (2 * p);
    GRID_STRIDE(r, sa_n + 1) {
        const uint64_t kr = r < sa_n ? tag_key(tw, ent, r, p) : top;
        const uint64_t lo = r > 0 ? tag_key(tw, ent, r - 1, p) + 1 : 0;
        if (lo > kr) continue;
        if (kr - lo < PT_SMALL) {
            for (uint64_t x = lo; x <= kr; x++) table[x] = r;
        } else {
            const unsigned long long slot = atomicAdd(nbig, 1ull);
            if (slot < big_cap) {
                big[3 * slot] = lo;
                big[3 * slot + 1] = kr;
                big[3 * slot + 2] = r;
            }
        }
    }
}

__global__ void k_tt_big(const uint64_t* __restrict__ big, const unsigned long long* __restrict__ nbig,
                         uint64_t big_cap, uint64_t* __restrict__ table) {
    const uint64_t nb = *nbig < big_cap ? *nbig : big_cap;  // the host fails the build past the cap
    for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x)
        for (uint64_t x = big[3 * b] + threadIdx.x; x <= big[3 * b + 1]; x += blockDim.x) table[x] = big[3 * b + 2];
}

// count field: entry x gets min(table[x+1] - table[x], 2^24 - 1) in bits 40..63.  Thread
// x+1 only ever changes the high bits of entry x+1, so the rank read here is stable.
__global__ void k_tt_count(uint64_t* __restrict__ table, uint64_t keys) {
    GRID_STRIDE(x, keys) {
        const uint64_t a = table[x] & (SAS_SA40_MAX - 1), b = table[x + 1] & (SAS_SA40_MAX - 1);
        const uint64_t c = b - a < 0xFFFFFFull ? b - a : 0xFFFFFFull;
        table[x] = a | (c << 40);
    }
}

#ifndef SAS_TAG_ALLOC_FLAGS
#define SAS_TAG_ALLOC_FLAGS 0  // hipExtMallocWithFlags flags of the entries and table (A/B)
#endif
static int build_tagged(sas_index* x, uint32_t p) {
    const uint64_t sa_n = x->sa_n;
    if (p == 0) {
        uint32_t l4 = 0;  // ceil(log4(sa_n)): ~1-4 suffixes per bucket
        while (l4 < 32 && (1ull << (2 * l4)) < sa_n) l4++;
        p = l4 < 1 ? 1 : (l4 > 16 ? 16 : l4);
    }
    if (p > 17) SAS_FAIL(EINVAL, "SAS_BUILD_TAGGED: p must be 1..17");
    DevBuf ent;
    TRY(ent.alloc_flags(sa_n * 8 + 16, "tagged SA entries", SAS_TAG_ALLOC_FLAGS));
    HIP_TRY(hipMemset(ent.as<uint8_t>() + sa_n * 8, 0, 16));
    const dim3 g(grid_for(sa_n)), b(256);
    if (x->sa_w == 5)
        hipLaunchKernelGGL(k_tag_entries<5>, g, b, 0, 0, x->text_w, SaView<5>{x->sa}, sa_n, p, ent.as<uint64_t>());
    else
        hipLaunchKernelGGL(k_tag_entries<4>, g, b, 0, 0, x->text_w, SaView<4>{x->sa}, sa_n, p, ent.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    // the entries hold every SA value: the plain SA goes (80 GiB at n = 2^34)
    (void)hipFree(x->sa);
    x->sa = ent.as<uint8_t>();
    x->sa_w = 8;
    ent.release();
    const uint64_t keys = 1ull << (2 * p);
    const uint64_t cap = (keys + 1) / (PT_SMALL + 1) + 2;
    DevBuf t, big, nbig;
    TRY(t.alloc_flags((keys + 1) * 8 + 8, "tagged bucket table", SAS_TAG_ALLOC_FLAGS));
    TRY(big.alloc(cap * 24, "bucket table gap list"));
    TRY(nbig.alloc(8, "bucket table gap count"));
    HIP_TRY(hipMemset(nbig.p, 0, 8));
    hipLaunchKernelGGL(k_tt_fill<SaView<8>>, dim3(grid_for(sa_n + 1)), b, 0, 0, x->text_w, SaView<8>{x->sa}, sa_n, p,
                       t.as<uint64_t>(), big.as<uint64_t>(), nbig.as<unsigned long long>(), cap);
    hipLaunchKernelGGL(k_tt_big, dim3(4096), b, 0, 0, big.as<uint64_t>(), nbig.as<unsigned long long>(), cap,
                       t.as<uint64_t>());
    hipLaunchKernelGGL(k_tt_count, dim3(grid_for(keys)), b, 0, 0, t.as<uint64_t>(), keys);
    HIP_TRY(hipGetLastError());
    uint64_t nb = 0;
    HIP_TRY(hipMemcpy(&nb, nbig.p, 8, hipMemcpyDeviceToHost));
    if (nb > cap) SAS_FAIL(EFAULT, "bucket table: gap list overflow");  // cannot happen: gaps are disjoint
    x->tag_table = t.as<uint64_t>();
    t.release();
    x->tag_p = p;
    return 0;
}

// ------------------------------------------------------------------ C ABI
static void free_index(sas_index* x) {
    if (!x) return;
    void* ptrs[] = {x->text_w, x->sa, x->lcp, x->llcp, x->prefix, x->stree, x->rel, x->scratch,
                     x->sec_inner, x->sec_leaves, x->quad_inner, x->quad_leaves, x->tag_table, x->tag_lines, x->tag_ovf,
                     x->tag_first, x->text2_base};
    for (void* p : ptrs) if (p) (void)hipFree(p);
    sas_stage_pool_free(x->stage);
    if (x->route_pool) {  // its blocks were freed stream-ordered: drain before destroying
        (void)hipSetDevice(x->device);
        (void)hipDeviceSynchronize();
        (void)hipMemPoolDestroy(x->route_pool);
    }
    delete x;
}

extern "C" int sas_free(sas_index* index) {
    free_index(index);
    return 0;
}

static uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// full = the SA must be a permutation of 0..n (false for a shard's rank range)
static int verify_sa(const uint64_t* tw, uint64_t n, const uint8_t* sa, uint32_t w, uint64_t sa_n, bool full) {
    DevBuf bitmap, bad;
    uint64_t words = (n + 31) / 32;
    if (full) {
        TRY(bitmap.alloc(words * 4, "verify bitmap"));
        HIP_TRY(hipMemset(bitmap.p, 0, words * 4));
    }
    TRY(bad.alloc(16, "verify flags"));
    HIP_TRY(hipMemset(bad.p, 0, 16));
    if (w == 8)
        hipLaunchKernelGGL(k_verify_adj<8>, dim3(grid_for(sa_n)), dim3(256), 0, 0, tw, n, SaView<8>{sa}, sa_n,
                           full ? bitmap.as<uint32_t>() : nullptr, bad.as<uint32_t>());
    else if (w == 5)
        hipLaunchKernelGGL(k_verify_adj<5>, dim3(grid_for(sa_n)), dim3(256), 0, 0, tw, n, SaView<5>{sa}, sa_n,
                           full ? bitmap.as<uint32_t>() : nullptr, bad.as<uint32_t>());
    else
        hipLaunchKernelGGL(k_verify_adj<4>, dim3(grid_for(sa_n)), dim3(256), 0, 0, tw, n, SaView<4>{sa}, sa_n,
                           full ? bitmap.as<uint32_t>() : nullptr, bad.as<uint32_t>());
    if (full)
        hipLaunchKernelGGL(k_count_bits, dim3(grid_for(words)), dim3(256), 0, 0, bitmap.as<uint32_t>(), words,
                           reinterpret_cast<unsigned long long*>(bad.as<uint32_t>() + 2));
    HIP_TRY(hipGetLastError());
    uint32_t h[4];
    HIP_TRY(hipMemcpy(h, bad.p, 16, hipMemcpyDeviceToHost));
    uint64_t seen = (uint64_t)h[2] | ((uint64_t)h[3] << 32);
    if (h[0] & 1) SAS_FAIL(EINVAL, "suffix array holds an entry >= n");
    if (h[0] & 2) SAS_FAIL(EINVAL, "suffix array not sorted: adjacent suffixes not strictly increasing");
    if (full && seen != n) SAS_FAIL(EINVAL, "suffix array is not a permutation of 0..n");
    return 0;
}

extern "C" int sas_verify(const sas_index* index) {
    if (!index) SAS_FAIL(EINVAL, "sas_verify: null index");
    if (index->tag_lines)
        SAS_FAIL(ENOTSUP, "sas_verify: a bucket-line index holds no SA array (verify at build: SAS_BUILD_VERIFY)");
    HIP_TRY(hipSetDevice(index->device));
    return verify_sa(index->text_w, index->n, index->sa, index->sa_w, index->sa_n, index->sa_n == index->n);
}

// ------------------------------------------------------------------ bucket lines
// SAS_BUILD_TAG_LINES: the tagged entries as one 128-B line per p-char bucket (common.hpp,
// sas_index::tag_lines): the header {overflow offset | min(count, 2^24 - 1) << 40} and the
// 48-bit entries {SA | tag << sb} of ranks first .. first + 19, split into u16 high and u32
// low halves; the overflow array with the entries of ranks first + 20 .. first + count of
// every bucket of >= 20 suffixes; the first-rank table (range and SA-by-rank calls, saturated
// counts); a second copy of the packed text 64 B off the 128-B line grid (tl_text).  Built
// from the SA: first ranks (k_tt_fill), overflow offsets (a block scan of max(count - 19,
// 0)), then every slot and overflow entry from SA[r] and its text.  Peak: the SA, the lines
// and the first-rank table.
#define TL_BLOCK 1024
#define TL_PER 4  // buckets per thread in the offset scan

// the entry of rank r: {SA | tag << sb}; rank sa_n (past the index): every bit set, the SA
// field standing for next_pos and the tag the maximum
template <int W>
__device__ __forceinline__ uint64_t tl_make(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n, uint64_t r,
                                            uint32_t p, uint32_t sb) {
    if (r >= sa_n) return (1ull << 48) - 1;
    const uint64_t s = sa[r];
    return s | ((uint64_t)tl_tag_of_key(text_chars32(tw, s), p, tl_tag_bits(sb)) << sb);
}
__device__ __forceinline__ uint64_t tl_tag_max(uint64_t e, uint32_t sb) { return e | (((1ull << 48) - 1) & ~tl_sa_mask(sb)); }

// overflow entries of bucket b: ranks first + 20 .. first + count (the last, rank first + count,
// is the next bucket's first suffix)
__device__ __forceinline__ uint64_t tl_ovf_need(const uint64_t* __restrict__ t, uint64_t b) {
    const uint64_t c = t[b + 1] - t[b];
    return c >= SAS_TL_SLOTS ? c - SAS_TL_SLOTS + 1 : 0;
}

__device__ __forceinline__ uint64_t tl_block_excl_scan(uint64_t v, uint64_t* lds, uint64_t* total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = (uint64_t)__shfl_up((long long)inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (uint32_t w = 0; w < nw; w++) {
            const uint64_t t = lds[w];
            lds[w] = acc;
            acc += t;
        }
        lds[nw] = acc;
    }
    __syncthreads();
    *total = lds[nw];
    return lds[wid] + inc - v;
}

__global__ __launch_bounds__(TL_BLOCK) void k_tl_sums(const uint64_t* __restrict__ t, uint64_t keys,
                                                      uint64_t* __restrict__ bsum) {
    __shared__ uint64_t lds[TL_BLOCK / 64 + 1];
    const uint64_t b0 = ((uint64_t)blockIdx.x * TL_BLOCK + threadIdx.x) * TL_PER;
    uint64_t v = 0;
    for (int k = 0; k < TL_PER; k++)
        if (b0 + k < keys) v += tl_ovf_need(t, b0 + k);
    uint64_t tot;
    tl_block_excl_scan(v, lds, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// headers: line b's {overflow offset | count << 40} (bsum: exclusive block offsets)
__global__ __launch_bounds__(TL_BLOCK) void k_tl_hdr(const uint64_t* __restrict__ t, uint64_t keys,
                                                     const uint64_t* __restrict__ bsum, uint64_t* __restrict__ lines) {
    __shared__ uint64_t lds[TL_BLOCK / 64 + 1];
    const uint64_t b0 = ((uint64_t)blockIdx.x * TL_BLOCK + threadIdx.x) * TL_PER;
    uint64_t need[TL_PER], v = 0;
    for (int k = 0; k < TL_PER; k++) {
        need[k] = b0 + k < keys ? tl_ovf_need(t, b0 + k) : 0;
        v += need[k];
    }
    uint64_t tot;
    uint64_t off = bsum[blockIdx.x] + tl_block_excl_scan(v, lds, &tot);
    for (int k = 0; k < TL_PER; k++) {
        const uint64_t b = b0 + k;
        if (b < keys) {
            const uint64_t c = t[b + 1] - t[b];
            lines[b * 16] = off | ((c < 0xFFFFFFull ? c : 0xFFFFFFull) << 40);
            off += need[k];
        }
    }
}

// slot j of line b: rank first + j; a slot past the bucket's count (a later bucket's suffix,
// > every query routed to b) carries the maximal tag, so a lookup's count of the slots whose
// tag is < q's never passes it and needs no count
template <int W>
__global__ void k_tl_slots(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n, uint32_t p, uint32_t sb,
                           uint64_t keys, const uint64_t* __restrict__ t, uint64_t* __restrict__ lines) {
    GRID_STRIDE(k, keys * SAS_TL_SLOTS) {
        const uint64_t b = k / SAS_TL_SLOTS, j = k - b * SAS_TL_SLOTS;
        const uint64_t first = t[b], c = t[b + 1] - first;
        uint64_t e = tl_make<W>(tw, sa, sa_n, first + j, p, sb);
        if (j >= c) e = tl_tag_max(e, sb);
        reinterpret_cast<uint16_t*>(lines + b * 16)[4 + j] = (uint16_t)(e >> 32);
        reinterpret_cast<uint32_t*>(lines + b * 16)[12 + j] = (uint32_t)e;
    }
}

// A bucket's overflow entries, ranks first + 20 .. first + count (the last one the next
// bucket's first suffix with the maximal tag).  One thread per bucket writes up to
// TL_OVF_SMALL of them; a longer bucket (a low-complexity text: a poly-A run at p = 15 is
// millions of suffixes) goes to a list whose buckets whole workgroups fill (k_tl_ovf_big),
// so no bucket waits on one thread's serial tail.
#define TL_OVF_SMALL 256
template <int W>
__global__ void k_tl_ovf(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n, uint32_t p, uint32_t sb,
                         uint64_t keys, const uint64_t* __restrict__ t, const uint64_t* __restrict__ lines,
                         uint64_t* __restrict__ ovf, uint64_t* __restrict__ big, unsigned long long* __restrict__ nbig,
                         uint64_t cap) {
    GRID_STRIDE(b, keys) {
        const uint64_t first = t[b], c = t[b + 1] - first;
        if (c < SAS_TL_SLOTS) continue;
        if (c - SAS_TL_SLOTS >= TL_OVF_SMALL) {
            const unsigned long long k = atomicAdd(nbig, 1ull);
            if (k < cap) big[k] = b;
            continue;
        }
        const uint64_t o = lines[b * 16] & (SAS_SA40_MAX - 1);
        for (uint64_t j = SAS_TL_SLOTS; j <= c; j++) {
            const uint64_t e = tl_make<W>(tw, sa, sa_n, first + j, p, sb);
            ovf[o + j - SAS_TL_SLOTS] = j == c ? tl_tag_max(e, sb) : e;
        }
    }
}

template <int W>
__global__ void k_tl_ovf_big(const uint64_t* __restrict__ tw, SaView<W> sa, uint64_t sa_n, uint32_t p, uint32_t sb,
                             const uint64_t* __restrict__ t, const uint64_t* __restrict__ lines,
                             uint64_t* __restrict__ ovf, const uint64_t* __restrict__ big,
                             const unsigned long long* __restrict__ nbig, uint64_t big_cap) {
    const uint64_t nb = *nbig < big_cap ? *nbig : big_cap;  // the host fails the build past the cap
    for (uint64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint64_t b = big[k];
        const uint64_t first = t[b], c = t[b + 1] - first;
        const uint64_t o = lines[b * 16] & (SAS_SA40_MAX - 1);
        for (uint64_t j = SAS_TL_SLOTS + threadIdx.x; j <= c; j += blockDim.x) {
            const uint64_t e = tl_make<W>(tw, sa, sa_n, first + j, p, sb);
            ovf[o + j - SAS_TL_SLOTS] = j == c ? tl_tag_max(e, sb) : e;
        }
    }
}

template <int W>
static int build_tag_lines_w(sas_index* x, uint32_t p) {
    const uint64_t sa_n = x->sa_n, keys = 1ull << (2 * p);
    uint32_t sb = 32;  // SA bits: the all-ones field (rank sa_n) must exceed every position < n
    while (sb < 40 && (x->n >> sb) != 0) sb++;
    if ((x->n >> sb) != 0) SAS_FAIL(ENOTSUP, "SAS_BUILD_TAG_LINES: n >= 2^40");
    const dim3 b(256);
    // 1. first rank of every bucket (the tagged table's fill, from the SA)
    const uint64_t cap = (keys + 1) / (PT_SMALL + 1) + 2;
    DevBuf t, big, nbig;
    TRY(t.alloc((keys + 1) * 8 + 8, "bucket first ranks"));
    TRY(big.alloc(cap * 24, "bucket table gap list"));
    TRY(nbig.alloc(8, "bucket table gap count"));
    HIP_TRY(hipMemset(nbig.p, 0, 8));
    hipLaunchKernelGGL(k_tt_fill<SaView<W>>, dim3(grid_for(sa_n + 1)), b, 0, 0, x->text_w, SaView<W>{x->sa}, sa_n, p,
                       t.as<uint64_t>(), big.as<uint64_t>(), nbig.as<unsigned long long>(), cap);
    hipLaunchKernelGGL(k_tt_big, dim3(4096), b, 0, 0, big.as<uint64_t>(), nbig.as<unsigned long long>(), cap,
                       t.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    uint64_t nb = 0;
    HIP_TRY(hipMemcpy(&nb, nbig.p, 8, hipMemcpyDeviceToHost));
    if (nb > cap) SAS_FAIL(EFAULT, "bucket lines: gap list overflow");
    big.alloc(0, "free");
    // 2. overflow offsets: block sums, their exclusive scan, the headers
    const uint64_t per_blk = (uint64_t)TL_BLOCK * TL_PER;
    const uint64_t nblk = (keys + per_blk - 1) / per_blk;
    DevBuf bsum, tmp, lines;
    TRY(bsum.alloc(nblk * 8, "bucket lines block sums"));
    hipLaunchKernelGGL(k_tl_sums, dim3((unsigned)nblk), dim3(TL_BLOCK), 0, 0, t.as<uint64_t>(), keys,
                       bsum.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    uint64_t last = 0;
    HIP_TRY(hipMemcpy(&last, bsum.as<uint64_t>() + nblk - 1, 8, hipMemcpyDeviceToHost));
    size_t tb = 0;
    HIP_TRY(rocprim::exclusive_scan(nullptr, tb, bsum.as<uint64_t>(), bsum.as<uint64_t>(), (uint64_t)0, (size_t)nblk,
                                    rocprim::plus<uint64_t>(), (hipStream_t)0));
    TRY(tmp.alloc(tb ? tb : 8, "scan scratch"));
    HIP_TRY(rocprim::exclusive_scan(tmp.p, tb, bsum.as<uint64_t>(), bsum.as<uint64_t>(), (uint64_t)0, (size_t)nblk,
                                    rocprim::plus<uint64_t>(), (hipStream_t)0));
    uint64_t lastx = 0;
    HIP_TRY(hipMemcpy(&lastx, bsum.as<uint64_t>() + nblk - 1, 8, hipMemcpyDeviceToHost));
    const uint64_t novf = lastx + last;
    TRY(lines.alloc(keys * 128, "bucket lines"));
    hipLaunchKernelGGL(k_tl_hdr, dim3((unsigned)nblk), dim3(TL_BLOCK), 0, 0, t.as<uint64_t>(), keys,
                       bsum.as<uint64_t>(), lines.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    bsum.alloc(0, "free");
    tmp.alloc(0, "free");
    // 3. the slots and the overflow entries, from the SA and the text
    DevBuf ovf;
    TRY(ovf.alloc(novf * 8 + 32, "bucket lines overflow"));
    HIP_TRY(hipMemset(ovf.as<uint8_t>() + novf * 8, 0, 32));  // pair loads may read 2 entries past the end
    hipLaunchKernelGGL(k_tl_slots<W>, dim3(grid_for(keys * SAS_TL_SLOTS)), b, 0, 0, x->text_w, SaView<W>{x->sa}, sa_n,
                       p, sb, keys, t.as<uint64_t>(), lines.as<uint64_t>());
    {
        // buckets of > TL_OVF_SMALL overflow entries: at most novf / TL_OVF_SMALL of them
        const uint64_t bcap = novf / TL_OVF_SMALL + 2;
        DevBuf bl, nbl;
        TRY(bl.alloc(bcap * 8, "overflow big-bucket list"));
        TRY(nbl.alloc(8, "overflow big-bucket count"));
        HIP_TRY(hipMemset(nbl.p, 0, 8));
        hipLaunchKernelGGL(k_tl_ovf<W>, dim3(grid_for(keys)), b, 0, 0, x->text_w, SaView<W>{x->sa}, sa_n, p, sb,
                           keys, t.as<uint64_t>(), lines.as<uint64_t>(), ovf.as<uint64_t>(), bl.as<uint64_t>(),
                           nbl.as<unsigned long long>(), bcap);
        hipLaunchKernelGGL(k_tl_ovf_big<W>, dim3(4096), b, 0, 0, x->text_w, SaView<W>{x->sa}, sa_n, p, sb,
                           t.as<uint64_t>(), lines.as<uint64_t>(), ovf.as<uint64_t>(), bl.as<uint64_t>(),
                           nbl.as<unsigned long long>(), bcap);
        HIP_TRY(hipGetLastError());
        uint64_t nb = 0;
        HIP_TRY(hipMemcpy(&nb, nbl.p, 8, hipMemcpyDeviceToHost));
        if (nb > bcap) SAS_FAIL(EFAULT, "bucket lines: overflow big-bucket list overflow");
        HIP_TRY(hipDeviceSynchronize());
    }
    // the lines and the overflow hold every SA value: the plain SA goes
    (void)hipFree(x->sa);
    x->sa = nullptr;
    x->sa_w = 8;
    x->tag_lines = lines.as<uint64_t>();
    lines.release();
    x->tag_ovf = ovf.as<uint64_t>();
    ovf.release();
    x->tag_first = t.as<uint64_t>();
    t.release();
    x->tag_ovf_n = novf;
    x->tag_p = p;
    x->tag_sb = sb;
    // 4. the second text copy, its word 0 at byte 64 of a 128-B line
    DevBuf t2;
    TRY(t2.alloc(x->text_words * 8 + 128, "packed text, second copy"));
    HIP_TRY(hipMemcpy(t2.as<uint8_t>() + 64, x->text_w, x->text_words * 8, hipMemcpyDeviceToDevice));
    x->text2_base = t2.release();
    x->text2 = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(x->text2_base) + 64);
    return 0;
}

static int build_tag_lines(sas_index* x, uint32_t p) {
    if (p == 0) {
        uint32_t l4 = 0;  // ceil(log4(sa_n)) - 2: ~4-16 suffixes per line
        while (l4 < 32 && (1ull << (2 * l4)) < x->sa_n) l4++;
        p = l4 < 3 ? 1 : l4 - 2;
        if (p > 15) p = 15;
    }
    if (p < 1 || p > 15) SAS_FAIL(EINVAL, "SAS_BUILD_TAG_LINES: p must be 1..15 (4^15 lines are 128 GiB)");
    return x->sa_w == 5 ? build_tag_lines_w<5>(x, p) : build_tag_lines_w<4>(x, p);
}

static int build_stree(sas_index* x) {
    uint64_t nk = x->sa_n;
    uint32_t height = tb_height(nk);
    if (height > SAS_STREE_MAX_LAYERS) SAS_FAIL(ENOTSUP, "S-tree too high");
    uint64_t ls[SAS_STREE_MAX_LAYERS], tot = 0;
    for (uint32_t h = 0; h < height; h++) {
        ls[h] = (tb_layer(nk, h, height) + 15) / 16;
        x->stree_off[h] = tot;
        tot += ls[h];
    }
    DevBuf t;
    TRY(t.alloc(tot * 64, "S-tree"));
    uint32_t* tree = t.as<uint32_t>();
    uint64_t ol = x->stree_off[height - 1];
    if (x->sa_w == 5)
        hipLaunchKernelGGL(k_keys16<5>, dim3(grid_for(ls[height - 1] * 16)), dim3(256), 0, 0, x->text_w,
                           SaView<5>{x->sa}, nk, tree + ol * 16, ls[height - 1] * 16);
    else
        hipLaunchKernelGGL(k_keys16<4>, dim3(grid_for(ls[height - 1] * 16)), dim3(256), 0, 0, x->text_w,
                           SaView<4>{x->sa}, nk, tree + ol * 16, ls[height - 1] * 16);
    for (int h = (int)height - 2; h >= 0; h--) {
        // internal nodes: slots B..N stay MAX (B == N == 16 here, so none)
        hipLaunchKernelGGL(k_stree_layer, dim3(grid_for(16 * ls[h])), dim3(256), 0, 0, tree, x->stree_off[h],
                           ls[h], ol, (uint32_t)h, height, nk);
    }
    HIP_TRY(hipGetLastError());
    x->stree = static_cast<uint32_t*>(t.release());
    x->stree_nodes = tot;
    x->stree_height = height;
    uint32_t lds_layers = 0;
    uint64_t lds_nodes = 0;
    for (uint32_t h = 0; h + 1 < height; h++) {
        if (lds_nodes + ls[h] > SAS_STREE_LDS_NODES) break;
        lds_nodes += ls[h];
        lds_layers++;
    }
    x->stree_lds_layers = lds_layers;
    x->stree_lds_nodes = (uint32_t)lds_nodes;
    return 0;
}

static int copy_in_sa(const void* src, uint8_t* dst, uint64_t bytes, bool dev) {
    HIP_TRY(hipMemcpy(dst, src, bytes, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    return 0;
}

// Caller's SA (host or device, 4 / 5 / 8 bytes per entry) -> this index's width.
template <int WI, int WO>
__global__ void k_convert_sa(const uint8_t* __restrict__ in, uint64_t n, uint8_t* __restrict__ out) {
    GRID_STRIDE(i, n) {
        uint64_t v;
        if (WI == 8) v = reinterpret_cast<const uint64_t*>(in)[i];
        else v = SaView<WI>{in}[i];
        sa_put<WO>(out, i, v);
    }
}

static int load_sa(const void* src, uint64_t n, int wi, bool dev, uint8_t* dst, uint32_t wo) {
    const uint64_t bytes = n * (uint64_t)wi;
    if ((uint32_t)wi == wo)
        return copy_in_sa(src, dst, bytes, dev);
    DevBuf staged;
    TRY(staged.alloc(bytes + 8, "caller SA staging"));
    TRY(copy_in_sa(src, staged.as<uint8_t>(), bytes, dev));
    const uint8_t* in = staged.as<uint8_t>();
    if (wi == 4 && wo == 5) hipLaunchKernelGGL((k_convert_sa<4, 5>), dim3(grid_for(n)), dim3(256), 0, 0, in, n, dst);
    else if (wi == 5 && wo == 4) hipLaunchKernelGGL((k_convert_sa<5, 4>), dim3(grid_for(n)), dim3(256), 0, 0, in, n, dst);
    else if (wi == 8 && wo == 4) hipLaunchKernelGGL((k_convert_sa<8, 4>), dim3(grid_for(n)), dim3(256), 0, 0, in, n, dst);
    else hipLaunchKernelGGL((k_convert_sa<8, 5>), dim3(grid_for(n)), dim3(256), 0, 0, in, n, dst);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    return 0;
}

// Common builder.  [rank_lo, rank_hi) = the SA ranks this index holds
// (the whole SA for sas_build, a shard's range for sas_build_shard).
static int build_impl(const uint8_t* text, uint64_t n, const void* sa_or_null, int sa_width, uint32_t flags,
                      uint64_t rank_lo, uint64_t rank_hi, sas_index** out, uint32_t part = 0, uint32_t parts = 0,
                      const ChaKey* gen = nullptr) {
    if (!out) SAS_FAIL(EINVAL, "sas_build: null out");
    *out = nullptr;
    if (n == 0) SAS_FAIL(EINVAL, "sas_build: empty text");
    if (!text && !gen) SAS_FAIL(EINVAL, "sas_build: null text");
    if (n >= SAS_SA40_MAX - 64) SAS_FAIL(ENOTSUP, "sas_build: n >= 2^40 - 64");
    const bool w5 = (flags & SAS_BUILD_SA40) || n >= (1ull << 32) - 64 || parts > 0;
    const uint32_t W = w5 ? 5 : 4;
    if (sa_or_null && sa_width != 4 && sa_width != 5 && sa_width != 8)
        SAS_FAIL(EINVAL, "sas_build: sa_width must be 4 (u32), 5 (packed 40-bit) or 8 (u64)");
    if (sa_or_null && sa_width == 4 && n > 0xFFFFFFFFull) SAS_FAIL(EINVAL, "sas_build: a u32 SA cannot index n >= 2^32");
    if (rank_lo >= rank_hi || rank_hi > n) SAS_FAIL(EINVAL, "sas_build_shard: empty or out-of-range rank range");
    if ((flags & SAS_BUILD_TAGGED) &&
        (flags & (SAS_BUILD_STREE | SAS_BUILD_SECTOR | SAS_BUILD_QUAD | SAS_BUILD_QUAD_COMPACT | SAS_BUILD_LLCP |
                  SAS_BUILD_PREFIX | SAS_BUILD_PREFIX_INLINE | SAS_BUILD_PREFIX_INLINE2 | SAS_BUILD_PREFIX_INLINE4)))
        SAS_FAIL(ENOTSUP, "SAS_BUILD_TAGGED replaces the SA: it combines with SAS_BUILD_LCP only, not with the "
                          "trees, LLCP or the prefix tables");
    // a bucket-line index serves SAS_ALGO_TAGGED only (no SA array): an LCP array, or the
    // binary-search pivot array, would be HBM nothing reads (64 GiB of LCP at n = 2^34)
    if ((flags & SAS_BUILD_TAG_LINES) && !(flags & SAS_BUILD_TAGGED))
        SAS_FAIL(EINVAL, "SAS_BUILD_TAG_LINES needs SAS_BUILD_TAGGED");
    if ((flags & SAS_BUILD_TAG_LINES) && (flags & (SAS_BUILD_LCP | SAS_BUILD_LLCP)))
        SAS_FAIL(ENOTSUP, "SAS_BUILD_TAG_LINES serves SAS_ALGO_TAGGED only: no LCP array");
    uint64_t t0 = now_ns();
    sas_index* x = new sas_index();
    x->n = n;
    x->rank_lo = rank_lo;
    x->sa_n = rank_hi - rank_lo;
    x->sa_w = W;
    HIP_TRY(hipGetDevice(&x->device));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, x->device) == hipSuccess) x->num_cus = prop.multiProcessorCount;
    struct Guard { sas_index*& p; ~Guard() { if (p) free_index(p); } } guard{x};
    bool dev = flags & SAS_DEVICE_PTRS;

    // text -> packed words (or random_string generated straight into them: sas_build_gen)
    DevBuf tbytes, bad, tw;
    x->text_words = (n + 31) / 32 + SAS_TEXT_PAD_WORDS;
    TRY(tw.alloc(x->text_words * 8, "packed text"));
    if (gen) {
        hipLaunchKernelGGL(k_gen_packed, dim3(grid_for(x->text_words)), dim3(256), 0, 0, *gen, n, tw.as<uint64_t>(),
                           x->text_words);
        HIP_TRY(hipGetLastError());
    } else {
        const uint8_t* dtext = text;
        if (!dev) {
            TRY(tbytes.alloc(n, "text bytes"));
            HIP_TRY(hipMemcpy(tbytes.p, text, n, hipMemcpyHostToDevice));
            dtext = tbytes.as<uint8_t>();
        }
        TRY(bad.alloc(4, "flag"));
        HIP_TRY(hipMemset(bad.p, 0, 4));
        hipLaunchKernelGGL(k_pack_text, dim3(grid_for(x->text_words)), dim3(256), 0, 0, dtext, n, tw.as<uint64_t>(),
                           x->text_words, bad.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        uint32_t hbad = 0;
        HIP_TRY(hipMemcpy(&hbad, bad.p, 4, hipMemcpyDeviceToHost));
        if (hbad) SAS_FAIL(EINVAL, "sas_build: text bytes must be DNA codes 0..3");
        tbytes.alloc(0, "free");
    }
    x->text_w = tw.as<uint64_t>();
    tw.release();

    if (parts > 0) {
        // part mode: only this part's SA rank range is ever built (sas_build40.hip)
        uint64_t s0 = now_ns(), lo = 0, cnt = 0, np = 0;
        uint8_t* local = nullptr;
        TRY(build_sa_part40(x->text_w, n, part, parts, &local, &lo, &cnt, &np, &x->stats.sa_rounds));
        x->sa = local;
        x->rank_lo = lo;
        x->sa_n = cnt;
        x->next_pos = np;
        HIP_TRY(hipDeviceSynchronize());
        x->stats.build_sa_ns = now_ns() - s0;
        if (flags & SAS_BUILD_VERIFY) TRY(verify_sa(x->text_w, n, x->sa, W, x->sa_n, false));
    } else {
    // global suffix array (caller's or built here), then this index's rank range
    DevBuf sa;
    // 40-bit: the pair loads' pad; u32: PLAIN's SA run loads the 16-B chunks covering its ranks
    const uint64_t sa_bytes_full = n * W + (W == 5 ? SAS_SA40_PAD : 16);
    TRY(sa.alloc(sa_bytes_full, "suffix array"));
    if (sa_or_null) {
        TRY(load_sa(sa_or_null, n, sa_width, dev, sa.as<uint8_t>(), W));
    } else {
        uint64_t s0 = now_ns();
        if (W == 5) {
            HIP_TRY(hipMemset(sa.p, 0, sa_bytes_full));
            uint64_t buckets = 0;
            TRY(build_sa_gpu40(x->text_w, n, sa.as<uint8_t>(), &x->stats.sa_rounds, &buckets));
        } else {
            TRY(build_sa_gpu(x->text_w, n, sa.as<uint32_t>(), &x->stats.sa_rounds, flags & SAS_BUILD_WIDE));
        }
        HIP_TRY(hipDeviceSynchronize());
        x->stats.build_sa_ns = now_ns() - s0;
    }
    if (flags & SAS_BUILD_VERIFY) TRY(verify_sa(x->text_w, n, sa.as<uint8_t>(), W, n, true));
    if (rank_hi < n) {
        uint8_t b[8] = {};
        HIP_TRY(hipMemcpy(b, sa.as<uint8_t>() + rank_hi * W, W, hipMemcpyDeviceToHost));
        uint64_t np = 0;
        for (uint32_t k = 0; k < W; k++) np |= (uint64_t)b[k] << (8 * k);
        x->next_pos = np;
    } else {
        x->next_pos = n;
    }
    if (x->sa_n == n) {
        x->sa = static_cast<uint8_t*>(sa.release());
    } else {
        DevBuf part;
        const uint64_t pb = x->sa_n * W + (W == 5 ? SAS_SA40_PAD : 16);
        TRY(part.alloc(pb, "suffix array shard"));
        HIP_TRY(hipMemset(part.p, 0, pb));
        HIP_TRY(hipMemcpy(part.p, sa.as<uint8_t>() + rank_lo * W, x->sa_n * W, hipMemcpyDeviceToDevice));
        sa.alloc(0, "free");
        x->sa = static_cast<uint8_t*>(part.release());
    }
    }  // part mode
    const uint64_t sa_n = x->sa_n;
    rank_lo = x->rank_lo;

    if (flags & (SAS_BUILD_LCP | SAS_BUILD_LLCP)) {
        DevBuf l;
        TRY(l.alloc(sa_n * 4, "lcp"));
        if (W == 5)
            hipLaunchKernelGGL(k_lcp<5>, dim3(grid_for(sa_n)), dim3(256), 0, 0, x->text_w, n, SaView<5>{x->sa}, sa_n,
                               l.as<uint32_t>());
        else
            hipLaunchKernelGGL(k_lcp<4>, dim3(grid_for(sa_n)), dim3(256), 0, 0, x->text_w, n, SaView<4>{x->sa}, sa_n,
                               l.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        x->lcp = static_cast<uint32_t*>(l.release());
    }
    if (flags & SAS_BUILD_LLCP) {
        DevBuf e;
        TRY(e.alloc(sa_n * 16, "llcp entries"));
        const uint32_t depths = 64 - __builtin_clzll(sa_n);  // binary_search iterations
        for (int d = (int)depths - 1; d >= 0; d--) {
            if (W == 5)
                hipLaunchKernelGGL(k_llcp_level<5>, dim3(grid_for(sa_n)), dim3(256), 0, 0, x->text_w, SaView<5>{x->sa},
                                   x->lcp, sa_n, (uint32_t)d, e.as<uint4>());
            else
                hipLaunchKernelGGL(k_llcp_level<4>, dim3(grid_for(sa_n)), dim3(256), 0, 0, x->text_w, SaView<4>{x->sa},
                                   x->lcp, sa_n, (uint32_t)d, e.as<uint4>());
        }
        HIP_TRY(hipGetLastError());
        x->llcp = e.as<uint4>();
        e.release();
    }
    if (flags & SAS_BUILD_STREE) TRY(build_stree(x));
    if (flags & SAS_BUILD_SECTOR) TRY(build_sector(x));
    if (flags & (SAS_BUILD_QUAD | SAS_BUILD_QUAD_COMPACT)) TRY(build_quad(x, (flags & SAS_BUILD_QUAD_COMPACT) != 0, flags & (SAS_BUILD_QUAD_ABS | SAS_BUILD_QUAD_REL)));
    if (flags & (SAS_BUILD_PREFIX | SAS_BUILD_PREFIX_INLINE | SAS_BUILD_PREFIX_INLINE2 | SAS_BUILD_PREFIX_INLINE4))
        TRY(build_prefix(x, (flags >> 16) & 31,
                         (flags & SAS_BUILD_PREFIX_INLINE4)   ? 4u
                         : (flags & SAS_BUILD_PREFIX_INLINE2) ? 2u
                         : (flags & SAS_BUILD_PREFIX_INLINE)  ? 1u : 0u));

    // the binary search's pivots (not for a bucket-line index: TAGGED never reads them)
    const uint32_t iters = 64 - __builtin_clzll(sa_n);  // ilog2(len) + 1 (sas/sa_search.rs:171)
    x->iters = iters;
    if (!(flags & SAS_BUILD_TAG_LINES)) {
        // the pivots of the first L iterations: SAS_TOP2_CACHE_LEVELS (27: 273 MiB of blocks)
        // unless the caller asks for another depth (SAS_BUILD_TOP2_LEVELS), rounded up to the
        // 4-level grid past the LDS levels.  The depth is never taken from free memory, so a
        // text always gets the same index.  The probe sequence, and so every result, is the
        // same at any depth.
        const uint32_t req = (flags >> 27) & 31u;
        rel_layout(iters, req ? req : SAS_TOP2_CACHE_LEVELS, &x->rel_lay);
        const RelLayout& lay = x->rel_lay;
        DevBuf rl;
        TRY(rl.alloc(lay.bytes, "rel"));
        HIP_TRY(hipMemset(rl.p, 0, lay.bytes));
        const uint64_t cnt = (1ull << lay.levels) - 1;
        const dim3 tb(256);
        if (W == 5)
            hipLaunchKernelGGL(k_rel<5>, dim3(grid_for(cnt)), tb, 0, 0, x->text_w, n, SaView<5>{x->sa}, sa_n,
                               rl.as<uint8_t>(), cnt, lay);
        else
            hipLaunchKernelGGL(k_rel<4>, dim3(grid_for(cnt)), tb, 0, 0, x->text_w, n, SaView<4>{x->sa}, sa_n,
                               rl.as<uint8_t>(), cnt, lay);
        HIP_TRY(hipGetLastError());
        x->rel = static_cast<uint8_t*>(rl.release());
    }
    if ((flags & SAS_BUILD_TAGGED) && (flags & SAS_BUILD_TAG_LINES)) TRY(build_tag_lines(x, (flags >> 16) & 31));
    else if (flags & SAS_BUILD_TAGGED) TRY(build_tagged(x, (flags >> 16) & 31));
    HIP_TRY(hipMalloc(&x->scratch, 64));
    HIP_TRY(hipMemset(x->scratch, 0, 64));
    HIP_TRY(hipDeviceSynchronize());

    sas_stats& st = x->stats;
    st.n = n;
    st.text_bytes = x->text_words * 8;
    st.sa_bytes = x->tag_lines ? x->tag_ovf_n * 8 : sa_n * x->sa_w;  // bucket lines: the overflow array
    st.sa_width = x->sa_w;
    st.lcp_bytes = x->lcp ? sa_n * 4 : 0;
    st.llcp_bytes = x->llcp ? sa_n * 16 : 0;
    st.prefix_bytes = x->prefix ? x->prefix_entries * x->prefix_w : 0;
    st.prefix_chars = x->prefix_chars;
    st.prefix_key_lo = x->prefix ? x->prefix_key_lo : 0;
    st.prefix_entries = x->prefix ? x->prefix_entries : 0;
    st.stree_bytes = x->stree_nodes * 64;
    st.stree_layers = x->stree_height;
    st.stree_lds_layers = x->stree_lds_layers;
    st.top_levels = x->rel ? x->rel_lay.levels < SAS_REL_LDS_LEVELS ? x->rel_lay.levels : SAS_REL_LDS_LEVELS : 0;
    st.iterations = x->iters;
    st.rank_lo = rank_lo;
    st.sa_entries = sa_n;
    st.next_pos = x->next_pos;
    st.sector_bytes = (x->sec_inner_nodes + x->sec_leaf_count) * 32;
    st.sector_layers = x->sec_leaves ? x->sec_inner_layers + 1 : 0;
    st.sector_lds_layers = x->sec_lds_layers;
    st.quad_bytes = (x->quad_inner_nodes + x->quad_leaf_count) * 64;
    st.quad_layers = x->quad_leaves ? x->quad_inner_layers + 1 : 0;
    st.quad_lds_layers = x->quad_lds_layers;
    st.quad_entry_bytes = x->quad_leaves ? (x->quad_compact ? 8 : 16) : 0;
    st.quad_fan = x->quad_leaves ? x->quad_fan : 0;
    st.top2_levels = x->rel ? x->rel_lay.levels : 0;
    st.tag_chars = x->tag_p;
    st.tag_table_bytes = x->tag_table   ? ((1ull << (2 * x->tag_p)) + 1) * 8
                         : x->tag_lines ? (1ull << (2 * x->tag_p)) * 128 + ((1ull << (2 * x->tag_p)) + 1) * 8 : 0;
    st.tag_line_slots = x->tag_lines ? SAS_TL_SLOTS : 0;
    st.tag_line_tag_bits = x->tag_lines ? tl_tag_bits(x->tag_sb) : 0;
    st.text2_bytes = x->text2 ? x->text_words * 8 : 0;
    st.tag_overflow_entries = x->tag_ovf_n;
    st.top2_bytes = 0;  // round 4: every pivot level is in the rel blocks
    st.rel_levels = x->rel ? x->rel_lay.levels : 0;
    st.rel_bytes = x->rel ? x->rel_lay.bytes : 0;
    st.index_bytes = st.text_bytes + st.sa_bytes + st.lcp_bytes + st.llcp_bytes + st.prefix_bytes + st.stree_bytes +
                     st.sector_bytes + st.quad_bytes + st.tag_table_bytes + st.text2_bytes + st.top2_bytes +
                     st.rel_bytes;
    st.build_total_ns = now_ns() - t0;
    *out = x;
    x = nullptr;  // disarm guard
    return 0;
}

extern "C" int sas_build(const uint8_t* text, uint64_t n, const void* sa_or_null, int sa_width, uint32_t flags,
                         sas_index** out) {
    return build_impl(text, n, sa_or_null, sa_width, flags, 0, n, out);
}

extern "C" int sas_build_shard(const uint8_t* text, uint64_t n, const void* sa_or_null, int sa_width,
                               uint64_t rank_lo, uint64_t rank_hi, uint32_t flags, sas_index** out) {
    return build_impl(text, n, sa_or_null, sa_width, flags, rank_lo, rank_hi, out);
}

extern "C" int sas_build_part(const uint8_t* text, uint64_t n, uint32_t part, uint32_t parts, uint32_t flags,
                              sas_index** out) {
    if (parts == 0 || part >= parts) SAS_FAIL(EINVAL, "sas_build_part: need part < parts");
    return build_impl(text, n, nullptr, 5, flags, 0, n, out, part, parts);
}

extern "C" int sas_build_gen(uint64_t seed, uint64_t n, uint32_t flags, sas_index** out) {
    ChaKey key;
    h_seed_from_u64(seed, key.k);
    return build_impl(nullptr, n, nullptr, 4, flags & ~SAS_DEVICE_PTRS, 0, n, out, 0, 0, &key);
}

extern "C" int sas_build_part_gen(uint64_t seed, uint64_t n, uint32_t part, uint32_t parts, uint32_t flags,
                                  sas_index** out) {
    if (parts == 0 || part >= parts) SAS_FAIL(EINVAL, "sas_build_part_gen: need part < parts");
    ChaKey key;
    h_seed_from_u64(seed, key.k);
    return build_impl(nullptr, n, nullptr, 5, flags & ~SAS_DEVICE_PTRS, 0, n, out, part, parts, &key);
}

extern "C" int sas_get_stats(const sas_index* index, sas_stats* out) {
    if (!index || !out) SAS_FAIL(EINVAL, "sas_get_stats: null argument");
    *out = index->stats;
    return 0;
}

static int copy_out(const void* src, void* dst, uint64_t bytes, uint32_t flags) {
    HIP_TRY(hipMemcpy(dst, src, bytes, (flags & SAS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int sas_copy_sa(const sas_index* index, uint32_t* dst, uint64_t count, uint32_t flags) {
    if (!index || !dst) SAS_FAIL(EINVAL, "sas_copy_sa: null argument");
    if (index->sa_w != 4) SAS_FAIL(EINVAL, "sas_copy_sa: the SA is not u32 (40-bit for n >= 2^32 or SAS_BUILD_SA40, or tagged): use sas_copy_sa64");
    if (count > index->sa_n) SAS_FAIL(EINVAL, "sas_copy_sa: count > number of SA entries");
    return copy_out(index->sa, dst, count * 4, flags);
}

extern "C" int sas_copy_sa_range(const sas_index* index, uint64_t start, uint64_t count, uint32_t* dst,
                                 uint32_t flags) {
    if (!index || (count && !dst)) SAS_FAIL(EINVAL, "sas_copy_sa_range: null argument");
    if (index->sa_w != 4) SAS_FAIL(EINVAL, "sas_copy_sa_range: the SA is not u32 (40-bit or tagged): use sas_copy_sa64");
    if (start < index->rank_lo || start - index->rank_lo + count > index->sa_n)
        SAS_FAIL(EINVAL, "sas_copy_sa_range: ranks outside this index");
    if (count == 0) return 0;
    return copy_out(index->sa + (start - index->rank_lo) * 4, dst, count * 4, flags);
}

// Substrings of the indexed text as byte codes: out[out_off[i] .. + len[i]) = text[pos[i] ..
// + len[i]), read from the packed copy, so a caller may drop its own byte copy of a large
// text after sas_build and still cut queries from it or check answers (the c3 bench).
// One thread per substring; bytes past the text end read 0 (the padding).
__global__ void k_extract(const uint64_t* __restrict__ tw, uint64_t n, const uint64_t* __restrict__ pos,
                          const uint32_t* __restrict__ len, const uint64_t* __restrict__ out_off, uint64_t count,
                          uint8_t* __restrict__ out) {
    GRID_STRIDE(i, count) {
        const uint64_t p = pos[i], o = out_off[i];
        const uint32_t L = len[i];
        for (uint32_t j = 0; j < L; j++) {
            const uint64_t c = p + j;
            out[o + j] = c < n ? (uint8_t)((tw[c >> 5] >> (62 - 2 * (c & 31))) & 3u) : (uint8_t)0;
        }
    }
}

extern "C" int sas_extract(const sas_index* index, const uint64_t* pos, const uint32_t* len, const uint64_t* out_off,
                           uint64_t count, uint8_t* out, void* stream, uint32_t flags) {
    if (!index || (count && (!pos || !len || !out_off || !out))) SAS_FAIL(EINVAL, "sas_extract: null argument");
    if (!(flags & SAS_DEVICE_PTRS)) SAS_FAIL(EINVAL, "sas_extract: device pointers only (SAS_DEVICE_PTRS)");
    if (count == 0) return 0;
    HIP_TRY(hipSetDevice(index->device));
    hipLaunchKernelGGL(k_extract, dim3(grid_for(count)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       index->text_w, index->n, pos, len, out_off, count, out);
    HIP_TRY(hipGetLastError());
    return 0;
}

template <int W>
__global__ void k_widen_sa(SaView<W> sa, uint64_t start, uint64_t count, uint64_t* __restrict__ out) {
    GRID_STRIDE(i, count) out[i] = sa[start + i];
}

// SAS_BUILD_TAG_LINES: SA[r] from the line of r's bucket (the last bucket whose first rank is
// <= r: a binary search over the first-rank table), its slot or its overflow entry
__global__ void k_tl_sa(const uint64_t* __restrict__ lines, const uint64_t* __restrict__ ovf,
                        const uint64_t* __restrict__ first, uint64_t keys, uint32_t sb, uint64_t start, uint64_t count,
                        uint64_t* __restrict__ out) {
    GRID_STRIDE(i, count) {
        const uint64_t r = start + i;
        uint64_t lo = 0, hi = keys;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (first[mid] > r) hi = mid;
            else lo = mid + 1;
        }
        const uint64_t b = lo - 1, j = r - first[b];
        const uint64_t e = j < SAS_TL_SLOTS ? tl_slot(lines, b, (uint32_t)j)
                                            : ovf[(lines[b * 16] & (SAS_SA40_MAX - 1)) + j - SAS_TL_SLOTS];
        out[i] = e & tl_sa_mask(sb);
    }
}

extern "C" int sas_copy_sa64(const sas_index* index, uint64_t start, uint64_t count, uint64_t* dst, uint32_t flags) {
    if (!index || (count && !dst)) SAS_FAIL(EINVAL, "sas_copy_sa64: null argument");
    if (start < index->rank_lo || start - index->rank_lo + count > index->sa_n)
        SAS_FAIL(EINVAL, "sas_copy_sa64: ranks outside this index");
    if (count == 0) return 0;
    HIP_TRY(hipSetDevice(index->device));
    DevBuf tmp;
    uint64_t* out = dst;
    if (!(flags & SAS_DEVICE_PTRS)) {
        TRY(tmp.alloc(count * 8, "sa64 staging"));
        out = tmp.as<uint64_t>();
    }
    uint64_t s0 = start - index->rank_lo;
    if (index->tag_lines)
        hipLaunchKernelGGL(k_tl_sa, dim3(grid_for(count)), dim3(256), 0, 0, index->tag_lines, index->tag_ovf,
                           index->tag_first, 1ull << (2 * index->tag_p), index->tag_sb, s0, count, out);
    else if (index->sa_w == 8)
        hipLaunchKernelGGL(k_widen_sa<8>, dim3(grid_for(count)), dim3(256), 0, 0, SaView<8>{index->sa}, s0, count, out);
    else if (index->sa_w == 5)
        hipLaunchKernelGGL(k_widen_sa<5>, dim3(grid_for(count)), dim3(256), 0, 0, SaView<5>{index->sa}, s0, count, out);
    else
        hipLaunchKernelGGL(k_widen_sa<4>, dim3(grid_for(count)), dim3(256), 0, 0, SaView<4>{index->sa}, s0, count, out);
    HIP_TRY(hipGetLastError());
    if (!(flags & SAS_DEVICE_PTRS)) HIP_TRY(hipMemcpy(dst, out, count * 8, hipMemcpyDeviceToHost));
    else HIP_TRY(hipDeviceSynchronize());
    return 0;
}

extern "C" int sas_copy_lcp(const sas_index* index, uint32_t* dst, uint64_t count, uint32_t flags) {
    if (!index || !dst) SAS_FAIL(EINVAL, "sas_copy_lcp: null argument");
    if (!index->lcp) SAS_FAIL(EINVAL, "sas_copy_lcp: index built without SAS_BUILD_LCP");
    if (count > index->sa_n) SAS_FAIL(EINVAL, "sas_copy_lcp: count > number of SA entries");
    return copy_out(index->lcp, dst, count * 4, flags);
}
