// sst.hip -- GPU static search tree over sorted u32 keys (drop-in for the
// reference's static-search-tree crate, sst/).
//
// Layouts are built on the host exactly as the reference builds them, then
// moved to HBM; queries run one lane per query with the top tree layers
// staged in LDS:
//   SST_SORTED     SortedVec::binary_search          sst/binary_search.rs:37-49
//   SST_EYTZINGER  Eytzinger::search_branchless      sst/eytzinger.rs:90-102,19-31
//   SST_STREE16/15 STree::search (find_popcnt)       sst/s_tree.rs:196-206, sst/node.rs:93-109
#include "common.hpp"

#include <cstring>
#include <vector>

#define SST_BLOCK 1024
// query stream of the u32 kernels: the next query of this lane (group) is loaded while the
// current one's nodes are in flight (SST_QPREFETCH), and the query and answer streams can
// bypass L2 (SST_NT_IO: non-temporal loads and stores).  Same-box A/B at 2^28 keys, 10^7
// queries, one table placement (tools/ab_sst_var.py, profiles/r5/placement/): prefetch takes
// DirectMap from 0.211 to 0.207 ms (its one entry read no longer waits behind the query's
// round trip) and leaves the S-trees and SortedVec within 0.3%; NT I/O gains nothing beside
// it.  Where the 8 GiB table lands moves DirectMap far more (0.235 vs 0.209 ms).
#ifndef SST_QPREFETCH
#define SST_QPREFETCH 1
#endif
#ifndef SST_NT_IO
#define SST_NT_IO 0
#endif
__device__ __forceinline__ uint32_t sst_qload(const uint32_t* qs, uint64_t i) {
    return SST_NT_IO ? __builtin_nontemporal_load(qs + i) : qs[i];
}
__device__ __forceinline__ void sst_out(uint32_t* out, uint64_t i, uint32_t v) {
    if (SST_NT_IO) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
}
// the query stream of one lane (group): get(i) returns query i; with SST_QPREFETCH query
// i + stride is loaded then, so the next iteration does not start with a dependent round trip
struct SstQueries {
    const uint32_t* qs;
    uint64_t nq, stride;
    uint32_t nxt;
    __device__ SstQueries(const uint32_t* q, uint64_t n, uint64_t i0, uint64_t s)
        : qs(q), nq(n), stride(s), nxt((SST_QPREFETCH && i0 < n) ? sst_qload(q, i0) : 0u) {}
    __device__ __forceinline__ uint32_t get(uint64_t i) {
        if (!SST_QPREFETCH) return sst_qload(qs, i);
        const uint32_t q = nxt;
        if (i + stride < nq) nxt = sst_qload(qs, i + stride);
        return q;
    }
};
#define SST_EYT_LDS 8192  // first 13 Eytzinger levels (32 KiB) in LDS


struct SstArgs {
    const uint32_t* nodes;
    uint64_t n;
    uint64_t off[SAS_STREE_MAX_LAYERS];
    uint32_t lds_off[SAS_STREE_MAX_LAYERS];
    uint32_t height;
    uint32_t B;
    uint32_t lds_layers;
    uint32_t lds_nodes;
    uint32_t eyt_iters;
    const uint32_t* qs;
    uint64_t nq;
    uint32_t* out;
    uint64_t* rank;
    const uint32_t* prefix_map;  // PartitionedSTree16M
    uint32_t shift;
    uint32_t parts;
    uint32_t leaf_nt;  // leaf layer read non-temporal (> SAS_NT_BYTES)
    const uint4* direct;  // SST_DIRECT_MAP: [2^b + 1] entries {index, key, next key, next-but-one}
    uint64_t root_stride;  // SST_PARTITIONED*: elements between two parts' root windows
    uint64_t l1_mul;       // and the first step's multiplier (k_sst_part4)
    uint64_t bpp;          // Compact: nodes per part (0 otherwise)
};

// count of keys < q under SIGNED compare (find_popcnt, sst/node.rs:93-109)
__device__ __forceinline__ uint32_t popcnt_find(const uint4* node, int32_t q) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint4 v = node[j];
        c += (q > (int32_t)v.x) + (q > (int32_t)v.y) + (q > (int32_t)v.z) + (q > (int32_t)v.w);
    }
    return c;
}

template <bool TOP>
__global__ __launch_bounds__(SST_BLOCK) void k_sst_stree(SstArgs a) {
    __shared__ uint4 s_nodes[TOP ? SAS_STREE_LDS_NODES * 4 : 1];
    const uint4* g = reinterpret_cast<const uint4*>(a.nodes);
    if (TOP) {
        for (uint32_t h = 0; h < a.lds_layers; h++) {
            uint32_t cnt = ((h + 1 < a.lds_layers) ? a.lds_off[h + 1] : a.lds_nodes) - a.lds_off[h];
            for (uint32_t w = threadIdx.x; w < cnt * 4; w += blockDim.x)
                s_nodes[a.lds_off[h] * 4 + w] = g[a.off[h] * 4 + w];
        }
        __syncthreads();
    }
    const uint32_t B = a.B;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t q = a.qs[i];
        uint64_t k = 0;
        for (uint32_t h = 0; h + 1 < a.height; h++) {
            const uint4* node = (TOP && h < a.lds_layers) ? s_nodes + (a.lds_off[h] + k) * 4 : g + (a.off[h] + k) * 4;
            k = k * (B + 1) + popcnt_find(node, (int32_t)q);
        }
        uint64_t o = a.off[a.height - 1];
        uint32_t idx = popcnt_find(g + (o + k) * 4, (int32_t)q);
        a.out[i] = a.nodes[(o + k + idx / 16) * 16 + idx % 16];
        if (a.rank) a.rank[i] = k * B + idx;
    }
}

// Same search, 4 lanes per query: lane j loads keys 4j..4j+3 of each 64-B node,
// so a node costs one memory request instead of four (treebench);
// the group sums its counts with DPP.  The answer key is taken from the lane that
// holds it (no reload of the leaf); only idx == 16 (every key of the leaf < q,
// STree16) reads the next leaf's first key, as the reference does.
template <bool TOP>
__global__ __launch_bounds__(SST_BLOCK, 8) void k_sst_stree4(SstArgs a) {
    __shared__ uint4 s_nodes[TOP ? SAS_STREE_LDS_NODES * 4 : 1];
    const uint4* g = reinterpret_cast<const uint4*>(a.nodes);
    if (TOP) {
        for (uint32_t h = 0; h < a.lds_layers; h++) {
            uint32_t cnt = ((h + 1 < a.lds_layers) ? a.lds_off[h + 1] : a.lds_nodes) - a.lds_off[h];
            for (uint32_t w = threadIdx.x; w < cnt * 4; w += blockDim.x)
                s_nodes[a.lds_off[h] * 4 + w] = g[a.off[h] * 4 + w];
        }
        __syncthreads();
    }
    const uint32_t B = a.B, sub = threadIdx.x & (QUAD_G - 1);
    const uint32_t lds_layers = TOP ? a.lds_layers : 0;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    const uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G;
    SstQueries qs(a.qs, a.nq, i0, stride);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        const int32_t q = (int32_t)qs.get(i);
        auto cnt4 = [&](uint4 v) -> uint32_t {
            return quad_sum((q > (int32_t)v.x) + (q > (int32_t)v.y) + (q > (int32_t)v.z) + (q > (int32_t)v.w));
        };
        uint64_t k = 0;
        uint32_t h = 0;
        for (; h < lds_layers && h + 1 < a.height; h++) k = k * (B + 1) + cnt4(s_nodes[(a.lds_off[h] + k) * 4 + sub]);
        for (; h + 1 < a.height; h++) k = k * (B + 1) + cnt4(g[(a.off[h] + k) * 4 + sub]);
        const uint64_t o = a.off[a.height - 1];
        const uint4 v = load4(g + (o + k) * 4 + sub, a.leaf_nt);
        const uint32_t idx = cnt4(v);
        // this lane's candidate key for idx % 4, then taken from lane idx / 4 of the group
        const uint32_t r = idx & 3;
        uint32_t mine = r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w;
        const int src = (int)((threadIdx.x & 63) & ~3u) + (int)((idx >> 2) & 3);
        uint32_t val = (uint32_t)__shfl((int)mine, src, 64);
        if (sub == 0) {
            if (idx >= 16) val = a.nodes[(o + k + 1) * 16];
            sst_out(a.out, i, val);
            if (a.rank) a.rank[i] = k * B + idx;
        }
    }
}

// PartitionedSTree16M::search (sst/partitioned_s_tree.rs:833-877): layer 0 is a
// flat separator array entered through prefix_map[q >> shift] (a 16-key window
// read at key granularity); below it the usual 17-ary left-max descent.
__global__ __launch_bounds__(SST_BLOCK) void k_sst_pmap(SstArgs a) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t q = a.qs[i];
        uint32_t p = q >> a.shift;
        if (p >= a.parts) p = a.parts - 1;  // q above every key's prefix (UB in the reference)
        uint64_t key = a.prefix_map[p];      // key index in layer 0
        if (a.height >= 2) {
            const uint32_t* l0 = a.nodes + a.off[0] * 16 + key;
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) c += (int32_t)q > (int32_t)l0[j];
            uint64_t k = key + c;  // node index in layer 1
            for (uint32_t h = 1; h + 1 < a.height; h++) {
                const uint4* node = reinterpret_cast<const uint4*>(a.nodes) + (a.off[h] + k) * 4;
                k = k * 17 + popcnt_find(node, (int32_t)q);
            }
            const uint4* leaf = reinterpret_cast<const uint4*>(a.nodes) + (a.off[a.height - 1] + k) * 4;
            uint32_t idx = popcnt_find(leaf, (int32_t)q);
            a.out[i] = a.nodes[(a.off[a.height - 1] + k) * 16 + idx];
            if (a.rank) a.rank[i] = k * 16 + idx;
        } else {
            const uint32_t* l0 = a.nodes + a.off[0] * 16 + key;
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) c += (int32_t)q > (int32_t)l0[j];
            a.out[i] = l0[c];
            if (a.rank) a.rank[i] = key + c;
        }
    }
}

// 4-lane cooperative version: the 16-key window (lane j: keys 4j..4j+3, any
// alignment) and every 64-B node are one request per group.
__global__ __launch_bounds__(SST_BLOCK, 8) void k_sst_pmap4(SstArgs a) {
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    const uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G;
    SstQueries qs(a.qs, a.nq, i0, stride);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        const int32_t q = (int32_t)qs.get(i);
        uint32_t p = (uint32_t)q >> a.shift;
        if (p >= a.parts) p = a.parts - 1;  // q above every key's prefix (UB in the reference)
        const uint64_t key = a.prefix_map[p];
        const uint32_t* l0 = a.nodes + a.off[0] * 16 + key + 4 * sub;
        const uint32_t w0 = l0[0], w1 = l0[1], w2 = l0[2], w3 = l0[3];
        const uint32_t c0 = quad_sum((q > (int32_t)w0) + (q > (int32_t)w1) + (q > (int32_t)w2) + (q > (int32_t)w3));
        uint32_t val;
        uint64_t rank;
        if (a.height >= 2) {
            uint64_t k = key + c0;  // node index in layer 1
            auto cnt4 = [&](uint4 v) -> uint32_t {
                return quad_sum((q > (int32_t)v.x) + (q > (int32_t)v.y) + (q > (int32_t)v.z) + (q > (int32_t)v.w));
            };
            const uint4* g = reinterpret_cast<const uint4*>(a.nodes);
            for (uint32_t h = 1; h + 1 < a.height; h++) k = k * 17 + cnt4(g[(a.off[h] + k) * 4 + sub]);
            const uint64_t o = a.off[a.height - 1];
            const uint4 v = load4(g + (o + k) * 4 + sub, a.leaf_nt);
            const uint32_t idx = cnt4(v);
            const uint32_t r = idx & 3;
            uint32_t mine = r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w;
            val = (uint32_t)__shfl((int)mine, (int)((threadIdx.x & 63) & ~3u) + (int)((idx >> 2) & 3), 64);
            if (idx >= 16) val = a.nodes[(o + k + 1) * 16];
            rank = k * 16 + idx;
        } else {
            const uint32_t r = c0 & 3;
            uint32_t mine = r == 0 ? w0 : r == 1 ? w1 : r == 2 ? w2 : w3;
            val = (uint32_t)__shfl((int)mine, (int)((threadIdx.x & 63) & ~3u) + (int)((c0 >> 2) & 3), 64);
            if (c0 >= 16) val = a.nodes[a.off[0] * 16 + key + 16];
            rank = key + c0;
        }
        if (sub == 0) {
            sst_out(a.out, i, val);
            if (a.rank) a.rank[i] = rank;
        }
    }
}

// PartitionedSTree<16,16,{Simple,Compact,L1,Overlapping}>::search (sst/partitioned_s_tree.rs:
// 654-831), one 4-lane group per query (lane j: keys 4j..4j+3 of each 16-key window).  In
// elements of the node array: the root window of part P starts at off[0]*16 + P*root_stride
// (Simple / L1: one node per part; Compact: the part's packed tree, bpp nodes; Overlapping:
// 16 - overlap keys per part, read unaligned); the first step goes to node
// P*root_stride*l1_mul/16 + c of layer 1 (Compact: c inside the part), then k*17 + c; the
// answer is key idx of the leaf window (idx = 16: the next window's first key).
__global__ __launch_bounds__(SST_BLOCK, 8) void k_sst_part4(SstArgs a) {
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    const bool compact = a.bpp != 0;
    const uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G;
    SstQueries qs(a.qs, a.nq, i0, stride);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        const int32_t q = (int32_t)qs.get(i);
        uint64_t part = (uint32_t)q >> a.shift;
        if (part >= a.parts) part = a.parts - 1;  // q above every key's prefix (UB in the reference)
        auto cnt4 = [&](uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) -> uint32_t {
            return quad_sum((q > (int32_t)w0) + (q > (int32_t)w1) + (q > (int32_t)w2) + (q > (int32_t)w3));
        };
        const uint64_t cbase = compact ? part * a.bpp : 0;
        uint64_t e = a.off[0] * 16 + part * a.root_stride;  // the window read now (elements)
        const uint32_t* r0 = a.nodes + e + 4 * sub;  // any alignment (Overlapping)
        uint32_t w0 = r0[0], w1 = r0[1], w2 = r0[2], w3 = r0[3];
        uint32_t c = cnt4(w0, w1, w2, w3);
        if (a.height >= 2) {
            uint64_t k = compact ? c : part * a.root_stride * a.l1_mul / 16 + c;
            const uint4* g = reinterpret_cast<const uint4*>(a.nodes);
            for (uint32_t h = 1; h < a.height; h++) {
                e = (a.off[h] + cbase + k) * 16;
                const uint4 v = (h + 1 == a.height) ? load4(g + e / 4 + sub, a.leaf_nt) : g[e / 4 + sub];
                w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
                c = cnt4(w0, w1, w2, w3);
                k = k * 17 + c;
            }
        }
        const uint32_t r = c & 3;
        const uint32_t mine = r == 0 ? w0 : r == 1 ? w1 : r == 2 ? w2 : w3;
        uint32_t val = (uint32_t)__shfl((int)mine, (int)((threadIdx.x & 63) & ~3u) + (int)((c >> 2) & 3), 64);
        if (c >= 16) val = a.nodes[e + 16];
        if (sub == 0) sst_out(a.out, i, val);
    }
}

__global__ __launch_bounds__(SST_BLOCK) void k_sst_eytzinger(SstArgs a) {
    __shared__ uint32_t s_e[SST_EYT_LDS];
    uint64_t len = a.n + 1;
    uint32_t lds = len < SST_EYT_LDS ? (uint32_t)len : SST_EYT_LDS;
    for (uint32_t w = threadIdx.x; w < lds; w += blockDim.x) s_e[w] = a.nodes[w];
    __syncthreads();
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t q = a.qs[i];
        uint64_t idx = 1;
        for (uint32_t it = 0; it < a.eyt_iters; it++) {
            uint32_t v = idx < lds ? s_e[idx] : a.nodes[idx];
            idx = 2 * idx + (q > v ? 1 : 0);
        }
        bool inb = idx < len;  // get_next_index_branchless (sst/eytzinger.rs:19-31)
        uint32_t v = a.nodes[inb ? idx : 0];
        idx = 2 * idx + (((q > v) || !inb) ? 1 : 0);
        idx >>= (__ffsll((long long)~idx));  // search_result_to_index: >> (trailing_ones + 1)
        a.out[i] = a.nodes[idx];
    }
}

__global__ __launch_bounds__(SST_BLOCK) void k_sst_sorted(SstArgs a) {
    const uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    SstQueries qs(a.qs, a.nq, i0, stride);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        const uint32_t q = qs.get(i);
        uint64_t l = 0, r = a.n;
        while (l < r) {
            uint64_t m = (l + r) >> 1;
            if (a.nodes[m] < q) l = m + 1;
            else r = m;
        }
        sst_out(a.out, i, l < a.n ? a.nodes[l] : 0xFFFFFFFFu);
        if (a.rank) a.rank[i] = l;
    }
}

// ------------------------------------------------------------------ SST_DIRECT_MAP
// Bucket x = the keys whose top b of 31 bits are x (key >> (31 - b)); entry x holds the
// first index r whose key is >= x's start and keys r, r+1, r+2 (MAX past the end), so
// the answer to q is one of them unless three keys of q's bucket are < q.  A query
// above i32::MAX takes the last entry (index n, MAX): no key is >= it.
__device__ __forceinline__ uint4 direct_entry(const uint32_t* vals, uint64_t n, uint64_t r) {
    auto v = [&](uint64_t i) -> uint32_t { return i < n ? vals[i] : 0xFFFFFFFFu; };
    return make_uint4((uint32_t)r, v(r), v(r + 1), v(r + 2));
}

// index r starting a new bucket fills entries (bucket(r-1), bucket(r)] (r = n: up to 2^b);
// gaps over 256 entries go to a list that whole workgroups fill
__global__ void k_direct_fill(const uint32_t* __restrict__ vals, uint64_t n, uint32_t b, uint4* __restrict__ t,
                              uint64_t* __restrict__ big, unsigned long long* __restrict__ nbig, uint64_t cap) {
    const uint32_t sh = 31 - b;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r <= n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t kr = r < n ? (vals[r] >> sh) : (1ull << b);
        const uint64_t lo = r > 0 ? (vals[r - 1] >> sh) + 1 : 0;
        if (lo > kr) continue;
        if (kr - lo < 256) {
            const uint4 e = direct_entry(vals, n, r);
            for (uint64_t x = lo; x <= kr; x++) t[x] = e;
        } else {
            const unsigned long long s = atomicAdd(nbig, 1ull);
            if (s < cap) {
                big[3 * s] = lo;
                big[3 * s + 1] = kr;
                big[3 * s + 2] = r;
            }
        }
    }
}

__global__ void k_direct_big(const uint32_t* __restrict__ vals, uint64_t n, const uint64_t* __restrict__ big,
                             const unsigned long long* __restrict__ nbig, uint4* __restrict__ t) {
    for (uint64_t g = blockIdx.x; g < *nbig; g += gridDim.x) {
        const uint4 e = direct_entry(vals, n, big[3 * g + 2]);
        for (uint64_t x = big[3 * g] + threadIdx.x; x <= big[3 * g + 1]; x += blockDim.x) t[x] = e;
    }
}

// one lane per query: one 16-B read, the first of its three keys >= q; else a binary
// search over the bucket's remaining keys [r + 3, entry(x + 1).index)
__global__ __launch_bounds__(SST_BLOCK, 8) void k_sst_direct(SstArgs a) {
    const uint32_t sh = 31 - a.shift;  // a.shift holds b here
    const uint64_t top = 1ull << a.shift;
    const uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    SstQueries qs(a.qs, a.nq, i0, stride);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        const uint32_t q = qs.get(i);
        uint64_t x = q >> sh;
        x = x < top ? x : top;
        const uint4 e = nt_load4(a.direct + x);
        uint64_t r;
        uint32_t v;
        if (e.y >= q) { r = e.x; v = e.y; }
        else if (e.z >= q) { r = (uint64_t)e.x + 1; v = e.z; }
        else if (e.w >= q) { r = (uint64_t)e.x + 2; v = e.w; }
        else {
            uint64_t l = (uint64_t)e.x + 3, h = a.direct[x + 1].x;
            while (l < h) {
                const uint64_t m = (l + h) >> 1;
                if (a.nodes[m] < q) l = m + 1;
                else h = m;
            }
            r = l;
            v = l < a.n ? a.nodes[l] : 0xFFFFFFFFu;
        }
        sst_out(a.out, i, v);
        if (a.rank) a.rank[i] = r < a.n ? r : a.n;
    }
}

#include "sst_host.hpp"

// ------------------------------------------------------------------ C ABI
extern "C" int sst_build(const uint32_t* sorted_vals, uint64_t n, int layout, uint32_t flags, sst_index** out) {
    if (!out) SAS_FAIL(EINVAL, "sst_build: null out");
    *out = nullptr;
    if (n == 0 || !sorted_vals) SAS_FAIL(EINVAL, "sst_build: empty input (the reference asserts n > 0)");
    for (uint64_t i = 1; i < n; i++)
        if (sorted_vals[i - 1] > sorted_vals[i]) SAS_FAIL(EINVAL, "sst_build: values are not sorted");
    sst_index* x = new sst_index();
    x->layout = layout;
    x->flags = flags;
    x->n = n;
    HIP_TRY(hipGetDevice(&x->num_cus));  // temporarily the device id
    {
        hipDeviceProp_t prop;
        int dev = x->num_cus;
        x->num_cus = 256;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) x->num_cus = prop.multiProcessorCount;
    }
    std::vector<uint32_t> host, pmap;
    int rc = 0;
    switch (layout) {
        case SST_SORTED:
            host.assign(sorted_vals, sorted_vals + n);
            break;
        case SST_EYTZINGER:
            build_eytzinger_host(sorted_vals, n, host);
            {
                uint64_t len = n + 1;
                x->height = 63 - __builtin_clzll(len);  // num_iters = ilog2(len)
            }
            break;
        case SST_STREE16:
        case SST_STREE15:
            rc = build_stree_host(sorted_vals, n, layout == SST_STREE16 ? 16 : 15, flags & SST_LEFT_MAX,
                                  flags & SST_REVERSE, flags & SST_FULL, host, x);
            break;
        case SST_PARTITIONED_MAP:
            rc = build_pmap_host(sorted_vals, n, SST_PART_BITS_OF(flags), host, pmap, x);
            break;
        case SST_PARTITIONED:
        case SST_PARTITIONED_COMPACT:
        case SST_PARTITIONED_L1:
        case SST_PARTITIONED_OVERLAP:
            rc = build_part_host(sorted_vals, n, SST_PART_BITS_OF(flags), layout, host, x);
            break;
        case SST_DIRECT_MAP:
            host.assign(sorted_vals, sorted_vals + n);  // the sorted keys (the fallback search)
            if (sorted_vals[n - 1] > SST_MAX) {  // buckets cover the 31-bit key space
                rc = EINVAL;
                sas_set_error(EINVAL, "sst_build: SST_DIRECT_MAP keys must be <= i32::MAX");
                break;
            }
            {
                uint32_t b = SST_PART_BITS_OF(flags);
                if (b == 0) {
                    b = 1;
                    while ((1ull << b) < n && b < 30) b++;
                    b = b + 1 < 30 ? b + 1 : 30;  // ceil(log2 n) + 1
                }
                if (b > 30) { rc = EINVAL; sas_set_error(EINVAL, "sst_build: SST_DIRECT_MAP needs b <= 30"); }
                x->shift = b;
            }
            break;
        default:
            rc = EINVAL;
            sas_set_error(EINVAL, "sst_build: unknown layout");
    }
    if (rc) { delete x; return rc; }
    x->words = host.size();
    // one guard node of MAX keys after the array: a leaf search with idx == 16 on the
    // last leaf (no sentinel in the input) reads the "next" node (sst/s_tree.rs:205)
    host.insert(host.end(), 16, SST_MAX);
    hipError_t e = hipMalloc(&x->nodes, host.size() * 4);
    if (e != hipSuccess) { delete x; SAS_FAIL(ENOMEM, "sst_build: hipMalloc failed"); }
    e = hipMemcpy(x->nodes, host.data(), host.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(x->nodes); delete x; SAS_FAIL(EIO, "sst_build: upload failed"); }
    if (layout == SST_DIRECT_MAP) {
        const uint32_t b = x->shift;
        const uint64_t entries = (1ull << b) + 1, cap = entries / 257 + 2;
        void *big = nullptr, *nb = nullptr;
        e = hipMalloc(&x->direct, entries * 16);
        if (e == hipSuccess) e = hipMalloc(&big, cap * 24);
        if (e == hipSuccess) e = hipMalloc(&nb, 8);
        if (e == hipSuccess) e = hipMemset(nb, 0, 8);
        if (e == hipSuccess) {
            const unsigned g = (unsigned)((n + 1 + 255) / 256 < 262144 ? (n + 1 + 255) / 256 : 262144);
            hipLaunchKernelGGL(k_direct_fill, dim3(g), dim3(256), 0, 0, x->nodes, n, b, x->direct,
                               static_cast<uint64_t*>(big), static_cast<unsigned long long*>(nb), cap);
            hipLaunchKernelGGL(k_direct_big, dim3(4096), dim3(256), 0, 0, x->nodes, n, static_cast<uint64_t*>(big),
                               static_cast<unsigned long long*>(nb), x->direct);
            e = hipDeviceSynchronize();
        }
        if (big) (void)hipFree(big);
        if (nb) (void)hipFree(nb);
        if (e != hipSuccess) {
            if (x->direct) (void)hipFree(x->direct);
            (void)hipFree(x->nodes);
            delete x;
            SAS_FAIL(ENOMEM, "sst_build: direct map build failed");
        }
    }
    if (!pmap.empty()) {
        x->pmap_words = pmap.size();
        e = hipMalloc(&x->prefix_map, pmap.size() * 4);
        if (e == hipSuccess) e = hipMemcpy(x->prefix_map, pmap.data(), pmap.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) { (void)hipFree(x->nodes); delete x; SAS_FAIL(ENOMEM, "sst_build: prefix map upload failed"); }
    }
    *out = x;
    return 0;
}

extern "C" int sst_free(sst_index* x) {
    if (x) {
        if (x->nodes) (void)hipFree(x->nodes);
        if (x->prefix_map) (void)hipFree(x->prefix_map);
        if (x->direct) (void)hipFree(x->direct);
        delete x;
    }
    return 0;
}

extern "C" uint64_t sst_size(const sst_index* x) {
    // SearchIndex::size(): bytes of the node / value array (sst/lib.rs:35-36), plus
    // the prefix map for PartitionedSTree16M (sst/partitioned_s_tree.rs:100-102)
    return x ? (x->words + x->pmap_words) * 4 + (x->direct ? ((1ull << x->shift) + 1) * 16 : 0) : 0;
}

extern "C" uint64_t sst_layers(const sst_index* x) {
    if (!x) return 0;
    switch (x->layout) {
        case SST_SORTED: return 64 - __builtin_clzll(x->n);              // ilog2(len)+1 (binary_search.rs:29-31)
        case SST_EYTZINGER: return 64 - __builtin_clzll(x->n + 1);       // ilog2(len)+1 (eytzinger.rs:72-74)
        case SST_PARTITIONED_MAP: return x->height + 1;                  // offsets.len() + MAP (partitioned_s_tree.rs:104-106)
        case SST_DIRECT_MAP: return 1;                                   // the table (the sorted keys are a fallback)
        default: return x->height;                                       // offsets.len() (s_tree.rs:52-54)
    }
}

extern "C" int sst_copy_nodes(const sst_index* x, uint32_t* dst, uint64_t count) {
    if (!x || !dst || count > x->words) SAS_FAIL(EINVAL, "sst_copy_nodes: bad argument");
    HIP_TRY(hipMemcpy(dst, x->nodes, count * 4, hipMemcpyDeviceToHost));
    return 0;
}

static int sst_launch(const sst_index* x, SstArgs& a, uint32_t flags, hipStream_t st) {
    uint64_t blocks = (a.nq + SST_BLOCK - 1) / SST_BLOCK;
    uint64_t cap = (uint64_t)x->num_cus * 2;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return 0;
    dim3 grid((unsigned)blocks), block(SST_BLOCK);
    if (x->layout == SST_SORTED) {
        hipLaunchKernelGGL(k_sst_sorted, grid, block, 0, st, a);
    } else if (x->layout == SST_EYTZINGER) {
        hipLaunchKernelGGL(k_sst_eytzinger, grid, block, 0, st, a);
    } else if (x->layout == SST_DIRECT_MAP) {
        hipLaunchKernelGGL(k_sst_direct, grid, block, 0, st, a);
    } else {
        // S-tree layouts: the 4-lane cooperative kernels (one request per node)
        uint64_t b4 = (a.nq * QUAD_G + SST_BLOCK - 1) / SST_BLOCK;
        dim3 grid4((unsigned)(b4 < cap ? b4 : cap));
        if (x->layout == SST_PARTITIONED_MAP) hipLaunchKernelGGL(k_sst_pmap4, grid4, block, 0, st, a);
        else if (x->layout >= SST_PARTITIONED) hipLaunchKernelGGL(k_sst_part4, grid4, block, 0, st, a);
        else if (flags & SST_NO_LDS_TOP) hipLaunchKernelGGL(k_sst_stree4<false>, grid4, block, 0, st, a);
        else hipLaunchKernelGGL(k_sst_stree4<true>, grid4, block, 0, st, a);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

static void sst_fill(const sst_index* x, SstArgs& a) {
    a.nodes = x->nodes;
    a.n = x->n;
    uint32_t lo = 0;
    for (uint32_t h = 0; h < SAS_STREE_MAX_LAYERS; h++) {
        a.off[h] = x->off[h];
        a.lds_off[h] = lo;
        if (h < x->lds_layers) lo += (uint32_t)x->layer_nodes[h];
    }
    a.height = x->height;
    a.B = x->B;
    a.lds_layers = x->lds_layers;
    a.lds_nodes = x->lds_nodes;
    a.eyt_iters = x->height;
    a.prefix_map = x->prefix_map;
    a.shift = x->shift;
    a.parts = x->parts;
    a.leaf_nt = x->height > 0 && x->layer_nodes[x->height - 1] * 64 > SAS_NT_BYTES;
    a.direct = x->direct;
    a.root_stride = x->root_stride;
    a.l1_mul = x->l1_mul;
    a.bpp = x->bpp;
}

extern "C" int sst_query(const sst_index* x, const uint32_t* qs, uint64_t nq, uint32_t* out_val, uint64_t* out_rank,
                         void* stream, uint32_t flags) {
    if (!x) SAS_FAIL(EINVAL, "sst_query: null index");
    if (nq == 0) return 0;
    if (!qs || !out_val) SAS_FAIL(EINVAL, "sst_query: null qs/out_val");
    if (out_rank && x->layout == SST_EYTZINGER) SAS_FAIL(EINVAL, "sst_query: Eytzinger layout has no rank output");
    if (out_rank && x->layout >= SST_PARTITIONED)
        SAS_FAIL(EINVAL, "sst_query: partitioned layouts pad every part's leaves: no rank output");
    hipStream_t st = static_cast<hipStream_t>(stream);
    SstArgs a{};
    sst_fill(x, a);
    a.nq = nq;
    bool dev = flags & SST_DEVICE_PTRS;
    void *dq = nullptr, *dout = nullptr, *drank = nullptr;
    struct Free { void** p; ~Free() { if (*p) (void)hipFree(*p); } } f1{&dq}, f2{&dout}, f3{&drank};
    if (dev) {
        a.qs = qs;
        a.out = out_val;
        a.rank = out_rank;
    } else {
        // host pointers: plain hipMalloc + synchronous copies (see sas_search.hip)
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMalloc(&dq, nq * 4));
        HIP_TRY(hipMalloc(&dout, nq * 4));
        if (out_rank) HIP_TRY(hipMalloc(&drank, nq * 8));
        HIP_TRY(hipMemcpy(dq, qs, nq * 4, hipMemcpyHostToDevice));
        a.qs = static_cast<uint32_t*>(dq);
        a.out = static_cast<uint32_t*>(dout);
        a.rank = static_cast<uint64_t*>(drank);
    }
    int rc = sst_launch(x, a, flags, st);
    if (rc) return rc;
    if (!dev) {
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(out_val, dout, nq * 4, hipMemcpyDeviceToHost));
        if (out_rank) HIP_TRY(hipMemcpy(out_rank, drank, nq * 8, hipMemcpyDeviceToHost));
    }
    return 0;
}

extern "C" int sst_time_query(const sst_index* x, const uint32_t* d_qs, uint64_t nq, uint32_t* d_out, int reps,
                              void* stream, uint32_t flags, double* kernel_ns) {
    if (!x || !d_qs || !d_out || reps < 1) SAS_FAIL(EINVAL, "sst_time_query: bad argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    SstArgs a{};
    sst_fill(x, a);
    a.nq = nq;
    a.qs = d_qs;
    a.out = d_out;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, st));
    for (int r = 0; r < reps; r++) {
        int rc = sst_launch(x, a, flags, st);
        if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(e1, st));
    HIP_TRY(hipEventSynchronize(e1));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    if (kernel_ns) *kernel_ns = ms * 1e6 / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}
