// treebench.hip -- price candidate search-tree layouts on MI355X before building them.
//
// Each lane runs one "lookup": a dependent chain of random accesses, one per tree
// layer, each into its own region whose size is that layer's footprint and whose
// width is that layer's node width (32 B = one sector, 128 B = one line).  The
// chain is dependent (the next address mixes in the loaded value) like a real
// descent.  NT = 1 issues the DRAM-level accesses (regions >= 1 GiB) as
// non-temporal loads so they do not evict the upper layers from L2 / MALL.
//
//   usage: treebench <lookups> <reps> <layout>...   layout = "W:MiB,W:MiB,..." (W in bytes, MiB may be fractional)
//   W = 1064 / 1128: a 64-B / 128-B node loaded cooperatively by 4 / 8 lanes (16 B each, one
//   request), the lanes of a group sharing one lookup (ps are then per lookup, not per lane)
//   e.g.   treebench 10000000 5 32:0.285,32:2.56,32:23.1,32:207,32:1864,32:16384
//
// Prints one JSON line per (layout, NT): lookups/s and ns per lookup.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/treebench tools/treebench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define MAXL 12
struct Layout {
    int L;
    uint64_t base[MAXL];   // byte offset of each region
    uint64_t units[MAXL];  // number of nodes in the region
    int width[MAXL];       // 32, 64 or 128
    int nt[MAXL];          // non-temporal loads for this region
};

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__device__ __forceinline__ uint64_t node_idx_coop(uint64_t h, uint64_t units) { return ((h >> 32) * units) >> 32; }

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// io != nullptr: each lookup also streams its 32-B query in (8 B per lane of the
// group) and writes an 8-B result (lane 0), as the real search kernels do.
struct Io { const uint8_t* q; uint64_t* res; };

template <int G>
__global__ __launch_bounds__(1024, 8) void k_chain(const uint8_t* __restrict__ p, Layout lay, uint64_t lookups,
                                                   uint32_t seed, uint32_t* out, Io io = Io{nullptr, nullptr}) {
    uint32_t acc = 0;
    const uint32_t sub = threadIdx.x % G;  // lane within a cooperative group of G lanes
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < lookups * G;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t i = t / G;
        uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + seed);
        uint32_t dep = 0;
        if (io.q) {
            const uint2 qv = *reinterpret_cast<const uint2*>(io.q + i * 32 + 8 * (sub % 4));
            h ^= (uint64_t)(qv.x & 0x80000000u);  // qv top bit 0: a data dependence, no value change
        }
        for (int l = 0; l < lay.L; l++) {
            // one 64-bit multiply per level (cheap, like a real descent's address math);
            // dep's top bit is 0 (buffer = 0x01): a true data dependence
            h = h * 0x9E3779B97F4A7C15ull + l + (dep & 0x80000000u);
            uint64_t node = ((h >> 32) * lay.units[l]) >> 32;
            const u32x4* v = reinterpret_cast<const u32x4*>(p + lay.base[l] + node * lay.width[l]);
            if (lay.width[l] < 16) {
                dep = *reinterpret_cast<const uint32_t*>(v);
                continue;
            }
            if (lay.width[l] > 1000) {  // cooperative: 16 B per lane, combine over the group
                int wb = lay.width[l] - 1000;
                const u32x4* node = reinterpret_cast<const u32x4*>(p + lay.base[l] + node_idx_coop(h, lay.units[l]) * wb);
                u32x4 t = node[sub % (wb / 16)];
                uint32_t d = t.x ^ t.y ^ t.z ^ t.w;
                for (int o = 1; o < G; o <<= 1) d ^= __shfl_xor(d, o, G);
                dep = d;
                continue;
            }
            u32x4 t = lay.nt[l] ? ld<true>(v) : ld<false>(v);
            if (lay.width[l] >= 32) { u32x4 t2 = lay.nt[l] ? ld<true>(v + 1) : ld<false>(v + 1); t ^= t2; }
            if (lay.width[l] >= 64) { t ^= ld<false>(v + 2) ^ ld<false>(v + 3); }
            if (lay.width[l] >= 128) { t ^= ld<false>(v + 4) ^ ld<false>(v + 5) ^ ld<false>(v + 6) ^ ld<false>(v + 7); }
            dep = t.x ^ t.y ^ t.z ^ t.w;
        }
        if (io.res && sub == 0) io.res[i] = dep;
        acc ^= dep;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Two independent lookups per lane group, their levels interleaved (ILP = 2):
// cooperative 64-B levels only (W = 1064), G = 4.
// XCD-partitioned replay (G = 4): workgroups are dispatched round-robin to the 8
// XCDs, so block b runs on XCD b % 8; its lookups only touch that XCD's eighth of
// every level (as if the queries had been bucketed by key range per XCD).
__global__ __launch_bounds__(1024, 8) void k_chain_xcd(const uint8_t* __restrict__ p, Layout lay, uint64_t lookups,
                                                       uint32_t seed, uint32_t* out) {
    const int G = 4;
    uint32_t acc = 0;
    const uint32_t sub = threadIdx.x % G, xcd = blockIdx.x % 8;
    const uint64_t groups = ((uint64_t)gridDim.x * blockDim.x) / G;
    for (uint64_t g = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; g < lookups; g += groups) {
        uint64_t h = mix(g * 0x9E3779B97F4A7C15ull + seed);
        uint32_t dep = 0;
        for (int l = 0; l < lay.L; l++) {
            h = h * 0x9E3779B97F4A7C15ull + l + (dep & 0x80000000u);
            const int wb = lay.width[l] - 1000;
            const uint64_t part = lay.units[l] / 8 ? lay.units[l] / 8 : 1;
            const uint64_t node = (lay.units[l] >= 8 ? xcd * part : 0) + (((h >> 32) * part) >> 32);
            const u32x4* v = reinterpret_cast<const u32x4*>(p + lay.base[l] + node * wb);
            u32x4 t = v[sub % (wb / 16)];
            uint32_t d = t.x ^ t.y ^ t.z ^ t.w;
            for (int o = 1; o < G; o <<= 1) d ^= __shfl_xor(d, o, G);
            dep = d;
        }
        acc ^= dep;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(1024, 8) void k_chain_ilp2(const uint8_t* __restrict__ p, Layout lay, uint64_t lookups,
                                                        uint32_t seed, uint32_t* out) {
    const int G = 4;
    uint32_t acc = 0;
    const uint32_t sub = threadIdx.x % G;
    const uint64_t groups = ((uint64_t)gridDim.x * blockDim.x) / G;
    for (uint64_t g = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; 2 * g < lookups; g += groups) {
        uint64_t ha = mix((2 * g) * 0x9E3779B97F4A7C15ull + seed), hb = mix((2 * g + 1) * 0x9E3779B97F4A7C15ull + seed);
        uint32_t da = 0, db = 0;
        for (int l = 0; l < lay.L; l++) {
            ha = ha * 0x9E3779B97F4A7C15ull + l + (da & 0x80000000u);
            hb = hb * 0x9E3779B97F4A7C15ull + l + (db & 0x80000000u);
            int wb = lay.width[l] - 1000;
            const u32x4* na = reinterpret_cast<const u32x4*>(p + lay.base[l] + node_idx_coop(ha, lay.units[l]) * wb);
            const u32x4* nb = reinterpret_cast<const u32x4*>(p + lay.base[l] + node_idx_coop(hb, lay.units[l]) * wb);
            u32x4 ta = na[sub % (wb / 16)], tb = nb[sub % (wb / 16)];
            uint32_t xa = ta.x ^ ta.y ^ ta.z ^ ta.w, xb = tb.x ^ tb.y ^ tb.z ^ tb.w;
            for (int o = 1; o < G; o <<= 1) { xa ^= __shfl_xor(xa, o, G); xb ^= __shfl_xor(xb, o, G); }
            da = xa; db = xb;
        }
        acc ^= da ^ db;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// TB_MIXED=G: one lookup per LANE; cooperative levels (W > 1000) are read by the lane's
// group of G for each of its G lookups in turn (G independent 16-B loads per lane, issued
// together, one request per node), per-lane levels by the lane alone (the k_sa_quad4x
// pattern).  TB_QBYTES=B: each lookup first reads B query bytes, a wave's 64 queries as one
// contiguous span with coalesced 16-B loads (the wave-staged queries of k_sa_tagged).
template <int G>
__global__ __launch_bounds__(256, 5) void k_chain_mixed(const uint8_t* __restrict__ p, Layout lay, uint64_t lookups,
                                                        uint32_t seed, uint32_t* out, const uint8_t* __restrict__ qb,
                                                        uint32_t qbytes) {
    uint32_t acc = 0;
    const uint32_t sub = threadIdx.x % G, lane = threadIdx.x & 63;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lookups;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + seed);
        uint32_t dep = 0;
        if (qb) {
            const uint64_t wbase = (i - lane) * qbytes;
            uint32_t x = 0;
            for (uint32_t o = lane * 16; o < 64 * qbytes; o += 64 * 16) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(qb + wbase + o);
                x ^= v.x ^ v.w;
            }
            h ^= (uint64_t)(x & 0x80000000u);
        }
        for (int l = 0; l < lay.L; l++) {
            h = h * 0x9E3779B97F4A7C15ull + l + (dep & 0x80000000u);
            if (lay.width[l] > 1000) {
                const int wb = lay.width[l] - 1000;
                u32x4 t[G];
#pragma unroll
                for (int k = 0; k < G; k++) {
                    const uint64_t hk = __shfl(h, (int)((lane & ~(uint32_t)(G - 1)) + k), 64);
                    const u32x4* node = reinterpret_cast<const u32x4*>(p + lay.base[l] + node_idx_coop(hk, lay.units[l]) * wb);
                    t[k] = node[sub % (wb / 16)];
                }
                uint32_t mine = 0;
#pragma unroll
                for (int k = 0; k < G; k++) {
                    uint32_t d = t[k].x ^ t[k].y ^ t[k].z ^ t[k].w;
                    for (int o = 1; o < G; o <<= 1) d ^= __shfl_xor(d, o, G);
                    mine = (sub == (uint32_t)k) ? d : mine;
                }
                dep = mine;
                continue;
            }
            const uint64_t node = ((h >> 32) * lay.units[l]) >> 32;
            const u32x4* v = reinterpret_cast<const u32x4*>(p + lay.base[l] + node * lay.width[l]);
            if (lay.width[l] < 16) {
                dep = lay.width[l] == 8 ? (uint32_t)*reinterpret_cast<const uint64_t*>(v)
                                        : *reinterpret_cast<const uint32_t*>(v);
                continue;
            }
            u32x4 t = __builtin_nontemporal_load(v);
            if (lay.width[l] >= 32) t ^= __builtin_nontemporal_load(v + 1);
            dep = t.x ^ t.y ^ t.z ^ t.w;
        }
        acc ^= dep;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: treebench <lookups> <reps> <layout>...\n"); return 2; }
    uint64_t lookups = strtoull(argv[1], 0, 10);
    int reps = atoi(argv[2]);
    std::vector<Layout> lays;
    std::vector<std::string> names;
    uint64_t maxbytes = 0;
    for (int a = 3; a < argc; a++) {
        Layout L{};
        char buf[1024];
        strncpy(buf, argv[a], sizeof buf - 1);
        uint64_t off = 0;
        for (char* tok = strtok(buf, ","); tok && L.L < MAXL; tok = strtok(nullptr, ",")) {
            int w = atoi(tok);
            double mib = atof(strchr(tok, ':') + 1);
            uint64_t bytes = (uint64_t)(mib * 1048576.0);
            int wb = w > 1000 ? w - 1000 : w;
            L.width[L.L] = w;
            L.units[L.L] = bytes / wb ? bytes / wb : 1;
            L.base[L.L] = off;
            L.nt[L.L] = 0;
            off += ((L.units[L.L] * wb + 4095) / 4096) * 4096;
            L.L++;
        }
        if (off > maxbytes) maxbytes = off;
        lays.push_back(L);
        names.push_back(argv[a]);
    }
    uint8_t* p;
    uint32_t* out;
    CHECK(hipMalloc(&out, 64));
    // TB_SEPARATE=1: every level in its own allocation, as the real index arrays are
    // (p = 0, base[l] = the level's device address)
    const bool separate = getenv("TB_SEPARATE") != nullptr;
    // TB_FRAG=<KiB>: before the levels are allocated, fill ~48 GiB with chunks of that
    // size and free every other one, so the levels land on scattered physical memory
    std::vector<void*> frag;
    if (getenv("TB_FRAG")) {
        const size_t chunk = (size_t)atoll(getenv("TB_FRAG")) << 10;
        for (size_t tot = 0; tot < (48ull << 30); tot += chunk) {
            void* q;
            if (hipMalloc(&q, chunk) != hipSuccess) break;
            frag.push_back(q);
        }
        for (size_t i = 0; i < frag.size(); i += 2) CHECK(hipFree(frag[i]));
        fprintf(stderr, "TB_FRAG: %zu chunks of %zu KiB, freed every other\n", frag.size(), chunk >> 10);
    }
    if (!separate) {
        CHECK(hipMalloc(&p, maxbytes));
        CHECK(hipMemset(p, 1, maxbytes));
    } else {
        p = nullptr;
        for (auto& L : lays) {
            for (int l = 0; l < L.L; l++) {
                const int wb = L.width[l] > 1000 ? L.width[l] - 1000 : L.width[l];
                uint8_t* q;
                CHECK(hipMalloc(&q, L.units[l] * wb + 64));
                CHECK(hipMemset(q, 1, L.units[l] * wb + 64));
                L.base[l] = (uint64_t)(uintptr_t)q;
            }
        }
    }
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    dim3 blk(1024), grd(cus * 2);
    Io io{nullptr, nullptr};
    if (getenv("TB_IO")) {
        uint8_t* qbuf;
        uint64_t* rbuf;
        CHECK(hipMalloc(&qbuf, lookups * 32 + 64));
        CHECK(hipMemset(qbuf, 1, lookups * 32 + 64));
        CHECK(hipMalloc(&rbuf, lookups * 8));
        io = Io{qbuf, rbuf};
    }
    const uint32_t mqb = getenv("TB_QBYTES") ? (uint32_t)atoi(getenv("TB_QBYTES")) : 0;
    uint8_t* mq = nullptr;
    if (mqb) {
        CHECK(hipMalloc(&mq, lookups * mqb + 1024));
        CHECK(hipMemset(mq, 1, lookups * mqb + 1024));
    }
    for (size_t k = 0; k < lays.size(); k++) {
        for (int nt = 0; nt < 1; nt++) {
            Layout L = lays[k];
            for (int l = 0; l < L.L; l++) L.nt[l] = nt && L.width[l] < 1000 && (L.units[l] * L.width[l] >= (1ull << 30));
            int G = 1;
            for (int l = 0; l < L.L; l++) if (L.width[l] > 1000) G = (L.width[l] - 1000) / 16 > G ? (L.width[l] - 1000) / 16 : G;
            bool ilp2 = getenv("TB_ILP2") != nullptr;
            bool xcdp = getenv("TB_XCD") != nullptr;
            const int mixed = getenv("TB_MIXED") ? atoi(getenv("TB_MIXED")) : 0;
            auto launch = [&](uint32_t sd) {
                if (mixed) {
                    const dim3 b2(256), g2(cus * 5);
                    if (mixed == 8) hipLaunchKernelGGL(k_chain_mixed<8>, g2, b2, 0, 0, p, L, lookups, sd, out, mq, mqb);
                    else if (mixed == 4) hipLaunchKernelGGL(k_chain_mixed<4>, g2, b2, 0, 0, p, L, lookups, sd, out, mq, mqb);
                    else hipLaunchKernelGGL(k_chain_mixed<1>, g2, b2, 0, 0, p, L, lookups, sd, out, mq, mqb);
                } else if (xcdp) hipLaunchKernelGGL(k_chain_xcd, grd, blk, 0, 0, p, L, lookups, sd, out);
                else if (ilp2) hipLaunchKernelGGL(k_chain_ilp2, grd, blk, 0, 0, p, L, lookups, sd, out);
                else if (G == 8) hipLaunchKernelGGL(k_chain<8>, grd, blk, 0, 0, p, L, lookups, sd, out, io);
                else if (G == 4) hipLaunchKernelGGL(k_chain<4>, grd, blk, 0, 0, p, L, lookups, sd, out, io);
                else hipLaunchKernelGGL(k_chain<1>, grd, blk, 0, 0, p, L, lookups, sd, out, io);
            };
            launch(1u);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++) launch(2u + r);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("{\"layout\": \"%s\", \"nt_dram\": %d, \"lookups\": %llu, \"ms\": %.4f, \"lookups_per_s\": %.4g, "
                   "\"ps_per_lookup\": %.1f}\n",
                   names[k].c_str(), nt, (unsigned long long)lookups, ms, lookups / (ms * 1e-3),
                   ms * 1e9 / lookups);
            fflush(stdout);
        }
    }
    return 0;
}
