// randbench.hip -- calibrate rocprofv3 memory-side counters and the random-access
// ceiling of MI355X HBM for the access shapes the search kernels use.
//
//   stream16 : coalesced 16 B/lane streaming read of the whole buffer (known bytes)
//   rand4    : independent random 4-B loads (one per lane per step)
//   rand8x2  : random 8-B + the next 8-B word (text_chars32 shape)
//   rand64   : random 64-B node, 4 x 16-B loads by one lane (S-tree node shape)
//   rand128  : random 128-B line, 8 x 16-B loads by one lane
//   rand16   : one random 16-B slot per lane
//   rand32pair: one random 32-B slot per lane pair, 16 B per lane (the PREFIX entry read)
//   rand32pair_nt: the same with non-temporal loads (as k_sa_prefix2 issues them)
//
// argv: buffer MiB, accesses, reps, allocation (0 hipMalloc, 1 hipDeviceMallocUncached,
// 2 hipDeviceMallocFinegrained), shapes to run (bit mask, default all)
//
// Prints one JSON line per kernel: accesses/s and bytes moved per the access shape.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/randbench tools/randbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__global__ void k_stream16(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// SHAPE: 0 = 4 B, 1 = 2 x 8 B, 2 = 64 B, 3 = 128 B ; steps independent accesses per lane
template <int SHAPE>
__global__ __launch_bounds__(1024) void k_rand(const uint8_t* __restrict__ p, uint64_t bytes, uint64_t accesses,
                                               uint32_t seed, uint32_t* out) {
    uint32_t acc = 0;
    uint64_t lines = bytes / 128;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; SHAPE < 5 && i < accesses;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + seed);
        uint64_t line = h % lines;
        const uint8_t* b = p + line * 128;
        if (SHAPE == 0) {
            acc ^= *reinterpret_cast<const uint32_t*>(b + ((h >> 40) & 31) * 4);
        } else if (SHAPE == 1) {
            const uint64_t* w = reinterpret_cast<const uint64_t*>(b + ((h >> 40) & 7) * 8);
            uint64_t x = w[0] ^ w[1];
            acc ^= (uint32_t)x ^ (uint32_t)(x >> 32);
        } else if (SHAPE == 2) {
            const uint4* v = reinterpret_cast<const uint4*>(b + ((h >> 40) & 1) * 64);
#pragma unroll
            for (int k = 0; k < 4; k++) { uint4 t = v[k]; acc ^= t.x ^ t.y ^ t.z ^ t.w; }
        } else if (SHAPE == 3) {
            const uint4* v = reinterpret_cast<const uint4*>(b);
#pragma unroll
            for (int k = 0; k < 8; k++) { uint4 t = v[k]; acc ^= t.x ^ t.y ^ t.z ^ t.w; }
        } else if (SHAPE == 4) {  // one lane, one random 16-B slot (one-suffix inline entry)
            const uint4 t = reinterpret_cast<const uint4*>(b)[(h >> 40) & 7];
            acc ^= t.x ^ t.y ^ t.z ^ t.w;
        }
    }
    if (SHAPE == 5) {  // lane pairs share one random 32-B slot, 16 B each (k_sa_prefix2's entry read)
        const uint32_t sub = threadIdx.x & 1;
        for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 2; i < accesses;
             i += (uint64_t)gridDim.x * blockDim.x / 2) {
            uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + seed);
            const uint8_t* b = p + (h % lines) * 128 + ((h >> 40) & 3) * 32;
            const uint4 t = reinterpret_cast<const uint4*>(b)[sub];
            acc ^= t.x ^ t.y ^ t.z ^ t.w;
        }
    }
    if (SHAPE == 6) {  // SHAPE 5 with non-temporal loads
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const uint32_t sub = threadIdx.x & 1;
        for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 2; i < accesses;
             i += (uint64_t)gridDim.x * blockDim.x / 2) {
            uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + seed);
            const uint8_t* b = p + (h % lines) * 128 + ((h >> 40) & 3) * 32;
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + sub);
            acc ^= t.x ^ t.y ^ t.z ^ t.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 4096ull) << 20;  // MiB
    uint64_t accesses = argc > 2 ? strtoull(argv[2], 0, 10) : 100000000ull;
    int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int alloc = argc > 4 ? atoi(argv[4]) : 0;
    const unsigned mask = argc > 5 ? (unsigned)strtoul(argv[5], 0, 0) : 0x7fu;
    uint8_t* p;
    uint32_t* out;
    if (alloc == 0) CHECK(hipMalloc(&p, bytes));
    else CHECK(hipExtMallocWithFlags((void**)&p, bytes, alloc == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(p, 1, bytes));
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float ms;
    auto report = [&](const char* name, double acc, double bytes_per) {
        printf("{\"kernel\": \"%s\", \"alloc\": %d, \"buffer_MiB\": %llu, \"accesses\": %.0f, \"ms\": %.4f, \"accesses_per_s\": %.4g, "
               "\"GBps_at_shape_bytes\": %.1f, \"GBps_at_128B_lines\": %.1f}\n",
               name, alloc, (unsigned long long)(bytes >> 20), acc, ms, acc / (ms * 1e-3), acc * bytes_per / (ms * 1e-3) / 1e9,
               acc * (bytes_per < 128 ? 128 : bytes_per) / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    dim3 blk(1024), grd(cus * 2);
    // warm + timed stream
    hipLaunchKernelGGL(k_stream16, grd, blk, 0, 0, (const uint4*)p, bytes / 16, out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_stream16, grd, blk, 0, 0, (const uint4*)p, bytes / 16, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    report("stream16", (double)(bytes / 16), 16);
#define RUN(S, NAME, BPER)                                                                                    \
    if (mask & (1u << S)) {                                                                                 \
    hipLaunchKernelGGL(k_rand<S>, grd, blk, 0, 0, p, bytes, accesses, 1u, out);                             \
    CHECK(hipDeviceSynchronize());                                                                          \
    CHECK(hipEventRecord(e0));                                                                              \
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_rand<S>, grd, blk, 0, 0, p, bytes, accesses, 2u + r, out); \
    CHECK(hipEventRecord(e1));                                                                              \
    CHECK(hipEventSynchronize(e1));                                                                         \
    CHECK(hipEventElapsedTime(&ms, e0, e1));                                                                \
    ms /= reps;                                                                                             \
    report(NAME, (double)accesses, BPER);                                                                   \
    }
    RUN(0, "rand4", 4)
    RUN(1, "rand8x2", 16)
    RUN(2, "rand64", 64)
    RUN(3, "rand128", 128)
    RUN(4, "rand16", 16)
    RUN(5, "rand32pair", 32)
    RUN(6, "rand32pair_nt", 32)
    return 0;
}
