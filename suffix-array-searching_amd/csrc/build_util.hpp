// build_util.hpp -- host helpers shared by the index builders (sas_build.hip,
// sas_build40.hip): launch sizing, owning device buffers, error plumbing.
#pragma once
#include "common.hpp"

static inline unsigned grid_for(uint64_t count, unsigned block = 256) {
    uint64_t g = (count + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 262144) g = 262144;  // grid-stride beyond
    return (unsigned)g;
}

#define GRID_STRIDE(i, count) \
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (count); i += (uint64_t)gridDim.x * blockDim.x)

struct MaxOp {
    __device__ __host__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
struct MaxOp64 {
    __device__ __host__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    template <class T> T* as() { return static_cast<T*>(p); }
    int alloc(size_t bytes, const char* what) {
        if (p) { (void)hipFree(p); p = nullptr; }
        hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
        if (e != hipSuccess) {
            p = nullptr;
            sas_set_error(ENOMEM, std::string("hipMalloc(") + what + ", " + std::to_string(bytes) + " B): " +
                                      hipGetErrorString(e));
            return ENOMEM;
        }
        return 0;
    }
    // hipExtMallocWithFlags (e.g. hipDeviceMallocContiguous) when mflags != 0, plain
    // hipMalloc if that fails or mflags == 0
    int alloc_flags(size_t bytes, const char* what, unsigned mflags) {
        if (mflags) {
            if (p) { (void)hipFree(p); p = nullptr; }
            if (hipExtMallocWithFlags(&p, bytes ? bytes : 1, mflags) == hipSuccess) return 0;
            p = nullptr;
            (void)hipGetLastError();
        }
        return alloc(bytes, what);
    }
    void* release() { void* q = p; p = nullptr; return q; }
};

#define TRY(x) do { int rc_ = (x); if (rc_) return rc_; } while (0)


// Declared here, defined in sas_build40.hip: the bucketed builder of a packed
// 40-bit SA (n up to 2^40 as HBM allows).  sa5: device, 5*n + SAS_SA40_PAD bytes.
int build_sa_gpu40(const uint64_t* tw, uint64_t n, uint8_t* sa5, uint32_t* rounds_out, uint64_t* buckets_out);
// Part builder (sas_build_part): the SA rank range of part `part` of `parts`
// (contiguous 7-mer bins), packed 40-bit; returns the device buffer, the range and
// SA[rank_hi] (n if none).
int build_sa_part40(const uint64_t* tw, uint64_t n, uint32_t part, uint32_t parts, uint8_t** sa5_out,
                    uint64_t* rank_lo, uint64_t* count, uint64_t* next_pos, uint32_t* rounds_out);
