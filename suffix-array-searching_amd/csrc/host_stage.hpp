// host_stage.hpp -- host-pointer search calls: reusable pinned staging and a chunked
// H2D / kernel / D2H pipeline over several HIP streams ("pinned staging
// buffers"; the reference hands host slices straight to its CPU search,
// sas/sa_search.rs:437-451).
//
// A call cuts its queries into chunks of at most SAS_STAGE_BYTES staged bytes.  Chunk c
// uses slot c % SAS_STAGE_SLOTS: the calling thread (with the host worker pool) fills the
// slot's pinned input while the GPU runs the chunks before it; the slot's stream copies the
// chunk in, searches it and copies the positions back into pinned memory, from where they
// are copied to the caller's array when the slot comes round again.  Slots (pinned + device
// buffers, streams) belong to the index and are reused by later calls; concurrent calls on
// one index each take their own set.
#pragma once
#include "common.hpp"

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#ifndef SAS_STAGE_BYTES
#define SAS_STAGE_BYTES (16u << 20)
#endif
#define SAS_STAGE_SLOTS 3
#ifndef SAS_STAGE_PACK_Q
#define SAS_STAGE_PACK_Q (1u << 19)  // queries per chunk when packing on the host
#endif

// ---------------------------------------------------------------- host worker pool
// A fixed set of worker threads (the CPU share of this process: its affinity mask, at most
// 16, or SAS_HOST_THREADS) that run `fn(part)` for part in [0, parts) together with the
// calling thread.  One job at a time; the workers are never joined (process lifetime).
class HostPool {
   public:
    // one pool per process: a child forked after the pool started has none of its worker
    // threads, so it builds its own (the parent's stays, unused)
    static HostPool& get() {
        static std::mutex mu;
        static HostPool* p = nullptr;
        std::lock_guard<std::mutex> g(mu);
        if (!p || p->pid_ != getpid()) p = new HostPool();
        return *p;
    }
    int size() const { return (int)workers_ + 1; }
    void run(int parts, const std::function<void(int)>& fn) {
        if (parts <= 1 || workers_ == 0) {
            for (int i = 0; i < parts; i++) fn(i);
            return;
        }
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            parts_ = parts;
            next_.store(0);
            active_ = workers_;
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return active_ == 0; });
        job_ = nullptr;
    }

   private:
    HostPool() {
        int n = 1;
        cpu_set_t cs;
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
        n = std::min(n, 16);
        if (const char* e = getenv("SAS_HOST_THREADS")) n = std::max(1, atoi(e));
        workers_ = (unsigned)(n > 1 ? n - 1 : 0);
        pid_ = getpid();
        for (unsigned i = 0; i < workers_; i++) std::thread([this] { loop(); }).detach();
    }
    void work() {
        for (int i; (i = next_.fetch_add(1)) < parts_;) (*job_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> g(mu_);
            if (--active_ == 0) done_cv_.notify_all();
        }
    }
    unsigned workers_ = 0;
    pid_t pid_ = 0;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int parts_ = 0;
    std::atomic<int> next_{0};
    unsigned active_ = 0;
    uint64_t gen_ = 0;
};

// memcpy split over the pool for large copies
static inline void par_memcpy(void* dst, const void* src, size_t bytes) {
    const size_t piece = 2u << 20;
    if (bytes < 2 * piece) {
        memcpy(dst, src, bytes);
        return;
    }
    const int parts = (int)std::min<size_t>((bytes + piece - 1) / piece, (size_t)HostPool::get().size() * 2);
    const size_t step = (bytes + parts - 1) / parts;
    HostPool::get().run(parts, [&](int i) {
        const size_t s = (size_t)i * step;
        if (s < bytes) memcpy((uint8_t*)dst + s, (const uint8_t*)src + s, std::min(step, bytes - s));
    });
}

// 8 byte codes (little-endian: byte k = char k) -> 16 bits, char 0 in bits 15..14 (the
// device's MSB-first packing, common.hpp pack4)
static inline uint64_t host_pack8(uint64_t v) {
    uint64_t x = __builtin_bswap64(v & 0x0303030303030303ull);
    x = (x | (x >> 6)) & 0x000F000F000F000Full;
    x = (x | (x >> 12)) & 0x000000FF000000FFull;
    return (x | (x >> 24)) & 0xFFFFull;
}

// BMI2 variant: pext gathers the 2 code bits of 8 bytes at once (char k at bits 2k, first
// char lowest); the 32 groups are then reversed (bytes by bswap, groups within a byte by two
// swaps) so that the first char lands in bits 63..62.
__attribute__((target("bmi2"))) static inline uint64_t host_pack32_bmi2(const uint8_t* q, uint64_t* bad) {
    uint64_t v[4];
    memcpy(v, q, 32);
    *bad |= v[0] | v[1] | v[2] | v[3];
    const uint64_t M = 0x0303030303030303ull;
    uint64_t p = __builtin_ia32_pext_di(v[0], M) | (__builtin_ia32_pext_di(v[1], M) << 16) |
                 (__builtin_ia32_pext_di(v[2], M) << 32) | (__builtin_ia32_pext_di(v[3], M) << 48);
    p = __builtin_bswap64(p);
    p = ((p >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((p & 0x0F0F0F0F0F0F0F0Full) << 4);
    return ((p >> 2) & 0x3333333333333333ull) | ((p & 0x3333333333333333ull) << 2);
}

__attribute__((target("bmi2"))) static uint8_t host_pack_words_bmi2(const uint8_t* q, uint32_t m, uint64_t nq,
                                                                    uint64_t* out) {
    uint64_t bad = 0;
    if (m == 32) {
        for (uint64_t i = 0; i < nq; i++, q += 32) out[i] = host_pack32_bmi2(q, &bad);
    } else {
        for (uint64_t i = 0; i < nq; i++, q += m) {
            uint8_t b[32] = {0};
            memcpy(b, q, m);
            out[i] = host_pack32_bmi2(b, &bad);
        }
    }
    uint8_t r = 0;
    for (int k = 0; k < 8; k++) r |= (uint8_t)(bad >> (8 * k));
    return r;
}

static inline bool host_has_bmi2() {
    static const bool has = __builtin_cpu_supports("bmi2");
    return has;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// AVX2 variant for m = 32 (one query = one 32-B vector): vpmaddubsw joins char pairs
// (4·c0 + c1), vpmaddwd joins pairs of those (64·c0 + 16·c1 + 4·c2 + c3, the byte of 4
// chars, first char high), vpshufb + a dword gather bring the 8 bytes together in char
// order, and a byte swap puts the first char in bits 63..62.
typedef char sas_v32qi __attribute__((vector_size(32)));
typedef short sas_v16hi __attribute__((vector_size(32)));
typedef int sas_v8si __attribute__((vector_size(32)));
typedef long long sas_v4di __attribute__((vector_size(32)));

__attribute__((target("avx2"))) static uint8_t host_pack32_words_avx2(const uint8_t* q, uint64_t nq, uint64_t* out) {
    const sas_v32qi pair = {4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1,
                            4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1, 4, 1};
    const sas_v16hi quad = {16, 1, 16, 1, 16, 1, 16, 1, 16, 1, 16, 1, 16, 1, 16, 1};
    const sas_v32qi pick = {0, 4, 8, 12, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128,
                            0, 4, 8, 12, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128, -128};
    sas_v4di acc = {0, 0, 0, 0};
    for (uint64_t i = 0; i < nq; i++, q += 32) {
        sas_v32qi v;
        memcpy(&v, q, 32);
        acc |= (sas_v4di)v;
        const sas_v16hi p2 = __builtin_ia32_pmaddubsw256(v, pair);
        const sas_v8si p4 = __builtin_ia32_pmaddwd256(p2, quad);
        const sas_v8si b = (sas_v8si)__builtin_ia32_pshufb256((sas_v32qi)p4, pick);
        const uint64_t w = (uint64_t)(uint32_t)b[0] | ((uint64_t)(uint32_t)b[4] << 32);
        out[i] = __builtin_bswap64(w);
    }
    const uint64_t bad = (uint64_t)(acc[0] | acc[1] | acc[2] | acc[3]);
    uint8_t r = 0;
    for (int k = 0; k < 8; k++) r |= (uint8_t)(bad >> (8 * k));
    return r;
}

static inline bool host_has_avx2() {
    static const bool has = __builtin_cpu_supports("avx2") && getenv("SAS_NO_AVX2") == nullptr;
    return has;
}
#endif

// fixed-length queries of m <= 32 chars -> 2-bit packed words (first char in bits 63..62,
// zero padded); returns the OR of every byte (a code > 3 shows in the bits 0xFC)
static inline uint8_t host_pack_words(const uint8_t* q, uint32_t m, uint64_t nq, uint64_t* out) {
#if !defined(__HIP_DEVICE_COMPILE__)
    if (m == 32 && host_has_avx2()) return host_pack32_words_avx2(q, nq, out);
#endif
    if (host_has_bmi2()) return host_pack_words_bmi2(q, m, nq, out);
    uint64_t bad = 0;
    if (m == 32) {
        for (uint64_t i = 0; i < nq; i++, q += 32) {
            uint64_t v[4];
            memcpy(v, q, 32);
            bad |= v[0] | v[1] | v[2] | v[3];
            out[i] = host_pack8(v[0]) << 48 | host_pack8(v[1]) << 32 | host_pack8(v[2]) << 16 | host_pack8(v[3]);
        }
    } else {
        for (uint64_t i = 0; i < nq; i++, q += m) {
            uint8_t b[32] = {0};
            memcpy(b, q, m);
            uint64_t v[4];
            memcpy(v, b, 32);
            bad |= v[0] | v[1] | v[2] | v[3];
            out[i] = host_pack8(v[0]) << 48 | host_pack8(v[1]) << 32 | host_pack8(v[2]) << 16 | host_pack8(v[3]);
        }
    }
    uint8_t r = 0;
    for (int k = 0; k < 8; k++) r |= (uint8_t)(bad >> (8 * k));
    return r;
}

// ---------------------------------------------------------------- staging slots
struct StageSlot {
    hipStream_t st = nullptr;
    uint8_t* h_in = nullptr;     // pinned: query bytes or packed words
    uint64_t* h_off = nullptr;   // pinned: ragged offsets (relative to the chunk)
    uint32_t* h_len = nullptr;   // pinned: ragged lengths
    uint64_t* h_out = nullptr;   // pinned: positions
    uint32_t* h_pr = nullptr;    // pinned: probe counts
    uint32_t* h_bad = nullptr;   // pinned: the chunk's invalid-code flag
    uint8_t* d_in = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_len = nullptr;
    uint64_t* d_out = nullptr;
    uint32_t* d_pr = nullptr;
    uint32_t* d_bad = nullptr;
    // the chunk in flight: its queries [s, e) of the call
    bool busy = false;
    uint64_t s = 0, e = 0;
};

struct StageSet {
    StageSlot slot[SAS_STAGE_SLOTS];
    uint64_t cap_bytes = 0;  // h_in / d_in
    uint64_t cap_q = 0;      // queries per chunk (offsets, lengths, positions, probes)
};

struct StagePool {
    std::mutex mu;
    std::vector<StageSet*> free_sets;
    int device = 0;
};

static inline void stage_set_free(StageSet* s) {
    if (!s) return;
    for (auto& sl : s->slot) {
        if (sl.st) (void)hipStreamSynchronize(sl.st);
        void* hp[] = {sl.h_in, sl.h_off, sl.h_len, sl.h_out, sl.h_pr, sl.h_bad};
        for (void* p : hp) if (p) (void)hipHostFree(p);
        void* dp[] = {sl.d_in, sl.d_off, sl.d_len, sl.d_out, sl.d_pr, sl.d_bad};
        for (void* p : dp) if (p) (void)hipFree(p);
        if (sl.st) (void)hipStreamDestroy(sl.st);
    }
    delete s;
}

static inline int stage_set_new(StageSet** out) {
    StageSet* s = new StageSet();
    s->cap_bytes = SAS_STAGE_BYTES;
    s->cap_q = SAS_STAGE_BYTES / 8;
    const uint64_t B = s->cap_bytes + 64, Q = s->cap_q;
    for (auto& sl : s->slot) {
        hipError_t e = hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_in, B, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_off, Q * 8, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_len, Q * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_out, Q * 8, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_pr, Q * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&sl.h_bad, 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_in, B);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_off, Q * 8);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_len, Q * 4);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_out, Q * 8);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_pr, Q * 4);
        if (e == hipSuccess) e = hipMalloc((void**)&sl.d_bad, 4);
        if (e != hipSuccess) {
            stage_set_free(s);
            const int c = sas_errno_of(e);
            sas_set_error(c, std::string("host staging buffers: ") + hipGetErrorString(e));
            return c;
        }
        if (sl.d_in) (void)hipMemset(sl.d_in + s->cap_bytes, 0, 64);  // slack after the last query
    }
    *out = s;
    return 0;
}

// Take a slot set of the index (allocating one on first use), give it back after the call.
struct StageLease {
    StagePool* pool = nullptr;
    StageSet* set = nullptr;
    ~StageLease() {
        if (!set) return;
        for (auto& sl : set->slot) {  // an early error return may leave chunks in flight
            if (sl.busy) (void)hipStreamSynchronize(sl.st);
            sl.busy = false;
        }
        std::lock_guard<std::mutex> g(pool->mu);
        pool->free_sets.push_back(set);
    }
};

static std::mutex g_stage_create_mu;

static inline int stage_acquire(const sas_index* x, StageLease* lease) {
    {
        std::lock_guard<std::mutex> g(g_stage_create_mu);
        if (!x->stage) {
            x->stage = new StagePool();
            x->stage->device = x->device;
        }
    }
    lease->pool = x->stage;
    {
        std::lock_guard<std::mutex> g(x->stage->mu);
        if (!x->stage->free_sets.empty()) {
            lease->set = x->stage->free_sets.back();
            x->stage->free_sets.pop_back();
            return 0;
        }
    }
    return stage_set_new(&lease->set);
}
