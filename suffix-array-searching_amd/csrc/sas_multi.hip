// sas_multi.hip -- one process driving several GPUs through the C ABI (SURVEY §8b:
// "Multi-GPU is via sas_build_multi(..., int ngpu, int mode /*REPLICATE,SHARD*/)").
//
// The production multi-GPU path is one process per GPU over torch.distributed /
// RCCL (bench.py, sas_amd/shard.py).  This is the same two modes for a host that
// wants a single handle over several devices, with no collective library:
//   REPLICATE: every device holds the whole index; a batch is cut into contiguous
//              query chunks (the reference's rayon chunking, sst/bin/bench.rs:558-573),
//              one host thread per device runs its chunk.
//   SHARD:     device g holds only part g of the SA rank space (sas_build_part);
//              every query is routed on the first device (sas_route_batch against the
//              parts' first suffixes), the queries of each part are searched on its
//              device, and the positions are scattered back into query order.
// A device may appear more than once in `devices` (two parts on one GPU), which
// is how the multi-part logic is tested on a one-GPU machine.
#include <thread>
#include <vector>

#include "build_util.hpp"
#include "common.hpp"

struct sas_multi {
    int mode = SAS_MULTI_REPLICATE;
    uint64_t n = 0;
    std::vector<int> devices;
    std::vector<sas_index*> parts;
    std::vector<uint64_t> splitters;  // text position of the first suffix of parts 1..P-1
};

static void multi_free(sas_multi* M) {
    if (!M) return;
    for (sas_index* x : M->parts)
        if (x) sas_free(x);
    delete M;
}

// Run f(g) for every part on its own host thread; first nonzero status wins (its
// message is copied into this thread's sas_last_error).
template <class F>
static int for_each_part(const sas_multi* M, F f) {
    const size_t P = M->devices.size();
    std::vector<int> rc(P, 0);
    std::vector<std::string> msg(P);
    std::vector<std::thread> th;
    for (size_t g = 0; g < P; g++) {
        th.emplace_back([&, g] {
            hipError_t e = hipSetDevice(M->devices[g]);
            rc[g] = e == hipSuccess ? f(g) : sas_errno_of(e);
            if (rc[g]) msg[g] = sas_last_error();
        });
    }
    for (auto& t : th) t.join();
    for (size_t g = 0; g < P; g++)
        if (rc[g]) {
            sas_set_error(rc[g], "part " + std::to_string(g) + ": " + msg[g]);
            return rc[g];
        }
    return 0;
}

extern "C" int sas_build_multi(const uint8_t* text, uint64_t n, const int* devices, int ngpu, int mode,
                               uint32_t flags, sas_multi** out) {
    if (!out || !devices || ngpu < 1 || ngpu > SAS_MAX_SPLIT + 1) SAS_FAIL(EINVAL, "sas_build_multi: bad arguments");
    if (mode != SAS_MULTI_REPLICATE && mode != SAS_MULTI_SHARD) SAS_FAIL(EINVAL, "sas_build_multi: unknown mode");
    if (flags & SAS_DEVICE_PTRS) SAS_FAIL(EINVAL, "sas_build_multi: text must be a host pointer");
    *out = nullptr;
    int count = 0;
    HIP_TRY(hipGetDeviceCount(&count));
    for (int g = 0; g < ngpu; g++)
        if (devices[g] < 0 || devices[g] >= count) SAS_FAIL(EINVAL, "sas_build_multi: no such device");
    sas_multi* M = new sas_multi();
    M->mode = mode;
    M->n = n;
    M->devices.assign(devices, devices + ngpu);
    M->parts.assign(ngpu, nullptr);
    int rc = for_each_part(M, [&](size_t g) {
        if (mode == SAS_MULTI_REPLICATE) return sas_build(text, n, nullptr, 0, flags, &M->parts[g]);
        return sas_build_part(text, n, (uint32_t)g, (uint32_t)ngpu, flags, &M->parts[g]);
    });
    if (!rc && mode == SAS_MULTI_SHARD) {
        for (int g = 1; g < ngpu && !rc; g++) {
            sas_stats st;
            uint64_t pos = 0;
            rc = sas_get_stats(M->parts[g], &st);
            if (!rc) rc = sas_copy_sa64(M->parts[g], st.rank_lo, 1, &pos, 0);
            M->splitters.push_back(pos);
        }
    }
    if (rc) {
        multi_free(M);
        return rc;
    }
    *out = M;
    return 0;
}

extern "C" int sas_multi_free(sas_multi* M) {
    multi_free(M);
    return 0;
}

extern "C" int sas_multi_parts(const sas_multi* M) { return M ? (int)M->parts.size() : 0; }

extern "C" int sas_multi_get_stats(const sas_multi* M, int part, sas_stats* out) {
    if (!M || part < 0 || part >= (int)M->parts.size()) SAS_FAIL(EINVAL, "sas_multi_get_stats: bad part");
    return sas_get_stats(M->parts[part], out);
}

extern "C" int sas_search_multi(const sas_multi* M, const uint8_t* qbytes, const uint64_t* qoff,
                                const uint32_t* qlen, uint64_t nq, int algo, uint64_t* out_pos, uint32_t flags) {
    if (!M) SAS_FAIL(EINVAL, "sas_search_multi: null handle");
    if (flags & SAS_DEVICE_PTRS) SAS_FAIL(EINVAL, "sas_search_multi: host pointers only");
    if (nq == 0) return 0;
    if (!qbytes || !qoff || !qlen || !out_pos) SAS_FAIL(EINVAL, "sas_search_multi: null argument");
    const size_t P = M->parts.size();
    if (M->mode == SAS_MULTI_REPLICATE) {
        return for_each_part(M, [&](size_t g) {
            const uint64_t s = nq * g / P, e = nq * (g + 1) / P;
            if (e == s) return 0;
            return sas_search_batch(M->parts[g], qbytes, qoff + s, qlen + s, e - s, algo, out_pos + s, nullptr,
                                    nullptr, flags);
        });
    }
    // SHARD: route on part 0's device, group by part (stable), search, scatter back
    std::vector<uint32_t> dest(nq);
    HIP_TRY(hipSetDevice(M->devices[0]));
    TRY(sas_route_batch(M->parts[0], M->splitters.data(), (uint32_t)M->splitters.size(), qbytes, qoff, qlen, nq,
                        dest.data(), nullptr, flags));
    std::vector<std::vector<uint64_t>> ids(P);
    for (uint64_t k = 0; k < nq; k++) ids[dest[k]].push_back(k);
    return for_each_part(M, [&](size_t g) {
        const std::vector<uint64_t>& I = ids[g];
        if (I.empty()) return 0;
        std::vector<uint64_t> off(I.size()), pos(I.size());
        std::vector<uint32_t> len(I.size());
        for (size_t j = 0; j < I.size(); j++) {
            off[j] = qoff[I[j]];
            len[j] = qlen[I[j]];
        }
        int rc = sas_search_batch(M->parts[g], qbytes, off.data(), len.data(), I.size(), algo, pos.data(), nullptr,
                                  nullptr, flags);
        if (rc) return rc;
        for (size_t j = 0; j < I.size(); j++) out_pos[I[j]] = pos[j];
        return 0;
    });
}
