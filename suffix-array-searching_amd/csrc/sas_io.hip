// sas_io.hip -- real-data inputs for the lookup path.
//
//   sas_read_fasta  replaces read_fasta_file (sas/util.rs:144-169): every record's
//                   sequence, concatenated; A/C/G/T/a/c/g/t -> 0..3 and EVERY other
//                   byte (N, IUPAC codes, ...) -> 0, exactly like the reference's
//                   zero-initialised `map` (:145-155).  FASTA ('>' headers, multi-line
//                   sequences) and FASTQ (4-line records) as needletail parses them;
//                   gzip input is rejected (ENOTSUP).
//   sas_kmer_keys   replaces the --human key extraction of sst/bin/bench.rs:58-76:
//                   vals[j] = 2-bit packed chars [j, j+k) & (4^k - 1) & i32::MAX,
//                   for j < min(n, limit + k - 1) - (k - 1), then vals[0] = i32::MAX.
#include "common.hpp"

#include <cstdio>
#include <vector>

static inline int code_of(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 0;  // sas/util.rs:145 map = [0; 256]
    }
}

extern "C" int sas_read_fasta(const char* path, uint8_t* out, uint64_t cap, uint64_t* len) {
    if (!path || !len) SAS_FAIL(EINVAL, "sas_read_fasta: null argument");
    FILE* f = fopen(path, "rb");
    if (!f) SAS_FAIL(ENOENT, std::string("sas_read_fasta: cannot open ") + path);
    struct Closer { FILE* f; ~Closer() { fclose(f); } } closer{f};
    std::vector<unsigned char> buf(1 << 20);
    size_t got = fread(buf.data(), 1, buf.size(), f);
    if (got >= 2 && buf[0] == 0x1f && buf[1] == 0x8b) SAS_FAIL(ENOTSUP, "sas_read_fasta: gzip input not supported");
    if (got == 0) { *len = 0; return 0; }
    const bool fastq = buf[0] == '@';
    if (!fastq && buf[0] != '>') SAS_FAIL(EINVAL, "sas_read_fasta: not a FASTA/FASTQ file");
    uint64_t n = 0;
    // line state machine: FASTA: '>' lines are headers, others sequence;
    // FASTQ: lines cycle header / sequence / '+' / quality.
    bool at_line_start = true, header = false;
    int fq_line = 0;  // FASTQ: 0 header, 1 seq, 2 plus, 3 qual
    bool seq_line = false;
    for (;;) {
        for (size_t i = 0; i < got; i++) {
            unsigned char c = buf[i];
            if (at_line_start) {
                at_line_start = false;
                if (fastq) {
                    seq_line = (fq_line == 1);
                } else {
                    header = (c == '>');
                    seq_line = !header;
                }
            }
            if (c == '\n') {
                at_line_start = true;
                if (fastq) fq_line = (fq_line + 1) & 3;
                continue;
            }
            if (c == '\r' || !seq_line) continue;
            if (out) {
                if (n >= cap) SAS_FAIL(ENOMEM, "sas_read_fasta: output buffer too small");
                out[n] = (uint8_t)code_of(c);
            }
            n++;
        }
        got = fread(buf.data(), 1, buf.size(), f);
        if (got == 0) break;
    }
    *len = n;
    return 0;
}

__global__ void k_kmer_keys(const uint8_t* __restrict__ text, uint64_t count, uint32_t k, uint32_t* __restrict__ out) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < count;
         j += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t dummy = 0;
        uint64_t w = pack_query_word(text + j, k, 0, &dummy);  // chars j..j+k in the top 2k bits
        uint64_t key = w >> (64 - 2 * k);
        out[j] = j == 0 ? 0x7fffffffu : ((uint32_t)key & 0x7fffffffu);
    }
}

extern "C" int sas_kmer_keys(const uint8_t* text, uint64_t n, uint32_t k, uint64_t limit, uint32_t* out,
                             uint64_t* count, uint32_t flags) {
    if (!count || (n && !text)) SAS_FAIL(EINVAL, "sas_kmer_keys: null argument");
    if (k == 0 || k > 16) SAS_FAIL(EINVAL, "sas_kmer_keys: k must be in 1..16 (u32 keys)");
    uint64_t end = n < limit + k - 1 ? n : limit + k - 1;
    uint64_t cnt = end >= k - 1 ? end - (k - 1) : 0;
    *count = cnt;
    if (cnt == 0 || !out) return 0;
    bool dev = flags & SAS_DEVICE_PTRS;
    void *dt = nullptr, *dout = nullptr;
    struct Free { void** p; ~Free() { if (*p) (void)hipFree(*p); } } f1{&dt}, f2{&dout};
    const uint8_t* tptr = text;
    uint32_t* optr = out;
    uint64_t tb = cnt + k - 1;
    if (!dev) {
        HIP_TRY(hipMalloc(&dt, tb + 64));
        HIP_TRY(hipMemcpy(dt, text, tb, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&dout, cnt * 4));
        tptr = static_cast<const uint8_t*>(dt);
        optr = static_cast<uint32_t*>(dout);
    }
    uint64_t blocks = (cnt + 255) / 256;
    if (blocks > 262144) blocks = 262144;
    hipLaunchKernelGGL(k_kmer_keys, dim3((unsigned)blocks), dim3(256), 0, 0, tptr, cnt, k, optr);
    HIP_TRY(hipGetLastError());
    if (!dev) HIP_TRY(hipMemcpy(out, optr, cnt * 4, hipMemcpyDeviceToHost));
    else HIP_TRY(hipDeviceSynchronize());
    return 0;
}
