// common.hpp -- shared host/device pieces of libsas_amd.so.
//
// Data layout in HBM:
//   text   : 2-bit packed DNA, u64 words, MSB-first (char p lives in word p/32,
//            bits 63-2*(p%32) .. 62-2*(p%32)), followed by SAS_TEXT_PAD_WORDS
//            zero words.  Unsigned compare of packed words == lexicographic
//            compare of the chars (codes 0..3, sas/util.rs:9-15).
//   sa     : suffix array, u32[n] (sa_w = 4) or packed 40-bit little-endian
//            (sa_w = 5: entry i in bytes 5i..5i+4, 8 pad bytes) for n >= 2^32
//            or SAS_BUILD_SA40.
//   lcp    : u32[n], lcp[0] = 0, lcp[r] = lcp(SA[r-1], SA[r]).
//   stree  : STree<16,16>-shaped B+ tree over key16[r] = first 16 chars of
//            suffix SA[r] (zero padded), internal layers first, the leaf layer
//            IS the key16 array (padded with 0xFFFFFFFF to a node multiple).
//   top    : Eytzinger array of the first TOP_LEVELS levels of the lockstep
//            binary search: pivot SA value + 32-char key, staged into LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <errno.h>
#include <string>

#include "../../include/sas.h"
#include "../../include/sst.h"

#define SAS_TEXT_PAD_WORDS 4
// The binary search's pivots are prefix-relative blocks ("rel", round 4): levels in groups of
// up to 4 (SAS_REL_GROUP); a group rooted at level d0 holds one block per root node, 2^h u16
// slots for an h-level group (32 B at h = 4, 16 B below): slot 0 = P, the lcp (capped at
// SAS_REL_PMAX) of the block interval's bounds SA[l - 1] and SA[r] (0 at the array's ends;
// bit 15 flags a block with a pivot whose suffix ends before char P + 8),
// slots 1.. = chars [P, P + 8) of the pivots of its subtree in local Eytzinger order.  Every
// suffix strictly inside the interval, and every query q with SA[l - 1] < q <= SA[r], starts
// with those P chars, so chars [P, P + 8) decide key < q unless they tie (then the SA value
// and the text).  Levels 0..14 (groups rooted at 0, 4, 8 and a 3-level one at 12: 72.5 KiB)
// are staged in LDS, two workgroups a CU; past them one 16-B pair read of a block (one
// request) serves 4 levels.  PLAIN, LCP, LLCP and INLINE all read them (LCP / LLCP take
// exact lcps off the keys).  History: round 2 read a 16-B {32-char key, SA} entry per level
// (PLAIN 7.15 ms per 10^7 without pivots, 4.27 with 23 levels, 2.71 with 30;
// profiles/r2/ab_top2_*.txt), round 4 first 3 levels of 16-char keys in a 128-B line (2.97 ms
// at 23 levels), then rel blocks past 14 LDS levels of 16-char keys (1.70 ms at 26).  The
// depth is a build parameter (SAS_BUILD_TOP2_LEVELS(L) in sas.h, rounded up to the group
// grid), never derived from free memory: the default SAS_TOP2_CACHE_LEVELS reach 27 levels
// with 273 MiB of blocks.
#define SAS_TOP2_CACHE_LEVELS 27
#define SAS_TOP2_MAX_LEVELS 31
#define SAS_REL_GROUP 4
#define SAS_REL_PMAX 24          // P + 8 <= 32: q's chars [P, P + 8) come from its first word
#define SAS_REL_LDS_LEVELS 15    // levels staged in LDS
#define SAS_REL_LDS_BYTES (32 * (1 + 16 + 256) + 16 * 4096)  // their blocks: 74272 B
#define SAS_REL_MAX_GROUPS 8     // 4 LDS groups + 4 of levels 15..30
struct RelLayout {
    uint64_t base[SAS_REL_MAX_GROUPS];  // byte offset of group g
    uint8_t d0[SAS_REL_MAX_GROUPS];     // its root level
    uint8_t h[SAS_REL_MAX_GROUPS];      // its levels (block bytes: 32 at h = 4, else 16)
    uint32_t groups;                    // groups in all
    uint32_t lds_groups;                // the first ones, staged in LDS
    uint32_t levels;                    // levels the blocks serve
    uint32_t lds_bytes;                 // bytes of the LDS groups (a multiple of 16)
    uint64_t bytes;                     // the array's bytes
};
// the layout for a depth of L levels (clamped to the iteration count; past the LDS levels
// rounded up to whole 4-level groups)
static inline void rel_layout(uint32_t iters, uint32_t L, RelLayout* y) {
    *y = RelLayout{};
    uint32_t R = L < iters ? L : iters;
    if (R > SAS_REL_LDS_LEVELS)
        R = SAS_REL_LDS_LEVELS + (R - SAS_REL_LDS_LEVELS + SAS_REL_GROUP - 1) / SAS_REL_GROUP * SAS_REL_GROUP;
    if (R > iters) R = iters;
    uint64_t b = 0;
    uint32_t g = 0;
    for (uint32_t d0 = 0; d0 < R; g++) {
        uint32_t h = SAS_REL_GROUP;
        if (d0 < SAS_REL_LDS_LEVELS && d0 + h > SAS_REL_LDS_LEVELS) h = SAS_REL_LDS_LEVELS - d0;
        if (d0 + h > R) h = R - d0;
        y->base[g] = b;
        y->d0[g] = (uint8_t)d0;
        y->h[g] = (uint8_t)h;
        b += (uint64_t)(h == SAS_REL_GROUP ? 32 : 16) << d0;
        d0 += h;
        if (d0 <= SAS_REL_LDS_LEVELS) {
            y->lds_groups = g + 1;
            y->lds_bytes = (uint32_t)b;
        }
    }
    y->groups = g;
    y->levels = R;
    y->bytes = b;
}
#define SAS_STREE_B 16                // keys per node / branching factor - 1
#define SAS_STREE_MAX_LAYERS 16
#define SAS_STREE_LDS_NODES 1024      // <= 64 KiB of top S-tree layers in LDS
#define SAS_KEY_MAX 0xFFFFFFFFu       // padding key of the SA S-tree (unsigned)
#define SAS_SECTOR_FAN 9              // sector tree: 8 separators, 9 children per 32-B node
#define SAS_SECTOR_MAX_LAYERS 24
#define SAS_SECTOR_LDS_NODES 2048     // <= 64 KiB of top sector-tree layers in LDS
#define SAS_QUAD_FAN 17               // quad tree, absolute nodes: 16 u32 separators, 17 children
#define SAS_QUAD_RFAN 31              // quad tree, prefix-relative nodes: 30 u16 separators, 31 children
#define SAS_QUAD_RMAXD 13             // relative nodes: at most 13 shared chars in the 27-bit header
#define SAS_MAX_SPLIT 1024            // sharded mode: at most 1025 parts
#define SAS_QUAD_MAX_INNER 10         // inner layers the (unrolled) descent supports; leaf index < 2^32
#define SAS_QUAD_MAX_LDS 4            // of which at most this many LDS-staged
#define SAS_QUAD_MAX_LAYERS 16
#define SAS_QUAD_LDS_NODES 1024       // <= 64 KiB of top quad-tree layers in LDS

// ---------------------------------------------------------------- errors
void sas_set_error(int code, const std::string& msg);
int sas_errno_of(hipError_t e);

#define SAS_FAIL(code, msg)                  \
    do {                                     \
        sas_set_error((code), (msg));        \
        return (code);                       \
    } while (0)

#define HIP_TRY(expr)                                                              \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess) {                                                    \
            int c_ = sas_errno_of(e_);                                             \
            sas_set_error(c_, std::string(#expr) + ": " + hipGetErrorString(e_));  \
            return c_;                                                             \
        }                                                                          \
    } while (0)

// ---------------------------------------------------------------- index structs
struct StagePool;                     // host_stage.hpp: pinned staging of host-pointer calls
void sas_stage_pool_free(StagePool*);  // sas_search.hip
struct sas_index {
    uint64_t n = 0;               // text length (chars)
    uint64_t sa_n = 0;            // SA entries held (= n, or a shard's rank range)
    uint64_t rank_lo = 0;         // global rank of sa[0]
    uint64_t next_pos = 0;        // global SA[rank_lo + sa_n] (n if none): answer when q > every held suffix
    int device = 0;
    int num_cus = 256;
    uint64_t* text_w = nullptr;  // packed text
    uint64_t text_words = 0;
    uint8_t* sa = nullptr;        // sa_w bytes per entry (SaView<4> / SaView<5>)
    uint32_t sa_w = 4;
    uint32_t* lcp = nullptr;
    uint8_t* prefix = nullptr;    // SAS_BUILD_PREFIX: first rank per p-char key, entry j for key
    uint32_t prefix_chars = 0;    // prefix_key_lo + j; prefix_w bytes per entry (4: u32; 5: packed
    uint32_t prefix_w = 4;        // 40-bit, for a 40-bit SA; 16 G: G inline slots)
    uint64_t prefix_key_lo = 0;   // whole index: 0 and 4^p + 1 entries; a part (a rank range of the
    uint64_t prefix_entries = 0;  // SA): its first key .. its last key + 2 (pt_slot, sas_search.hip)
    bool prefix_hi40 = false;     // inline slots of a text >= 2^32 chars: bits 32..39 of each slot's SA
                                  // value in slot 1's rank word (only slot 0's rank is read); with two
                                  // slots also bits 32..39 of slot 0's rank (a part of >= 2^32 suffixes)
    uint4* llcp = nullptr;        // SAS_BUILD_LLCP: {SA[m], Llcp, Rlcp, 2 x 16 chars} per rank m (sas_build.hip)
    uint32_t* stree = nullptr;   // all nodes, 16 u32 each
    uint64_t stree_nodes = 0;
    uint32_t stree_height = 0;
    uint64_t stree_off[SAS_STREE_MAX_LAYERS] = {};
    uint32_t stree_lds_layers = 0;
    uint32_t stree_lds_nodes = 0;
    uint8_t* rel = nullptr;       // the prefix-relative pivot blocks (rel_lay), their first groups staged in LDS
    RelLayout rel_lay{};
    uint32_t iters = 0;           // ilog2(n) + 1
    uint32_t* scratch = nullptr;  // device flag word(s) for kernels (invalid query codes)
    // sector tree (SAS_ALGO_SECTOR): 32-B nodes
    uint32_t* sec_inner = nullptr;   // internal nodes, 8 u32 16-char separators each, root first
    uint4* sec_leaves = nullptr;     // leaf i = 2 x uint4: {key(2i) lo,hi, key(2i+1) lo,hi},
                                     // {sa(2i) lo32, sa(2i+1) lo32, hi8(2i) | hi8(2i+1) << 8, 0}
    uint64_t sec_leaf_count = 0;
    uint64_t sec_off[SAS_SECTOR_MAX_LAYERS] = {};  // node offsets of the internal layers
    uint32_t sec_inner_layers = 0;   // internal layers (the leaf layer not counted)
    uint32_t sec_lds_layers = 0;
    uint32_t sec_lds_nodes = 0;
    uint64_t sec_inner_nodes = 0;
    // quad tree (SAS_ALGO_QUAD): 64-B nodes, one 4-lane cooperative load each
    uint4* quad_inner = nullptr;     // internal nodes (4 x uint4 each), root first: prefix-relative
                                     // (quad_fan 31) or 16 u32 16-char separators (quad_fan 17)
    uint4* quad_leaves = nullptr;    // entry x = {key lo, key hi, sa lo32, sa bits 32..39}; leaf = 4 entries
                                     // compact (SAS_BUILD_QUAD_COMPACT): entry x = key64 only; leaf = 8 entries
    uint32_t quad_compact = 0;       // 1: key-only leaves, SA values read from `sa`
    uint64_t quad_leaf_count = 0;
    uint64_t quad_off[SAS_QUAD_MAX_LAYERS] = {};
    uint32_t quad_fan = SAS_QUAD_RFAN;  // children per inner node; 31 = prefix-relative layout
    uint32_t quad_inner_layers = 0;
    uint32_t quad_lds_layers = 0;
    uint32_t quad_lds_nodes = 0;
    uint64_t quad_inner_nodes = 0;
    // SAS_BUILD_TAGGED: `sa` holds u64 entries {SA 40 bits | chars [tag_p, tag_p + 12) << 40}
    // (sa_w = 8) and tag_table[x] = {first rank whose tag_p-char key is >= x (40 bits) |
    // min(rank count of key x, 2^24 - 1) << 40} for x in [0, 4^tag_p]
    uint64_t* tag_table = nullptr;
    uint32_t tag_p = 0;
    // SAS_BUILD_TAG_LINES (no SA, no tag_table): line b = 128 B {header u64: overflow offset |
    // min(count, 2^24 - 1) << 40; u16 hi[20]; u32 lo[20]}, slot j = the 48-bit entry
    // {SA (tag_sb bits) | tag << tag_sb} of rank first + j split as hi[j] << 32 | lo[j]
    // (tl_slot below; an SA field of all ones stands for rank sa_n); tag_ovf holds the entries
    // of ranks first + SAS_TL_SLOTS .. first + count (u64, same format) of every bucket with
    // count >= SAS_TL_SLOTS, bucket after bucket; tag_first[b] = bucket b's first rank
    uint64_t* tag_lines = nullptr;
    uint64_t* tag_ovf = nullptr;
    uint64_t tag_ovf_n = 0;
    uint64_t* tag_first = nullptr;
    uint32_t tag_sb = 40;          // SA bits of a line entry: max(32, bit length of n)
    uint64_t* text2 = nullptr;     // SAS_BUILD_TAG_LINES: the packed text again, 64 B off the
    void* text2_base = nullptr;    // 128-B line grid (text2 = text2_base + 64 B; tl_text)
    sas_stats stats = {};
    mutable StagePool* stage = nullptr;  // created by the first host-pointer search
    mutable hipMemPool_t route_pool = nullptr;  // stream-ordered scratch of sas_route_pack (first use)
};

struct sst_index {
    int layout = 0;
    uint32_t flags = 0;
    uint64_t n = 0;
    uint32_t B = 16, N = 16;
    uint32_t* nodes = nullptr;  // device: STree nodes / Eytzinger vals / sorted vals
    uint64_t words = 0;         // u32 words in `nodes`
    uint32_t height = 0;
    uint64_t off[SAS_STREE_MAX_LAYERS] = {};
    uint64_t layer_nodes[SAS_STREE_MAX_LAYERS] = {};
    uint32_t lds_layers = 0;
    uint32_t lds_nodes = 0;
    int num_cus = 256;
    uint32_t* prefix_map = nullptr;  // PartitionedSTree16M
    uint4* direct = nullptr;         // SST_DIRECT_MAP entries [2^shift... see sst.hip]
    uint64_t pmap_words = 0;
    uint32_t shift = 0;
    uint32_t parts = 0;
    // SST_PARTITIONED*: the root window's element stride per part and the first step's
    // multiplier (sst/partitioned_s_tree.rs:654-831), nodes per part (Compact)
    uint64_t root_stride = 16, l1_mul = 17;
    uint64_t bpp = 0;
};

// ---------------------------------------------------------------- suffix-array element access
#define SAS_SA40_PAD 8           // bytes after a packed 40-bit SA (aligned 8-B reads)
#define SAS_SA40_MAX (1ull << 40)
// SAS_BUILD_LLCP entries: SA (40 bits) | Llcp << 40 | Rlcp << 52 + 16 chars after each lcp
#define SAS_LLCP_CAP 4095u

// W = 8: the tagged SA of SAS_BUILD_TAGGED, u64 entries {SA 40 bits | 12 chars << 40}
// (sas_build.hip, build_tagged): the SA value is the low 40 bits.
#define SAS_TAG_CHARS 12
// Bucket lines (SAS_BUILD_TAG_LINES): 20 entries of 48 bits per 128-B line, {SA | tag << sb}
// with sb = max(32, bit length of n) SA bits and 48 - sb tag bits (the bits of chars [p, ...)
// after the bucket's p chars: 13 bits at n = 2^34, 16 below 2^32).  In the line the entry is
// split: u16 hi[j] = entry >> 32 at u16 4 + j, u32 lo[j] at u32 12 + j, so an 8-lane group
// reading 16 B per lane holds the header and hi[0..3] (lane 0), hi[4..11], hi[12..19] (lanes
// 1, 2) and lo[4s - 12 ..] (lanes 3..7).
#define SAS_TL_SLOTS 20
__host__ __device__ __forceinline__ uint64_t tl_sa_mask(uint32_t sb) { return (1ull << sb) - 1; }
__host__ __device__ __forceinline__ uint32_t tl_tag_bits(uint32_t sb) { return 48 - sb; }
// the tag of a packed 32-char key: tb bits from char p (the bucket's p chars are the key's first)
__host__ __device__ __forceinline__ uint32_t tl_tag_of_key(uint64_t k64, uint32_t p, uint32_t tb) {
    return (uint32_t)((k64 << (2 * p)) >> (64 - tb));
}
__device__ __forceinline__ uint64_t tl_slot(const uint64_t* __restrict__ lines, uint64_t b, uint32_t j) {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(lines + b * 16);
    const uint32_t* l = reinterpret_cast<const uint32_t*>(lines + b * 16);
    return ((uint64_t)h[4 + j] << 32) | l[12 + j];
}
template <int W>
struct SaView {
    const uint8_t* p;
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const {
        if (W == 4) return reinterpret_cast<const uint32_t*>(p)[i];
        if (W == 8) return reinterpret_cast<const uint64_t*>(p)[i] & (SAS_SA40_MAX - 1);
        // 5-byte entry at byte 5i: two aligned u32 loads (same 128-B line except
        // when straddling one) and a funnel shift
        uint64_t o = 5 * i;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(p + (o & ~3ull));
        uint64_t v = ((uint64_t)w[1] << 32) | w[0];
        return (v >> (8 * (o & 3))) & (SAS_SA40_MAX - 1);
    }
};

// Writes: byte stores, so neighbouring entries written by other lanes never race.
template <int W>
__device__ __forceinline__ void sa_put(uint8_t* p, uint64_t i, uint64_t v) {
    if (W == 8) {
        reinterpret_cast<uint64_t*>(p)[i] = v;
        return;
    }
    if (W == 4) {
        reinterpret_cast<uint32_t*>(p)[i] = (uint32_t)v;
        return;
    }
    uint8_t* b = p + 5 * i;
#pragma unroll
    for (int k = 0; k < 5; k++) b[k] = (uint8_t)(v >> (8 * k));
}

// ---------------------------------------------------------------- 4-lane (quad) groups
#define QUAD_G 4

// Sum over the 4 lanes of a quad with DPP quad_perm moves (VALU, no LDS crossbar):
// [1,0,3,2] = lane ^ 1 (0xB1), [2,3,0,1] = lane ^ 2 (0x4E).
__device__ __forceinline__ uint32_t quad_sum(uint32_t c) {
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xF, 0xF, false);
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xF, 0xF, false);
    return c;
}

// 4-bit mask of the group's lanes with b set (bit j = lane j of the group)
__device__ __forceinline__ uint32_t quad_mask(bool b) {
    uint64_t bal = __ballot(b);
    return (uint32_t)(bal >> (threadIdx.x & 60)) & 0xFu;
}

// ---------------------------------------------------------------- device helpers
// Non-temporal loads for arrays far larger than the 256 MiB Infinity Cache (more than
// SAS_NT_BYTES): they then do not evict the upper tree layers from L2.  Measured on the
// quad tree (sas_search.hip, quad_nt_from): -6% at n = 2^30; on a level that partly
// fits the Infinity Cache (554 MB) they made the kernel slower.
#ifndef SAS_NT_BYTES
#define SAS_NT_BYTES (3ull * (256ull << 20))
#endif
typedef unsigned int sas_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load4(const uint4* p) {
    const sas_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const sas_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 load4(const uint4* p, bool nt) { return nt ? nt_load4(p) : *p; }

__device__ __forceinline__ uint64_t chars_mask(uint32_t c) {
    // top 2c bits set, c in [0, 32]
    return c == 0 ? 0ull : (~0ull << (64 - 2 * c));
}

// 32 chars of the packed text starting at char p (zero beyond n: padding).
__device__ __forceinline__ uint64_t text_chars32(const uint64_t* __restrict__ tw, uint64_t p) {
    uint64_t w = p >> 5;
    uint32_t s = (uint32_t)(p & 31) << 1;
    uint64_t a = tw[w];
    uint64_t b = tw[w + 1];
    return s ? ((a << s) | (b >> (64 - s))) : a;
}

// Pack 4 byte-codes (little-endian u32, each byte 0..3) into 8 bits, first char high.
__device__ __forceinline__ uint32_t pack4(uint32_t x) {
    return ((x & 3u) << 6) | (((x >> 8) & 3u) << 4) | (((x >> 16) & 3u) << 2) | ((x >> 24) & 3u);
}

static __device__ __forceinline__ uint64_t pack_query_word_slow(const uint8_t* __restrict__ q, uint32_t m,
                                                                     uint32_t base, uint32_t* bad);

// Word j (chars 32j .. 32j+31, zero padded) of a byte-coded query of length m.
__device__ __forceinline__ uint64_t pack_query_word(const uint8_t* __restrict__ q, uint32_t m, uint32_t j,
                                                    uint32_t* bad) {
    uint32_t base = j * 32;
    uint64_t w = 0;
    if (base >= m) return 0;
    if (base + 32 <= m && ((((uintptr_t)(q + base)) & 15) == 0)) {
        const uint4* p = reinterpret_cast<const uint4*>(q + base);
        uint4 a = p[0], b = p[1];
        uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            *bad |= v[i] & 0xFCFCFCFCu;
            w = (w << 8) | pack4(v[i]);
        }
        return w;
    }
    return pack_query_word_slow(q, m, base, bad);
}

// Unaligned / partial word.
static __device__ __forceinline__ uint64_t pack_query_word_slow(const uint8_t* __restrict__ q, uint32_t m,
                                                                     uint32_t base, uint32_t* bad) {
    uint64_t w = 0;
    // Unaligned / partial word: read the 16-B aligned blocks that intersect the
    // c valid bytes (each block holds at least one valid byte, so it can never
    // touch a page outside the buffer) and realign with v_alignbyte_b32.
    uint32_t c = m - base < 32 ? m - base : 32;
    // aligned block pointer by pointer arithmetic (an int-to-pointer cast would drop
    // the global address space and compile to FLAT loads)
    uint32_t s = (uint32_t)(((uintptr_t)(q + base)) & 15);
    const uint4* p = reinterpret_cast<const uint4*>(q + base - s);
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4 b0 = p[0];
    uint4 b1 = (s + c > 16) ? p[1] : z;
    uint4 b2 = (s + c > 32) ? p[2] : z;
    uint32_t d[13] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w, 0u};
    uint32_t qi = s >> 2, sb = s & 3;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t lo = d[k], hi = d[k + 1];
        lo = (qi == 1) ? d[k + 1] : lo;
        hi = (qi == 1) ? d[k + 2] : hi;
        lo = (qi == 2) ? d[k + 2] : lo;
        hi = (qi == 2) ? d[k + 3] : hi;
        lo = (qi == 3) ? d[k + 3] : lo;
        hi = (qi == 3) ? d[k + 4] : hi;
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sb);
        int valid = (int)c - 4 * k;  // bytes of this dword inside the query
        uint32_t bm = valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * valid)));
        v &= bm;
        *bad |= v & 0xFCFCFCFCu;
        w = (w << 8) | pack4(v);
    }
    return w;
}

template <int QW>
struct QueryRegs {
    uint64_t w[QW];
    const uint8_t* bytes;
    uint32_t m;

    __device__ __forceinline__ void load(const uint8_t* q, uint32_t len, uint32_t* bad) {
        bytes = q;
        m = len;
#pragma unroll
        for (int j = 0; j < QW; j++) w[j] = pack_query_word(q, len, j, bad);
    }
    // aligned word j (static select over the register copy; beyond QW, repack from bytes).
    // An instance with QW <= 2 only ever runs batches whose queries fit its words (qw_for:
    // 1 for m <= 32, 2 for m <= 64; an unknown longest query gives 4), so past them it is 0
    // and no repacking code is compiled (the register spills it cost, round 6); the two
    // kernels that run longer queries on two register words use QueryRegsRepack
    __device__ __forceinline__ uint64_t word(uint32_t j) const {
        if (j < (uint32_t)QW) {
            uint64_t r = w[0];
#pragma unroll
            for (int k = 1; k < QW; k++) r = (j == (uint32_t)k) ? w[k] : r;
            return r;
        }
        if (QW <= 2) return 0;
        uint32_t dummy = 0;
        return pack_query_word(bytes, m, j, &dummy);
    }
    // 32 chars starting at char offset off (unaligned)
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        uint32_t j = off >> 5, s = (off & 31) << 1;
        uint64_t a = word(j);
        if (s == 0) return a;
        return (a << s) | (word(j + 1) >> (64 - s));
    }
};

// QueryRegs for a kernel launched only with m <= 32 QW: every word is in registers and the
// words past them are 0, so no code repacks words from the bytes (k_sa_quad_llcp)
template <int QW>
struct QueryRegsExact : QueryRegs<QW> {
    __device__ __forceinline__ uint64_t word(uint32_t j) const {
        uint64_t r = 0;
#pragma unroll
        for (int k = 0; k < QW; k++) r = (j == (uint32_t)k) ? this->w[k] : r;
        return r;
    }
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        const uint32_t j = off >> 5, s = (off & 31) << 1;
        const uint64_t a = word(j);
        if (s == 0) return a;
        return (a << s) | (word(j + 1) >> (64 - s));
    }
};

// QueryRegs whose words past the registers are repacked from the bytes at any QW (k_sa_quad4x
// and k_sa_quad_llcp hold two register words for queries of any length)
template <int QW>
struct QueryRegsRepack : QueryRegs<QW> {
    __device__ __forceinline__ uint64_t word(uint32_t j) const {
        if (j < (uint32_t)QW) return QueryRegs<QW>::word(j);
        uint32_t dummy = 0;
        return pack_query_word(this->bytes, this->m, j, &dummy);
    }
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        const uint32_t j = off >> 5, s = (off & 31) << 1;
        const uint64_t a = word(j);
        if (s == 0) return a;
        return (a << s) | (word(j + 1) >> (64 - s));
    }
};

// Rust slice order `t[p..n] < q`, with the first h chars known equal.
// Returns lt; *lcp = lcp(t[p..n], q) (capped at min(n-p, m)).
template <int QW, class Q>
__device__ __forceinline__ bool suffix_less_from(const uint64_t* __restrict__ tw, uint64_t n, uint64_t p,
                                                 const Q& q, uint32_t h, uint32_t* lcp) {
    uint64_t lenS = n - p;
    uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    if (h < L) {
        // consecutive 32-char windows share a text word: carry it, one new load per window
        uint64_t w = (p + h) >> 5;
        const uint32_t sh = (uint32_t)((p + h) & 31) << 1;
        uint64_t lo = tw[w];
        for (uint32_t off = h; off < L; off += 32) {
            const uint64_t hi = tw[++w];
            const uint32_t c = L - off < 32 ? L - off : 32;
            const uint64_t mk = chars_mask(c);
            const uint64_t a = (sh ? ((lo << sh) | (hi >> (64 - sh))) : lo) & mk;
            const uint64_t b = q.chars32(off) & mk;
            if (a != b) {
                *lcp = off + (uint32_t)(__clzll(a ^ b) >> 1);
                return a < b;
            }
            lo = hi;
        }
    }
    *lcp = L;
    return lenS < (uint64_t)q.m;
}

// suffix_less_from reading the packed text as 16-B aligned word pairs: a compare that runs
// over several 32-char windows costs half the load instructions (and L1->L2 requests) of
// one 8-B load per window.  The text carries SAS_TEXT_PAD_WORDS zero words, so the pair
// after the last word is readable.
template <int QW, class Q>
__device__ __forceinline__ bool suffix_less_from_x2(const uint64_t* __restrict__ tw, uint64_t n, uint64_t p,
                                                    const Q& q, uint32_t h, uint32_t* lcp) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const uint64_t lenS = n - p;
    const uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    if (h < L) {
        uint64_t w = (p + h) >> 5;
        const uint32_t sh = (uint32_t)((p + h) & 31) << 1;
        const u64x2* tp = reinterpret_cast<const u64x2*>(tw);
        u64x2 pr = tp[w >> 1];
        uint64_t lo = (w & 1) ? pr.y : pr.x;
        bool nxt = (w & 1) == 0;  // pr.y is word w + 1
        for (uint32_t off = h; off < L; off += 32) {
            uint64_t hi;
            if (nxt) {
                hi = pr.y;
            } else {
                pr = tp[(w + 1) >> 1];
                hi = pr.x;
            }
            nxt = !nxt;
            w++;
            const uint32_t c = L - off < 32 ? L - off : 32;
            const uint64_t mk = chars_mask(c);
            const uint64_t a = (sh ? ((lo << sh) | (hi >> (64 - sh))) : lo) & mk;
            const uint64_t b = q.chars32(off) & mk;
            if (a != b) {
                *lcp = off + (uint32_t)(__clzll(a ^ b) >> 1);
                return a < b;
            }
            lo = hi;
        }
    }
    *lcp = L;
    return lenS < (uint64_t)q.m;
}

// suffix_less_from_x2 with the first PRE word pairs the compare can need loaded together:
// a positive query matches its own suffix to the end, so the compare always runs over every
// window and the plain loop's pair loads form a dependent chain ((m - h) / 64 round trips).
// Windows past the preloaded 2 PRE - 2 continue as suffix_less_from_x2 does.
// tw2: the same text 64 B off the 128-B line grid (bucket lines, sas_index::text2), or tw: the
// pairs are read from the copy in which they lie in one 128-B line when only one copy has that
// (any run of <= 4 pairs lies in one line of one of the two copies).
template <int PRE, class Q>
__device__ __forceinline__ bool suffix_less_from_pre(const uint64_t* __restrict__ tw, const uint64_t* __restrict__ tw2,
                                                     uint64_t n, uint64_t p, const Q& q, uint32_t h, uint32_t* lcp) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const uint64_t lenS = n - p;
    const uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    if (h < L) {
        const uint64_t w0 = (p + h) >> 5;
        const uint32_t sh = (uint32_t)((p + h) & 31) << 1;
        const uint32_t o = (uint32_t)(w0 & 1);
        const uint32_t nwin = (L - h + 31) >> 5;  // windows; window r reads words w0 + r, w0 + r + 1
        const uint32_t npair = (o + nwin) / 2 + 1;  // pairs holding words w0 .. w0 + nwin
        const uint64_t P0 = w0 >> 1, P1 = P0 + (npair < (uint32_t)PRE ? npair : (uint32_t)PRE) - 1;
        const bool two = (P0 >> 3) != (P1 >> 3) && ((P0 + 4) >> 3) == ((P1 + 4) >> 3);
        const u64x2* tp = reinterpret_cast<const u64x2*>(two ? tw2 : tw) + P0;
        uint64_t W[2 * PRE];
#pragma unroll
        for (int j = 0; j < PRE; j++) {
            const u64x2 v = (uint32_t)j < npair ? tp[j] : u64x2{0ull, 0ull};
            W[2 * j] = v.x;
            W[2 * j + 1] = v.y;
        }
#pragma unroll
        for (int r = 0; r < 2 * PRE - 2; r++) {
            const uint32_t off = h + 32u * r;
            if (off >= L) {
                *lcp = L;
                return lenS < (uint64_t)q.m;
            }
            const uint64_t lo = o ? W[r + 1] : W[r], hi = o ? W[r + 2] : W[r + 1];
            const uint32_t c = L - off < 32 ? L - off : 32;
            const uint64_t mk = chars_mask(c);
            const uint64_t a = (sh ? ((lo << sh) | (hi >> (64 - sh))) : lo) & mk;
            const uint64_t b = q.chars32(off) & mk;
            if (a != b) {
                *lcp = off + (uint32_t)(__clzll(a ^ b) >> 1);
                return a < b;
            }
        }
        const uint32_t h2 = h + 32u * (2 * PRE - 2);
        if (h2 < L) return suffix_less_from_x2<1>(tw, n, p, q, h2, lcp);
    }
    *lcp = L;
    return lenS < (uint64_t)q.m;
}

// Same decision when the first 32 chars of the suffix are already known (key).
template <int QW, class Q>
__device__ __forceinline__ bool suffix_less_key(const uint64_t* __restrict__ tw, uint64_t n, uint64_t p,
                                                uint64_t key, const Q& q, uint32_t h,
                                                uint32_t* lcp) {
    uint64_t lenS = n - p;
    uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    if (h < 32) {
        uint32_t c = L < 32 ? L : 32;
        uint64_t mk = chars_mask(c);
        uint64_t a = key & mk, b = q.w[0] & mk;
        if (a != b) {
            *lcp = (uint32_t)(__clzll(a ^ b) >> 1);
            return a < b;
        }
        if (L <= 32) {
            *lcp = L;
            return lenS < (uint64_t)q.m;
        }
        h = 32;
    }
    return suffix_less_from<QW>(tw, n, p, q, h, lcp);
}

// ---------------------------------------------------------------- wave-staged queries
// The 64 queries of a wavefront (consecutive query ids) usually sit in one contiguous span
// of the caller's buffer.  Loading them lane by lane costs one L1->L2 request per 16-B piece
// of every query (the configs[3] shape: ~12 of its ~19 requests per lookup); instead the
// wave reads the span once, coalesced (lane l reads 16-B block l, l+64, ...), packs it 2 bits
// per char into LDS, and each lane reads its query words from there.  A span longer than
// SAS_WQ_WORDS - 1 words (16,608 chars: 64 queries of 256 chars and the 16-B alignment fit,
// configs[3]'s longest) falls back to per-lane loads.
#ifndef SAS_WQ_WORDS
#define SAS_WQ_WORDS 520
#endif
// 16-B blocks a lane loads before it packs any (0: the plain loop)
#ifndef SAS_WQ_UNROLL
#define SAS_WQ_UNROLL 8
#endif

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = (uint64_t)__shfl_xor((long long)v, o);
        v = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = (uint64_t)__shfl_xor((long long)v, o);
        v = t > v ? t : v;
    }
    return v;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// 16 byte codes -> 32 bits, first char in bits 31..30
__device__ __forceinline__ uint32_t pack16(uint4 v) {
    return (pack4(v.x) << 24) | (pack4(v.y) << 16) | (pack4(v.z) << 8) | pack4(v.w);
}

// Stage the span of this wave's queries (qo = byte offset of this lane's query in qbytes, m
// its length, act = the lane holds a query).  Wave-uniform result: true = staged, *lo16 = the
// byte offset of LDS char 0 (the span's first byte rounded down to 16 B).  Every 16-B block
// read holds a byte of the span, which lies inside the caller's buffer.
__device__ __forceinline__ bool wave_stage_queries(const uint8_t* __restrict__ qbytes, uint64_t qo, uint32_t m,
                                                   bool act, uint32_t* L32, uint64_t* lo16) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lo = wave_min_u64(act && m ? qo : ~0ull);
    const uint64_t hi = wave_max_u64(act && m ? qo + m : 0ull);
    wave_sync_lds();  // the previous batch's reads of L32 are done
    if (hi == 0) {  // no lane has a char to stage
        *lo16 = 0;
        if (lane < 2) L32[lane] = 0;
        wave_sync_lds();
        return true;
    }
    const uint64_t base = lo & ~15ull;
    const uint64_t span = hi - base;
    if (span > (uint64_t)(SAS_WQ_WORDS - 1) * 32) return false;
    const uint32_t nblk = (uint32_t)((span + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(qbytes + base);
#if SAS_WQ_UNROLL > 1
    // all of a lane's blocks in flight before the first wait: the span (~8 blocks per lane at
    // configs[3]'s mean length) costs one memory round trip, not one per pair of blocks.  The
    // lookup state is not live yet, so the buffer costs no occupancy
    for (uint32_t b0 = lane; b0 < nblk; b0 += 64 * SAS_WQ_UNROLL) {
        uint4 v[SAS_WQ_UNROLL];
#pragma unroll
        for (int k = 0; k < SAS_WQ_UNROLL; k++) {
            const uint32_t b = b0 + 64u * k;
            v[k] = b < nblk ? src[b] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < SAS_WQ_UNROLL; k++) {
            const uint32_t b = b0 + 64u * k;
            if (b < nblk) L32[b ^ 1] = pack16(v[k]);
        }
    }
#else
    for (uint32_t b = lane; b < nblk; b += 64) L32[b ^ 1] = pack16(src[b]);
#endif
    // zero the rest of the last word and one guard word after it
    const uint32_t nw = (nblk + 1) >> 1, z = nblk + lane;
    if (z < 2 * nw + 2) L32[z ^ 1] = 0;
    wave_sync_lds();
    *lo16 = base;
    return true;
}

// A query read from the wave's LDS words (same interface as QueryRegs: m, w[0], word,
// chars32; chars past m read as 0).
struct WaveQuery {
    const uint64_t* L;
    uint32_t qo;  // the query's first char in L
    uint32_t m;
    uint64_t w[1];
    __device__ __forceinline__ void init(const uint32_t* L32, uint32_t off, uint32_t len) {
        L = reinterpret_cast<const uint64_t*>(L32);
        qo = off;
        m = len;
        w[0] = chars32(0);
    }
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        if (off >= m) return 0;
        const uint32_t c = qo + off, k = c >> 5, s = (c & 31) << 1;
        uint64_t v = L[k];
        if (s) v = (v << s) | (L[k + 1] >> (64 - s));
        return v & chars_mask(m - off < 32 ? m - off : 32);
    }
    __device__ __forceinline__ uint64_t word(uint32_t j) const { return chars32(j << 5); }
};

// A query that is a slice of the indexed text (SAS_QUERIES_ARE_SLICES, the reference's
// borrowed &t[i..i + len] queries, sas/util.rs:18-26): its chars come from the packed text
// on demand, and `pos` tells a lookup where one occurrence starts.
struct TextQuery {
    const uint64_t* tw;
    uint64_t pos;
    uint32_t m;
    uint64_t w[1];
    __device__ __forceinline__ void init(const uint64_t* t, uint64_t p, uint32_t len) {
        tw = t;
        pos = p;
        m = len;
        w[0] = chars32(0);
    }
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        if (off >= m) return 0;
        return text_chars32(tw, pos + off) & chars_mask(m - off < 32 ? m - off : 32);
    }
    __device__ __forceinline__ uint64_t word(uint32_t j) const { return chars32(j << 5); }
};

// the text position a query is known to occur at (TextQuery), else none
template <class Q>
__device__ __forceinline__ uint64_t query_source(const Q&) { return ~0ull; }
template <>
__device__ __forceinline__ uint64_t query_source<TextQuery>(const TextQuery& q) { return q.pos; }

// A query read from its bytes on demand (the fallback of spread-out batches): word 0 in a
// register, later windows packed from global memory when a compare reaches them.
struct ByteQuery {
    const uint8_t* bytes;
    uint32_t m;
    uint64_t w[1];
    __device__ __forceinline__ void init(const uint8_t* q, uint32_t len) {
        bytes = q;
        m = len;
        uint32_t dummy = 0;
        w[0] = pack_query_word(q, len, 0, &dummy);
    }
    __device__ __forceinline__ uint64_t word(uint32_t j) const {
        if (j == 0) return w[0];
        uint32_t dummy = 0;
        return pack_query_word(bytes, m, j, &dummy);
    }
    __device__ __forceinline__ uint64_t chars32(uint32_t off) const {
        const uint32_t j = off >> 5, s = (off & 31) << 1;
        const uint64_t a = word(j);
        if (s == 0) return a;
        return (a << s) | (word(j + 1) >> (64 - s));
    }
};
