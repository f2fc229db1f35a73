// sas_search.hip -- batched suffix-array lookup kernels for gfx950 (MI355X).
//
// Every algorithm returns SA[lower_bound(q)] under Rust slice order, i.e. the
// result of binary_search (sas/sa_search.rs:98-112), bit for bit.
//
//   PLAIN  one lane per query, the whole wave64 walks 64 queries in lockstep for
//          ilog2(n)+1 iterations exactly like binary_search_batch<64>
//          (sas/sa_search.rs:157-196).  The first levels' pivots come from the
//          prefix-relative blocks (common.hpp RelLayout): 15 levels from LDS, then
//          4 levels per request, the rest from SA words and text windows.  The
//          lane remembers SA[r] of the last right move, so the final `sa[l]`
//          (:195) needs no extra load unless a key decided it.
//   LCP    PLAIN + Manber-Myers mlr skipping: chars [0, min(llcp, rlcp)) are known
//          equal and are not compared again (sas/sa_search.rs:344-345 TODO).
//   LLCP   PLAIN's probes with Manber-Myers' Llcp/Rlcp accelerant (SAS_BUILD_LLCP):
//          below the cached top levels a probe reads one 16-B {SA, Llcp, Rlcp,
//          16 chars after each} entry; it decides from the lcps alone unless they
//          tie, and a tie compares the inlined chars before any text.
//   SECTOR / QUAD  B-trees over the fused (32-char key, SA) leaf entries.
//   PREFIX the reference's prefix table made live (sas/sa_search.rs:59-95): the
//          rank range of q's first p chars, then binary_search over it on the
//          fused leaf entries; with inline tables one G-lane group reads the first
//          G suffixes of the range as one request (the headline, k_sa_prefix2).
//   STREE  descend an STree<16,16> over the 16-char keys of the SA (top layers in
//          LDS), giving the key range [r0, r1) of suffixes whose padded 16-char
//          prefix equals the query's; the lower bound lies in [r0, r1] and is
//          found by an exact binary search there (mlr skipping from char 16).
//
// Text compares are 2-bit packed: 32 chars per u64 compare.
#include "common.hpp"
#include "host_stage.hpp"

#include <rocprim/device/device_scan.hpp>

#include <chrono>
#include <type_traits>
#include <vector>

#define SEARCH_BLOCK 1024
#define TRY_RC(x) do { int rc_ = (x); if (rc_) return rc_; } while (0)
#define BLOCKS_PER_CU 2
// the binary searches (k_sa_binary: PLAIN, LCP, LLCP) and the S-tree descents (k_sa_stree,
// k_sa_stree4x: STREE, STREE_LLCP): workgroup size and workgroups per CU.
// The launch bound follows them (waves per SIMD = block x blocks / 256), which caps the VGPRs:
// 1024 x 2 -> 8 waves, 64 VGPRs; 768 x 2 -> 6 waves, 80 VGPRs (the LDS pivot groups, 72.5 KiB
// a workgroup, allow two workgroups a CU either way)
#ifndef SAS_BIN_BLOCK
#define SAS_BIN_BLOCK 768
#endif
#ifndef SAS_BIN_BPC
#define SAS_BIN_BPC 2
#endif
#define SAS_BIN_WAVES (SAS_BIN_BLOCK * SAS_BIN_BPC / 256)
// ... for queries past 64 chars (4 or 8 query words in registers): an A/B hook
#ifndef SAS_BIN_BLOCK_LONG
#define SAS_BIN_BLOCK_LONG SAS_BIN_BLOCK
#endif
#define BIN_BLOCK(QW) ((QW) <= 2 ? SAS_BIN_BLOCK : SAS_BIN_BLOCK_LONG)
#define BIN_WAVES(QW) (BIN_BLOCK(QW) * SAS_BIN_BPC / 256)
// STREE at m <= 32: one lane per query (k_sa_stree4x) instead of a 4-lane group (A/B hook)
#ifndef SAS_STREE_PERLANE
#define SAS_STREE_PERLANE 0
#endif

struct SearchArgs {
    const uint64_t* tw;
    uint64_t n;          // text length
    uint64_t sa_n;       // SA entries held by this index
    uint64_t next_pos;   // answer when the lower bound is sa_n (n for a whole index)
    uint64_t rank_lo;    // global rank of sa[0]
    const uint8_t* sa;       // SaView<W> (u32 or packed 40-bit)
    const uint4* llcp;       // SAS_BUILD_LLCP entries (k_sa_binary<.., BS_LLCP, ..>)
    const uint8_t* prefix;   // SAS_BUILD_PREFIX table (k_sa_prefix): u32 or packed 40-bit entries
    uint32_t prefix_chars;
    uint32_t prefix_w;       // bytes per table entry (4 or 5)
    uint32_t prefix_hi40;    // inline slots: SA bits 32..39 in slot 1's rank word
    uint64_t pt_base;        // the table's first key (0, or a part's first suffix's key)
    uint64_t pt_jmax;        // its last entry a lookup may start at (entries - 2)
    const uint8_t* rel;      // the prefix-relative pivot blocks (common.hpp RelLayout)
    RelLayout rel_lay;
    uint32_t iters;
    const uint32_t* stree;
    uint64_t stree_off[SAS_STREE_MAX_LAYERS];
    uint32_t stree_height;
    uint32_t stree_lds_layers;
    uint32_t stree_lds_nodes;
    const uint32_t* sec_inner;
    const uint4* sec_leaves;
    uint64_t sec_off[SAS_SECTOR_MAX_LAYERS];
    uint32_t sec_inner_layers;
    uint32_t sec_lds_layers;
    uint32_t sec_lds_nodes;
    const uint4* quad_inner;
    const uint4* quad_leaves;
    uint64_t quad_off[SAS_QUAD_MAX_LAYERS];
    uint64_t quad_leaf_count;
    uint32_t stree_leaf_nt;  // S-tree leaf layer (16-char keys) read non-temporal
    uint32_t quad_fan;
    uint32_t quad_nt_from;   // first inner layer read with non-temporal loads
    uint32_t quad_leaf_nt;   // leaves read with non-temporal loads
    uint32_t quad_inner_layers;
    uint32_t quad_lds_layers;
    uint32_t quad_lds_nodes;
    const uint64_t* tag_table;  // SAS_BUILD_TAGGED bucket table (sa = tagged entries, W = 8)
    uint32_t tag_p;
    const uint64_t* tag_lines;  // SAS_BUILD_TAG_LINES: 128-B bucket lines (common.hpp)
    const uint64_t* tag_ovf;    // and their overflow entries
    const uint64_t* tag_first;  // and the buckets' first ranks
    const uint64_t* tw2;        // and the second text copy (tl_text)
    uint32_t tag_sb;            // SA bits of a line entry
    const uint8_t* qbytes;
    const uint64_t* qwords;  // sas_search_packed: 2-bit packed fixed-length queries (PREFIX)
    const uint64_t* qoff;
    const uint32_t* qlen;
    uint32_t m_fixed;
    uint32_t m_max;          // longest query of the batch when the host knows it (0: unknown)
    uint64_t nq;
    uint64_t* out_pos;
    uint32_t* out_probes;
    uint32_t* bad;
    const uint64_t* bcounts; // sas_search_buckets: queries per bucket (null: every slot is a query)
    uint32_t bcap;           // slots per bucket
};

// sas_search_buckets (the sharded step's received slots): slot i is place i % bcap of
// bucket i / bcap, and only places below that bucket's count hold a query; the others are
// skipped (no reads, no output).  The host checks nq = buckets x bcap < 2^32.
__device__ __forceinline__ bool slot_live(const SearchArgs& a, uint64_t i) {
    if (!a.bcounts) return true;
    const uint32_t b = (uint32_t)i / a.bcap;
    return (uint64_t)((uint32_t)i - b * a.bcap) < a.bcounts[b];
}

__device__ __forceinline__ void query_ptr(const SearchArgs& a, uint64_t i, const uint8_t** qb, uint32_t* m) {
    if (a.qoff) {
        *qb = a.qbytes + a.qoff[i];
        *m = a.qlen[i];
    } else {
        *qb = a.qbytes + i * (uint64_t)a.m_fixed;
        *m = a.m_fixed;
    }
}

// ------------------------------------------------------------------ PLAIN / LCP
template <int W>
using sa_val_t = typename std::conditional<W == 4, uint32_t, uint64_t>::type;

// LLCP tie: the first h chars of suffix p are known equal to q's; inl = the suffix's
// chars [h, h + 16) from its LLCP entry.  Same result as suffix_less_from(.., h, ..),
// which only runs when those 16 chars match and both strings go on.
template <int QW, class Q>
__device__ __forceinline__ bool llcp_tie_less(const uint64_t* __restrict__ tw, uint64_t n, uint64_t p,
                                              const Q& q, uint32_t h, uint32_t inl, uint32_t* lcp) {
    const uint64_t lenS = n - p;
    const uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    if (h < L) {
        const uint32_t c = L - h < 16 ? L - h : 16;
        const uint32_t mk = ~0u << (32 - 2 * c);  // c >= 1
        const uint32_t av = inl & mk, bv = (uint32_t)(q.chars32(h) >> 32) & mk;
        if (av != bv) {
            *lcp = h + (uint32_t)(__clz(av ^ bv) >> 1);
            return av < bv;
        }
        if (h + 16 < L) return suffix_less_from<QW>(tw, n, p, q, h + 16, lcp);
    }
    *lcp = L;
    return lenS < (uint64_t)q.m;
}

// The table entry of p-char key K: K - pt_base, clamped to the table.  A whole index's table
// holds every key (pt_base 0, pt_jmax 4^p - 1: the identity).  A part's holds its first
// suffix's key .. its last one's and two entries of rank sa_n: a key below the interval
// clamps to entry 0, whose suffixes (like every suffix of the part) are > q, so the lower
// bound is rank 0 from either; a key above it to entry jmax, the empty range at sa_n
__device__ __forceinline__ uint64_t pt_slot(const SearchArgs& a, uint64_t K) {
    K = K > a.pt_base ? K - a.pt_base : 0;
    return K < a.pt_jmax ? K : a.pt_jmax;
}
// Rank of inline entry j (16 G bytes): slot 0's rank word, and for two slots beside a text of
// >= 2^32 chars bits 32..39 from slot 1's (a part of >= 2^32 suffixes)
template <int G, bool HI40>
__device__ __forceinline__ uint64_t pt_rank(const uint4* t, uint64_t j) {
    const uint64_t r = t[G * j].z;
    if (!(HI40 && G == 2)) return r;
    return r | ((uint64_t)((t[G * j + 1].z >> 16) & 0xFFu) << 32);
}
// prefix_range (sas/sa_search.rs:86-95): the SA ranks [lo, hi) whose p-char key is K,
// from the prefix table in any of its entry formats
__device__ __forceinline__ void prefix_range(const SearchArgs& a, uint64_t K, uint64_t* lo, uint64_t* hi) {
    K = pt_slot(a, K);
    if (a.prefix_w >= 16) {  // inline entries: rank in the first slot's .z
        const uint4* t = reinterpret_cast<const uint4*>(a.prefix);
        if (a.prefix_w == 32 && a.prefix_hi40) {
            *lo = pt_rank<2, true>(t, K);
            *hi = pt_rank<2, true>(t, K + 1);
        } else {
            const uint64_t st = a.prefix_w / 16;
            *lo = t[st * K].z;
            *hi = t[st * (K + 1)].z;
        }
    } else if (a.prefix_w == 5) {
        const SaView<5> v{a.prefix};
        *lo = v[K];
        *hi = v[K + 1];
    } else {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(a.prefix);
        *lo = t[K];
        *hi = t[K + 1];
    }
}

// MODE 0: PLAIN, 1: LCP (mlr), 2: LLCP (Manber-Myers with the Llcp/Rlcp entries)
// RANGE (SAS_PREFIX_RANGE, PLAIN / LCP without the LDS top): start from the prefix
// table's range for q's first p chars instead of [0, sa_n), exactly as the reference's
// binary_search does (sas/sa_search.rs:98-101) once its p is not 0
// PLAIN over a u32 SA: a range of at most this many ranks (4 or 8; 0: off) has its SA words
// loaded together for the remaining probes
#ifndef SAS_PLAIN_SA_RUN
#define SAS_PLAIN_SA_RUN 8
#endif
static_assert(SAS_PLAIN_SA_RUN == 0 || SAS_PLAIN_SA_RUN == 4 || SAS_PLAIN_SA_RUN == 8, "SAS_PLAIN_SA_RUN: 0, 4 or 8");
#define BS_PLAIN 0
#define BS_MLR 1
#define BS_LLCP 2
// LLCP: a range of at most this many ranks (0: off, 2..4) has its 16-B entries loaded together
// (consecutive ranks: one or two lines) for the remaining probes (A/B hook)
#ifndef SAS_LLCP_RUN
#define SAS_LLCP_RUN 0
#endif
static_assert(SAS_LLCP_RUN == 0 || (SAS_LLCP_RUN >= 2 && SAS_LLCP_RUN <= 4), "SAS_LLCP_RUN: 0 or 2..4");
// The rel blocks' LDS groups (common.hpp RelLayout) into a workgroup's LDS: 16-B copies
__device__ __forceinline__ void stage_rel(uint4* s, const uint8_t* __restrict__ rel, uint32_t bytes) {
    const uint4* src = reinterpret_cast<const uint4*>(rel);
    for (uint32_t w = threadIdx.x; w < bytes / 16; w += blockDim.x) s[w] = src[w];
}
// Node k's block at level it (the root of group g, hh levels): from LDS for the staged groups,
// else two (one) 16-B loads of one line, issued together (one request)
__device__ __forceinline__ void rel_block(const SearchArgs& a, const uint4* s, uint32_t g, uint32_t it, uint32_t k,
                                          uint32_t hh, uint4& b0, uint4& b1) {
    const uint64_t off = a.rel_lay.base[g] + ((uint64_t)(k - (1u << it)) << (hh == SAS_REL_GROUP ? 5 : 4));
    if (g < a.rel_lay.lds_groups) {
        const uint32_t w = (uint32_t)off >> 4;
        b0 = s[w];
        if (hh == SAS_REL_GROUP) b1 = s[w + 1];
    } else {
        const uint4* p = reinterpret_cast<const uint4*>(a.rel + off);
        b0 = p[0];
        if (hh == SAS_REL_GROUP) b1 = p[1];
    }
}
// Slot j (1..15) of a block: the pivot's chars [P, P + 8) (slot 0 = P)
__device__ __forceinline__ uint32_t rel_slot(const uint4& b0, const uint4& b1, uint32_t j) {
    const uint4 v = j >= 8 ? b1 : b0;
    const uint32_t cw = (j >> 1) & 3u;
    const uint32_t wv = cw == 0 ? v.x : cw == 1 ? v.y : cw == 2 ? v.z : v.w;
    return ((j & 1u) ? (wv >> 16) : wv) & 0xFFFFu;
}
// EXQ (QW >= 4): launched only with m <= 32 QW, the query words all in registers (QueryRegsExact:
// no repacking code, fewer registers; the plain form repacks words past them from the bytes)
template <int QW, int MODE, bool TOP, int W, bool RANGE = false, bool EXQ = false>
__global__ __launch_bounds__(BIN_BLOCK(QW), BIN_WAVES(QW)) void k_sa_binary(SearchArgs a) {
    using QR = typename std::conditional<EXQ && (QW > 2), QueryRegsExact<QW>, QueryRegs<QW>>::type;
    // the prefix-relative pivot blocks, the first 15 levels' from LDS (common.hpp RelLayout)
    __shared__ uint4 s_rel[TOP ? SAS_REL_LDS_BYTES / 16 : 1];
    const SaView<W> sa{a.sa};
    if (TOP) {
        stage_rel(s_rel, a.rel, a.rel_lay.lds_bytes);
        __syncthreads();
    }
    uint32_t bad = 0;
    const uint64_t n = a.n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (!slot_live(a, i)) continue;
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QR q;
        q.load(qb, m, &bad);

        // ranks fit 32 bits beside a u32 SA (sa_n < 2^32): fewer registers for l, r, mid
        using rank_t = sa_val_t<W>;
        rank_t l = 0, r = (rank_t)a.sa_n;
        uint32_t k = 1, probes = 0, llcp = 0, rlcp = 0;
        sa_val_t<W> pr = 0;  // SA[r] while prv
        bool prv = false;
        if (RANGE) {
            uint64_t l64, r64;
            prefix_range(a, q.w[0] >> (64 - 2 * a.prefix_chars), &l64, &r64);
            l = (rank_t)l64;
            r = (rank_t)r64;
            probes = 1;  // the reference's cnt counts the table read (:87-89)
        }
        // one probe's outcome: the reference's l / r update (sas/sa_search.rs:102-110); pk:
        // p is known (PLAIN's blocked pivot levels may decide from the key alone)
        auto take = [&](rank_t mid, bool lt, uint32_t lcp, sa_val_t<W> p, bool pk) {
            probes++;
            if (lt) {
                l = mid + 1;
                llcp = lcp;
            } else {
                r = mid;
                rlcp = lcp;
                pr = p;
                prv = pk;
            }
        };
        uint32_t it = 0;
        if (TOP) {
            // the prefix-relative blocks, 4 levels from one 32-B block (LDS, or two 16-B loads
            // of one line: one request): the 8 chars after the block bounds' common prefix of P
            // chars decide each probe unless they tie with q's (then the SA value -- LLCP: from
            // its entry -- and the text from char P + c).  q starts with those P chars
            // (common.hpp), and a key padded past its suffix's end that differs from q there is
            // a proper prefix of q (key < q)
            for (uint32_t g = 0; g < a.rel_lay.groups; ++g) {
                const uint32_t hh = a.rel_lay.h[g];
                uint4 b0 = make_uint4(0, 0, 0, 0), b1 = b0;
                if (l < r) rel_block(a, s_rel, g, it, k, hh, b0, b1);
                const uint32_t P = b0.x & 0x7FFFu;
                const uint32_t c0 = q.m > P ? q.m - P : 0u;
                // LCP / LLCP need exact lcps: a block flagged (bit 15) as holding a pivot whose
                // suffix ends inside its key compares no key chars (every probe: the entry and
                // the text from P)
                const uint32_t c = (MODE != BS_PLAIN && (b0.x & 0x8000u)) ? 0u : c0 < 8 ? c0 : 8u;
                const uint32_t mk = c ? (0xFFFFu << (16 - 2 * c)) & 0xFFFFu : 0u;
                const uint32_t qk = (uint32_t)((q.w[0] << (2 * P)) >> 48) & mk;
                for (uint32_t t = 0; t < hh; ++t, ++it) {
                    if (!(l < r)) continue;
                    const rank_t mid = (rank_t)(((uint64_t)l + r) >> 1);
                    const uint32_t key = rel_slot(b0, b1, (1u << t) | (k & ((1u << t) - 1u))) & mk;
                    // LCP / LLCP: lcp = P + the first differing char
                    sa_val_t<W> p = 0;
                    uint32_t lcp = key != qk ? P + (((uint32_t)__clz(key ^ qk) - 16u) >> 1) : 0u;
                    bool lt, pk = false;
                    if (key != qk) {
                        lt = key < qk;
                    } else {
                        if (MODE == BS_LLCP) {
                            const uint4 e = a.llcp[mid];
                            p = (sa_val_t<W>)((uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32));
                        } else {
                            p = (sa_val_t<W>)sa[mid];
                        }
                        // chars [0, P + c) are known equal
                        lt = suffix_less_from<QW>(a.tw, n, p, q, P + c, &lcp);
                        pk = true;
                    }
                    k = 2 * k + (lt ? 1u : 0u);
                    take(mid, lt, lcp, p, pk);
                }
            }
        }
        bool run = false;  // PLAIN, u32 SA: the range's SA words are in sc0..sc2 (from rank rb)
        uint32_t rb = 0;   // LLCP (SAS_LLCP_RUN): the range's entries are in sc0..sc3 (from rank rl)
        uint4 sc0 = make_uint4(0, 0, 0, 0), sc1 = sc0, sc2 = sc0, sc3 = sc0;
        rank_t rl = 0;
        for (; it < a.iters; ++it) {
            if (l < r) {
                const rank_t mid = (rank_t)(((uint64_t)l + r) >> 1);
                const uint32_t h = MODE != BS_PLAIN ? (llcp < rlcp ? llcp : rlcp) : 0u;
                sa_val_t<W> p;
                uint32_t lcp;
                bool lt;
                if (MODE == BS_LLCP) {
                    // one 16-B read: SA[mid], the lcps of the pivot with the interval's
                    // bounds L = SA[l-1] (< q) and R = SA[r] (>= q), and 16 pivot chars
                    // after each.  Manber-Myers: with llcp >= rlcp, Llcp > llcp puts the
                    // pivot on L's side of q (< q, same lcp), Llcp < llcp on R's side
                    // (> q, lcp = Llcp); symmetric with Rlcp.  A tie (or a capped value)
                    // compares from the known lcp, first against the inlined chars.
                    uint4 e;
                    if (SAS_LLCP_RUN) {
                        if (!run && r - l <= SAS_LLCP_RUN) {
                            run = true;
                            rl = l;
                            const uint4* c = a.llcp + l;  // consecutive 16-B entries: one or two lines
                            sc0 = c[0];
                            if (r - l > 1) sc1 = c[1];
                            if (SAS_LLCP_RUN > 2 && r - l > 2) sc2 = c[2];
                            if (SAS_LLCP_RUN > 3 && r - l > 3) sc3 = c[3];
                        }
                        if (run) {
                            const uint32_t o = (uint32_t)(mid - rl);
                            e = o == 0 ? sc0 : o == 1 ? sc1 : (SAS_LLCP_RUN > 3 && o == 3) ? sc3 : sc2;
                        } else {
                            e = a.llcp[mid];
                        }
                    } else {
                        e = a.llcp[mid];
                    }
                    p = (sa_val_t<W>)((uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32));
                    const uint32_t x = (e.y >> 8) & SAS_LLCP_CAP, y = e.y >> 20;
                    uint32_t hh = 0, inl = 0;
                    bool decided = true;
                    if (llcp >= rlcp) {
                        if (x > llcp) { lt = true; lcp = llcp; }
                        else if (x < llcp && x < SAS_LLCP_CAP) { lt = false; lcp = x; }
                        else { decided = false; hh = x; inl = e.z; }
                    } else {
                        if (y > rlcp) { lt = false; lcp = rlcp; }
                        else if (y < rlcp && y < SAS_LLCP_CAP) { lt = true; lcp = y; }
                        else { decided = false; hh = y; inl = e.w; }
                    }
                    if (!decided) {
                        lt = llcp_tie_less<QW>(a.tw, n, p, q, hh, inl, &lcp);
                    }
                } else if (MODE == BS_PLAIN && W == 4 && SAS_PLAIN_SA_RUN) {
                    // the last probes' SA words: once the range holds <= SAS_PLAIN_SA_RUN ranks,
                    // the 16-B chunks covering it are loaded together (one request) and the
                    // remaining probes take their SA values from registers
                    if (!run && r - l <= SAS_PLAIN_SA_RUN) {
                        run = true;
                        rb = l & ~3u;
                        const uint4* c = reinterpret_cast<const uint4*>(a.sa) + (rb >> 2);
                        sc0 = c[0];
                        if (((uint32_t)r - 1) - rb >= 4) sc1 = c[1];
                        if (SAS_PLAIN_SA_RUN > 4 && ((uint32_t)r - 1) - rb >= 8) sc2 = c[2];
                    }
                    if (run) {
                        const uint32_t o = (uint32_t)mid - rb;
                        const uint4 v = o < 4 ? sc0 : (SAS_PLAIN_SA_RUN > 4 && o >= 8 ? sc2 : sc1);
                        const uint32_t oo = o & 3;
                        p = (sa_val_t<W>)(oo == 0 ? v.x : oo == 1 ? v.y : oo == 2 ? v.z : v.w);
                    } else {
                        p = (sa_val_t<W>)sa[mid];
                    }
                    lt = suffix_less_from<QW>(a.tw, n, p, q, h, &lcp);
                } else {
                    p = (sa_val_t<W>)sa[mid];
                    lt = suffix_less_from<QW>(a.tw, n, p, q, h, &lcp);
                }
                take(mid, lt, lcp, p, true);
            }
        }
        // SA[r] not seen yet: r never moved (RANGE: the table's range end) or moved last on a
        // pivot decided from its key alone (rare below a 23-level array: a right move on
        // every one of the last levels' SA probes would have to be missing)
        if (!prv && r < a.sa_n) {
            if (MODE == BS_LLCP) {  // LLCP reads its own entries only
                const uint4 e = a.llcp[r];
                pr = (sa_val_t<W>)((uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32));
            } else {
                pr = (sa_val_t<W>)sa[r];
            }
        }
        a.out_pos[i] = (r >= a.sa_n) ? a.next_pos : (uint64_t)pr;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ STREE
// 4-lane cooperative node reads (one request per 64-B node): lane
// j holds keys 4j..4j+3, the group sums its counts with DPP.
__device__ __forceinline__ uint32_t quad_cnt_lt(uint4 v, uint32_t K) {
    return quad_sum((v.x < K) + (v.y < K) + (v.z < K) + (v.w < K));
}
__device__ __forceinline__ uint32_t quad_cnt_eq(uint4 v, uint32_t K) {
    return quad_sum((v.x == K) + (v.y == K) + (v.z == K) + (v.w == K));
}

// Descend the internal layers for key K; returns the leaf node index (within
// the leaf layer).  sst/s_tree.rs:196-203 with unsigned keys.  LDS layers, then
// HBM layers (separate loops: ds_read / global_load, not FLAT).
__device__ __forceinline__ uint64_t stree_descend(const SearchArgs& a, const uint4* s_nodes, uint32_t K,
                                                  uint32_t sub) {
    uint64_t k = 0;
    const uint4* g = reinterpret_cast<const uint4*>(a.stree);
    uint32_t h = 0;
    for (; h < a.stree_lds_layers && h + 1 < a.stree_height; h++)
        k = k * (SAS_STREE_B + 1) + quad_cnt_lt(s_nodes[(a.stree_off[h] + k) * 4 + sub], K);
    for (; h + 1 < a.stree_height; h++) k = k * (SAS_STREE_B + 1) + quad_cnt_lt(g[(a.stree_off[h] + k) * 4 + sub], K);
    return k;
}

// The exact lower bound of q inside [r0, r1], the run of suffixes whose padded 16-char key
// is q's (the S-tree descent's result); returns its position.
// LT = false: binary search over [r0, r1] with mlr skipping from char 16 (SA + text reads).
// LT = true (SAS_ALGO_STREE_LLCP): the LLCP entries (Manber-Myers Llcp / Rlcp, SAS_BUILD_LLCP)
//   belong to the implicit binary-search tree over the whole SA, so the tail walks that tree
//   from its root: a mid outside the run is decided by the S-tree keys with no read (below r0:
//   < q; at or past r1: > q), a mid inside reads its 16-B entry and applies the LLCP rules of
//   k_sa_binary.  A bound outside the run has an lcp with q below 16 that no compare measured;
//   the first entry read after it supplies it: for a suffix a < the run (key16(a) < K) and b in
//   the run, lcp(a, b) = lcp(a, q), and symmetrically for the right bound (up to a text-end
//   suffix b shorter than 16 chars, where lcp(b, c) may fall below lcp(q, c)).  Taking the
//   entry's own Llcp / Rlcp for such a side makes that side tie (Llcp = llcp), so a probe
//   decided on it always compares (from its lcp, which b shares with q either way); a side
//   inside the run carries an exact lcp from an earlier compare or rule.  So every rule is
//   applied on an exact lcp and the result is binary_search's.
template <int QW, int W, bool LT, class Q>
__device__ __forceinline__ uint64_t stree_tail(const SearchArgs& a, const Q& q, uint32_t m, uint64_t r0,
                                               uint64_t r1, uint32_t* probes) {
    const SaView<W> sa{a.sa};
    const uint64_t n = a.n, sa_n = a.sa_n;
    if (!LT) {
        // exact lower bound inside [r0, r1]: chars [0, min(16, m)) match every suffix there
        const uint32_t h16 = m < 16 ? m : 16;
        uint64_t l = r0, r = r1;
        uint32_t llcp = h16, rlcp = h16;
        sa_val_t<W> pr = 0;
        bool have = false;
        while (l < r) {
            const uint64_t mid = (l + r) >> 1;
            const sa_val_t<W> p = (sa_val_t<W>)sa[mid];
            uint32_t lcp;
            const uint32_t h = llcp < rlcp ? llcp : rlcp;
            const bool lt = suffix_less_from<QW>(a.tw, n, p, q, h, &lcp);
            (*probes)++;
            if (lt) {
                l = mid + 1;
                llcp = lcp;
            } else {
                r = mid;
                rlcp = lcp;
                pr = p;
                have = true;
            }
        }
        if (l >= sa_n) return a.next_pos;
        return have ? (uint64_t)pr : (uint64_t)sa[l];
    }
    uint64_t l = 0, r = sa_n, pr = 0;
    uint32_t llcp = 0, rlcp = 0;
    bool have = false;
    for (;;) {
        // the walk to the next mid inside the run, ALU only: the lanes of a wave reach their
        // in-run mids at different depths, and one load per outer iteration keeps their
        // reads in lockstep (a load inside the walk would serialise their latencies)
        uint64_t mid = 0;
        while (l < r) {
            mid = (l + r) >> 1;
            if (mid < r0) l = mid + 1;       // key16 < K: < q, no read
            else if (mid >= r1) r = mid;     // key16 > K: > q, no read
            else break;
        }
        if (!(l < r)) break;
        const uint4 e = a.llcp[mid];
        const uint64_t p = (uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32);
        const uint32_t x = (e.y >> 8) & SAS_LLCP_CAP, y = e.y >> 20;
        if (l <= r0) llcp = x;  // the left bound SA[l - 1] lies before the run (or l = 0)
        if (r >= r1) rlcp = y;  // the right bound SA[r] lies past it (or r = sa_n)
        (*probes)++;
        bool lt;
        uint32_t lcp, hh = 0, inl = 0;
        bool decided = true;
        if (llcp >= rlcp) {
            if (x > llcp) { lt = true; lcp = llcp; }
            else if (x < llcp && x < SAS_LLCP_CAP) { lt = false; lcp = x; }
            else { decided = false; hh = x; inl = e.z; }
        } else {
            if (y > rlcp) { lt = false; lcp = rlcp; }
            else if (y < rlcp && y < SAS_LLCP_CAP) { lt = true; lcp = y; }
            else { decided = false; hh = y; inl = e.w; }
        }
        if (!decided) lt = llcp_tie_less<QW>(a.tw, n, p, q, hh, inl, &lcp);
        if (lt) {
            l = mid + 1;
            llcp = lcp;
        } else {
            r = mid;
            rlcp = lcp;
            pr = p;
            have = true;
        }
    }
    if (r >= sa_n) return a.next_pos;
    if (have) return pr;
    const uint4 e = a.llcp[r];  // r moved only past the run (or is r1 itself)
    return (uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32);
}

// One 4-lane group per query.  The S-tree descent and the leaf scans are
// cooperative; the exact tail search in [r0, r1] (SA + text reads) runs on all
// four lanes identically, so its loads coalesce to one request each.
template <int QW, int W>
__global__ __launch_bounds__(SAS_BIN_BLOCK, SAS_BIN_WAVES) void k_sa_stree(SearchArgs a) {
    __shared__ uint4 s_nodes[SAS_STREE_LDS_NODES * 4];
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.stree);
        for (uint32_t w = threadIdx.x; w < a.stree_lds_nodes * 4; w += blockDim.x) s_nodes[w] = g[w];
        __syncthreads();
    }
    uint32_t bad = 0;
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const uint4* g = reinterpret_cast<const uint4*>(a.stree);
    const uint64_t ol = a.stree_off[a.stree_height - 1];
    const uint64_t sa_n = a.sa_n;
    const uint64_t leaf_nodes = (sa_n + 15) / 16;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G; i < a.nq; i += stride) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint32_t K = (uint32_t)(q.w[0] >> 32);  // padded 16-char key of q
        uint32_t probes = a.stree_height - 1;

        uint64_t k = stree_descend(a, s_nodes, K, sub);
        const uint4 lv = load4(g + (ol + k) * 4 + sub, a.stree_leaf_nt);
        const uint32_t c = quad_cnt_lt(lv, K), e = quad_cnt_eq(lv, K);
        probes++;
        uint64_t r0 = k * 16 + c;
        uint64_t r1 = r0 + e;
        if (c + e == 16) {  // the run of equal keys may continue in the next leaves
            uint64_t kk = k + 1;
            int steps = 0;
            for (; kk < leaf_nodes && steps < 4; kk++, steps++) {
                const uint32_t e2 = quad_cnt_eq(g[(ol + kk) * 4 + sub], K);
                probes++;
                r1 += e2;
                if (e2 < 16) break;
            }
            if (kk < leaf_nodes && steps == 4) {  // long run: lower_bound(K + 1)
                if (K == SAS_KEY_MAX) {
                    r1 = sa_n;
                } else {
                    uint64_t k2 = stree_descend(a, s_nodes, K + 1, sub);
                    probes += a.stree_height - 1;
                    r1 = k2 * 16 + quad_cnt_lt(g[(ol + k2) * 4 + sub], K + 1);
                    probes++;
                }
            }
        }
        if (r0 > sa_n) r0 = sa_n;
        if (r1 > sa_n) r1 = sa_n;
        const uint64_t pos = stree_tail<QW, W, false>(a, q, m, r0, r1, &probes);
        if (sub == 0) {
            a.out_pos[i] = pos;
            if (a.out_probes) a.out_probes[i] = probes;
        }
    }
    if (bad) atomicOr(a.bad, 1u);
}



// Long queries (QW > 1): one query per LANE, four queries per 4-lane group.
// The group walks the S-tree cooperatively for each of its four queries in turn
// (one request per 64-B node, the 16-char key taken from the owning lane), then
// every lane runs the exact tail search of its own query in parallel: the descent
// costs one request per node as in k_sa_stree, and the tail keeps the per-lane
// parallelism of a one-lane-per-query search (the text compares of long queries dominate).
template <int QW, int W, bool LT = false, bool EXQ = false>
__global__ __launch_bounds__(BIN_BLOCK(QW), BIN_WAVES(QW)) void k_sa_stree4x(SearchArgs a) {
    using QR = typename std::conditional<EXQ && (QW > 2), QueryRegsExact<QW>, QueryRegs<QW>>::type;
    __shared__ uint4 s_nodes[SAS_STREE_LDS_NODES * 4];
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.stree);
        for (uint32_t w = threadIdx.x; w < a.stree_lds_nodes * 4; w += blockDim.x) s_nodes[w] = g[w];
        __syncthreads();
    }
    uint32_t bad = 0;
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~3u);
    const uint4* g = reinterpret_cast<const uint4*>(a.stree);
    const uint64_t ol = a.stree_off[a.stree_height - 1];
    const uint64_t sa_n = a.sa_n;
    const uint64_t leaf_nodes = (sa_n + 15) / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // the loop runs while ANY query of the group is in range (group-uniform)
    for (uint64_t gi = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) - sub; gi < a.nq; gi += stride) {
        const uint64_t i = gi + sub;
        const bool mine = i < a.nq;
        const uint8_t* qb;
        uint32_t m = 0;
        QR q;
        if (mine) {
            query_ptr(a, i, &qb, &m);
            q.load(qb, m, &bad);
        } else {
            q.bytes = a.qbytes;
            q.m = 0;
            for (int j = 0; j < QW; j++) q.w[j] = 0;
        }
        const uint32_t Kmine = (uint32_t)(q.w[0] >> 32);  // padded 16-char key of this lane's query
        uint32_t probes = 0;
        uint64_t my_r0 = 0, my_r1 = 0;
        for (uint32_t j = 0; j < QUAD_G; j++) {
            if (gi + j >= a.nq) break;  // group-uniform
            const uint32_t K = (uint32_t)__shfl((int)Kmine, lane0 + (int)j, 64);
            uint32_t pr_j = a.stree_height - 1;
            const uint64_t k = stree_descend(a, s_nodes, K, sub);
            const uint4 lv = load4(g + (ol + k) * 4 + sub, a.stree_leaf_nt);
            const uint32_t c = quad_cnt_lt(lv, K), e = quad_cnt_eq(lv, K);
            pr_j++;
            uint64_t r0 = k * 16 + c, r1 = r0 + e;
            if (c + e == 16) {
                uint64_t kk = k + 1;
                int steps = 0;
                for (; kk < leaf_nodes && steps < 4; kk++, steps++) {
                    const uint32_t e2 = quad_cnt_eq(g[(ol + kk) * 4 + sub], K);
                    pr_j++;
                    r1 += e2;
                    if (e2 < 16) break;
                }
                if (kk < leaf_nodes && steps == 4) {
                    if (K == SAS_KEY_MAX) {
                        r1 = sa_n;
                    } else {
                        const uint64_t k2 = stree_descend(a, s_nodes, K + 1, sub);
                        pr_j += a.stree_height;
                        r1 = k2 * 16 + quad_cnt_lt(g[(ol + k2) * 4 + sub], K + 1);
                    }
                }
            }
            if (sub == j) {
                my_r0 = r0 > sa_n ? sa_n : r0;
                my_r1 = r1 > sa_n ? sa_n : r1;
                probes = pr_j;
            }
        }
        if (!mine) continue;
        // exact lower bound of this lane's query inside [r0, r1] (per lane)
        const uint64_t pos = stree_tail<QW, W, LT>(a, q, m, my_r0, my_r1, &probes);
        a.out_pos[i] = pos;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ SECTOR
// Lower bound = first rank x with suffix(x) >= q.  In the sector tree that
// predicate is read off the fused leaf entry (key = first 32 chars, sa):
//   key != K64(q)          ->  key > K64
//   key == K64, m <= 32    ->  n - sa >= m   (equal padded prefixes: the shorter
//                                             suffix is a proper prefix of q)
//   key == K64, m > 32     ->  exact compare from char 32 (text read)
// suffix(p) < q when the first 32 chars are known equal (m > 32).  The windows
// past char 32 are all needed when q occurs at p (every positive answer), so the
// text words are loaded in chunks of up to 4 windows before any compare: their
// latencies overlap instead of chaining load -> compare -> branch per window.
template <int QW>
__device__ __forceinline__ bool tail_less32(const uint64_t* __restrict__ tw, uint64_t n, uint64_t p,
                                            const QueryRegs<QW>& q) {
    const uint64_t lenS = n - p;
    const uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
    const uint64_t w0 = (p + 32) >> 5;
    const uint32_t sh = (uint32_t)(p & 31) << 1;
    for (uint32_t off = 32, wi = 0; off < L; off += 128, wi += 4) {
        uint64_t wd[5];
#pragma unroll
        for (int i = 0; i < 5; i++) wd[i] = (off + 32 * i <= L + 31) ? tw[w0 + wi + i] : 0ull;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t o = off + 32 * i;
            if (o >= L) break;
            const uint32_t c = L - o < 32 ? L - o : 32;
            const uint64_t mk = chars_mask(c);
            const uint64_t t = (sh ? ((wd[i] << sh) | (wd[i + 1] >> (64 - sh))) : wd[i]) & mk;
            const uint64_t b = q.chars32(o) & mk;
            if (t != b) return t < b;
        }
    }
    return lenS < (uint64_t)q.m;
}

// PREFETCH: load the tail's text words up front (tail_less32); measured faster for
// the per-lane sector kernel, slower for the 4-lane quad kernel (register spills).
// SHORT1: QW == 1 means m <= 32 (qw_for), so the text compare is dead code there;
// false for kernels that hold fewer query words in registers than the query has.
template <int QW, bool PREFETCH = false, bool SHORT1 = true, class Q = QueryRegs<QW>>
__device__ __forceinline__ bool sector_ge(uint64_t key, uint64_t p, uint64_t K64, const SearchArgs& a,
                                          const Q& q) {
    if (key != K64) return key > K64;
    if ((SHORT1 && QW == 1) || q.m <= 32) return (a.n - p) >= (uint64_t)q.m;
    if (PREFETCH) return !tail_less32<QW>(a.tw, a.n, p, q);
    uint32_t lcp;
    return !suffix_less_from<QW>(a.tw, a.n, p, q, 32, &lcp);
}

// SA value of leaf entry j (0/1) from the leaf's second 16 B: low word + bits 32..39
__device__ __forceinline__ uint64_t sector_sa(uint4 sv, uint32_t j) {
    uint32_t lo = j ? sv.y : sv.x;
    return (uint64_t)lo | ((uint64_t)((sv.z >> (8 * j)) & 0xFF) << 32);
}

__device__ __forceinline__ void sector_entry(const uint4* __restrict__ leaves, uint64_t x, uint64_t* key, uint64_t* p) {
    const uint64_t* kk = reinterpret_cast<const uint64_t*>(leaves + 2 * (x >> 1));
    *key = kk[x & 1];
    *p = sector_sa(leaves[2 * (x >> 1) + 1], (uint32_t)(x & 1));
}

// UPPER predicate for occurrence ranges: the first min(m, len) chars of
// suffix(x) compare > q (x is past every suffix that starts with q).
//   m <= 32: key > Q3, Q3 = q's 32-char key padded with 3s instead of 0s
//   m >  32: key != K64 -> key > K64; else exact compare from char 32
template <int QW>
__device__ __forceinline__ bool sector_gt_prefix(uint64_t key, uint64_t p, uint64_t K64, uint64_t Q3,
                                                 const SearchArgs& a, const QueryRegs<QW>& q) {
    if (QW == 1 || q.m <= 32) return key > Q3;
    if (key != K64) return key > K64;
    uint32_t lcp;
    bool lt = suffix_less_from<QW>(a.tw, a.n, p, q, 32, &lcp);
    return !lt && lcp < q.m;
}

// First local rank x with pred(x) (pred monotone over ranks, false before the
// routed leaf), by descent on the 16-char key R16, the routed leaf, and an
// exponential + binary search on the leaf array for runs that cross leaves.
template <int QW, bool UPPER>
__device__ __forceinline__ uint64_t sector_bound(const SearchArgs& a, const uint4* s_nodes, const QueryRegs<QW>& q,
                                                 uint64_t K64, uint64_t Q3, uint32_t* probes, uint64_t* px) {
    const uint64_t sa_n = a.sa_n;
    const uint4* leaves = a.sec_leaves;
    const uint4* g = reinterpret_cast<const uint4*>(a.sec_inner);
    const uint32_t R16 = (uint32_t)(((UPPER && q.m <= 32) ? Q3 : K64) >> 32);
    auto pred = [&](uint64_t key, uint64_t p) -> bool {
        return UPPER ? sector_gt_prefix<QW>(key, p, K64, Q3, a, q) : sector_ge<QW, true>(key, p, K64, a, q);
    };
    uint64_t k = 0;
    auto count8 = [&](uint4 v0, uint4 v1) -> uint32_t {
        return (v0.x < R16) + (v0.y < R16) + (v0.z < R16) + (v0.w < R16) + (v1.x < R16) + (v1.y < R16) +
               (v1.z < R16) + (v1.w < R16);
    };
    // LDS layers, then HBM layers (separate loops: ds_read / global_load, not FLAT)
    uint32_t h = 0;
    for (; h < a.sec_lds_layers; h++) {
        const uint4* node = s_nodes + (a.sec_off[h] + k) * 2;
        k = k * SAS_SECTOR_FAN + count8(node[0], node[1]);
    }
    for (; h < a.sec_inner_layers; h++) {
        const uint4* node = g + (a.sec_off[h] + k) * 2;
        k = k * SAS_SECTOR_FAN + count8(node[0], node[1]);
    }
    *probes += a.sec_inner_layers;
    // leaf k: entries 2k, 2k+1 (everything before 2k fails pred)
    // (non-temporal loads here measured 8% slower: tools/ab_nt2.sh)
    uint4 kv = leaves[2 * k], sv = leaves[2 * k + 1];
    (*probes)++;
    uint64_t key0 = (uint64_t)kv.x | ((uint64_t)kv.y << 32), key1 = (uint64_t)kv.z | ((uint64_t)kv.w << 32);
    const uint64_t p0 = sector_sa(sv, 0), p1 = sector_sa(sv, 1);
    if (2 * k < sa_n && pred(key0, p0)) {
        *px = p0;
        return 2 * k;
    }
    if (2 * k + 1 < sa_n && pred(key1, p1)) {
        *px = p1;
        return 2 * k + 1;
    }
    // rare: a run of entries sharing the routing key continues to the right --
    // exponential search, then binary search, on the leaf array
    uint64_t lo = 2 * k + 2, step = 1, hi;
    if (lo >= sa_n) return sa_n;
    for (;;) {
        hi = lo + step - 1;
        if (hi >= sa_n) { hi = sa_n; break; }
        uint64_t kk, pp;
        sector_entry(leaves, hi, &kk, &pp);
        (*probes)++;
        if (pred(kk, pp)) break;
        lo = hi + 1;
        step *= 2;
    }
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        uint64_t kk, pp;
        sector_entry(leaves, mid, &kk, &pp);
        (*probes)++;
        if (pred(kk, pp)) hi = mid;
        else lo = mid + 1;
    }
    if (lo < sa_n) {
        uint64_t kk;
        sector_entry(leaves, lo, &kk, px);
    }
    return lo;
}

__device__ __forceinline__ void stage_sector_top(const SearchArgs& a, uint4* s_nodes) {
    const uint4* g = reinterpret_cast<const uint4*>(a.sec_inner);
    for (uint32_t w = threadIdx.x; w < a.sec_lds_nodes * 2; w += blockDim.x) s_nodes[w] = g[w];
    __syncthreads();
}

template <int QW>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_sector(SearchArgs a) {
    __shared__ uint4 s_nodes[SAS_SECTOR_LDS_NODES * 2];
    stage_sector_top(a, s_nodes);
    uint32_t bad = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        uint32_t probes = 0;
        uint64_t px = 0;
        uint64_t x = sector_bound<QW, false>(a, s_nodes, q, q.w[0], 0, &probes, &px);
        a.out_pos[i] = (x >= a.sa_n) ? a.next_pos : px;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// Occurrence ranges: global ranks [lo, hi) of the suffixes that start with q.
// out_pos = lo, out_hi = hi (both rank_lo-based).
template <int QW>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_sector_range(SearchArgs a, uint64_t* out_hi) {
    __shared__ uint4 s_nodes[SAS_SECTOR_LDS_NODES * 2];
    stage_sector_top(a, s_nodes);
    uint32_t bad = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        uint32_t probes = 0;
        uint64_t px = 0;
        uint64_t lo = sector_bound<QW, false>(a, s_nodes, q, K64, Q3, &probes, &px);
        uint64_t hi = sector_bound<QW, true>(a, s_nodes, q, K64, Q3, &probes, &px);
        if (hi < lo) hi = lo;
        a.out_pos[i] = a.rank_lo + lo;
        out_hi[i] = a.rank_lo + hi;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ QUAD
// Levels far larger than the 256 MiB Infinity Cache (quad_nt_from.., the leaves when
// quad_leaf_nt) are read with non-temporal loads so they do not evict the upper layers
// from L2; the query stream and the positions likewise (SAS_QUAD_NT_IO).  Same-box
// A/B at n = 2^30 (tools/ab_nt.sh): absolute layout 0.760 -> 0.713 ms, relative
// 0.790 -> 0.734 ms; NT on a level that partly fits the Infinity Cache (the 554 MB
// relative leaf-parent layer, the 59 MB absolute one) made it slower.
#ifndef SAS_QUAD_NT_IO
#define SAS_QUAD_NT_IO 1
#endif
__device__ __forceinline__ uint4 quad_leaf_load(const SearchArgs& a, const uint4* p) {
    return a.quad_leaf_nt ? nt_load4(p) : *p;
}

// A 4-lane group per query.  Every node is 64 B and the group loads it with one
// 16-B load per lane, which the memory system serves as ONE request (a per-lane
// 32-B node costs two): tools/treebench measured 19-22 ps per DRAM-level 64-B
// group load vs 26.5 ps for a per-lane 32-B node.  Inner nodes: 16 left-max
// 16-char separators, 17-ary; lane j counts its 4, the group sums by shuffles.
// Leaves: 4 entries {key64, SA}, lane j evaluates entry j, a group ballot picks
// the first entry >= q.  All branches are group-uniform.
// m <= 32 queries at an 8-B aligned address with m % 8 == 0 (the headline shape):
// lane j of the group loads bytes 8j..8j+7 (one contiguous 32-B request per query
// instead of two 16-B halves per lane) and packs them to 16 bits; the group ORs the
// four parts with DPP quad_perm moves.
__device__ __forceinline__ uint64_t quad_key32(const uint8_t* __restrict__ qb, uint32_t m, uint32_t sub,
                                               uint32_t* bad) {
    uint32_t part = 0;
    if (8 * sub < m) {
        uint2 v;
        if (SAS_QUAD_NT_IO) {  // the query stream is read once: keep it out of L2
            const uint64_t w = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(qb + 8 * sub));
            v = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
        } else {
            v = *reinterpret_cast<const uint2*>(qb + 8 * sub);
        }
        *bad |= (v.x | v.y) & 0xFCFCFCFCu;
        part = (pack4(v.x) << 8) | pack4(v.y);
    }
    // chars 8j..8j+7 -> bits 63-16j .. 48-16j
    uint32_t hi = (sub < 2) ? (part << (16 - 16 * sub)) : 0u;
    uint32_t lo = (sub >= 2) ? (part << (16 - 16 * (sub - 2))) : 0u;
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x4E, 0xF, 0xF, false);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x4E, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

// Leaf formats (KO = key-only, SAS_BUILD_QUAD_COMPACT):
//   fused: entry x = 16 B {key64, SA lo32, SA bits 32..39}, 4 per 64-B leaf
//   KO:    entry x = key64, 8 per 64-B leaf; SA values come from the SA array
// Per-lane reads of one entry (the tails of the 4x kernel, INLINE's probes):
template <bool KO>
__device__ __forceinline__ uint64_t quad_entry_key(const SearchArgs& a, uint64_t x) {
    if (KO) return reinterpret_cast<const uint64_t*>(a.quad_leaves)[x];
    const uint2 k = reinterpret_cast<const uint2*>(a.quad_leaves)[2 * x];
    return (uint64_t)k.x | ((uint64_t)k.y << 32);
}
template <bool KO, int W>
__device__ __forceinline__ uint64_t quad_entry_sa(const SearchArgs& a, uint64_t x) {
    if (KO) return SaView<W>{a.sa}[x];
    const uint2 s = reinterpret_cast<const uint2*>(a.quad_leaves)[2 * x + 1];
    return (uint64_t)s.x | ((uint64_t)(s.y & 0xFFu) << 32);
}

#define QUAD_NO_SA (~0ull)  // "SA value not read yet" (never a valid 40-bit SA)

// Evaluate leaf L for the bound's predicate (UPPER = false: suffix(x) >= q;
// UPPER = true: the first min(m, len) chars of suffix(x) are > q, sector_gt_prefix).
// Returns the first qualifying entry of the leaf (EPL if none; entries x >= sa_n
// never qualify) and *p = its SA value, group-uniform (KO: QUAD_NO_SA when the
// predicate did not need it).  Fused leaves: lane j holds entry j; KO leaves: lane j
// holds entries 2j, 2j+1 and reads an SA value only for an entry whose key ties q's.
template <int QW, bool UPPER, bool KO, int W>
__device__ __forceinline__ uint32_t quad_leaf(const SearchArgs& a, const QueryRegs<QW>& q, uint64_t K64, uint64_t Q3,
                                              uint64_t L, uint32_t sub, uint64_t* p) {
    const int lane0 = (int)((threadIdx.x & 63) & ~3u);
    const uint4 e = quad_leaf_load(a, a.quad_leaves + 4 * L + sub);
    // short-circuit: padding entries (x >= sa_n) carry all-ones keys/SA and must never
    // reach the predicate (its m > 32 text compare would read past the text)
    auto pred = [&](uint64_t key, uint64_t pp) -> bool {
        return UPPER ? sector_gt_prefix<QW>(key, pp, K64, Q3, a, q) : sector_ge<QW>(key, pp, K64, a, q);
    };
    if (!KO) {
        const uint64_t x = 4 * L + sub;
        const uint64_t key = (uint64_t)e.x | ((uint64_t)e.y << 32);
        const uint64_t pp = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
        const uint32_t mk = quad_mask(x < a.sa_n && pred(key, pp));
        const uint32_t f = mk ? (uint32_t)__builtin_ctz(mk) : 4u;
        *p = __shfl((unsigned long long)pp, lane0 + (int)(f & 3), 64);
        return f;
    }
    const uint64_t x0 = 8 * L + 2 * sub;
    const uint64_t k0 = (uint64_t)e.x | ((uint64_t)e.y << 32), k1 = (uint64_t)e.z | ((uint64_t)e.w << 32);
    // the SA value matters only on a tie with q's 32-char key (UPPER with m <= 32: never)
    const bool tie_ok = !(UPPER && q.m <= 32);
    uint64_t p0 = QUAD_NO_SA, p1 = QUAD_NO_SA;
    if (tie_ok && k0 == K64 && x0 < a.sa_n) p0 = quad_entry_sa<true, W>(a, x0);
    if (tie_ok && k1 == K64 && x0 + 1 < a.sa_n) p1 = quad_entry_sa<true, W>(a, x0 + 1);
    const bool t0 = x0 < a.sa_n && pred(k0, p0);
    const bool t1 = x0 + 1 < a.sa_n && pred(k1, p1);
    const uint32_t many = quad_mask(t0 || t1), m0 = quad_mask(t0);
    if (!many) {
        *p = QUAD_NO_SA;
        return 8;
    }
    const uint32_t j = (uint32_t)__builtin_ctz(many);
    const uint32_t s = ((m0 >> j) & 1u) ? 0u : 1u;  // entry 2j (t0) or 2j+1
    *p = __shfl((unsigned long long)(s ? p1 : p0), lane0 + (int)j, 64);
    return 2 * j + s;
}

// Inner-node descent of the 4-lane group to the leaf for routing key R (a padded
// 32-char key).  Absolute nodes (quad_fan 17): lane j counts its 4 of the 16 u32
// 16-char separators < R's first 16 chars.  Prefix-relative nodes (quad_fan 31,
// k_quad_rel_layer): lane 0's word 0 is the header {d, P}, broadcast to the group;
// if R's first d chars equal P, the child is the count of 16-bit separators below
// R's chars [d, d+8); if they are below P every entry of the subtree is >= R (child
// 0), if above, every entry is < R (the last child; a layer's last node, which may
// have fewer children, has d = 0, so it never answers "above").  Either way every
// entry before the chosen child is < R, the invariant the leaf search needs.
typedef short quad_short2 __attribute__((ext_vector_type(2)));
// sign bits (15, 31) of the saturating packed i16 difference w - tt: set where the
// 16-bit half of w is below tt's (both stored XOR 0x8000, so signed order = unsigned)
__device__ __forceinline__ uint32_t lt2_signs(uint32_t w, uint32_t tt) {
    const quad_short2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(quad_short2, w),
                                                        __builtin_bit_cast(quad_short2, tt));
    return __builtin_bit_cast(uint32_t, d);
}

// m0 = 0 on lane 0 of the group (its word 0 is the header), 0x80008000 elsewhere
__device__ __forceinline__ uint32_t quad_rel_child(uint4 v, uint64_t R, uint32_t m0) {
    const uint32_t hdr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x00, 0xF, 0xF, false);
    const uint64_t full = R >> (48 - ((hdr >> 26) & 62u));  // R's chars [0, d + 8)
    const uint32_t Qd = (uint32_t)(full >> 16), P = hdr & 0x7FFFFFFu;
    const uint32_t T = (uint32_t)full & 0xFFFFu;
    const uint32_t tt = (T | (T << 16)) ^ 0x80008000u;
    uint32_t c = __builtin_popcount(lt2_signs(v.x, tt) & m0);
    c += __builtin_popcount(lt2_signs(v.y, tt) & 0x80008000u);
    c += __builtin_popcount(lt2_signs(v.z, tt) & 0x80008000u);
    c += __builtin_popcount(lt2_signs(v.w, tt) & 0x80008000u);
    c = quad_sum(c);
    return Qd == P ? c : (Qd < P ? 0u : SAS_QUAD_RFAN - 1);
}

__device__ __forceinline__ uint32_t quad_abs_child(uint4 v, uint32_t R16) {
    return quad_sum((v.x < R16) + (v.y < R16) + (v.z < R16) + (v.w < R16));
}

// Both loops are unrolled over the layer index so the per-layer offsets (kernel
// arguments) are loop-invariant scalar loads hoisted out of the query loop; the leaf
// index fits 32 bits (build_quad refuses more than 2^32 leaves).
template <bool REL>
__device__ __forceinline__ uint32_t quad_descend_t(const SearchArgs& a, const uint4* s_nodes, uint64_t R, uint32_t sub) {
    const uint32_t R16 = (uint32_t)(R >> 32);
    const uint32_t m0 = sub ? 0x80008000u : 0u;
    uint32_t k = 0;
    // LDS layers, then HBM layers: separate loops keep the loads ds_read / global_load
    // (a pointer select between the two address spaces compiles to FLAT loads)
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_LDS; h++) {
        if (h < a.quad_lds_layers) {
            const uint4 v = s_nodes[((uint32_t)a.quad_off[h] + k) * 4 + sub];
            k = REL ? k * SAS_QUAD_RFAN + quad_rel_child(v, R, m0) : k * SAS_QUAD_FAN + quad_abs_child(v, R16);
        }
    }
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_INNER; h++) {
        if (h >= a.quad_lds_layers && h < a.quad_inner_layers) {
            const uint4* pv = a.quad_inner + (a.quad_off[h] + k) * 4 + sub;
            const uint4 v = h >= a.quad_nt_from ? nt_load4(pv) : *pv;
            k = REL ? k * SAS_QUAD_RFAN + quad_rel_child(v, R, m0) : k * SAS_QUAD_FAN + quad_abs_child(v, R16);
        }
    }
    return k;
}

__device__ __forceinline__ uint64_t quad_descend(const SearchArgs& a, const uint4* s_nodes, uint64_t R, uint32_t sub) {
    return a.quad_fan == SAS_QUAD_RFAN ? quad_descend_t<true>(a, s_nodes, R, sub)
                                       : quad_descend_t<false>(a, s_nodes, R, sub);
}

// First local rank with the bound's predicate (monotone over ranks): descent on the
// 16-char routing key, the routed leaf, then (rare) an exponential + binary search
// over later leaves for a run of equal routing keys that crosses leaves.  Returns
// sa_n if no entry qualifies; *px = SA at the returned rank (group-uniform;
// QUAD_NO_SA if a KO leaf did not need it).
template <int QW, bool UPPER, bool KO, int W>
__device__ __forceinline__ uint64_t quad_bound(const SearchArgs& a, const uint4* s_nodes, const QueryRegs<QW>& q,
                                               uint64_t K64, uint64_t Q3, uint32_t sub, uint32_t* probes,
                                               uint64_t* px) {
    constexpr uint32_t EPL = KO ? 8 : 4;
    const uint64_t nl = a.quad_leaf_count;
    const uint64_t k = quad_descend(a, s_nodes, (UPPER && q.m <= 32) ? Q3 : K64, sub);
    *probes += a.quad_inner_layers + 1;
    // routed leaf k: every entry before it fails the predicate
    uint64_t pl;
    uint32_t f = quad_leaf<QW, UPPER, KO, W>(a, q, K64, Q3, k, sub, &pl);
    uint64_t L = k;
    if (f == EPL) {
        // leaf nl = virtual: past every entry
        uint64_t lo = k + 1, step = 1, hi = nl;
        while (lo < nl) {
            hi = lo + step - 1;
            if (hi >= nl) { hi = nl; break; }
            uint64_t pp;
            (*probes)++;
            if (quad_leaf<QW, UPPER, KO, W>(a, q, K64, Q3, hi, sub, &pp) < EPL) break;
            lo = hi + 1;
            step *= 2;
            hi = nl;
        }
        while (lo < hi) {
            uint64_t mid = (lo + hi) >> 1;
            uint64_t pp;
            (*probes)++;
            if (quad_leaf<QW, UPPER, KO, W>(a, q, K64, Q3, mid, sub, &pp) < EPL) hi = mid;
            else lo = mid + 1;
        }
        L = lo;
        if (L < nl) {
            f = quad_leaf<QW, UPPER, KO, W>(a, q, K64, Q3, L, sub, &pl);
            (*probes)++;
        }
    }
    if (f == EPL) return a.sa_n;
    *px = pl;
    return EPL * L + f;
}

__device__ __forceinline__ void stage_quad_top(const SearchArgs& a, uint4* s_nodes) {
    for (uint32_t w = threadIdx.x; w < a.quad_lds_nodes * 4; w += blockDim.x) s_nodes[w] = a.quad_inner[w];
    __syncthreads();
}

template <int QW, bool KO, int W>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_quad(SearchArgs a) {
    __shared__ uint4 s_nodes[SAS_QUAD_LDS_NODES * 4];
    stage_quad_top(a, s_nodes);
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    uint32_t bad = 0;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G; i < a.nq; i += stride) {
        if (!slot_live(a, i)) continue;  // group-uniform: the 4 lanes share i
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        if (QW == 1 && a.qoff == nullptr && (m & 7) == 0 && (((uintptr_t)qb) & 7) == 0) {
            q.bytes = qb;
            q.m = m;
            q.w[0] = quad_key32(qb, m, sub, &bad);
        } else {
            q.load(qb, m, &bad);
        }
        uint32_t probes = 0;
        uint64_t px = 0;
        const uint64_t x = quad_bound<QW, false, KO, W>(a, s_nodes, q, q.w[0], 0, sub, &probes, &px);
        if (KO && x < a.sa_n && px == QUAD_NO_SA) px = quad_entry_sa<true, W>(a, x);  // group-uniform address
        if (sub == 0) {
            const uint64_t res = (x >= a.sa_n) ? a.next_pos : px;
            if (SAS_QUAD_NT_IO) __builtin_nontemporal_store(res, a.out_pos + i);
            else a.out_pos[i] = res;
            if (a.out_probes) a.out_probes[i] = probes;
        }
    }
    if (bad) atomicOr(a.bad, 1u);
}

// tail_less32 prefetch in the 4x tails: measured 4-6% slower (more spills), so off
// query words the 4x kernel holds in registers (later words are repacked from the
// bytes): 2 measured ~2% faster than 4/8 (fewer spills) on ragged 8..256 queries
#ifndef SAS_QUAD4X_MAXREGS
#define SAS_QUAD4X_MAXREGS 2
#endif
#ifndef SAS_QUAD4X_PREFETCH
#define SAS_QUAD4X_PREFETCH false
#endif
// The per-lane finish of k_sa_quad4x: every entry before x0 is < q (the routed leaf's count
// of 32-char keys below q's); key0 / p0 = entry x0's key and SA value when the leaf read
// delivered them (known).  The predicate at x0 (a key tie: one text compare from char 32),
// and in the rare case it fails an exponential + binary search over the following entries.
// Returns the position.
template <int QW, bool KO, int W, class Q>
__device__ __forceinline__ uint64_t quad_x0_finish(const SearchArgs& a, const Q& q, uint64_t K64,
                                                   uint64_t x0, bool known, uint64_t key0, uint64_t p0,
                                                   uint32_t* probes) {
    const uint64_t sa_n = a.sa_n;
    bool ok = false;
    if (x0 < sa_n) {
        const uint64_t key = known ? key0 : quad_entry_key<KO>(a, x0);
        if (key != K64) {
            ok = key > K64;
        } else {
            if (p0 == QUAD_NO_SA) p0 = quad_entry_sa<KO, W>(a, x0);
            ok = sector_ge<QW, SAS_QUAD4X_PREFETCH, false, Q>(key, p0, K64, a, q);
        }
        if (!known) (*probes)++;
    }
    uint64_t x = x0;
    if (!ok && x0 < sa_n) {  // rare: exponential + binary search over x0+1 ..
        auto pred = [&](uint64_t y) -> bool {
            const uint64_t key = quad_entry_key<KO>(a, y);
            if (key != K64) return key > K64;
            return sector_ge<QW, SAS_QUAD4X_PREFETCH, false, Q>(key, quad_entry_sa<KO, W>(a, y), K64, a, q);
        };
        uint64_t lo = x0 + 1, hi = sa_n, step = 1;
        while (lo < sa_n) {
            hi = lo + step - 1;
            if (hi >= sa_n) { hi = sa_n; break; }
            (*probes)++;
            if (pred(hi)) break;
            lo = hi + 1;
            step *= 2;
            hi = sa_n;
        }
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            (*probes)++;
            if (pred(mid)) hi = mid;
            else lo = mid + 1;
        }
        x = lo;
        p0 = QUAD_NO_SA;
    }
    if (x >= sa_n) return a.next_pos;
    return (p0 != QUAD_NO_SA) ? p0 : quad_entry_sa<KO, W>(a, x);
}

// Long queries (QW > 1), as k_sa_stree4x: one query per LANE, four per 4-lane group.
// The group descends the quad tree and reads the routed leaf cooperatively for each
// of its four queries in turn (one request per 64-B node), which places each query
// at x0 = the first entry of that leaf whose 32-char key is >= its own (the entry's
// key and fused SA value travel to the owning lane by a shuffle).  Every entry
// before x0 is < q.  Then every lane finishes its own query: the predicate at x0
// (typically a key tie -> one text compare from char 32, the part that dominates for
// long queries), and in the rare case it fails an exponential + binary search over
// the following entries.
// RP: queries longer than QW register words (their later words repacked from the bytes)
template <int QW, bool KO, int W, bool RP>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_quad4x(SearchArgs a) {
    using QR = typename std::conditional<RP, QueryRegsRepack<QW>, QueryRegs<QW>>::type;
    constexpr uint32_t EPL = KO ? 8 : 4;
    __shared__ uint4 s_nodes[SAS_QUAD_LDS_NODES * 4];
    stage_quad_top(a, s_nodes);
    uint32_t bad = 0;
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~3u);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // the loop runs while ANY query of the group is in range (group-uniform)
    for (uint64_t gi = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) - sub; gi < a.nq; gi += stride) {
        const uint64_t i = gi + sub;
        const bool mine = i < a.nq;
        const uint8_t* qb;
        uint32_t m = 0;
        QR q;
        if (mine) {
            query_ptr(a, i, &qb, &m);
            q.load(qb, m, &bad);
        } else {
            q.bytes = a.qbytes;
            q.m = 0;
            for (int j = 0; j < QW; j++) q.w[j] = 0;
        }
        const uint64_t Kmine = q.w[0];  // padded 32-char key of this lane's query
        uint32_t probes = a.quad_inner_layers + 1;
        uint64_t x0 = 0, key0 = 0, p0 = QUAD_NO_SA;
        bool known = false;
        for (uint32_t j = 0; j < QUAD_G; j++) {
            if (gi + j >= a.nq) break;  // group-uniform
            const uint64_t K64 = __shfl((unsigned long long)Kmine, lane0 + (int)j, 64);
            const uint64_t k = quad_descend(a, s_nodes, K64, sub);
            const uint4 e = quad_leaf_load(a, a.quad_leaves + 4 * k + sub);
            uint64_t ksel, psel = QUAD_NO_SA;
            uint32_t c;
            if (KO) {
                const uint64_t ka = (uint64_t)e.x | ((uint64_t)e.y << 32), kb = (uint64_t)e.z | ((uint64_t)e.w << 32);
                c = quad_sum((ka < K64) + (kb < K64));
                ksel = (c & 1) ? kb : ka;
            } else {
                ksel = (uint64_t)e.x | ((uint64_t)e.y << 32);
                psel = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
                c = quad_sum(ksel < K64);
            }
            const int src = lane0 + (int)((KO ? c >> 1 : c) & 3);
            const uint64_t kc = __shfl((unsigned long long)ksel, src, 64);
            const uint64_t pc = KO ? QUAD_NO_SA : __shfl((unsigned long long)psel, src, 64);
            if (sub == j) {
                x0 = EPL * k + c;
                known = c < EPL;  // else x0 starts the next leaf: nothing read for it yet
                key0 = kc;
                p0 = known ? pc : QUAD_NO_SA;
            }
        }
        if (!mine) continue;
        const uint64_t pos = quad_x0_finish<QW, KO, W, QR>(a, q, Kmine, x0, known, key0, p0, &probes);
        a.out_pos[i] = pos;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}


// quad_x0_finish for a query of m <= 32 chars on fused leaves: the 32-char key and the
// suffix length decide every entry (sector_ge's m <= 32 case), so no text is compared
__device__ __forceinline__ uint64_t quad_short_finish(const SearchArgs& a, uint64_t K64, uint32_t m, uint64_t x0,
                                                      bool known, bool eq0, uint64_t p0, uint32_t* probes) {
    const uint64_t sa_n = a.sa_n;
    auto pred = [&](uint64_t y, uint64_t* py) -> bool {
        const uint4 e = a.quad_leaves[y];
        const uint64_t key = (uint64_t)e.x | ((uint64_t)e.y << 32);
        *py = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
        if (key != K64) return key > K64;
        return a.n - *py >= (uint64_t)m;
    };
    if (x0 >= sa_n) return a.next_pos;
    bool ok;
    if (known) {
        ok = !eq0 || a.n - p0 >= (uint64_t)m;
    } else {
        ok = pred(x0, &p0);
        (*probes)++;
    }
    if (ok) return p0;
    // rare: exponential + binary search over x0+1 ..
    uint64_t lo = x0 + 1, hi = sa_n, step = 1, py;
    while (lo < sa_n) {
        hi = lo + step - 1;
        if (hi >= sa_n) { hi = sa_n; break; }
        (*probes)++;
        if (pred(hi, &py)) break;
        lo = hi + 1;
        step *= 2;
        hi = sa_n;
    }
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        (*probes)++;
        if (pred(mid, &py)) hi = mid;
        else lo = mid + 1;
    }
    if (lo >= sa_n) return a.next_pos;
    (*probes)++;
    pred(lo, &py);
    return py;
}

// ------------------------------------------------------------------ QUAD_LLCP
// configs[2] as one kernel (SAS_ALGO_QUAD_LLCP): QUAD's descent over the fused 32-char keys,
// and where the routed leaf does not settle the query, Manber-Myers LLCP skipping
// (the SAS_BUILD_LLCP entries, as stree_tail<.., true>) inside the run of suffixes that share
// q's key.  Absolute layout (quad_fan 17: 16-char left-max separators), fused leaves.
//
// The descent routes on q's 16-char key K16, so leaf k holds the first suffix whose 16-char key
// is >= K16 (s0 = 4k + count(key16 < K16)), and every suffix before it has key16 < K16.  At
// every inner node the group also counts the separators <= K16: the first level where that
// count exceeds the < K16 one is where the path of K16 + 1 leaves q's path (a run of equal
// 16-char keys spans at most a few leaves, so the paths part near the leaves), and the
// suffixes past q's 16-char run are found by descending from there -- one or two requests
// instead of a second descent from the root.  From the leaves' 32-char keys:
//   L0 = 4k + count(key64 < K64): every suffix before L0 is < q;
//   U  = the first suffix whose key64 > K64 (leaf k, or the leaf of K16 + 1 when it holds a
//        key <= K64), else the end s1 of the 16-char run: every suffix from U on is > q.
// A query that the leaf settles (the common case on random text: U <= L0 + 1) costs QUAD's
// reads and at most one text compare (k_sa_quad4x's).  Otherwise the LLCP walk runs from the
// root of the entries' implicit binary-search tree: a mid below L0 goes right and one at or
// past U goes left with no read; a mid in [L0, U) reads its 16-B entry.  A bound that no read
// measured takes an lcp as stree_tail does -- the entry's own Llcp / Rlcp, which makes that
// side tie (so the probe compares from there) -- except a left bound inside leaf k, whose exact
// lcp with q the leaf's 32-char key gives (min(first differing char, suffix length)).  That
// substitution is sound because every mid read lies in q's 16-char run [s0, s1), and in q's
// 32-char run when both L0 and U are exact at 32 chars (kappa = 32): then a ties' compare
// starts at char kappa (a suffix shorter than kappa in the run is a proper prefix of q).
// Queries of <= 32 chars in a ragged batch finish as k_sa_quad4x's do (their 32-char key
// decides every entry).  out_probes: inner levels + leaves + entries + text compares read.
template <int QW, class Q>
__device__ __forceinline__ bool qllcp_tie_less(const SearchArgs& a, uint64_t p, const Q& q, uint32_t hh, uint32_t inl,
                                               uint32_t kappa, uint32_t* lcp) {
    const uint64_t lenS = a.n - p;
    if (lenS < kappa) {  // its padded key matched q's: a proper prefix of q (m > 32)
        *lcp = (uint32_t)lenS;
        return true;
    }
    uint32_t h = kappa;
    if (hh + 16 > kappa) {
        // llcp_tie_less: the entry's 16 chars after hh first (those below kappa compare equal)
        const uint32_t L = lenS < (uint64_t)q.m ? (uint32_t)lenS : q.m;
        if (hh < L) {
            const uint32_t c = L - hh < 16 ? L - hh : 16;
            const uint32_t mk = ~0u << (32 - 2 * c);
            const uint32_t av = inl & mk, bv = (uint32_t)(q.chars32(hh) >> 32) & mk;
            if (av != bv) {
                *lcp = hh + (uint32_t)(__clz(av ^ bv) >> 1);
                return av < bv;
            }
        }
        h = hh + 16;
    }
    return suffix_less_from<QW>(a.tw, a.n, p, q, h, lcp);
}

#define QLLCP_NONE 0xFFu

// k_sa_quad_llcp's workgroup size (two workgroups a CU): 768 -> 6 waves a SIMD, 80 VGPRs;
// 512 -> 4 waves, 128 VGPRs
#ifndef SAS_QLLCP_BLOCK
#define SAS_QLLCP_BLOCK 768
#endif
// ... for m > 64 (4 or 8 query words in registers)
#ifndef SAS_QLLCP_BLOCK_LONG
#define SAS_QLLCP_BLOCK_LONG 768
#endif
#define QLLCP_BLOCK(QW) ((QW) <= 2 ? SAS_QLLCP_BLOCK : SAS_QLLCP_BLOCK_LONG)
// descent on K16 recording where K16 + 1's path parts from it (level, node index one level down)
__device__ __forceinline__ uint32_t quad_descend_split(const SearchArgs& a, const uint4* s_nodes, uint32_t K16,
                                                       uint32_t sub, uint32_t* dlev, uint32_t* dnode) {
    uint32_t k = 0, dl = QLLCP_NONE, dn = 0;
    auto step = [&](uint4 v, uint32_t h) {
        const uint32_t lt = (v.x < K16) + (v.y < K16) + (v.z < K16) + (v.w < K16);
        const uint32_t le = (v.x <= K16) + (v.y <= K16) + (v.z <= K16) + (v.w <= K16);
        const uint32_t cc = quad_sum(lt | (le << 8));
        const uint32_t c = cc & 0xFFu, c2 = cc >> 8;
        if (dl == QLLCP_NONE && c2 > c) {
            dl = h;
            dn = k * SAS_QUAD_FAN + c2;
        }
        k = k * SAS_QUAD_FAN + c;
    };
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_LDS; h++)
        if (h < a.quad_lds_layers) step(s_nodes[((uint32_t)a.quad_off[h] + k) * 4 + sub], h);
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_INNER; h++) {
        if (h >= a.quad_lds_layers && h < a.quad_inner_layers) {
            const uint4* pv = a.quad_inner + (a.quad_off[h] + k) * 4 + sub;
            step(h >= a.quad_nt_from ? nt_load4(pv) : *pv, h);
        }
    }
    *dlev = dl;
    *dnode = dn;
    return k;
}

// K16 + 1's descent from node k of level h0 (separators <= K16 = < K16 + 1)
__device__ __forceinline__ uint32_t quad_descend_from(const SearchArgs& a, const uint4* s_nodes, uint32_t h0,
                                                      uint32_t k, uint32_t K16, uint32_t sub) {
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_LDS; h++) {
        if (h >= h0 && h < a.quad_lds_layers) {
            const uint4 v = s_nodes[((uint32_t)a.quad_off[h] + k) * 4 + sub];
            k = k * SAS_QUAD_FAN + quad_sum((v.x <= K16) + (v.y <= K16) + (v.z <= K16) + (v.w <= K16));
        }
    }
#pragma unroll
    for (uint32_t h = 0; h < SAS_QUAD_MAX_INNER; h++) {
        if (h >= h0 && h >= a.quad_lds_layers && h < a.quad_inner_layers) {
            const uint4* pv = a.quad_inner + (a.quad_off[h] + k) * 4 + sub;
            const uint4 v = h >= a.quad_nt_from ? nt_load4(pv) : *pv;
            k = k * SAS_QUAD_FAN + quad_sum((v.x <= K16) + (v.y <= K16) + (v.z <= K16) + (v.w <= K16));
        }
    }
    return k;
}

// the per-query state a lane keeps between the group steps, packed (k_sa_quad_llcp)
#define QL_C16(st) ((st) & 7u)           // leaf k's keys16 < K16
#define QL_C64(st) (((st) >> 3) & 7u)    // leaf k's keys64 < K64 (4: none >= K64 in it)
#define QL_FU(st) (((st) >> 6) & 7u)     // U = 4 kU + FU
#define QL_KNOWN (1u << 9)               // leaf k holds a key >= K64 (L0 exact at 32 chars)
#define QL_EQ0 (1u << 10)                // ... and it is K64
#define QL_UK (1u << 11)                 // U known
#define QL_X32 (1u << 12)                // U exact at 32 chars too: q's 32-char run
#define QL_LAM0 (1u << 13)               // entry L0 compared below q: L0 + 1, its lcp in lcp0
#define QL_END (1u << 14)                // q's 16-char run reaches the end: U = sa_n
#define QL_DLEV(st) ((st) >> 24)         // where K16 + 1's path parts from q's (QLLCP_NONE: not)
// leaf k's keys all below q's (L0 past it): read the next entry to settle q as k_sa_quad4x
// would (1), or go to the walk from L0 = 4k + 4 with kappa 16 (0), or read it only when just
// leaf k's last entry shares q's 16-char key (2).  On random text that is the usual shape of
// the case (one other suffix with q's 16-char key below q, a leaf boundary between them) and
// the next entry is q's; on repetitive text a 16-char run fills more of the leaf and the
// next entry is rarely L0 itself, so the read would mostly be wasted
#ifndef SAS_QLLCP_NEXT
#define SAS_QLLCP_NEXT 2
#endif

// k_sa_quad_llcp: the group step (descent, leaf, counts), the settle (k_sa_quad4x's reads: the
// first entry not below q's 32-char key and at most one compare), then for what that does not
// settle U (where the run leaves leaf k; cooperative) and the LLCP walk.  (Round 6 also
// measured it split in two kernels, the unsettled queries' state handed over in a list: the
// list's scattered query and result accesses cost more than the split saved)
// EXACT: launched only with m <= 32 QW (QueryRegsExact: no repacking from the bytes);
// R32: sa_n < 2^32, the walk's ranks in 32 bits
template <int QW, bool EXACT, bool R32>
__global__ __launch_bounds__(QLLCP_BLOCK(QW), QLLCP_BLOCK(QW) * 2 / 256) void k_sa_quad_llcp(SearchArgs a) {
    using QR = typename std::conditional<EXACT, QueryRegsExact<QW>, QueryRegsRepack<QW>>::type;
    __shared__ uint4 s_nodes[SAS_QUAD_LDS_NODES * 4];
    stage_quad_top(a, s_nodes);
    uint32_t bad = 0;
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~3u);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t gi = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) - sub; gi < a.nq; gi += stride) {
        const uint64_t i = gi + sub;
        const bool mine = i < a.nq;
        const uint8_t* qb;
        uint32_t m = 0;
        QR q;
        if (mine) {
            query_ptr(a, i, &qb, &m);
            q.load(qb, m, &bad);
        } else {
            q.bytes = a.qbytes;
            q.m = 0;
            for (int j = 0; j < QW; j++) q.w[j] = 0;
        }
        const uint64_t Kmine = q.w[0];
        uint32_t probes = a.quad_inner_layers + 1;
        // this lane's query, from its group step: leaf k, the leaf kU of U, the packed counts and
        // flags (QL_*), leaf k's entries' lcps with q (8 bits each), K16 + 1's node below its
        // parting level, and the SA values at L0 and U when a leaf read delivered them
        uint32_t kq = 0, st = 0, lam = 0, dnode = 0;
        uint64_t p0 = QUAD_NO_SA;
        for (uint32_t j = 0; j < QUAD_G; j++) {
            if (gi + j >= a.nq) break;  // group-uniform
            const uint64_t K64 = __shfl((unsigned long long)Kmine, lane0 + (int)j, 64);
            const uint32_t K16 = (uint32_t)(K64 >> 32);
            uint32_t dl, dn;
            const uint32_t k = quad_descend_split(a, s_nodes, K16, sub, &dl, &dn);
            const uint4 e = quad_leaf_load(a, a.quad_leaves + 4 * (uint64_t)k + sub);
            const uint64_t key = (uint64_t)e.x | ((uint64_t)e.y << 32);
            const uint32_t cc = quad_sum((uint32_t)(e.y < K16) | ((uint32_t)(key < K64) << 8) |
                                         ((uint32_t)(key <= K64) << 16));
            const uint32_t c16 = cc & 0xFFu, c64 = (cc >> 8) & 0xFFu, le64 = cc >> 16;
            // this entry's lcp with q: min(first differing char of the 32-char keys, length)
            uint32_t d = key == K64 ? 32u : (uint32_t)__clzll(key ^ K64) >> 1;
            if (4 * (uint64_t)k + sub < a.sa_n) {
                const uint64_t len = a.n - ((uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32));
                if ((uint64_t)d > len) d = (uint32_t)len;
            }
            const uint32_t lamj = quad_sum(d << (8 * sub));  // disjoint bytes: the sum is the OR
            const uint32_t eq0 = (uint32_t)__shfl((int)(e.x == (uint32_t)K64 && e.y == K16), lane0 + (int)(c64 & 3), 64);
            const uint32_t z0 = (uint32_t)__shfl((int)e.z, lane0 + (int)(c64 & 3), 64);
            const uint32_t w0 = (uint32_t)__shfl((int)e.w, lane0 + (int)(c64 & 3), 64);
            if (sub == j) {
                kq = k;
                lam = lamj;
                dnode = dn;
                st = c16 | (c64 << 3) | (dl << 24);
                if (c64 < 4) {
                    st |= QL_KNOWN | QL_X32 | (eq0 ? QL_EQ0 : 0u);
                    p0 = (uint64_t)z0 | ((uint64_t)(w0 & 0xFFu) << 32);
                }
                if (le64 < 4) {  // leaf k holds the first key > K64
                    st |= QL_UK | (le64 << 6);
                } else if (K16 == 0xFFFFFFFFu) {  // q's 16-char run reaches the end
                    st = (st & ~QL_X32) | QL_UK | QL_END;
                }
            }
        }
        uint64_t pos = 0;
        bool done = !mine;
        uint32_t lcp0 = 0;
        if (mine && m <= 32) {
            // the 32-char key decides every entry: k_sa_quad4x's finish
            pos = quad_short_finish(a, Kmine, m, 4 * (uint64_t)kq + QL_C64(st), (st & QL_KNOWN) != 0,
                                    (st & QL_EQ0) != 0, p0, &probes);
            done = true;
        } else if (mine && 4 * (uint64_t)kq + QL_C64(st) >= a.sa_n) {
            pos = a.next_pos;
            done = true;
        } else if (mine) {
            if (!(st & QL_KNOWN) && (SAS_QLLCP_NEXT == 1 || (SAS_QLLCP_NEXT == 2 && QL_C16(st) == 3))) {
                // leaf k's keys are all below q's: the next entry, as k_sa_quad4x reads it (a
                // key still below q's leaves L0 inexact at 32 chars, the walk's kappa 16)
                const uint4 e = a.quad_leaves[4 * (uint64_t)kq + 4];
                const uint64_t key = (uint64_t)e.x | ((uint64_t)e.y << 32);
                probes++;
                if (key >= Kmine) {
                    st |= QL_KNOWN | ((st & QL_END) ? 0u : QL_X32) | (key == Kmine ? QL_EQ0 : 0u);
                    p0 = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
                }
            }
            if (st & QL_KNOWN) {
                // the first suffix not below q's 32-char key: > it, or one compare from char 32
                // (k_sa_quad4x's common case); below q, it is the walk's exact left bound
                if (!(st & QL_EQ0) || (probes++, !suffix_less_from<QW>(a.tw, a.n, p0, q, 32, &lcp0))) {
                    pos = p0;
                    done = true;
                } else {
                    st |= QL_LAM0;
                }
            }
        }
        uint32_t kU = kq;
        // U for the queries whose 32-char run leaves leaf k: the leaf of K16 + 1, from where its
        // path parts from q's (near the leaves: one or two requests)
        const bool needU = !done && !(st & QL_UK);
        const uint32_t nu = quad_mask(needU);  // group-uniform
        for (uint32_t j = 0; nu && j < QUAD_G; j++) {
            if (!(nu & (1u << j))) continue;
            const uint64_t K64 = __shfl((unsigned long long)Kmine, lane0 + (int)j, 64);
            const uint32_t K16 = (uint32_t)(K64 >> 32);
            const uint32_t dl = (uint32_t)__shfl((int)st, lane0 + (int)j, 64) >> 24;
            uint32_t ku = (uint32_t)__shfl((int)kq, lane0 + (int)j, 64);
            if (dl != QLLCP_NONE) {
                ku = quad_descend_from(a, s_nodes, dl + 1, (uint32_t)__shfl((int)dnode, lane0 + (int)j, 64), K16, sub);
                if (sub == j) probes += a.quad_inner_layers - dl;
            }
            const uint4 eU = quad_leaf_load(a, a.quad_leaves + 4 * (uint64_t)ku + sub);
            const uint64_t keyU = (uint64_t)eU.x | ((uint64_t)eU.y << 32);
            const uint32_t cu = quad_sum((uint32_t)(keyU <= K64) | ((uint32_t)(eU.y <= K16) << 8));
            const uint32_t le64U = cu & 0xFFu, le16U = cu >> 8;
            // a key <= K64 in the leaf: everything before it is too, and the next one is the
            // first key > K64; none: the 16-char run's end, exact at 16 chars
            const uint32_t f = le64U ? le64U : le16U;
            if (sub == j) {
                kU = ku;
                st = (st & ~(7u << 6)) | (f << 6) | QL_UK;
                if (!le64U) st &= ~QL_X32;
            }
        }
        if (!mine) continue;
        if (!done) {
            using rk_t = typename std::conditional<R32, uint32_t, uint64_t>::type;
            const rk_t sa_n = (rk_t)a.sa_n;
            const rk_t kb = 4 * (rk_t)kq;
            const rk_t s0 = kb + QL_C16(st);
            const rk_t L0 = kb + QL_C64(st) + ((st & QL_LAM0) ? 1 : 0);
            rk_t U = (st & QL_END) ? sa_n : 4 * (rk_t)kU + QL_FU(st);
            if (U >= sa_n) U = sa_n;
            const uint32_t kappa = (st & QL_X32) ? 32u : 16u;
            rk_t l = 0, r = sa_n;
            uint64_t pr = QUAD_NO_SA;
            uint32_t llcp = 0, rlcp = 0;
            for (;;) {
                rk_t mid = 0;
                while (l < r) {  // ALU only, as stree_tail
                    mid = (l + r) >> 1;
                    if (mid < L0) l = mid + 1;
                    else if (mid >= U) r = mid;
                    else break;
                }
                if (!(l < r)) break;
                const uint4 e = a.llcp[mid];
                const uint32_t x = (e.y >> 8) & SAS_LLCP_CAP, y = e.y >> 20;
                if (l <= s0) llcp = x;  // SA[l - 1] before q's 16-char run (or l = 0)
                else if (l <= L0)       // in leaf k, below q: exact
                    llcp = ((st & QL_LAM0) && l == L0) ? lcp0 : (lam >> (8 * (uint32_t)(l - 1 - kb))) & 0xFFu;
                if (r >= U) rlcp = y;   // SA[r] past q's run (or r = sa_n)
                probes++;
                bool lt;
                uint32_t lcp, hh = 0, inl = 0;
                bool decided = true;
                if (llcp >= rlcp) {
                    if (x > llcp) { lt = true; lcp = llcp; }
                    else if (x < llcp && x < SAS_LLCP_CAP) { lt = false; lcp = x; }
                    else { decided = false; hh = x; inl = e.z; }
                } else {
                    if (y > rlcp) { lt = false; lcp = rlcp; }
                    else if (y < rlcp && y < SAS_LLCP_CAP) { lt = true; lcp = y; }
                    else { decided = false; hh = y; inl = e.w; }
                }
                const uint64_t p = (uint64_t)e.x | ((uint64_t)(e.y & 0xFFu) << 32);
                if (!decided) lt = qllcp_tie_less<QW, QR>(a, p, q, hh, inl, kappa, &lcp);
                if (lt) {
                    l = mid + 1;
                    llcp = lcp;
                } else {
                    r = mid;
                    rlcp = lcp;
                    pr = p;
                }
            }
            if (r >= sa_n) pos = a.next_pos;
            else if (pr != QUAD_NO_SA) pos = pr;
            else {
                const uint4 eu = a.llcp[r];
                pos = (uint64_t)eu.x | ((uint64_t)(eu.y & 0xFFu) << 32);
                probes++;
            }
        }
        a.out_pos[i] = pos;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// Occurrence ranges on the quad tree: global ranks [lo, hi) of the suffixes
// that start with q (out_pos = lo, out_hi = hi), as k_sa_sector_range.
template <int QW, bool KO, int W>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_quad_range(SearchArgs a, uint64_t* out_hi) {
    __shared__ uint4 s_nodes[SAS_QUAD_LDS_NODES * 4];
    stage_quad_top(a, s_nodes);
    const uint32_t sub = threadIdx.x & (QUAD_G - 1);
    uint32_t bad = 0;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / QUAD_G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / QUAD_G; i < a.nq; i += stride) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        uint32_t probes = 0;
        uint64_t px = 0;
        const uint64_t lo = quad_bound<QW, false, KO, W>(a, s_nodes, q, K64, Q3, sub, &probes, &px);
        uint64_t hi = quad_bound<QW, true, KO, W>(a, s_nodes, q, K64, Q3, sub, &probes, &px);
        if (hi < lo) hi = lo;
        if (sub == 0) {
            a.out_pos[i] = a.rank_lo + lo;
            out_hi[i] = a.rank_lo + hi;
            if (a.out_probes) a.out_probes[i] = probes;
        }
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ INLINE
// binary_search_batch<64>'s probes (sas/sa_search.rs:157-196: same mids, same
// ilog2(n)+1 lockstep iterations, same LDS top as PLAIN) but each probe reads the
// quad leaves' entry: the 32-char key decides unless it equals the query's (then
// the SA value -- in the fused entry, or from the SA array for KO leaves -- and the
// text from char 32), so a len-32 probe is one memory request instead of an SA
// word + two text words.
template <int QW, bool TOP, bool KO, int W>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_inline(SearchArgs a) {
    __shared__ uint4 s_rel[TOP ? SAS_REL_LDS_BYTES / 16 : 1];  // the rel blocks' LDS groups
    if (TOP) {
        stage_rel(s_rel, a.rel, a.rel_lay.lds_bytes);
        __syncthreads();
    }
    uint32_t bad = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        uint64_t l = 0, r = a.sa_n, pr = QUAD_NO_SA;
        uint32_t k = 1, probes = 0;
        // selects, not a branch on ge: the branch form made the compiler store l or pr through a
        // selected pointer into scratch (24 B a lane, round 5's make resource)
        auto take = [&](uint64_t mid, bool ge, uint64_t p) {
            probes++;
            r = ge ? mid : r;
            pr = ge ? p : pr;
            l = ge ? l : mid + 1;
        };
        uint32_t it = 0;
        if (TOP) {
            // the prefix-relative blocks, as PLAIN reads them; an 8-char tie reads the probe's
            // own entry (key != K64 decides key > K64, the sector predicate)
            for (uint32_t g = 0; g < a.rel_lay.groups; ++g) {
                const uint32_t hh = a.rel_lay.h[g];
                uint4 b0 = make_uint4(0, 0, 0, 0), b1 = b0;
                if (l < r) rel_block(a, s_rel, g, it, (uint32_t)k, hh, b0, b1);
                const uint32_t P = b0.x & 0x7FFFu;
                const uint32_t c0 = q.m > P ? q.m - P : 0u;
                const uint32_t c = c0 < 8 ? c0 : 8u;
                const uint32_t mk = c ? (0xFFFFu << (16 - 2 * c)) & 0xFFFFu : 0u;
                const uint32_t qk = (uint32_t)((K64 << (2 * P)) >> 48) & mk;
                for (uint32_t t = 0; t < hh; ++t, ++it) {
                    if (!(l < r)) continue;
                    const uint64_t mid = (l + r) >> 1;
                    const uint32_t key = rel_slot(b0, b1, (1u << t) | (k & ((1u << t) - 1u))) & mk;
                    bool ge;
                    uint64_t p = QUAD_NO_SA;
                    if (key != qk) {
                        ge = key > qk;
                    } else {
                        uint64_t ek;
                        if (KO) {
                            ek = quad_entry_key<true>(a, mid);
                            p = ek == K64 ? quad_entry_sa<true, W>(a, mid) : QUAD_NO_SA;
                        } else {
                            const uint4 e = a.quad_leaves[mid];
                            ek = (uint64_t)e.x | ((uint64_t)e.y << 32);
                            p = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
                        }
                        ge = sector_ge<QW>(ek, p, K64, a, q);
                    }
                    k = 2 * k + (ge ? 0u : 1u);
                    take(mid, ge, p);
                }
            }
        }
        for (; it < a.iters; ++it) {
            if (l < r) {
                const uint64_t mid = (l + r) >> 1;
                uint64_t key, p;
                if (KO) {
                    key = quad_entry_key<true>(a, mid);
                    p = key == K64 ? quad_entry_sa<true, W>(a, mid) : QUAD_NO_SA;
                } else {
                    const uint4 e = a.quad_leaves[mid];
                    key = (uint64_t)e.x | ((uint64_t)e.y << 32);
                    p = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
                }
                take(mid, sector_ge<QW>(key, p, K64, a, q), p);
            }
        }
        // SA[r] not seen yet (a compact leaf's key, or a pivot decided by its first 16 chars)
        if (r >= a.sa_n) pr = a.next_pos;
        else if (pr == QUAD_NO_SA) pr = KO ? quad_entry_sa<true, W>(a, r) : quad_entry_sa<false, W>(a, r);
        a.out_pos[i] = pr;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ PREFIX
// The reference's prefix table, live (fill_prefix_table / prefix_range,
// sas/sa_search.rs:59-95; p = 0 there, :31).  One lane per query: K = q's first p
// chars zero padded; every suffix whose p-char key is < K is < q and every one whose
// key is > K is > q (zero padding keeps key order = slice order), so
// the lower bound lies in [table[K], table[K+1]], found by a binary search over the
// quad leaf entries of that range with the sector predicate.  At p = ceil(log4 n) + 1
// a random lookup is two memory requests: the table pair, then one leaf entry.
#ifndef SAS_PREFIX_NT
#define SAS_PREFIX_NT 1  // non-temporal table / entry loads (-3%, tools/ab_prefix.py)
#endif
#ifndef SAS_PREFIX_SPLITQ
#define SAS_PREFIX_SPLITQ 1  // lane pairs split a 32-B query load (k_sa_prefix2; -4%)
#endif
#ifndef SAS_PREFIX_QPREFETCH
#define SAS_PREFIX_QPREFETCH 1  // load the next query while this one's entry is in flight (-1%)
#endif
#ifndef SAS_PREFIX_NT_OUT
#define SAS_PREFIX_NT_OUT 0  // non-temporal position stores (k_sa_prefix2)
#endif
#ifndef SAS_PREFIX_QWMAX
#define SAS_PREFIX_QWMAX 8  // register-resident query words (later ones repacked from the bytes)
#endif
// k_sa_prefix2 on the headline shape (fixed 32-char queries, lane pairs): queries in flight
// per lane pair (round 6 A/B hook; 1 = one lookup at a time)
#ifndef SAS_PREFIX_ILP
#define SAS_PREFIX_ILP 1
#endif
#ifndef SAS_PREFIX_PAIR
#define SAS_PREFIX_PAIR 0  // table[K], table[K+1] as one dword-aligned 8-B load
#endif
template <int QW, bool KO, int W, int TW>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_prefix(SearchArgs a) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.prefix_chars;
    const uint64_t sa_n = a.sa_n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (!slot_live(a, i)) continue;
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        if (a.qwords) {  // packed fixed-length query: the key word itself
            q.bytes = nullptr;
            q.m = m;
            q.w[0] = a.qwords[i] & chars_mask(m);
        } else {
            q.load(qb, m, &bad);
        }
        const uint64_t K64 = q.w[0];
        const uint64_t K = pt_slot(a, K64 >> sh);
        uint64_t lo, hi = 0, pos = QUAD_NO_SA;
        const uint32_t* pt = reinterpret_cast<const uint32_t*>(a.prefix);
        const uint4* pt16 = reinterpret_cast<const uint4*>(a.prefix);
        bool have_hi = true;
        if (TW == 16) {
            // inline entry: the range's first suffix {key, rank, SA}; if it is >= q it is
            // the answer, and this was the only read
            const uint4 e0 = SAS_PREFIX_NT ? nt_load4(pt16 + K) : pt16[K];
            lo = e0.z;
            have_hi = false;
            if (lo >= sa_n) {
                pos = a.next_pos;
            } else if (sector_ge<QW>((uint64_t)e0.x | ((uint64_t)e0.y << 32), e0.w, K64, a, q)) {
                pos = e0.w;
            } else {
                hi = pt16[K + 1].z;
                have_hi = true;
            }
        } else if (TW == 5) {
            const SaView<5> v{a.prefix};
            lo = v[K];
            hi = v[K + 1];
        } else if (SAS_PREFIX_PAIR) {
            typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
            const u32x2_a4* pp2 = reinterpret_cast<const u32x2_a4*>(pt + K);
            const u32x2_a4 v = SAS_PREFIX_NT ? __builtin_nontemporal_load(pp2) : *pp2;
            lo = v.x;
            hi = v.y;
        } else if (SAS_PREFIX_NT) {
            lo = __builtin_nontemporal_load(pt + K);
            hi = __builtin_nontemporal_load(pt + K + 1);
        } else {
            lo = pt[K];
            hi = pt[K + 1];
        }
        const uint64_t lo0 = lo;
        uint64_t hi0 = hi;
        // binary_search over [table[K], table[K+1]) (sas/sa_search.rs:98-112); with inline
        // entries rank lo is already known to be < q.  A scan of short ranges with
        // independent loads measured slower (0.53 -> 0.60 ms at c1, 26.6 -> 39.4 ms at c3):
        // its key re-reads lengthen the dependent chain.
        if (pos == QUAD_NO_SA) {
            uint64_t pr = QUAD_NO_SA;
            if (TW == 16) lo++;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                uint64_t key, pp;
                if (KO) {
                    key = quad_entry_key<true>(a, mid);
                    pp = key == K64 ? quad_entry_sa<true, W>(a, mid) : QUAD_NO_SA;
                } else {
                    const uint4 e = SAS_PREFIX_NT ? nt_load4(a.quad_leaves + mid) : a.quad_leaves[mid];
                    key = (uint64_t)e.x | ((uint64_t)e.y << 32);
                    pp = (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
                }
                if (sector_ge<QW>(key, pp, K64, a, q)) {
                    hi = mid;
                    pr = pp;  // SA at rank hi (QUAD_NO_SA: not read); lo ends at hi
                } else {
                    lo = mid + 1;
                }
            }
            if (lo >= sa_n) pos = a.next_pos;
            else if (pr != QUAD_NO_SA) pos = pr;
            else pos = quad_entry_sa<KO, W>(a, lo);
        }
        // out_probes = the reference's cnt (sas/sa_search.rs:86-112): 1 for the table, then
        // binary_search's iterations over [table[K], table[K+1]), which end at rank lo
        uint32_t probes = 1;
        if (a.out_probes) {
            if (!have_hi) hi0 = pt16[K + 1].z;
            for (uint64_t l2 = lo0, h2 = hi0; l2 < h2; probes++) {
                const uint64_t mid = (l2 + h2) >> 1;
                if (mid < lo) l2 = mid + 1;
                else h2 = mid;
            }
        }
        a.out_pos[i] = pos;
        if (a.out_probes) a.out_probes[i] = probes;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// SAS_BUILD_PREFIX_INLINE2 / _INLINE4: 16·G-byte entries, the first G suffixes (ranks
// r .. r + G - 1) of the range of q's p-char key.  A G-lane group reads the entry as one
// request (16 B per lane), each lane tests one suffix, and the group ballot takes the
// first that is >= q; only if all are < q does the search go on in [r + G, table[K+1]).
// HI40 (a part index of a text >= 2^32 chars): slot 1's rank word holds bits 32..39 of
// every slot's SA value, one byte per slot.
// k_sa_prefix2's lookup of query i once its table entry e (entry K) is in: the pair's slots
// tested, the rare bisection past them, the position (and the reference's cnt) stored
template <int QW, int G, bool HI40>
__device__ __forceinline__ void prefix2_finish(const SearchArgs& a, const uint4* pt, uint64_t i, uint64_t K,
                                               const uint4& e, const QueryRegs<QW>& q, uint64_t K64, uint32_t sub,
                                               int lane0) {
    const uint64_t sa_n = a.sa_n;
    const uint32_t hb = HI40 ? (uint32_t)__shfl((int)e.z, lane0 + 1, 64) : 0u;
    // two slots beside a >= 2^32-char text: bits 32..39 of the rank in slot 1's rank word
    const uint64_t r0 = (uint64_t)(uint32_t)__shfl((int)e.z, lane0, 64) |
                        (HI40 && G == 2 ? (uint64_t)((hb >> 16) & 0xFFu) << 32 : 0ull);
    const uint64_t rank = r0 + sub;
    const uint64_t pe = HI40 ? ((uint64_t)e.w | ((uint64_t)((hb >> (8 * sub)) & 0xFFu) << 32)) : (uint64_t)e.w;
    // rank sa_n stands for "past every suffix": it is the answer if reached
    const bool ok = rank >= sa_n || sector_ge<QW>((uint64_t)e.x | ((uint64_t)e.y << 32), pe, K64, a, q);
    const uint32_t grp = (uint32_t)(__ballot(ok) >> lane0) & ((1u << G) - 1u);
    const uint32_t j = grp ? (uint32_t)__builtin_ctz(grp) : 0u;
    const uint32_t pw = (uint32_t)__shfl((int)e.w, lane0 + (int)j, 64);
    uint64_t ans, pos;
    if (grp) {
        ans = r0 + j;
        pos = ans >= sa_n ? a.next_pos : (HI40 ? ((uint64_t)pw | ((uint64_t)((hb >> (8 * j)) & 0xFFu) << 32)) : pw);
    } else {
        uint64_t lo = r0 + G, hi = pt_rank<G, HI40>(pt, K + 1), pr = QUAD_NO_SA;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            const uint4 f = SAS_PREFIX_NT ? nt_load4(a.quad_leaves + mid) : a.quad_leaves[mid];
            const uint64_t pp = (uint64_t)f.z | ((uint64_t)(f.w & 0xFFu) << 32);
            if (sector_ge<QW>((uint64_t)f.x | ((uint64_t)f.y << 32), pp, K64, a, q)) {
                hi = mid;
                pr = pp;
            } else {
                lo = mid + 1;
            }
        }
        ans = lo;
        if (lo >= sa_n) pos = a.next_pos;
        else if (pr != QUAD_NO_SA) pos = pr;
        else pos = quad_entry_sa<false, 4>(a, lo);
    }
    if (sub == 0) {
        if (SAS_PREFIX_NT_OUT) __builtin_nontemporal_store(pos, a.out_pos + i);
        else a.out_pos[i] = pos;
        if (a.out_probes) {  // the reference's cnt over [table[K], table[K+1])
            uint32_t probes = 1;
            for (uint64_t l2 = r0, h2 = pt_rank<G, HI40>(pt, K + 1); l2 < h2; probes++) {
                const uint64_t mid = (l2 + h2) >> 1;
                if (mid < ans) l2 = mid + 1;
                else h2 = mid;
            }
            a.out_probes[i] = probes;
        }
    }
}

template <int QW, int G, bool HI40 = false>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_prefix2(SearchArgs a) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.prefix_chars;
    const uint32_t sub = threadIdx.x & (G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~(uint32_t)(G - 1));
    const uint4* pt = reinterpret_cast<const uint4*>(a.prefix);
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / G;
    // fixed 32-char queries at 16-B aligned addresses: the pair splits each query load
    const bool split = SAS_PREFIX_SPLITQ && G == 2 && QW == 1 && a.qoff == nullptr && a.qwords == nullptr &&
                       a.m_fixed == 32 && a.bcounts == nullptr &&
                       (((uintptr_t)a.qbytes) & 15) == 0;
    auto qload = [&](uint64_t k) -> uint4 {
        const uint4* p = reinterpret_cast<const uint4*>(a.qbytes + k * 32) + sub;
        return SAS_QUAD_NT_IO ? nt_load4(p) : *p;
    };
    const uint64_t i0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G;
    if (SAS_PREFIX_ILP > 1 && split) {
        // two queries per lane pair in flight: i and i + stride, both table entries requested
        // before either is tested (the next two queries' loads overlap the lookups)
        auto pack_q = [&](const uint4& v, uint64_t k, QueryRegs<QW>& q) {
            bad |= (v.x | v.y | v.z | v.w) & 0xFCFCFCFCu;
            const uint32_t part = (pack4(v.x) << 24) | (pack4(v.y) << 16) | (pack4(v.z) << 8) | pack4(v.w);
            const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)part, 0xB1, 0xF, 0xF, false);
            q.bytes = a.qbytes + k * 32;
            q.m = 32;
            q.w[0] = sub ? (((uint64_t)other << 32) | part) : (((uint64_t)part << 32) | other);
        };
        const uint4 z = make_uint4(0, 0, 0, 0);
        uint4 va = i0 < a.nq ? qload(i0) : z, vb = i0 + stride < a.nq ? qload(i0 + stride) : z;
        for (uint64_t i = i0; i < a.nq; i += 2 * stride) {
            const uint64_t i2 = i + stride;
            const bool two = i2 < a.nq;  // group-uniform
            const uint4 ua = va, ub = vb;
            if (i + 2 * stride < a.nq) va = qload(i + 2 * stride);
            if (i2 + 2 * stride < a.nq) vb = qload(i2 + 2 * stride);
            QueryRegs<QW> qa, qb2;
            pack_q(ua, i, qa);
            pack_q(ub, i2, qb2);
            const uint64_t Ka = pt_slot(a, qa.w[0] >> sh), Kb = pt_slot(a, qb2.w[0] >> sh);
            const uint4 ea = SAS_PREFIX_NT ? nt_load4(pt + G * Ka + sub) : pt[G * Ka + sub];
            uint4 eb = z;
            if (two) eb = SAS_PREFIX_NT ? nt_load4(pt + G * Kb + sub) : pt[G * Kb + sub];
            prefix2_finish<QW, G, HI40>(a, pt, i, Ka, ea, qa, qa.w[0], sub, lane0);
            if (two) prefix2_finish<QW, G, HI40>(a, pt, i2, Kb, eb, qb2, qb2.w[0], sub, lane0);
        }
        if (bad) atomicOr(a.bad, 1u);
        return;
    }
    uint4 vnext = make_uint4(0, 0, 0, 0);
    if (SAS_PREFIX_QPREFETCH && split && i0 < a.nq) vnext = qload(i0);
    for (uint64_t i = i0; i < a.nq; i += stride) {
        if (!slot_live(a, i)) continue;  // group-uniform: the G lanes share i
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        if (a.qwords) {  // packed: the key word itself (both lanes, one 8-B request)
            q.bytes = nullptr;
            q.m = m;
            q.w[0] = a.qwords[i] & chars_mask(m);
        } else if (split) {
            // the pair splits the 32-B query: lane j packs bytes 16j..16j+15 to 32 bits,
            // then the halves are swapped within the pair (DPP quad_perm [1,0,3,2])
            uint4 v;
            if (SAS_PREFIX_QPREFETCH) {  // the next query's load overlaps this lookup
                v = vnext;
                if (i + stride < a.nq) vnext = qload(i + stride);
            } else {
                v = qload(i);
            }
            bad |= (v.x | v.y | v.z | v.w) & 0xFCFCFCFCu;
            const uint32_t part = (pack4(v.x) << 24) | (pack4(v.y) << 16) | (pack4(v.z) << 8) | pack4(v.w);
            const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)part, 0xB1, 0xF, 0xF, false);
            q.bytes = qb;
            q.m = m;
            q.w[0] = sub ? (((uint64_t)other << 32) | part) : (((uint64_t)part << 32) | other);
        } else {
            q.load(qb, m, &bad);  // every lane of the group: the same addresses, one request
        }
        const uint64_t K64 = q.w[0];
        const uint64_t K = pt_slot(a, K64 >> sh);
        const uint4 e = SAS_PREFIX_NT ? nt_load4(pt + G * K + sub) : pt[G * K + sub];
        prefix2_finish<QW, G, HI40>(a, pt, i, K, e, q, K64, sub, lane0);
    }
    if (bad) atomicOr(a.bad, 1u);
}

// Occurrence ranges from the prefix table (any entry format; Search::search_prefix,
// sas/util.rs:36-46): lo = the lower bound, bisected in [table[K], table[K+1]]; hi = the
// first suffix whose first min(m, len) chars are > q, bisected in the range of the
// routing key (q padded with 3s for m <= 32, its own key above), with the predicates of
// k_sa_quad_range over the quad leaves' entries.
template <int QW, bool KO, int W>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_prefix_range(SearchArgs a, uint64_t* out_hi) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.prefix_chars;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        // both bisections advance in lock step: two independent entry reads in flight per lane
        uint64_t lo, l1, hi, h1;
        prefix_range(a, K64 >> sh, &lo, &l1);
        prefix_range(a, (q.m <= 32 ? Q3 : K64) >> sh, &hi, &h1);
        while (lo < l1 || hi < h1) {
            const bool g0 = lo < l1, g1 = hi < h1;
            const uint64_t m0 = (lo + l1) >> 1, m1 = (hi + h1) >> 1;
            const uint64_t k0 = g0 ? quad_entry_key<KO>(a, m0) : 0;
            const uint64_t k1 = g1 ? quad_entry_key<KO>(a, m1) : 0;
            const uint64_t p0 = (g0 && k0 == K64) ? quad_entry_sa<KO, W>(a, m0) : QUAD_NO_SA;
            const uint64_t p1 = (g1 && q.m > 32 && k1 == K64) ? quad_entry_sa<KO, W>(a, m1) : QUAD_NO_SA;
            if (g0) {
                if (sector_ge<QW>(k0, p0, K64, a, q)) l1 = m0;
                else lo = m0 + 1;
            }
            if (g1) {
                if (sector_gt_prefix<QW>(k1, p1, K64, Q3, a, q)) h1 = m1;
                else hi = m1 + 1;
            }
        }
        if (hi < lo) hi = lo;
        a.out_pos[i] = a.rank_lo + lo;
        out_hi[i] = a.rank_lo + hi;
    }
    if (bad) atomicOr(a.bad, 1u);
}

template <bool KO, int W>
static void launch_prefix_range(int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a, uint64_t* dhi) {
    switch (qw) {
        case 1: hipLaunchKernelGGL((k_sa_prefix_range<1, KO, W>), grid, block, 0, st, a, dhi); break;
        case 2: hipLaunchKernelGGL((k_sa_prefix_range<2, KO, W>), grid, block, 0, st, a, dhi); break;
        case 4: hipLaunchKernelGGL((k_sa_prefix_range<4, KO, W>), grid, block, 0, st, a, dhi); break;
        default: hipLaunchKernelGGL((k_sa_prefix_range<8, KO, W>), grid, block, 0, st, a, dhi); break;
    }
}

// Occurrence ranges on a G-slot inline prefix table (SAS_BUILD_PREFIX_INLINE2 / _INLINE4):
// the G lanes of a query read its entry (the first G suffixes of the range of its p-char
// key) as one request and test both bounds' predicates on every slot: lo = the first slot
// >= q, hi = the first slot whose first min(m, len) chars are > q (m >= p: the suffixes
// starting with q all lie in the key's range).  A bound not inside the entry is bisected
// in [r + G, table[K + 1]) (hi, for m < p: in the range of the 3-padded key), both in
// lock step as k_sa_prefix_range does; every lane of the group runs the same loop (same
// addresses: one request per probe).
template <int QW, int G, bool HI40 = false>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_prefix2_range(SearchArgs a, uint64_t* out_hi) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.prefix_chars;
    const uint64_t sa_n = a.sa_n;
    const uint32_t sub = threadIdx.x & (G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~(uint32_t)(G - 1));
    const uint4* pt = reinterpret_cast<const uint4*>(a.prefix);
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; i < a.nq; i += stride) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);  // every lane of the group: the same addresses, one request
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        const uint64_t K = pt_slot(a, K64 >> sh);
        const uint4 e = pt[G * K + sub];
        const uint32_t hb = HI40 ? (uint32_t)__shfl((int)e.z, lane0 + 1, 64) : 0u;
        const uint64_t r0 = (uint64_t)(uint32_t)__shfl((int)e.z, lane0, 64) |
                            (HI40 && G == 2 ? (uint64_t)((hb >> 16) & 0xFFu) << 32 : 0ull);
        const uint64_t rank = r0 + sub;
        const uint64_t key = (uint64_t)e.x | ((uint64_t)e.y << 32);
        const uint64_t pe = HI40 ? ((uint64_t)e.w | ((uint64_t)((hb >> (8 * sub)) & 0xFFu) << 32)) : (uint64_t)e.w;
        // rank sa_n stands for "past every suffix": both bounds are reached there
        const bool past = rank >= sa_n;
        const bool ge = past || sector_ge<QW>(key, pe, K64, a, q);
        const bool whole = m >= a.prefix_chars;  // hi inside the key's range too
        const bool gt = past || (whole && sector_gt_prefix<QW>(key, pe, K64, Q3, a, q));
        const uint32_t mask = (1u << G) - 1u;
        const uint32_t gge = (uint32_t)(__ballot(ge) >> lane0) & mask;
        const uint32_t ggt = (uint32_t)(__ballot(gt) >> lane0) & mask;
        uint64_t lo, l1, hi, h1;
        if (gge) {
            lo = l1 = r0 + (uint32_t)__builtin_ctz(gge);
        } else {
            lo = r0 + G;
            l1 = pt_rank<G, HI40>(pt, K + 1);
        }
        if (whole) {
            if (ggt) {
                hi = h1 = r0 + (uint32_t)__builtin_ctz(ggt);
            } else {
                hi = r0 + G;
                h1 = gge ? pt_rank<G, HI40>(pt, K + 1) : l1;
            }
        } else {
            prefix_range(a, Q3 >> sh, &hi, &h1);
        }
        while (lo < l1 || hi < h1) {
            const bool g0 = lo < l1, g1 = hi < h1;
            const uint64_t m0 = (lo + l1) >> 1, m1 = (hi + h1) >> 1;
            const uint64_t k0 = g0 ? quad_entry_key<false>(a, m0) : 0;
            const uint64_t k1 = g1 ? quad_entry_key<false>(a, m1) : 0;
            const uint64_t p0 = (g0 && k0 == K64) ? quad_entry_sa<false, 4>(a, m0) : QUAD_NO_SA;
            const uint64_t p1 = (g1 && q.m > 32 && k1 == K64) ? quad_entry_sa<false, 4>(a, m1) : QUAD_NO_SA;
            if (g0) {
                if (sector_ge<QW>(k0, p0, K64, a, q)) l1 = m0;
                else lo = m0 + 1;
            }
            if (g1) {
                if (sector_gt_prefix<QW>(k1, p1, K64, Q3, a, q)) h1 = m1;
                else hi = m1 + 1;
            }
        }
        if (hi < lo) hi = lo;
        if (sub == 0) {
            a.out_pos[i] = a.rank_lo + lo;
            out_hi[i] = a.rank_lo + hi;
        }
    }
    if (bad) atomicOr(a.bad, 1u);
}

template <int G, bool HI40>
static void launch_prefix2_range_h(int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a,
                                   uint64_t* dhi) {
    switch (qw) {
        case 1: hipLaunchKernelGGL((k_sa_prefix2_range<1, G, HI40>), grid, block, 0, st, a, dhi); break;
        case 2: hipLaunchKernelGGL((k_sa_prefix2_range<2, G, HI40>), grid, block, 0, st, a, dhi); break;
        case 4: hipLaunchKernelGGL((k_sa_prefix2_range<4, G, HI40>), grid, block, 0, st, a, dhi); break;
        default: hipLaunchKernelGGL((k_sa_prefix2_range<8, G, HI40>), grid, block, 0, st, a, dhi); break;
    }
}

template <int G>
static void launch_prefix2_range(int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a, uint64_t* dhi) {
    if (a.prefix_hi40) launch_prefix2_range_h<G, true>(qw, grid, block, st, a, dhi);
    else launch_prefix2_range_h<G, false>(qw, grid, block, st, a, dhi);
}

// ------------------------------------------------------------------ INTERP
// interpolation_search<16> (sas/sa_search.rs:376-421), one lane per query.  string_value<16>
// (sas/util.rs:76-117) of a suffix is the high half of its 32-char packed key; of the query,
// the high half of its first packed word (zero padded past m).  The mid is the
// reference's l + (r-l)(q_val - l_val + 1) / (r_val - l_val + 2) in wrapping u64 arithmetic
// (its release build), clamped to [l + (r-l)/16, l + 15(r-l)/16] (:406-409), so l <= mid < r
// and every probe is an exact compare: the result is binary_search's, the probe count the
// reference's cnt.  FUSED: a probe reads the fused quad leaf entry {key64, SA} (one 16-B
// request); otherwise SA[mid], then the text window (two dependent requests), as the
// reference does.  range: start from the prefix table's range of q's first p chars (cnt + 1,
// sas/sa_search.rs:86-89).
template <int QW, int W, bool FUSED>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_interp(SearchArgs a, uint32_t range) {
    uint32_t bad = 0;
    const SaView<W> sa{a.sa};
    const uint64_t sa_n = a.sa_n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        uint64_t l = 0, r = sa_n;
        uint32_t cnt = 0;
        if (range) {
            prefix_range(a, K64 >> (64 - 2 * a.prefix_chars), &l, &r);
            cnt = 1;
        }
        auto probe = [&](uint64_t x, uint64_t* key) -> uint64_t {
            if (FUSED) {
                const uint4 e = nt_load4(a.quad_leaves + x);
                *key = (uint64_t)e.x | ((uint64_t)e.y << 32);
                return (uint64_t)e.z | ((uint64_t)(e.w & 0xFFu) << 32);
            }
            const uint64_t p = sa[x];
            *key = text_chars32(a.tw, p);
            return p;
        };
        uint64_t key = 0, l_val = 0, r_val = 1ull << 32, pr = QUAD_NO_SA;
        if (l < sa_n) {  // sa.suffix(l) (:378)
            (void)probe(l, &key);
            l_val = key >> 32;
        }
        if (r < sa_n) {  // sa.suffix(r) when r < len, else 4^K (:379-383)
            pr = probe(r, &key);
            r_val = key >> 32;
        }
        const uint64_t q_val = K64 >> 32;
        while (l < r) {
            cnt++;
            uint64_t mid = l + ((r - l) * (q_val - l_val + 1)) / (r_val - l_val + 2);
            const uint64_t low = l + (r - l) / 16, high = l + 15 * (r - l) / 16;
            mid = mid < low ? low : (mid > high ? high : mid);
            const uint64_t p = probe(mid, &key);
            if (sector_ge<QW>(key, p, K64, a, q)) {  // !(t < q)
                r = mid;
                r_val = key >> 32;
                pr = p;
            } else {
                l = mid + 1;
                l_val = key >> 32;
            }
        }
        a.out_pos[i] = l >= sa_n ? a.next_pos : pr;  // pr = SA[r] (read or moved), l == r
        if (a.out_probes) a.out_probes[i] = cnt;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ TAGGED
// SAS_BUILD_TAGGED (the configs[3] path): entries e[r] = {SA[r] 40 bits |
// chars [p, p+12) of that suffix << 40} in rank order, and the bucket table of the
// reference's prefix_range (sas/sa_search.rs:86-95) with p live: {first rank 40 bits |
// count 24 bits} per p-char key.  Every entry of q's bucket shares q's (zero-padded) first p
// chars, so the entry's tag extends that to a (p+12)-char key: "tag < q's tag" proves
// suffix < q, "tag > q's tag" proves suffix > q, and only a tie needs the length (m <= p+12)
// or an exact compare from char p+12 (the sector predicate with L = p + 12).  A lookup is:
// the bucket word (one aligned 8-B read), the first SAS_TAG_WIN entries of the bucket as
// 16-B entry pairs (a bucket holds ~4 suffixes at n = 4^p), the text past char p+12 of the
// single candidate whose tag ties q's (a positive query's own suffix; read as 16-B word
// pairs, suffix_less_from_x2), and its position straight from the entry.  Larger buckets
// continue with a binary search over the rest.
#ifndef SAS_TAG_WIN
#define SAS_TAG_WIN 8
#endif
#ifndef SAS_TAG_WINS
#define SAS_TAG_WINS 1
#endif
#define TAG_M40 (SAS_SA40_MAX - 1)
// text word pairs the tie compare loads together before its first compare (0: one pair at a
// time, suffix_less_from_x2)
#ifndef SAS_TAG_PRE
#define SAS_TAG_PRE 0
#endif
// waves per SIMD the long-query (QW >= SAS_TAG_LB_QW) instances are built for
#ifndef SAS_TAG_LB
#define SAS_TAG_LB 5
#endif
#ifndef SAS_TAG_LB_QW
#define SAS_TAG_LB_QW 1
#endif
// threads per block of k_sa_tagged (one wave per SIMD per block: the grid is num_cus x
// SAS_TAG_LB blocks)
#ifndef SAS_TAG_BLOCK
#define SAS_TAG_BLOCK 256
#endif

// chars [p, p+12) of a packed 32-char key (p + 12 <= 32)
__device__ __forceinline__ uint32_t tag_of_key(uint64_t k64, uint32_t p) { return (uint32_t)((k64 << (2 * p)) >> 40); }

// suffix(e) >= q, for an entry of q's bucket
template <int QW, class Q>
__device__ __forceinline__ bool tag_ge(uint64_t e, uint32_t Q12, const SearchArgs& a, const Q& q) {
    const uint32_t T = (uint32_t)(e >> 40);
    if (T != Q12) return T > Q12;
    const uint64_t p = e & TAG_M40;
    const uint32_t L = a.tag_p + SAS_TAG_CHARS;
    if (q.m <= L) return (a.n - p) >= (uint64_t)q.m;  // equal padded keys: a shorter suffix is a prefix of q
    uint32_t lcp;
#if SAS_TAG_PRE
    return !suffix_less_from_pre<SAS_TAG_PRE>(a.tw, a.tw, a.n, p, q, L, &lcp);
#else
    return !suffix_less_from_x2<QW>(a.tw, a.n, p, q, L, &lcp);
#endif
}

// the first min(m, len) chars of suffix(e) are > q, for an entry of the bucket of q's routing
// key (Q3 = q padded with 3s when m <= p + 12, else q's own; as sector_gt_prefix)
template <int QW, class Q>
__device__ __forceinline__ bool tag_gt_prefix(uint64_t e, uint32_t Q12, uint32_t Q3t, const SearchArgs& a,
                                              const Q& q) {
    const uint32_t T = (uint32_t)(e >> 40);
    const uint32_t L = a.tag_p + SAS_TAG_CHARS;
    if (q.m <= L) return T > Q3t;
    if (T != Q12) return T > Q12;
    uint32_t lcp;
    const bool lt = suffix_less_from_x2<QW>(a.tw, a.n, e & TAG_M40, q, L, &lcp);
    return !lt && lcp < q.m;
}

// ranks [lo, hi) of p-char key x (a saturated count reads the next bucket word)
__device__ __forceinline__ void tag_bucket(const SearchArgs& a, uint64_t x, uint64_t* lo, uint64_t* hi) {
    const uint64_t t = __builtin_nontemporal_load(a.tag_table + x);
    *lo = t & TAG_M40;
    const uint64_t c = t >> 40;
    *hi = c == 0xFFFFFFull ? (a.tag_table[x + 1] & TAG_M40) : *lo + c;
}

// One lookup on the tagged index (q: QueryRegs or WaveQuery).
template <int QW, class Q>
__device__ __forceinline__ void tagged_lookup(const SearchArgs& a, const Q& q, uint64_t i) {
    const uint64_t* ent = reinterpret_cast<const uint64_t*>(a.sa);
    const uint64_t sa_n = a.sa_n;
    const uint32_t sh = 64 - 2 * a.tag_p;
    const uint64_t K64 = q.w[0];
    const uint32_t Q12 = tag_of_key(K64, a.tag_p);
    uint64_t lo, hi;
    tag_bucket(a, K64 >> sh, &lo, &hi);
    // the bucket's suffixes are ranks [lo, hi); rank hi (the next bucket's first suffix, > q)
    // is the answer when all of them are < q, and is read only then (by the bisection
    // below, which ends at hi).  The window holds the first nw entries, loaded as 16-B
    // aligned entry pairs: half the load instructions of 8-B loads, and fewer L1->L2
    // requests and TLB lookups, which bound this kernel (the entries carry 16 bytes of
    // padding, so the pair holding rank sa_n - 1 is readable)
    // SAS_TAG_WINS windows of SAS_TAG_WIN entries are scanned before the bisection: a wave
    // waits for its slowest lane, and a bucket past one window (~2% of lanes at 4 suffixes
    // per bucket, so most waves hold one) costs one more dependent read instead of
    // log2(count - SAS_TAG_WIN) of them
    uint64_t ans = 0, pos = 0, start = lo;
    bool done = false;
#pragma unroll 1
    for (int w = 0; w < SAS_TAG_WINS; w++) {
        const uint64_t wb = lo + (uint64_t)w * SAS_TAG_WIN;
        const uint64_t rest = hi - wb;
        const uint32_t nw = rest < SAS_TAG_WIN ? (uint32_t)rest : (uint32_t)SAS_TAG_WIN;
        uint64_t e[SAS_TAG_WIN];
        {
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            const uint32_t o = (uint32_t)(wb & 1);
            const u64x2* ep = reinterpret_cast<const u64x2*>(ent + (wb & ~1ull));
            uint64_t w2[SAS_TAG_WIN + 2];
#pragma unroll
            for (int j = 0; j < SAS_TAG_WIN / 2 + 1; j++) {
                const u64x2 v = (2u * j < o + nw) ? __builtin_nontemporal_load(ep + j) : u64x2{0ull, 0ull};
                w2[2 * j] = v.x;
                w2[2 * j + 1] = v.y;
            }
#pragma unroll
            for (int j = 0; j < SAS_TAG_WIN; j++) e[j] = (uint32_t)j < nw ? (o ? w2[j + 1] : w2[j]) : 0ull;
        }
        // first slot whose tag is >= q's: every slot before it is < q (tags are sorted
        // within a bucket)
        uint32_t j0 = nw;
#pragma unroll
        for (int j = SAS_TAG_WIN - 1; j >= 0; j--)
            if ((uint32_t)j < nw && (uint32_t)(e[j] >> 40) >= Q12) j0 = (uint32_t)j;
        uint64_t ej = e[0];
#pragma unroll
        for (int j = 1; j < SAS_TAG_WIN; j++) ej = (j0 == (uint32_t)j) ? e[j] : ej;
        if (j0 < nw) {
            const uint64_t r = wb + j0;
            // a text-slice query t[src .. src + m) and the tying entry of suffix src: that
            // suffix starts with q, so it is >= q without reading the text (the slice must
            // lie inside the text)
            const uint64_t src = query_source(q);
            const bool own = src != ~0ull && src + q.m <= a.n && (ej & TAG_M40) == src && (uint32_t)(ej >> 40) == Q12;
            if (own || tag_ge<QW>(ej, Q12, a, q)) {
                ans = r;
                pos = ej & TAG_M40;
                done = true;
            }
            start = r + 1;  // a tag tie whose suffix is < q
            break;
        }
        start = wb + nw;  // the whole window is < q
        if (start >= hi) break;
    }
    if (!done) {  // binary search over the rest of the bucket (rank hi if nothing qualifies)
        uint64_t l2 = start, h2 = hi, pr = QUAD_NO_SA;
        while (l2 < h2) {
            const uint64_t mid = (l2 + h2) >> 1;
            const uint64_t f = __builtin_nontemporal_load(ent + mid);
            if (tag_ge<QW>(f, Q12, a, q)) {
                h2 = mid;
                pr = f & TAG_M40;
            } else {
                l2 = mid + 1;
            }
        }
        ans = l2;
        pos = l2 >= sa_n ? a.next_pos : (pr != QUAD_NO_SA ? pr : (ent[l2] & TAG_M40));
    }
    a.out_pos[i] = pos;
    if (a.out_probes) {  // the reference's cnt: the table, then binary_search over [lo, hi)
        uint32_t probes = 1;
        for (uint64_t l2 = lo, h2 = hi; l2 < h2; probes++) {
            const uint64_t mid = (l2 + h2) >> 1;
            if (mid < ans) l2 = mid + 1;
            else h2 = mid;
        }
        a.out_probes[i] = probes;
    }
}

// byte offset and length of query i
__device__ __forceinline__ void query_span(const SearchArgs& a, uint64_t i, uint64_t* off, uint32_t* m) {
    if (a.qoff) {
        *off = a.qoff[i];
        *m = a.qlen[i];
    } else {
        *off = i * (uint64_t)a.m_fixed;
        *m = a.m_fixed;
    }
}

#ifndef SAS_TAG_WQ
#define SAS_TAG_WQ 1
#endif

template <int QW>
__global__ __launch_bounds__(SAS_TAG_BLOCK, (QW >= SAS_TAG_LB_QW ? SAS_TAG_LB : 8)) void k_sa_tagged(SearchArgs a) {
    uint32_t bad = 0;
#if SAS_TAG_WQ
    // wave-uniform loop over batches of 64 consecutive queries; the batch's bytes are staged
    // through LDS (wave_stage_queries) unless they are spread out
    __shared__ uint32_t wq[SAS_TAG_BLOCK / 64][2 * SAS_WQ_WORDS];
    uint32_t* L32 = wq[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x + (threadIdx.x & ~63u); b0 < a.nq;
         b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = b0 + lane;
        const bool act = i < a.nq;
        uint64_t qo = 0;
        uint32_t m = 0;
        if (act) query_span(a, i, &qo, &m);
        uint64_t base;
        if (wave_stage_queries(a.qbytes, qo, m, act, L32, &base)) {
            if (act) {
                WaveQuery q;
                q.init(L32, (uint32_t)(qo - base), m);
                tagged_lookup<QW>(a, q, i);
            }
        } else if (act) {
            ByteQuery q;
            q.init(a.qbytes + qo, m);
            tagged_lookup<QW>(a, q, i);
        }
    }
#else
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        tagged_lookup<QW>(a, q, i);
    }
#endif
    if (bad) atomicOr(a.bad, 1u);
}

// SAS_QUERIES_ARE_SLICES: query i is the slice t[qoff[i] .. qoff[i] + qlen[i]) of the indexed
// text, read from the packed text (no query bytes), one lane per query.
template <int QW>
__global__ __launch_bounds__(SAS_TAG_BLOCK, SAS_TAG_LB) void k_sa_tagged_slices(SearchArgs a) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t qo;
        uint32_t m;
        query_span(a, i, &qo, &m);
        TextQuery q;
        q.init(a.tw, qo, m);
        tagged_lookup<QW>(a, q, i);
    }
}

// Occurrence ranges on the tagged index: lo = the lower bound in q's bucket, hi = the first
// suffix whose first min(m, len) chars are > q, in the bucket of the routing key; both
// bisections advance in lock step (two entry reads in flight).
template <int QW>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_tagged_range(SearchArgs a, uint64_t* out_hi) {
    uint32_t bad = 0;
    const uint64_t* ent = reinterpret_cast<const uint64_t*>(a.sa);
    const uint32_t sh = 64 - 2 * a.tag_p;
    const uint32_t L = a.tag_p + SAS_TAG_CHARS;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        const uint32_t Q12 = tag_of_key(K64, a.tag_p), Q3t = tag_of_key(Q3, a.tag_p);
        uint64_t lo, l1, hi, h1;
        tag_bucket(a, K64 >> sh, &lo, &l1);
        tag_bucket(a, (m <= L ? Q3 : K64) >> sh, &hi, &h1);
        while (lo < l1 || hi < h1) {
            const bool g0 = lo < l1, g1 = hi < h1;
            const uint64_t m0 = (lo + l1) >> 1, m1 = (hi + h1) >> 1;
            const uint64_t e0 = g0 ? __builtin_nontemporal_load(ent + m0) : 0;
            const uint64_t e1 = g1 ? __builtin_nontemporal_load(ent + m1) : 0;
            if (g0) {
                if (tag_ge<QW>(e0, Q12, a, q)) l1 = m0;
                else lo = m0 + 1;
            }
            if (g1) {
                if (tag_gt_prefix<QW>(e1, Q12, Q3t, a, q)) h1 = m1;
                else hi = m1 + 1;
            }
        }
        if (hi < lo) hi = lo;
        a.out_pos[i] = a.rank_lo + lo;
        out_hi[i] = a.rank_lo + hi;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// ------------------------------------------------------------------ TAGGED on bucket lines
// SAS_BUILD_TAG_LINES (sas_build.hip, build_tag_lines): line b holds bucket b's header
// {overflow offset | count} and the 48-bit entries {SA | tag << sb} of ranks first .. first +
// 19 (common.hpp: u16 high halves, then u32 low halves), so the bucket word and the first
// window of the tagged lookup above are one 128-B request, and 20 slots keep 98% of the
// positive lookups at ~16 suffixes per bucket inside it.  An 8-lane group reads the lines of
// its 8 queries (one per lane) together, 16 B per lane (lane 0 the header and hi[0..3], lanes
// 1 and 2 hi[4..19], lanes 3..7 lo[0..19]); per line lanes 0-2 count the slots whose tag is
// below the query's, the group sums the counts, and the lanes holding that slot's halves
// hand them to the query's lane; the rest -- the tie's text compare, a larger bucket's
// overflow window -- is per lane.  Slots past the bucket's count hold the next buckets' first
// suffixes with the maximal tag, so "every suffix of the bucket is < q" finds its answer (the
// first suffix after the bucket, rank first + count) in the same line whenever count < 20
// (and at overflow index count - 20 otherwise).
#define TL_G 8
// waves per SIMD the line kernels are built for: the 8 line loads a lane keeps in flight take
// 32 VGPRs (at 5 waves the kernel spills)
#ifndef SAS_TL_LB
#define SAS_TL_LB 4
#endif
#ifndef SAS_TL_WIN
#define SAS_TL_WIN 8  // overflow entries a lane reads before bisecting the rest
#endif

// entry j of bucket b: line slot j (j < 20) or overflow entry j - 20
__device__ __forceinline__ uint64_t tl_entry(const SearchArgs& a, uint64_t b, uint64_t ovf, uint64_t j) {
    return j < SAS_TL_SLOTS ? tl_slot(a.tag_lines, b, (uint32_t)j)
                            : __builtin_nontemporal_load(a.tag_ovf + ovf + (j - SAS_TL_SLOTS));
}

// bucket b's suffix count from its header word (a saturated count reads the first-rank table)
__device__ __forceinline__ uint64_t tl_count(const SearchArgs& a, uint64_t b, uint64_t h0) {
    const uint64_t c = h0 >> 40;
    return c == 0xFFFFFFull ? a.tag_first[b + 1] - a.tag_first[b] : c;
}

// chars known equal to q's when an entry's tag ties with q's: the bucket's p and the tag's whole chars
__device__ __forceinline__ uint32_t tl_known(const SearchArgs& a) { return a.tag_p + (tl_tag_bits(a.tag_sb) >> 1); }

// text word pairs a bucket-line lookup loads together for its tie's compare: 5 pairs (80 B)
// cover chars [p + 12, 256) of any suffix, so no compare of a query of <= 256 chars waits for a
// second round trip (loaded lazily they are ~3 dependent round trips of the whole wave).  Same
// box, 2*10^7 ragged 8..256 at n = 2^34: 5 pairs 1.91 ms, 4 pairs 1.99, 3 pairs 2.05-2.07
// (gpurun_out A/B, profiles/r3/); 0: the lazy pair loop (suffix_less_from_x2).  The pairs come
// from the text copy in which they lie in one 128-B line (sas_index::text2).
#ifndef SAS_TL_PRE
#define SAS_TL_PRE 5
#endif

// suffix(e) >= q for an entry of q's bucket (Qt: q's tag), the tie's text compare preloading
// (PRE) or pair by pair (the rare bisection and the range kernel)
template <int QW, bool PRE, class Q>
__device__ __forceinline__ bool tl_ge(uint64_t e, uint32_t Qt, const SearchArgs& a, const Q& q) {
    const uint32_t T = (uint32_t)(e >> a.tag_sb);
    if (T != Qt) return T > Qt;
    const uint64_t p = e & tl_sa_mask(a.tag_sb);
    const uint32_t L = tl_known(a);
    if (q.m <= L) return (a.n - p) >= (uint64_t)q.m;
    const uint64_t src = query_source(q);  // a text-slice query's own suffix starts with q
    if (src != ~0ull && src + q.m <= a.n && p == src) return true;
    uint32_t lcp;
#if SAS_TL_PRE
    if (PRE) return !suffix_less_from_pre<SAS_TL_PRE>(a.tw, a.tw2, a.n, p, q, L, &lcp);
#endif
    return !suffix_less_from_x2<QW>(a.tw, a.n, p, q, L, &lcp);
}

// the first min(m, len) chars of suffix(e) are > q, for an entry of the bucket of q's routing
// key (Q3t: the tag of q padded with 3s; as tag_gt_prefix)
template <int QW, class Q>
__device__ __forceinline__ bool tl_gt_prefix(uint64_t e, uint32_t Qt, uint32_t Q3t, const SearchArgs& a, const Q& q) {
    const uint32_t T = (uint32_t)(e >> a.tag_sb);
    const uint32_t L = tl_known(a);
    if (q.m <= L) return T > Q3t;
    if (T != Qt) return T > Qt;
    uint32_t lcp;
    const bool lt = suffix_less_from_x2<QW>(a.tw, a.n, e & tl_sa_mask(a.tag_sb), q, L, &lcp);
    return !lt && lcp < q.m;
}

// The lookup after the line: f = the number of the bucket's first 20 suffixes whose tag is
// below q's (20: all of them), ef = slot f's entry when f < 20, h0 = the line's header word
// {overflow offset | count}.  Slots past the bucket's count carry the maximal tag, so f <=
// count when count < 20, and f == count finds the first suffix after the bucket.  The answer
// is entry j of the bucket for the first j in [0, count] whose suffix is >= q (j = count: the
// next bucket's first suffix).  A wave waits for its slowest lane at every step, so the loads
// of the lanes that need the overflow window are issued before the other lanes' text compares
// wait for theirs: one round trip serves both.
template <int QW, class Q>
__device__ __forceinline__ void tl_finish(const SearchArgs& a, const Q& q, uint64_t i, uint64_t b, uint64_t h0,
                                          uint32_t f, uint64_t ef, uint32_t Qt) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const uint32_t sb = a.tag_sb;
    const uint64_t cnt = tl_count(a, b, h0), ovf = h0 & TAG_M40;
    // the overflow window [20, cnt] (entry cnt is >= q whatever its tag), as 16-B aligned pairs
    const bool ovfl = f >= SAS_TL_SLOTS && cnt > SAS_TL_SLOTS;
    const uint64_t rest = ovfl ? cnt + 1 - SAS_TL_SLOTS : 0;
    const uint32_t nw = rest < SAS_TL_WIN ? (uint32_t)rest : (uint32_t)SAS_TL_WIN;
    const uint32_t o = (uint32_t)(ovf & 1);
    uint64_t w2[SAS_TL_WIN + 2];
    if (ovfl) {
        const u64x2* ep = reinterpret_cast<const u64x2*>(a.tag_ovf + (ovf & ~1ull));
#pragma unroll
        for (int k = 0; k < SAS_TL_WIN / 2 + 1; k++) {
            const u64x2 v = (2u * k < o + nw) ? __builtin_nontemporal_load(ep + k) : u64x2{0ull, 0ull};
            w2[2 * k] = v.x;
            w2[2 * k + 1] = v.y;
        }
    }
    uint64_t j = 0, e = 0, start = SAS_TL_SLOTS, cj = 0, ce = 0;
    bool done = false, cand = false;  // cand: entry ce (index cj) needs the compare
    if (f < SAS_TL_SLOTS) {
        if (f >= cnt) {  // the first suffix after the bucket
            j = f;
            e = ef;
            done = true;
        } else {
            cand = true;
            cj = f;
            ce = ef;
        }
        start = (uint64_t)f + 1;  // a tie whose suffix is < q: the search goes on
    } else if (cnt == SAS_TL_SLOTS) {  // every suffix of the bucket is < q: the next one's first
        j = cnt;
        e = tl_entry(a, b, ovf, cnt);
        done = true;
    } else if (ovfl) {
        uint64_t ew[SAS_TL_WIN];
#pragma unroll
        for (int k = 0; k < SAS_TL_WIN; k++) ew[k] = (uint32_t)k < nw ? (o ? w2[k + 1] : w2[k]) : 0ull;
        uint32_t k0 = nw;
#pragma unroll
        for (int k = SAS_TL_WIN - 1; k >= 0; k--)
            if ((uint32_t)k < nw && (SAS_TL_SLOTS + k == cnt || (uint32_t)(ew[k] >> sb) >= Qt)) k0 = (uint32_t)k;
        uint64_t ek0 = ew[0];
#pragma unroll
        for (int k = 1; k < SAS_TL_WIN; k++) ek0 = (k0 == (uint32_t)k) ? ew[k] : ek0;
        if (k0 < nw) {
            const uint64_t r = SAS_TL_SLOTS + k0;
            if (r == cnt) {
                j = r;
                e = ek0;
                done = true;
            } else {
                cand = true;
                cj = r;
                ce = ek0;
            }
            start = r + 1;
        } else {
            start = SAS_TL_SLOTS + nw;
        }
    }
    if (cand && tl_ge<QW, true>(ce, Qt, a, q)) {  // one compare site: a slot's or the window's
        j = cj;
        e = ce;
        done = true;
    }
    if (!done && start == cnt) {  // the first suffix after the bucket
        j = cnt;
        e = tl_entry(a, b, ovf, cnt);
        done = true;
    }
    if (!done) {  // binary search over [start, cnt): entry cnt is >= q
        uint64_t l2 = start, h2 = cnt, pe = 0;
        bool have = false;
        while (l2 < h2) {
            const uint64_t mid = (l2 + h2) >> 1;
            const uint64_t fm = tl_entry(a, b, ovf, mid);
            if (tl_ge<QW, false>(fm, Qt, a, q)) {
                h2 = mid;
                pe = fm;
                have = true;
            } else {
                l2 = mid + 1;
            }
        }
        j = l2;
        e = (have && l2 < cnt) ? pe : tl_entry(a, b, ovf, l2);
    }
    const uint64_t s = e & tl_sa_mask(sb);
    a.out_pos[i] = s == tl_sa_mask(sb) ? a.next_pos : s;
    if (a.out_probes) {  // the reference's cnt: the table, then binary_search over [first, first + cnt)
        uint32_t probes = 1;
        for (uint64_t l2 = 0, h2 = cnt; l2 < h2; probes++) {
            const uint64_t mid = (l2 + h2) >> 1;
            if (mid < j) l2 = mid + 1;
            else h2 = mid;
        }
        a.out_probes[i] = probes;
    }
}

// Exchanges inside an aligned group of 8 lanes without address registers: ds_swizzle in bit
// mode (lane' = ((lane & and) | or) ^ xor within each 32-lane half) and DPP quad_perm.
__device__ __forceinline__ uint32_t g8_swz(uint32_t v, int pattern_k) {
    switch (pattern_k) {  // broadcast from lane k of the group: and 0x18, or k
        case 0: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (0 << 5));
        case 1: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (1 << 5));
        case 2: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (2 << 5));
        case 3: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (3 << 5));
        case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (4 << 5));
        case 5: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (5 << 5));
        case 6: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (6 << 5));
        default: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (7 << 5));
    }
}
// sum over the group of 8 (every lane gets it)
__device__ __forceinline__ uint32_t g8_sum(uint32_t c) {
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xF, 0xF, false);  // lane ^ 1
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xF, 0xF, false);  // lane ^ 2
    return c + (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x1F | (4 << 10));    // lane ^ 4
}
__device__ __forceinline__ uint32_t sel4(const uint4& v, uint32_t k) {
    const uint32_t lo = (k & 1) ? v.y : v.x, hi = (k & 1) ? v.w : v.z;
    return (k & 2) ? hi : lo;
}

// The cooperative part: every lane of the wave calls it together (act: the lane holds query
// i).  Lane s of a group holds 16 B of each of the group's 8 lines (common.hpp); per line
// lanes 0-2 count the slots whose tag is below the line's query's (the tag halves are the
// high bits of the u16 fields: h < Qt << (sb - 32)), the group sums the counts into f, and the
// lanes holding hi[f] ((f + 4) / 8) and lo[f] (3 + f / 4) hand them, with the header word, to
// the query's lane.
template <int QW, class Q>
__device__ __forceinline__ void tl_lookup(const SearchArgs& a, const Q& q, bool act, uint64_t i) {
    const uint32_t lane = threadIdx.x & 63, sub = lane & (TL_G - 1), g0 = lane & ~(uint32_t)(TL_G - 1);
    const uint32_t sh = 64 - 2 * a.tag_p, hs = a.tag_sb - 32;
    const uint64_t K64 = act ? q.w[0] : 0ull;
    const uint64_t b = K64 >> sh;
    const uint32_t Qt = tl_tag_of_key(K64, a.tag_p, tl_tag_bits(a.tag_sb));
    const uint4* L4 = reinterpret_cast<const uint4*>(a.tag_lines);
    uint4 v[TL_G];
#pragma unroll
    for (int k = 0; k < TL_G; k++) {
        const uint64_t bk = ((uint64_t)g8_swz((uint32_t)(b >> 32), k) << 32) | g8_swz((uint32_t)b, k);
        v[k] = nt_load4(L4 + bk * 8 + sub);
    }
    // tag fields of this lane's 16 B: lane 0 the upper 8 B (hi[0..3]), lanes 1 and 2 all of it;
    // a field h counts when h < Qt << (sb - 32), two fields per packed saturating subtract
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    const bool lo_tags = sub == 1 || sub == 2, hi_tags = sub <= 2;
    uint64_t my_h0 = 0, my_ef = 0;
    uint32_t my_f = 0;
#pragma unroll
    for (int k = 0; k < TL_G; k++) {
        const uint32_t Qs = g8_swz(Qt, k) << hs;  // (h >> hs) < Qt  <=>  h < Qt << hs
        const uint32_t Qp = Qs | (Qs << 16);
        const u16x2 Qlo = __builtin_bit_cast(u16x2, lo_tags ? Qp : 0u), Qhi = __builtin_bit_cast(u16x2, hi_tags ? Qp : 0u);
        const u16x2 acc =
            __builtin_elementwise_min(__builtin_elementwise_sub_sat(Qlo, __builtin_bit_cast(u16x2, v[k].x)), one) +
            __builtin_elementwise_min(__builtin_elementwise_sub_sat(Qlo, __builtin_bit_cast(u16x2, v[k].y)), one) +
            __builtin_elementwise_min(__builtin_elementwise_sub_sat(Qhi, __builtin_bit_cast(u16x2, v[k].z)), one) +
            __builtin_elementwise_min(__builtin_elementwise_sub_sat(Qhi, __builtin_bit_cast(u16x2, v[k].w)), one);
        const uint32_t f = g8_sum((uint32_t)acc.x + acc.y);
        const uint32_t fe = (f + 4) & 7;
        const uint32_t hw = (sel4(v[k], fe >> 1) >> ((fe & 1) * 16)) & 0xFFFFu;
        const uint32_t mine = sub < 3 ? hw : sel4(v[k], f & 3);
        const uint32_t hl = (f + 4) >> 3, ll = 3 + (f >> 2);
        const uint32_t hiv = (uint32_t)__shfl((int)mine, (int)(g0 + (hl < 2 ? hl : 2u)), 64);
        const uint32_t lov = (uint32_t)__shfl((int)mine, (int)(g0 + (ll < 7 ? ll : 7u)), 64);
        const uint64_t h0 = ((uint64_t)g8_swz(v[k].y, 0) << 32) | g8_swz(v[k].x, 0);
        if (sub == (uint32_t)k) {
            my_h0 = h0;
            my_f = f;
            my_ef = ((uint64_t)hiv << 32) | lov;
        }
        __builtin_amdgcn_sched_barrier(0);  // one line at a time: interleaved, the 8 spill
    }
    if (act) tl_finish<QW>(a, q, i, b, my_h0, my_f, my_ef, Qt);
}

template <int QW>
__global__ __launch_bounds__(SAS_TAG_BLOCK, SAS_TL_LB) void k_sa_tagged_lines(SearchArgs a) {
    // wave-uniform loop over batches of 64 consecutive queries, staged as in k_sa_tagged
    __shared__ uint32_t wq[SAS_TAG_BLOCK / 64][2 * SAS_WQ_WORDS];
    uint32_t* L32 = wq[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x + (threadIdx.x & ~63u); b0 < a.nq;
         b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = b0 + lane;
        const bool act = i < a.nq;
        uint64_t qo = 0;
        uint32_t m = 0;
        if (act) query_span(a, i, &qo, &m);
        uint64_t base;
        if (wave_stage_queries(a.qbytes, qo, m, act, L32, &base)) {
            WaveQuery q;
            q.init(L32, act ? (uint32_t)(qo - base) : 0u, act ? m : 0u);
            tl_lookup<QW>(a, q, act, i);
        } else {
            ByteQuery q;
            q.init(a.qbytes + qo, act ? m : 0u);
            tl_lookup<QW>(a, q, act, i);
        }
    }
}

// SAS_QUERIES_ARE_SLICES on bucket lines
template <int QW>
__global__ __launch_bounds__(SAS_TAG_BLOCK, SAS_TL_LB) void k_sa_tagged_lines_slices(SearchArgs a) {
    for (uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x + (threadIdx.x & ~63u); b0 < a.nq;
         b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = b0 + (threadIdx.x & 63);
        const bool act = i < a.nq;
        uint64_t qo = 0;
        uint32_t m = 0;
        if (act) query_span(a, i, &qo, &m);
        TextQuery q;
        q.init(a.tw, qo, m);
        tl_lookup<QW>(a, q, act, i);
    }
}

// Measured and not kept (profiles/r3/defer/, same box, 2*10^7 ragged 8..256 at n = 2^34):
// * two passes: the lanes whose answer lies past the line's 20 slots (~2% of lanes, in most
//   waves) wrote their query index into a per-wave list and a second kernel ran them whole,
//   so no wave waited for the overflow window and its second compare: 1.67 against 1.48 ms
//   (one list counter for the grid, claimed by an atomic per wave: 3.3 ms);
// * the next batch's query offsets and lengths loaded a batch ahead: 1.478 against 1.462 ms.
// The kernel is bound by the rate of its random requests (0.84 of the ceiling), not by the
// round trips of a wave's slowest lane.

// Occurrence ranges on bucket lines: both bounds bisected in their buckets (entries by
// bucket index: slot or overflow), as k_sa_tagged_range does over rank-ordered entries.
template <int QW>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_tagged_lines_range(SearchArgs a, uint64_t* out_hi) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.tag_p, tb = tl_tag_bits(a.tag_sb);
    const uint32_t L = tl_known(a);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.nq;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* qb;
        uint32_t m;
        query_ptr(a, i, &qb, &m);
        QueryRegs<QW> q;
        q.load(qb, m, &bad);
        const uint64_t K64 = q.w[0];
        const uint64_t Q3 = m >= 32 ? K64 : (K64 | (~0ull >> (2 * m)));
        const uint32_t Qt = tl_tag_of_key(K64, a.tag_p, tb), Q3t = tl_tag_of_key(Q3, a.tag_p, tb);
        const uint64_t b0 = K64 >> sh, b1 = (m <= L ? Q3 : K64) >> sh;
        const uint64_t h00 = a.tag_lines[b0 * 16], h10 = a.tag_lines[b1 * 16];
        const uint64_t o0 = h00 & TAG_M40, o1 = h10 & TAG_M40;
        uint64_t lo = 0, l1 = tl_count(a, b0, h00), hi = 0, h1 = tl_count(a, b1, h10);
        while (lo < l1 || hi < h1) {
            const bool g0 = lo < l1, g1 = hi < h1;
            const uint64_t m0 = (lo + l1) >> 1, m1 = (hi + h1) >> 1;
            const uint64_t e0 = g0 ? tl_entry(a, b0, o0, m0) : 0;
            const uint64_t e1 = g1 ? tl_entry(a, b1, o1, m1) : 0;
            if (g0) {
                if (tl_ge<QW, false>(e0, Qt, a, q)) l1 = m0;
                else lo = m0 + 1;
            }
            if (g1) {
                if (tl_gt_prefix<QW>(e1, Qt, Q3t, a, q)) h1 = m1;
                else hi = m1 + 1;
            }
        }
        uint64_t rlo = a.tag_first[b0] + lo, rhi = a.tag_first[b1] + hi;
        if (rhi < rlo) rhi = rlo;
        a.out_pos[i] = a.rank_lo + rlo;
        out_hi[i] = a.rank_lo + rhi;
    }
    if (bad) atomicOr(a.bad, 1u);
}

// Validation pass (SAS_VALIDATE, host-pointer calls): every byte of every query must be a
// DNA code 0..3, including those past the words a search kernel holds in registers.
__global__ void k_validate_queries(const uint8_t* __restrict__ qb, const uint64_t* __restrict__ qoff,
                                   const uint32_t* __restrict__ qlen, uint32_t m_fixed, uint64_t nq,
                                   uint32_t* __restrict__ bad) {
    uint32_t b = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* q = qoff ? qb + qoff[i] : qb + i * (uint64_t)m_fixed;
        const uint32_t m = qoff ? qlen[i] : m_fixed;
        for (uint32_t k = 0; k < m; k++) b |= q[k];
    }
    if (b & 0xFCu) atomicOr(bad, 1u);
}

// ------------------------------------------------------------------ host dispatch
template <int W>
static void launch_w(int algo, bool top, bool range, int qw, dim3 grid, dim3 block, hipStream_t st,
                     const SearchArgs& a) {
#define QW_CASE(KERNEL_T)                                                           \
    switch (qw) {                                                                   \
        case 1: hipLaunchKernelGGL(KERNEL_T(1), grid, block, 0, st, a); break;      \
        case 2: hipLaunchKernelGGL(KERNEL_T(2), grid, block, 0, st, a); break;      \
        case 4: hipLaunchKernelGGL(KERNEL_T(4), grid, block, 0, st, a); break;      \
        default: hipLaunchKernelGGL(KERNEL_T(8), grid, block, 0, st, a); break;     \
    }
    // the query words all in registers when the batch's longest query is known to fit them
    const bool exq = a.m_max && a.m_max <= 32u * (uint32_t)qw && qw <= 8;
#define QWX_CASE(KERNEL_T)                                                                      \
    switch (qw) {                                                                               \
        case 1: hipLaunchKernelGGL(KERNEL_T(1, false), grid, block, 0, st, a); break;           \
        case 2: hipLaunchKernelGGL(KERNEL_T(2, false), grid, block, 0, st, a); break;           \
        case 4:                                                                                 \
            if (exq) hipLaunchKernelGGL(KERNEL_T(4, true), grid, block, 0, st, a);              \
            else hipLaunchKernelGGL(KERNEL_T(4, false), grid, block, 0, st, a);                 \
            break;                                                                              \
        default:                                                                                \
            if (exq) hipLaunchKernelGGL(KERNEL_T(8, true), grid, block, 0, st, a);              \
            else hipLaunchKernelGGL(KERNEL_T(8, false), grid, block, 0, st, a);                 \
            break;                                                                              \
    }
#define K_PLAIN_TOP(Q, X) (k_sa_binary<Q, BS_PLAIN, true, W, false, X>)
#define K_PLAIN(Q, X) (k_sa_binary<Q, BS_PLAIN, false, W, false, X>)
#define K_LCP_TOP(Q, X) (k_sa_binary<Q, BS_MLR, true, W, false, X>)
#define K_LCP(Q, X) (k_sa_binary<Q, BS_MLR, false, W, false, X>)
#define K_LLCP_TOP(Q, X) (k_sa_binary<Q, BS_LLCP, true, W, false, X>)
#define K_LLCP(Q, X) (k_sa_binary<Q, BS_LLCP, false, W, false, X>)
#define K_PLAIN_RANGE(Q) (k_sa_binary<Q, BS_PLAIN, false, W, true>)
#define K_LCP_RANGE(Q) (k_sa_binary<Q, BS_MLR, false, W, true>)
#define K_STREE(Q) (k_sa_stree<Q, W>)
#define K_STREE4X(Q, X) (k_sa_stree4x<Q, W, false, X>)
#define K_STREE4X_LT(Q, X) (k_sa_stree4x<Q, W, true, X>)
#define K_SECTOR(Q) (k_sa_sector<Q>)
    if (algo == SAS_ALGO_PLAIN && range) {
        QW_CASE(K_PLAIN_RANGE)
    } else if (algo == SAS_ALGO_LCP && range) {
        QW_CASE(K_LCP_RANGE)
    } else if (algo == SAS_ALGO_PLAIN) {
        if (top) { QWX_CASE(K_PLAIN_TOP) } else { QWX_CASE(K_PLAIN) }
    } else if (algo == SAS_ALGO_LCP) {
        if (top) { QWX_CASE(K_LCP_TOP) } else { QWX_CASE(K_LCP) }
    } else if (algo == SAS_ALGO_LLCP) {
        if (top) { QWX_CASE(K_LLCP_TOP) } else { QWX_CASE(K_LLCP) }
    } else if (algo == SAS_ALGO_STREE) {
        // m <= 32: the cooperative kernel (descent dominates); longer: one lane per query
        if (qw == 1 && !SAS_STREE_PERLANE) hipLaunchKernelGGL(K_STREE(1), grid, block, 0, st, a);
        else { QWX_CASE(K_STREE4X) }
    } else if (algo == SAS_ALGO_STREE_LLCP) {
        // the same descent, the LLCP tail (stree_tail) on one lane per query at every m: the
        // tail's walk to its in-run mids diverges between queries, which a 4-lane group per
        // query would pay 4 times over (m = 32: 1.77 ms cooperative)
        QWX_CASE(K_STREE4X_LT)
    } else {  // SAS_ALGO_SECTOR: positions come from the fused leaves, W = 4 only
        QW_CASE(K_SECTOR)
    }
#undef QW_CASE
#undef QWX_CASE
}

// QUAD / INLINE: fused leaves read no SA (W = 4 instantiation only); KO leaves read
// SA values through SaView<W>.
template <bool KO, int W>
static void launch_quad(int algo, bool top, int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a) {
#define QW_CASE(KERNEL_T)                                                           \
    switch (qw) {                                                                   \
        case 1: hipLaunchKernelGGL(KERNEL_T(1), grid, block, 0, st, a); break;      \
        case 2: hipLaunchKernelGGL(KERNEL_T(2), grid, block, 0, st, a); break;      \
        case 4: hipLaunchKernelGGL(KERNEL_T(4), grid, block, 0, st, a); break;      \
        default: hipLaunchKernelGGL(KERNEL_T(8), grid, block, 0, st, a); break;     \
    }
#define K_INLINE_TOP(Q) (k_sa_inline<Q, true, KO, W>)
#define K_INLINE(Q) (k_sa_inline<Q, false, KO, W>)
#define K_PREFIX(Q) (k_sa_prefix<(Q < SAS_PREFIX_QWMAX ? Q : SAS_PREFIX_QWMAX), KO, W, 4>)
#define K_PREFIX5(Q) (k_sa_prefix<(Q < SAS_PREFIX_QWMAX ? Q : SAS_PREFIX_QWMAX), KO, W, 5>)
#define K_PREFIX2(Q) (k_sa_prefix2<Q, 2>)
#define K_PREFIX4(Q) (k_sa_prefix2<Q, 4>)
#define K_PREFIX2H(Q) (k_sa_prefix2<Q, 2, true>)
#define K_PREFIX4H(Q) (k_sa_prefix2<Q, 4, true>)
#define K_PREFIX16(Q) (k_sa_prefix<(Q < SAS_PREFIX_QWMAX ? Q : SAS_PREFIX_QWMAX), KO, W, 16>)
    if (algo == SAS_ALGO_QUAD) {
        // m <= 32: the cooperative kernel; longer: one lane per query (as STREE), two query
        // words in registers (m <= 64), later ones repacked from the bytes
        if (qw == 1) hipLaunchKernelGGL((k_sa_quad<1, KO, W>), grid, block, 0, st, a);
        else if (qw == 2) hipLaunchKernelGGL((k_sa_quad4x<2, KO, W, false>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((k_sa_quad4x<SAS_QUAD4X_MAXREGS, KO, W, true>), grid, block, 0, st, a);
    } else if (algo == SAS_ALGO_PREFIX) {
        if (a.prefix_w == 5) { QW_CASE(K_PREFIX5) }
        else if (a.prefix_w == 16 && !KO) { QW_CASE(K_PREFIX16) }
        else if (a.prefix_w == 32 && !KO && a.prefix_hi40) { QW_CASE(K_PREFIX2H) }
        else if (a.prefix_w == 64 && !KO && a.prefix_hi40) { QW_CASE(K_PREFIX4H) }
        else if (a.prefix_w == 32 && !KO) { QW_CASE(K_PREFIX2) }
        else if (a.prefix_w == 64 && !KO) { QW_CASE(K_PREFIX4) }
        else { QW_CASE(K_PREFIX) }
    } else {
        if (top) { QW_CASE(K_INLINE_TOP) } else { QW_CASE(K_INLINE) }
    }
#undef QW_CASE
}

// INTERP: fused quad leaves (W = 4 instantiation, no SA reads) or SA + text at any width
template <int W, bool FUSED>
static void launch_interp(int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a, uint32_t range) {
    switch (qw) {
        case 1: hipLaunchKernelGGL((k_sa_interp<1, W, FUSED>), grid, block, 0, st, a, range); break;
        case 2: hipLaunchKernelGGL((k_sa_interp<2, W, FUSED>), grid, block, 0, st, a, range); break;
        case 4: hipLaunchKernelGGL((k_sa_interp<4, W, FUSED>), grid, block, 0, st, a, range); break;
        default: hipLaunchKernelGGL((k_sa_interp<8, W, FUSED>), grid, block, 0, st, a, range); break;
    }
}

// Tagged indexes (sa_w = 8): TAGGED, and PLAIN / LCP reading the SA values from the entries
static void launch_w8(int algo, bool top, int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a) {
#define QW_CASE(KERNEL_T)                                                           \
    switch (qw) {                                                                   \
        case 1: hipLaunchKernelGGL(KERNEL_T(1), grid, block, 0, st, a); break;      \
        case 2: hipLaunchKernelGGL(KERNEL_T(2), grid, block, 0, st, a); break;      \
        case 4: hipLaunchKernelGGL(KERNEL_T(4), grid, block, 0, st, a); break;      \
        default: hipLaunchKernelGGL(KERNEL_T(8), grid, block, 0, st, a); break;     \
    }
#define K_TAGGED(Q) (k_sa_tagged<Q>)
    const bool exq = a.m_max && a.m_max <= 32u * (uint32_t)qw && qw <= 8;
#define QWX_CASE(KERNEL_T)                                                                      \
    switch (qw) {                                                                               \
        case 1: hipLaunchKernelGGL(KERNEL_T(1, false), grid, block, 0, st, a); break;           \
        case 2: hipLaunchKernelGGL(KERNEL_T(2, false), grid, block, 0, st, a); break;           \
        case 4:                                                                                 \
            if (exq) hipLaunchKernelGGL(KERNEL_T(4, true), grid, block, 0, st, a);              \
            else hipLaunchKernelGGL(KERNEL_T(4, false), grid, block, 0, st, a);                 \
            break;                                                                              \
        default:                                                                                \
            if (exq) hipLaunchKernelGGL(KERNEL_T(8, true), grid, block, 0, st, a);              \
            else hipLaunchKernelGGL(KERNEL_T(8, false), grid, block, 0, st, a);                 \
            break;                                                                              \
    }
#define K8_PLAIN_TOP(Q, X) (k_sa_binary<Q, BS_PLAIN, true, 8, false, X>)
#define K8_PLAIN(Q, X) (k_sa_binary<Q, BS_PLAIN, false, 8, false, X>)
#define K8_LCP_TOP(Q, X) (k_sa_binary<Q, BS_MLR, true, 8, false, X>)
#define K8_LCP(Q, X) (k_sa_binary<Q, BS_MLR, false, 8, false, X>)
    if (algo == SAS_ALGO_TAGGED) {
        QW_CASE(K_TAGGED)
    } else if (algo == SAS_ALGO_PLAIN) {
        if (top) { QWX_CASE(K8_PLAIN_TOP) } else { QWX_CASE(K8_PLAIN) }
    } else {
        if (top) { QWX_CASE(K8_LCP_TOP) } else { QWX_CASE(K8_LCP) }
    }
#undef QW_CASE
#undef QWX_CASE
}

static int launch_search(const sas_index* x, SearchArgs& a, int algo, int qw, uint32_t flags, hipStream_t st) {
    // PLAIN, LLCP and INLINE read the pivot levels past the LDS ones from the prefix-relative
    // blocks, which the build makes wherever the array has such levels
    const bool coop = (algo == SAS_ALGO_QUAD || algo == SAS_ALGO_QUAD_LLCP ||
                       (algo == SAS_ALGO_STREE && !SAS_STREE_PERLANE)) && qw == 1;
    // inline prefix tables with G slots: G lanes per query
    const uint64_t g = (algo == SAS_ALGO_PREFIX && x->prefix_w >= 32) ? x->prefix_w / 16 : 1;
    const uint64_t lanes = a.nq * (coop ? QUAD_G : g);
    // k_sa_binary (PLAIN / LCP / LLCP, any SA width) and the S-tree kernels have their own
    // workgroup shape
    const bool bin = algo == SAS_ALGO_PLAIN || algo == SAS_ALGO_LCP || algo == SAS_ALGO_LLCP ||
                     algo == SAS_ALGO_STREE || algo == SAS_ALGO_STREE_LLCP;
    // k_sa_binary / k_sa_stree4x instances: QW = qw (1, 2, 4, and 8 for anything longer);
    // QUAD_LLCP past 32 chars sizes its two kernels itself
    const uint64_t bs = bin ? (coop ? SAS_BIN_BLOCK : BIN_BLOCK(qw)) : SEARCH_BLOCK;
    uint64_t blocks = (lanes + bs - 1) / bs;
    uint64_t cap = (uint64_t)x->num_cus * (bin ? SAS_BIN_BPC : BLOCKS_PER_CU);
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return 0;
    dim3 grid((unsigned)blocks), block((unsigned)bs);
    bool top = !(flags & SAS_NO_LDS_TOP);
    const bool range = (flags & SAS_PREFIX_RANGE) != 0;
    if (algo == SAS_ALGO_TAGGED) {
        uint64_t tb = (a.nq + SAS_TAG_BLOCK - 1) / SAS_TAG_BLOCK;
        const uint64_t tcap = (uint64_t)x->num_cus * (x->tag_lines ? SAS_TL_LB : (qw >= SAS_TAG_LB_QW ? SAS_TAG_LB : 8));
        if (tb > tcap) tb = tcap;
        if (x->tag_lines) {
            const dim3 g((unsigned)tb), b(SAS_TAG_BLOCK);
            const bool sl = (flags & SAS_QUERIES_ARE_SLICES) != 0;
#define SAS_TL_LAUNCH(Q)                                                                           \
    if (sl) hipLaunchKernelGGL(k_sa_tagged_lines_slices<Q>, g, b, 0, st, a);                       \
    else hipLaunchKernelGGL(k_sa_tagged_lines<Q>, g, b, 0, st, a)
            switch (qw) {
                case 1: SAS_TL_LAUNCH(1); break;
                case 2: SAS_TL_LAUNCH(2); break;
                case 4: SAS_TL_LAUNCH(4); break;
                default: SAS_TL_LAUNCH(8); break;
            }
#undef SAS_TL_LAUNCH
        } else if (flags & SAS_QUERIES_ARE_SLICES) {
            const dim3 g((unsigned)tb), b(SAS_TAG_BLOCK);
            switch (qw) {
                case 1: hipLaunchKernelGGL(k_sa_tagged_slices<1>, g, b, 0, st, a); break;
                case 2: hipLaunchKernelGGL(k_sa_tagged_slices<2>, g, b, 0, st, a); break;
                case 4: hipLaunchKernelGGL(k_sa_tagged_slices<4>, g, b, 0, st, a); break;
                default: hipLaunchKernelGGL(k_sa_tagged_slices<8>, g, b, 0, st, a); break;
            }
        } else {
            launch_w8(algo, top, qw, dim3((unsigned)tb), dim3(SAS_TAG_BLOCK), st, a);
        }
    } else if (algo == SAS_ALGO_INTERP) {
        if (x->quad_leaves && !x->quad_compact) launch_interp<4, true>(qw, grid, block, st, a, range);
        else if (x->sa_w == 8) launch_interp<8, false>(qw, grid, block, st, a, range);
        else if (x->sa_w == 5) launch_interp<5, false>(qw, grid, block, st, a, range);
        else launch_interp<4, false>(qw, grid, block, st, a, range);
    } else if (x->sa_w == 8) {
        launch_w8(algo, top, qw, grid, block, st, a);
    } else if (algo == SAS_ALGO_QUAD_LLCP && qw == 1) {
        // m <= 32: QUAD (the 32-char key decides every entry)
        hipLaunchKernelGGL((k_sa_quad<1, false, 4>), grid, block, 0, st, a);
    } else if (algo == SAS_ALGO_QUAD_LLCP) {
        // longer: k_sa_quad_llcp (fused leaves, any SA width: the leaves and the LLCP entries carry
        // 40-bit positions), with every query word in registers when the batch's longest query
        // is known to fit them, else two words and the rest repacked from the bytes
        const bool exact = a.m_max && a.m_max <= 32u * (uint32_t)qw && qw <= 8;
        const bool r32 = a.sa_n < (1ull << 32);
        uint64_t gq = (a.nq + QLLCP_BLOCK(2) - 1) / QLLCP_BLOCK(2);
        if (gq > (uint64_t)x->num_cus * 2) gq = (uint64_t)x->num_cus * 2;
        const dim3 g1((unsigned)gq), b1((unsigned)(exact ? QLLCP_BLOCK(qw) : QLLCP_BLOCK(2)));
#define QLLCP_GO(Q, X)                                                                            \
    if (r32) hipLaunchKernelGGL((k_sa_quad_llcp<Q, X, true>), g1, b1, 0, st, a);                  \
    else hipLaunchKernelGGL((k_sa_quad_llcp<Q, X, false>), g1, b1, 0, st, a)
        if (!exact) { QLLCP_GO(2, false); }
        else if (qw == 2) { QLLCP_GO(2, true); }
        else if (qw == 4) { QLLCP_GO(4, true); }
        else { QLLCP_GO(8, true); }
#undef QLLCP_GO
    } else if (algo == SAS_ALGO_QUAD || algo == SAS_ALGO_INLINE || algo == SAS_ALGO_PREFIX) {
        if (!x->quad_compact) launch_quad<false, 4>(algo, top, qw, grid, block, st, a);
        else if (x->sa_w == 5) launch_quad<true, 5>(algo, top, qw, grid, block, st, a);
        else launch_quad<true, 4>(algo, top, qw, grid, block, st, a);
    } else if (x->sa_w == 5 && algo != SAS_ALGO_SECTOR) {
        launch_w<5>(algo, top, range, qw, grid, block, st, a);
    } else {
        launch_w<4>(algo, top, range, qw, grid, block, st, a);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

static int qw_for(uint64_t maxlen) {
    if (maxlen <= 32) return 1;
    if (maxlen <= 64) return 2;
    if (maxlen <= 128) return 4;
    return 8;
}

static void fill_args(const sas_index* x, SearchArgs& a) {
    a.tw = x->text_w;
    a.n = x->n;
    a.sa_n = x->sa_n;
    a.next_pos = x->next_pos;
    a.rank_lo = x->rank_lo;
    a.sa = x->sa;
    a.llcp = x->llcp;
    a.prefix = x->prefix;
    a.prefix_chars = x->prefix_chars;
    a.prefix_w = x->prefix_w;
    a.prefix_hi40 = x->prefix_hi40;
    a.pt_base = x->prefix_key_lo;
    a.pt_jmax = x->prefix_entries >= 2 ? x->prefix_entries - 2 : 0;
    a.rel = x->rel;
    a.rel_lay = x->rel_lay;
    a.iters = x->iters;
    a.stree = x->stree;
    for (int h = 0; h < SAS_STREE_MAX_LAYERS; h++) a.stree_off[h] = x->stree_off[h];
    a.stree_height = x->stree_height;
    a.stree_lds_layers = x->stree_lds_layers;
    a.stree_lds_nodes = x->stree_lds_nodes;
    a.sec_inner = x->sec_inner;
    a.sec_leaves = x->sec_leaves;
    for (int h = 0; h < SAS_SECTOR_MAX_LAYERS; h++) a.sec_off[h] = x->sec_off[h];
    a.sec_inner_layers = x->sec_inner_layers;
    a.sec_lds_layers = x->sec_lds_layers;
    a.sec_lds_nodes = x->sec_lds_nodes;
    // non-temporal levels, as for the quad tree below
    a.stree_leaf_nt = (x->sa_n + 15) / 16 * 64 > SAS_NT_BYTES;
    a.quad_inner = x->quad_inner;
    a.quad_leaves = x->quad_leaves;
    for (int h = 0; h < SAS_QUAD_MAX_LAYERS; h++) a.quad_off[h] = x->quad_off[h];
    a.quad_fan = x->quad_fan;
    {
        // non-temporal levels: footprint > 3x the 256 MiB Infinity Cache (see nt_load4)
        const uint64_t big = SAS_NT_BYTES / 64;  // in 64-B nodes
        const uint32_t H = x->quad_inner_layers;
        a.quad_nt_from = H;
        for (uint32_t h = 0; h < H; h++) {
            const uint64_t sz = (h + 1 < H ? x->quad_off[h + 1] : x->quad_inner_nodes) - x->quad_off[h];
            if (sz > big) { a.quad_nt_from = h; break; }
        }
        a.quad_leaf_nt = x->quad_leaf_count > big;
    }
    a.quad_leaf_count = x->quad_leaf_count;
    a.quad_inner_layers = x->quad_inner_layers;
    a.quad_lds_layers = x->quad_lds_layers;
    a.quad_lds_nodes = x->quad_lds_nodes;
    a.tag_table = x->tag_table;
    a.tag_p = x->tag_p;
    a.tag_lines = x->tag_lines;
    a.tag_ovf = x->tag_ovf;
    a.tag_first = x->tag_first;
    a.tw2 = x->text2 ? x->text2 : x->text_w;
    a.tag_sb = x->tag_sb;
}

// Algorithm / index / flag compatibility, shared by the search entry points.
static int check_algo(const sas_index* x, int algo, uint32_t flags, const char* where) {
    const std::string w(where);
    if (algo < SAS_ALGO_PLAIN || algo > SAS_ALGO_QUAD_LLCP) SAS_FAIL(EINVAL, w + ": unknown algo");
    if ((flags & SAS_PREFIX_RANGE) &&
        (!x->prefix || (algo != SAS_ALGO_PLAIN && algo != SAS_ALGO_LCP && algo != SAS_ALGO_INTERP)))
        SAS_FAIL(EINVAL, "SAS_PREFIX_RANGE: PLAIN / LCP / INTERP on an index with SAS_BUILD_PREFIX");
    if (algo == SAS_ALGO_PREFIX && !x->prefix) SAS_FAIL(EINVAL, "SAS_ALGO_PREFIX needs SAS_BUILD_PREFIX");
    if (algo == SAS_ALGO_LLCP && !x->llcp) SAS_FAIL(EINVAL, w + ": SAS_ALGO_LLCP needs SAS_BUILD_LLCP");
    if ((algo == SAS_ALGO_QUAD || algo == SAS_ALGO_INLINE) && !x->quad_leaves)
        SAS_FAIL(EINVAL, w + ": SAS_ALGO_QUAD / SAS_ALGO_INLINE need SAS_BUILD_QUAD");
    if (algo == SAS_ALGO_STREE && !x->stree) SAS_FAIL(EINVAL, w + ": SAS_ALGO_STREE needs SAS_BUILD_STREE");
    if (algo == SAS_ALGO_STREE_LLCP && (!x->stree || !x->llcp))
        SAS_FAIL(EINVAL, w + ": SAS_ALGO_STREE_LLCP needs SAS_BUILD_STREE and SAS_BUILD_LLCP");
    if (algo == SAS_ALGO_QUAD_LLCP &&
        (!x->quad_leaves || x->quad_compact || x->quad_fan != SAS_QUAD_FAN || !x->llcp || x->sa_w == 8))
        SAS_FAIL(EINVAL, w + ": SAS_ALGO_QUAD_LLCP needs SAS_BUILD_LLCP and SAS_BUILD_QUAD with fused leaves in the "
                             "absolute layout (SAS_BUILD_QUAD_ABS)");
    if (algo == SAS_ALGO_SECTOR && !x->sec_leaves) SAS_FAIL(EINVAL, w + ": SAS_ALGO_SECTOR needs SAS_BUILD_SECTOR");
    if (algo == SAS_ALGO_TAGGED && !x->tag_table && !x->tag_lines)
        SAS_FAIL(EINVAL, w + ": SAS_ALGO_TAGGED needs SAS_BUILD_TAGGED");
    if (x->tag_lines && (algo != SAS_ALGO_TAGGED || (flags & SAS_PREFIX_RANGE)))
        SAS_FAIL(ENOTSUP, w + ": a bucket-line index (SAS_BUILD_TAG_LINES) has no SA array: SAS_ALGO_TAGGED only");
    if (x->sa_w == 8 && algo != SAS_ALGO_PLAIN && algo != SAS_ALGO_LCP && algo != SAS_ALGO_INTERP &&
        algo != SAS_ALGO_TAGGED)
        SAS_FAIL(EINVAL, w + ": a tagged index (SAS_BUILD_TAGGED) serves TAGGED, PLAIN, LCP and INTERP");
    if (algo == SAS_ALGO_INTERP && x->n >= (1ull << 32))
        SAS_FAIL(ENOTSUP, w + ": interpolation_search<16> needs n < 2^32 (the reference asserts r_val * r "
                              "fits a usize, sas/sa_search.rs:389-392)");
    return 0;
}

struct DeviceBuf {
    void* p = nullptr;
    ~DeviceBuf() { if (p) (void)hipFree(p); }
};

// Occurrence-range kernel for the index's structures (defined with the range kernels below)
static void launch_range(const sas_index* x, const SearchArgs& a, int qw, uint32_t flags, hipStream_t st,
                         uint64_t* dhi);

// ------------------------------------------------------------------ host-pointer pipeline
void sas_stage_pool_free(StagePool* p) {
    if (!p) return;
    for (StageSet* s : p->free_sets) stage_set_free(s);
    delete p;
}

enum HostMode {
    HM_FIXED = 0,   // fixed-length query bytes, staged as bytes
    HM_RAGGED = 1,  // ragged query bytes, gathered chunk by chunk
    HM_PACK = 2,    // fixed-length bytes, m <= 32, PREFIX: packed to 2-bit words on the host
    HM_WORDS = 3,   // the caller's packed words (sas_search_packed)
};

// Synchronous search of host arrays through the index's pinned staging slots (host_stage.hpp).
// Returns with out_pos / out_probes filled; EINVAL (after the whole batch) if a query byte
// is not a DNA code.
// out_hi non-null: occurrence ranges (launch_range) instead of a search; a chunk then holds
// at most cap_q / 2 queries and its lo and hi share the slot's position buffers.
static int host_pipeline(const sas_index* x, int mode, const uint8_t* qbytes, const uint64_t* qoff,
                         const uint32_t* qlen, const uint64_t* qwords, uint32_t m, uint64_t nq, int algo,
                         uint64_t* out_pos, uint32_t* out_probes, hipStream_t user_st, uint32_t flags,
                         uint64_t* out_hi = nullptr) {
    StageLease lease;
    TRY_RC(stage_acquire(x, &lease));
    StageSet& S = *lease.set;
    const uint64_t cap_q = out_hi ? S.cap_q / 2 : S.cap_q;
    HIP_TRY(hipStreamSynchronize(user_st));  // the caller's earlier work on its stream
    const bool validate = mode == HM_FIXED || mode == HM_RAGGED;
    std::atomic<uint32_t> host_bad{0};
    uint32_t dev_bad = 0;
    HostPool& pool = HostPool::get();
    int err = 0;
    // pieces of one pool job: the copy-out of the slot's previous chunk (positions, probes;
    // the caller's pages are often touched here for the first time, so page faults spread
    // over the pool too) and the fill of the new chunk run together
    constexpr uint64_t OUT_PIECE = 1u << 17;  // positions per copy-out piece (1 MiB)
    auto copy_out = [&](const StageSlot& sl, uint64_t piece) {
        const uint64_t k = sl.e - sl.s, b = piece * OUT_PIECE, e = std::min(k, b + OUT_PIECE);
        memcpy(out_pos + sl.s + b, sl.h_out + b, (e - b) * 8);
        if (out_hi) memcpy(out_hi + sl.s + b, sl.h_out + k + b, (e - b) * 8);
        if (out_probes) memcpy(out_probes + sl.s + b, sl.h_pr + b, (e - b) * 4);
    };
    auto out_pieces = [&](const StageSlot& sl) -> int {
        return sl.busy ? (int)((sl.e - sl.s + OUT_PIECE - 1) / OUT_PIECE) : 0;
    };
    // SAS_STAGE_TRACE=1: per-phase host time of the call on stderr (tuning aid)
    static const bool trace = getenv("SAS_STAGE_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    double t_wait = 0, t_job = 0, t_enq = 0;
    auto t_all = clk::now();
    uint64_t s = 0;
    int chunks = 0;
    for (int c = 0; s < nq && !err; c++, chunks++) {
        StageSlot& sl = S.slot[c % SAS_STAGE_SLOTS];
        auto t0 = clk::now();
        if (sl.busy) {
            HIP_TRY(hipStreamSynchronize(sl.st));
            if (validate) dev_bad |= *sl.h_bad;
        }
        auto t1 = clk::now();
        t_wait += std::chrono::duration<double, std::milli>(t1 - t0).count();
        const int po = out_pieces(sl);
        SearchArgs a{};
        fill_args(x, a);
        a.m_fixed = m;
        uint64_t k = 0, in_bytes = 0;
        int qw = 1;
        // the new chunk: its extent, and a fill function over `pi` pieces
        int pi_n = 0;
        std::function<void(int)> fill;
        if (mode == HM_FIXED || mode == HM_WORDS) {
            const uint64_t unit = mode == HM_FIXED ? std::max(m, 1u) : 8;
            k = std::min<uint64_t>(nq - s, std::min<uint64_t>(S.cap_bytes / unit, cap_q));
            in_bytes = k * unit;
            const uint8_t* src = mode == HM_FIXED ? qbytes + s * m : reinterpret_cast<const uint8_t*>(qwords + s);
            const uint64_t piece = 1u << 20;
            pi_n = (int)((in_bytes + piece - 1) / piece);
            fill = [&sl, src, in_bytes, piece](int i) {
                const uint64_t b = (uint64_t)i * piece;
                memcpy(sl.h_in + b, src + b, std::min(piece, in_bytes - b));
            };
            if (mode == HM_FIXED) qw = qw_for(m);
            a.m_max = mode == HM_FIXED ? m : 0;
        } else if (mode == HM_PACK) {
            // smaller chunks than the byte modes: the host packing is the longest stage, and
            // the pipeline fills and drains faster
            k = std::min<uint64_t>(nq - s, std::min<uint64_t>(cap_q, SAS_STAGE_PACK_Q));
            in_bytes = k * 8;
            constexpr uint64_t per = 16384;
            pi_n = (int)((k + per - 1) / per);
            uint64_t* w = reinterpret_cast<uint64_t*>(sl.h_in);
            const uint8_t* src = qbytes + s * m;
            fill = [&host_bad, w, src, k, m](int i) {
                const uint64_t b = (uint64_t)i * per, e = std::min(k, b + per);
                if (host_pack_words(src + b * m, m, e - b, w + b) & 0xFC) host_bad.fetch_or(1);
            };
        } else {  // ragged: consecutive queries up to the byte and count caps (at least one)
            uint64_t bytes = 0, e = s;
            uint32_t maxlen = 0;
            while (e < nq && e - s < cap_q && (e == s || bytes + qlen[e] <= S.cap_bytes)) {
                sl.h_off[e - s] = bytes;
                sl.h_len[e - s] = qlen[e];
                bytes += qlen[e];
                maxlen = std::max(maxlen, qlen[e]);
                e++;
            }
            k = e - s;
            in_bytes = bytes;
            constexpr uint64_t per = 4096;
            const uint64_t s0 = s;
            pi_n = (int)((k + per - 1) / per);
            fill = [&sl, qbytes, qoff, k, s0](int i) {
                const uint64_t b = (uint64_t)i * per, ee = std::min(k, b + per);
                for (uint64_t j = b; j < ee; j++) memcpy(sl.h_in + sl.h_off[j], qbytes + qoff[s0 + j], sl.h_len[j]);
            };
            qw = qw_for(maxlen);
            a.m_max = maxlen ? maxlen : 1;
        }
        // h_out of this slot is read by the copy-out pieces before the new chunk's D2H is
        // queued below, so both can run in one job
        pool.run(po + pi_n, [&](int i) {
            if (i < po) copy_out(sl, (uint64_t)i);
            else fill(i - po);
        });
        auto t2 = clk::now();
        t_job += std::chrono::duration<double, std::milli>(t2 - t1).count();
        sl.busy = false;
        HIP_TRY(hipMemcpyAsync(sl.d_in, sl.h_in, in_bytes, hipMemcpyHostToDevice, sl.st));
        if (mode == HM_RAGGED) {
            HIP_TRY(hipMemcpyAsync(sl.d_off, sl.h_off, k * 8, hipMemcpyHostToDevice, sl.st));
            HIP_TRY(hipMemcpyAsync(sl.d_len, sl.h_len, k * 4, hipMemcpyHostToDevice, sl.st));
            a.qoff = sl.d_off;
            a.qlen = sl.d_len;
        }
        if (mode == HM_WORDS || mode == HM_PACK) a.qwords = reinterpret_cast<const uint64_t*>(sl.d_in);
        else a.qbytes = sl.d_in;
        a.nq = k;
        a.out_pos = sl.d_out;
        a.out_probes = out_probes ? sl.d_pr : nullptr;
        a.bad = x->scratch;
        if (validate) {
            HIP_TRY(hipMemsetAsync(sl.d_bad, 0, 4, sl.st));
            a.bad = sl.d_bad;
            uint64_t vb = (k + 255) / 256;
            if (vb > 65536) vb = 65536;
            hipLaunchKernelGGL(k_validate_queries, dim3((unsigned)vb), dim3(256), 0, sl.st, a.qbytes, a.qoff, a.qlen,
                               a.m_fixed, k, a.bad);
        }
        if (out_hi) {
            launch_range(x, a, qw, flags, sl.st, sl.d_out + k);
            HIP_TRY(hipGetLastError());
        } else if ((err = launch_search(x, a, algo, qw, flags | SAS_DEVICE_PTRS, sl.st))) {
            break;
        }
        HIP_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, (out_hi ? 2 : 1) * k * 8, hipMemcpyDeviceToHost, sl.st));
        if (out_probes) HIP_TRY(hipMemcpyAsync(sl.h_pr, sl.d_pr, k * 4, hipMemcpyDeviceToHost, sl.st));
        if (validate) HIP_TRY(hipMemcpyAsync(sl.h_bad, sl.d_bad, 4, hipMemcpyDeviceToHost, sl.st));
        sl.busy = true;
        sl.s = s;
        sl.e = s + k;
        s += k;
        t_enq += std::chrono::duration<double, std::milli>(clk::now() - t2).count();
    }
    // drain: the last chunks' copy-outs, all slots in one job
    if (!err) {
        int tot = 0, base[SAS_STAGE_SLOTS];
        for (int c = 0; c < SAS_STAGE_SLOTS; c++) {
            StageSlot& sl = S.slot[c];
            if (sl.busy) {
                HIP_TRY(hipStreamSynchronize(sl.st));
                if (validate) dev_bad |= *sl.h_bad;
            }
            base[c] = tot;
            tot += out_pieces(sl);
        }
        pool.run(tot, [&](int i) {
            int c = SAS_STAGE_SLOTS - 1;
            while (c > 0 && i < base[c]) c--;
            copy_out(S.slot[c], (uint64_t)(i - base[c]));
        });
        for (auto& sl : S.slot) sl.busy = false;
    }
    if (trace)
        fprintf(stderr, "[sas stage] mode %d nq %llu chunks %d threads %d: wait %.2f ms, fill+copy-out %.2f ms, "
                        "enqueue %.2f ms, total %.2f ms\n",
                mode, (unsigned long long)nq, chunks, pool.size(), t_wait, t_job, t_enq,
                std::chrono::duration<double, std::milli>(clk::now() - t_all).count());
    if (err) return err;
    if (dev_bad || host_bad.load()) SAS_FAIL(EINVAL, "search: query bytes must be DNA codes 0..3");
    return 0;
}

// Host-pointer calls stage through plain hipMalloc + synchronous copies: the
// stream-ordered allocator + pageable async copies raced on the null stream.
// queries t[qoff[k] .. qoff[k] + qlen[k]) of the indexed text (SAS_QUERIES_ARE_SLICES)
__global__ void k_validate_slices(const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qlen, uint64_t nq,
                                  uint64_t n, uint32_t* __restrict__ bad) {
    uint32_t b = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x)
        b |= (qoff[i] > n || qlen[i] > n - qoff[i]) ? 1u : 0u;
    if (b) atomicOr(bad, 1u);
}

static int slices_impl(const sas_index* x, const uint64_t* qoff, const uint32_t* qlen, uint64_t nq, int algo,
                       uint64_t* out_pos, uint32_t* out_probes, void* stream, uint32_t flags) {
    if (algo != SAS_ALGO_TAGGED) SAS_FAIL(EINVAL, "SAS_QUERIES_ARE_SLICES: SAS_ALGO_TAGGED only");
    if (!(flags & SAS_DEVICE_PTRS)) SAS_FAIL(EINVAL, "SAS_QUERIES_ARE_SLICES: device pointers only (SAS_DEVICE_PTRS)");
    if (!qoff || !qlen) SAS_FAIL(EINVAL, "SAS_QUERIES_ARE_SLICES: null qoff/qlen");
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.qoff = qoff;
    a.qlen = qlen;
    a.out_pos = out_pos;
    a.out_probes = out_probes;
    a.bad = x->scratch;
    // every slice inside the text: checked first, always (an out-of-range slice would read
    // past the packed text); the call synchronises to read the flag back
    DeviceBuf bflag;
    HIP_TRY(hipMalloc(&bflag.p, 4));
    HIP_TRY(hipMemsetAsync(bflag.p, 0, 4, st));
    uint64_t vb = (nq + 255) / 256;
    if (vb > 65536) vb = 65536;
    hipLaunchKernelGGL(k_validate_slices, dim3((unsigned)vb), dim3(256), 0, st, qoff, qlen, nq, x->n,
                       static_cast<uint32_t*>(bflag.p));
    uint32_t hbad = 0;
    HIP_TRY(hipMemcpyAsync(&hbad, bflag.p, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (hbad) SAS_FAIL(EINVAL, "SAS_QUERIES_ARE_SLICES: a slice reaches past the text");
    return launch_search(x, a, algo, 4, flags, st);
}

static int search_impl(const sas_index* x, const uint8_t* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                       uint32_t m_fixed, uint64_t nq, int algo, uint64_t* out_pos, uint32_t* out_probes,
                       void* stream, uint32_t flags) {
    if (!x) SAS_FAIL(EINVAL, "search: null index");
    TRY_RC(check_algo(x, algo, flags, "search"));
    if (nq == 0) return 0;
    if (!out_pos) SAS_FAIL(EINVAL, "search: null out_pos");
    if (flags & SAS_QUERIES_ARE_SLICES) return slices_impl(x, qoff, qlen, nq, algo, out_pos, out_probes, stream, flags);
    if (!qbytes) SAS_FAIL(EINVAL, "search: null qbytes");
    bool ragged = qoff != nullptr;
    if (ragged && !qlen) SAS_FAIL(EINVAL, "search: qoff without qlen");
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    bool dev = flags & SAS_DEVICE_PTRS;

    if (!dev) {
        // host arrays: the pinned, chunked pipeline (host_pipeline) unless one query alone
        // exceeds a staging chunk
        uint64_t maxlen = m_fixed;
        if (ragged)
            for (uint64_t k = 0; k < nq; k++) maxlen = qlen[k] > maxlen ? qlen[k] : maxlen;
        if (maxlen <= SAS_STAGE_BYTES) {
            const bool pack = !ragged && algo == SAS_ALGO_PREFIX && m_fixed > 0 && m_fixed <= 32 &&
                              !(flags & SAS_PREFIX_RANGE);
            return host_pipeline(x, ragged ? HM_RAGGED : (pack ? HM_PACK : HM_FIXED), qbytes, qoff, qlen, nullptr,
                                 m_fixed, nq, algo, out_pos, out_probes, st, flags);
        }
    }
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.m_fixed = m_fixed;
    // invalid-code flag: a per-call word when it is read back, so that concurrent calls
    // on other streams (allowed: the index is immutable) never see each other's flags;
    // otherwise the index's write-only sink
    a.bad = x->scratch;
    bool check_bad = !dev || (flags & SAS_VALIDATE);
    DeviceBuf bflag;
    if (check_bad) {
        HIP_TRY(hipMalloc(&bflag.p, 4));
        HIP_TRY(hipMemsetAsync(bflag.p, 0, 4, st));
        a.bad = static_cast<uint32_t*>(bflag.p);
    }

    int qw = 4;
    DeviceBuf bqb, bqoff, bqlen, bout, bprobes;
    if (dev) {
        a.qbytes = qbytes;
        a.qoff = qoff;
        a.qlen = qlen;
        a.out_pos = out_pos;
        a.out_probes = out_probes;
        if (!ragged) qw = qw_for(m_fixed);
        a.m_max = ragged ? 0 : m_fixed;
    } else {
        uint64_t span;
        uint64_t maxlen = m_fixed;
        if (ragged) {
            span = 0;
            maxlen = 0;
            for (uint64_t k = 0; k < nq; k++) {
                uint64_t e = qoff[k] + qlen[k];
                if (e > span) span = e;
                if (qlen[k] > maxlen) maxlen = qlen[k];
            }
        } else {
            span = nq * (uint64_t)m_fixed;
        }
        qw = qw_for(maxlen);
        a.m_max = maxlen ? (uint32_t)maxlen : 1;
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMalloc(&bqb.p, span + 64));
        if (span) HIP_TRY(hipMemcpy(bqb.p, qbytes, span, hipMemcpyHostToDevice));
        a.qbytes = static_cast<const uint8_t*>(bqb.p);
        if (ragged) {
            HIP_TRY(hipMalloc(&bqoff.p, nq * 8));
            HIP_TRY(hipMalloc(&bqlen.p, nq * 4));
            HIP_TRY(hipMemcpy(bqoff.p, qoff, nq * 8, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(bqlen.p, qlen, nq * 4, hipMemcpyHostToDevice));
            a.qoff = static_cast<const uint64_t*>(bqoff.p);
            a.qlen = static_cast<const uint32_t*>(bqlen.p);
        }
        HIP_TRY(hipMalloc(&bout.p, nq * 8));
        a.out_pos = static_cast<uint64_t*>(bout.p);
        if (out_probes) {
            HIP_TRY(hipMalloc(&bprobes.p, nq * 4));
            a.out_probes = static_cast<uint32_t*>(bprobes.p);
        }
    }
    if (check_bad) {  // every query byte, not only those the search kernel packs
        uint64_t vb = (nq + 255) / 256;
        if (vb > 65536) vb = 65536;
        hipLaunchKernelGGL(k_validate_queries, dim3((unsigned)vb), dim3(256), 0, st, a.qbytes, a.qoff, a.qlen,
                           a.m_fixed, nq, a.bad);
    }
    int rc = launch_search(x, a, algo, qw, flags, st);
    if (rc) return rc;
    if (check_bad || !dev) {
        HIP_TRY(hipStreamSynchronize(st));
        uint32_t hbad = 0;
        if (check_bad) HIP_TRY(hipMemcpy(&hbad, a.bad, 4, hipMemcpyDeviceToHost));
        if (!dev) {
            HIP_TRY(hipMemcpy(out_pos, a.out_pos, nq * 8, hipMemcpyDeviceToHost));
            if (out_probes) HIP_TRY(hipMemcpy(out_probes, a.out_probes, nq * 4, hipMemcpyDeviceToHost));
        }
        if (hbad) SAS_FAIL(EINVAL, "search: query bytes must be DNA codes 0..3");
    }
    return 0;
}

extern "C" int sas_search_batch(const sas_index* index, const uint8_t* qbytes, const uint64_t* qoff,
                                const uint32_t* qlen, uint64_t nq, int algo, uint64_t* out_pos, uint32_t* out_probes,
                                void* stream, uint32_t flags) {
    if (nq && (!qoff || !qlen)) SAS_FAIL(EINVAL, "sas_search_batch: null qoff/qlen");
    return search_impl(index, qbytes, qoff, qlen, 0, nq, algo, out_pos, out_probes, stream, flags);
}

extern "C" int sas_search_fixed(const sas_index* index, const uint8_t* qbytes, uint32_t m, uint64_t nq, int algo,
                                uint64_t* out_pos, uint32_t* out_probes, void* stream, uint32_t flags) {
    return search_impl(index, qbytes, nullptr, nullptr, m, nq, algo, out_pos, out_probes, stream, flags);
}

__global__ void k_pack_queries(const uint8_t* __restrict__ qb, uint32_t m, uint64_t nq, uint64_t* __restrict__ out,
                               uint32_t* __restrict__ bad) {
    uint32_t b = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = pack_query_word(qb + i * (uint64_t)m, m, 0, &b);
    if (b) atomicOr(bad, 1u);
}

extern "C" int sas_pack_queries(const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t* out_words, void* stream,
                                uint32_t flags) {
    if (m > 32) SAS_FAIL(EINVAL, "sas_pack_queries: m must be <= 32");
    if (nq == 0) return 0;
    if (!qbytes || !out_words) SAS_FAIL(EINVAL, "sas_pack_queries: null argument");
    if (!(flags & SAS_DEVICE_PTRS)) {  // host arrays: the staging pipeline's packer on the host pool
        std::atomic<uint32_t> bad{0};
        constexpr uint64_t per = 16384;
        HostPool::get().run((int)((nq + per - 1) / per), [&](int i) {
            const uint64_t b = (uint64_t)i * per, e = std::min(nq, b + per);
            if (host_pack_words(qbytes + b * m, m, e - b, out_words + b) & 0xFC) bad.fetch_or(1);
        });
        if (bad.load()) SAS_FAIL(EINVAL, "sas_pack_queries: query bytes must be DNA codes 0..3");
        return 0;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    DeviceBuf bflag;
    HIP_TRY(hipMalloc(&bflag.p, 4));
    HIP_TRY(hipMemsetAsync(bflag.p, 0, 4, st));
    uint64_t blocks = (nq + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_pack_queries, dim3((unsigned)blocks), dim3(256), 0, st, qbytes, m, nq, out_words,
                       static_cast<uint32_t*>(bflag.p));
    HIP_TRY(hipGetLastError());
    uint32_t hbad = 0;
    HIP_TRY(hipMemcpyAsync(&hbad, bflag.p, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (hbad) SAS_FAIL(EINVAL, "sas_pack_queries: query bytes must be DNA codes 0..3");
    return 0;
}

extern "C" int sas_search_packed(const sas_index* x, const uint64_t* qwords, uint32_t m, uint64_t nq, int algo,
                                 uint64_t* out_pos, uint32_t* out_probes, void* stream, uint32_t flags) {
    if (!x) SAS_FAIL(EINVAL, "sas_search_packed: null index");
    if (algo != SAS_ALGO_PREFIX) SAS_FAIL(EINVAL, "sas_search_packed: SAS_ALGO_PREFIX only");
    if (!x->prefix) SAS_FAIL(EINVAL, "sas_search_packed: needs SAS_BUILD_PREFIX");
    if (m > 32) SAS_FAIL(EINVAL, "sas_search_packed: m must be <= 32");
    if (nq == 0) return 0;
    if (!qwords || !out_pos) SAS_FAIL(EINVAL, "sas_search_packed: null argument");
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!(flags & SAS_DEVICE_PTRS))  // host words: the pinned staging pipeline
        return host_pipeline(x, HM_WORDS, nullptr, nullptr, nullptr, qwords, m, nq, algo, out_pos, out_probes, st,
                             flags);
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.m_fixed = m;
    a.bad = x->scratch;  // packed words hold no invalid codes
    a.qwords = qwords;
    a.out_pos = out_pos;
    a.out_probes = out_probes;
    return launch_search(x, a, algo, 1, flags, st);
}

extern "C" int sas_search_buckets(const sas_index* x, const void* queries, uint32_t m, uint32_t nbuckets,
                                  uint64_t cap, const uint64_t* counts, int algo, uint64_t* out_pos, void* stream,
                                  uint32_t flags) {
    if (!x) SAS_FAIL(EINVAL, "sas_search_buckets: null index");
    TRY_RC(check_algo(x, algo, flags & ~SAS_PREFIX_RANGE, "sas_search_buckets"));
    if (!(flags & SAS_DEVICE_PTRS)) SAS_FAIL(EINVAL, "sas_search_buckets: device pointers only (SAS_DEVICE_PTRS)");
    if (flags & SAS_PREFIX_RANGE) SAS_FAIL(EINVAL, "sas_search_buckets: SAS_PREFIX_RANGE is not supported");
    const bool packed = (flags & SAS_ROUTE_PACKED) != 0;
    if (m == 0 || (packed && (m > 32 || algo != SAS_ALGO_PREFIX)))
        SAS_FAIL(EINVAL, "sas_search_buckets: m >= 1; packed words need SAS_ALGO_PREFIX and m <= 32");
    // the kernels that skip unfilled slots: one lane (or one lane group) per query
    const bool ok = algo == SAS_ALGO_PLAIN || algo == SAS_ALGO_LCP || algo == SAS_ALGO_LLCP ||
                    algo == SAS_ALGO_PREFIX || (algo == SAS_ALGO_QUAD && m <= 32);
    if (!ok || x->sa_w == 8) SAS_FAIL(ENOTSUP, "sas_search_buckets: PLAIN, LCP, LLCP, PREFIX, or QUAD with m <= 32");
    const uint64_t nq = (uint64_t)nbuckets * cap;
    if (nq == 0) return 0;
    if (cap >= (1ull << 32) || nq >= (1ull << 32)) SAS_FAIL(EINVAL, "sas_search_buckets: buckets x cap >= 2^32");
    if (!queries || !counts || !out_pos) SAS_FAIL(EINVAL, "sas_search_buckets: null argument");
    HIP_TRY(hipSetDevice(x->device));
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.m_fixed = m;
    a.m_max = m;
    a.bad = x->scratch;  // device pointers: codes unchecked, as sas_search_fixed without SAS_VALIDATE
    if (packed) a.qwords = static_cast<const uint64_t*>(queries);
    else a.qbytes = static_cast<const uint8_t*>(queries);
    a.out_pos = out_pos;
    a.bcounts = counts;
    a.bcap = (uint32_t)cap;
    return launch_search(x, a, algo, packed ? 1 : qw_for(m), flags, static_cast<hipStream_t>(stream));
}

extern "C" int sas_time_fixed(const sas_index* x, const uint8_t* d_qbytes, uint32_t m, uint64_t nq, int algo,
                              uint64_t* d_out_pos, int reps, void* stream, uint32_t flags, double* kernel_ns,
                              double* call_ns) {
    if (!x || !d_qbytes || !d_out_pos || reps < 1) SAS_FAIL(EINVAL, "sas_time_fixed: bad argument");
    TRY_RC(check_algo(x, algo, flags, "sas_time_fixed"));
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.m_fixed = m;
    a.m_max = m;
    a.qbytes = d_qbytes;
    a.out_pos = d_out_pos;
    a.bad = x->scratch;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipStreamSynchronize(st));
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventRecord(e0, st));
    for (int r = 0; r < reps; r++) {
        int rc = launch_search(x, a, algo, qw_for(m), flags | SAS_DEVICE_PTRS, st);
        if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(e1, st));
    HIP_TRY(hipEventSynchronize(e1));
    auto t1 = std::chrono::steady_clock::now();
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    if (kernel_ns) *kernel_ns = ms * 1e6 / reps;
    if (call_ns) *call_ns = std::chrono::duration<double, std::nano>(t1 - t0).count() / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

// ------------------------------------------------------------------ sharded-mode routing
// Routing compares a query with the splitter suffixes by their first 32 chars (staged in
// LDS once per block: sk[w] = text_chars32 at splitter w) and reads the text only on a tie
// of those keys (distinct 32-char keys order as the strings do, zero padding included,
// as sector_ge relies on): the shard of q = the number of splitter suffixes < q.
__device__ __forceinline__ void stage_split_keys(const uint64_t* __restrict__ tw, const uint64_t* __restrict__ sp,
                                                 uint32_t nsplit, uint64_t* sk) {
    for (uint32_t w = threadIdx.x; w < nsplit; w += blockDim.x) sk[w] = text_chars32(tw, sp[w]);
}

template <int QW>
__device__ __forceinline__ uint32_t route_of(const uint64_t* __restrict__ tw, uint64_t n,
                                             const uint64_t* __restrict__ sp, const uint64_t* sk, uint32_t nsplit,
                                             const QueryRegs<QW>& q) {
    uint32_t lo = 0, hi = nsplit, lcp;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t kk = sk[mid];
        const bool less = kk != q.w[0] ? kk < q.w[0] : suffix_less_from<QW>(tw, n, sp[mid], q, 0, &lcp);
        if (less) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_route(const uint64_t* __restrict__ tw, uint64_t n,
                                               const uint64_t* __restrict__ sp, uint32_t nsplit,
                                               const uint8_t* __restrict__ qbytes, uint32_t m,
                                               const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qlen,
                                               uint64_t nq, uint32_t* __restrict__ out, uint32_t* bad) {
    __shared__ uint64_t sk[SAS_MAX_SPLIT];
    stage_split_keys(tw, sp, nsplit, sk);
    __syncthreads();
    uint32_t b = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x) {
        QueryRegs<4> q;
        if (qoff) q.load(qbytes + qoff[i], qlen[i], &b);  // ragged (sas_route_batch)
        else q.load(qbytes + i * (uint64_t)m, m, &b);
        out[i] = route_of<4>(tw, n, sp, sk, nsplit, q);
    }
    if (b) atomicOr(bad, 1u);
}

// Fixed-length (qoff == nullptr) or ragged routing, host or device pointers.
static int route_impl(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit, const uint8_t* qbytes,
                      uint32_t m, const uint64_t* qoff, const uint32_t* qlen, uint64_t nq, uint32_t* out_shard,
                      void* stream, uint32_t flags) {
    if (!x || (nsplit && !splitter_pos) || (nq && (!qbytes || !out_shard))) SAS_FAIL(EINVAL, "sas_route: null argument");
    if (qoff && !qlen) SAS_FAIL(EINVAL, "sas_route_batch: qoff without qlen");
    if (nsplit > SAS_MAX_SPLIT) SAS_FAIL(EINVAL, "sas_route: too many splitters");
    if (nq == 0) return 0;
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    bool dev = flags & SAS_DEVICE_PTRS;
    DeviceBuf bsp, bq, bout, boff, blen;
    const uint64_t* dsp = splitter_pos;
    const uint8_t* dq = qbytes;
    const uint64_t* doff = qoff;
    const uint32_t* dlen = qlen;
    uint32_t* dout = out_shard;
    if (!dev) {
        uint64_t span = nq * (uint64_t)m;
        if (qoff) {
            span = 0;
            for (uint64_t k = 0; k < nq; k++) span = qoff[k] + qlen[k] > span ? qoff[k] + qlen[k] : span;
        }
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMalloc(&bsp.p, nsplit * 8 + 8));
        if (nsplit) HIP_TRY(hipMemcpy(bsp.p, splitter_pos, nsplit * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&bq.p, span + 64));
        if (span) HIP_TRY(hipMemcpy(bq.p, qbytes, span, hipMemcpyHostToDevice));
        if (qoff) {
            HIP_TRY(hipMalloc(&boff.p, nq * 8));
            HIP_TRY(hipMalloc(&blen.p, nq * 4));
            HIP_TRY(hipMemcpy(boff.p, qoff, nq * 8, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(blen.p, qlen, nq * 4, hipMemcpyHostToDevice));
            doff = static_cast<const uint64_t*>(boff.p);
            dlen = static_cast<const uint32_t*>(blen.p);
        }
        HIP_TRY(hipMalloc(&bout.p, nq * 4));
        dsp = static_cast<const uint64_t*>(bsp.p);
        dq = static_cast<const uint8_t*>(bq.p);
        dout = static_cast<uint32_t*>(bout.p);
    }
    uint64_t blocks = (nq + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_route, dim3((unsigned)blocks), dim3(256), 0, st, x->text_w, x->n, dsp, nsplit, dq, m, doff,
                       dlen, nq, dout, x->scratch);
    HIP_TRY(hipGetLastError());
    if (!dev) {
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(out_shard, dout, nq * 4, hipMemcpyDeviceToHost));
    }
    return 0;
}

extern "C" int sas_route(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit, const uint8_t* qbytes,
                         uint32_t m, uint64_t nq, uint32_t* out_shard, void* stream, uint32_t flags) {
    return route_impl(x, splitter_pos, nsplit, qbytes, m, nullptr, nullptr, nq, out_shard, stream, flags);
}

extern "C" int sas_route_batch(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit,
                               const uint8_t* qbytes, const uint64_t* qoff, const uint32_t* qlen, uint64_t nq,
                               uint32_t* out_shard, void* stream, uint32_t flags) {
    if (nq && (!qoff || !qlen)) SAS_FAIL(EINVAL, "sas_route_batch: null qoff/qlen");
    return route_impl(x, splitter_pos, nsplit, qbytes, 0, qoff, qlen, nq, out_shard, stream, flags);
}

// ------------------------------------------------------------------ route + pack (sharded step)
// One sharded-mode step needs the queries grouped by destination shard.  This is
// a counting sort by destination, fused with the routing and the byte copy:
//   k_route_count    dest[i] (as in sas_route) + per-block histogram of dest (LDS
//                    atomics) -> cnt[w * nblk + b] (+ the packed word, SAS_ROUTE_PACKED)
//   exclusive scan   -> base[w * nblk + b] = first send slot of (bucket w, block b)
//   k_pack_scatter   slot = base + LDS-atomic rank; copy the query's m bytes to
//                    send[slot * m]; slot_of[i] = slot (positions come back in
//                    send order and are gathered with it)
// Order inside a bucket is not stable (it need not be: every slot is recorded).
#define PACK_BLOCK 1024
#define PACK_ITEMS 8
#define PACK_CHUNK (PACK_BLOCK * PACK_ITEMS)
#ifndef SAS_ROUTE_ITEMS
#define SAS_ROUTE_ITEMS 8
#endif

// route + per-block histogram in one pass over the queries: dest[i] = the shard of query i
// (as k_route; no splitters: shard 0 without reading the query), and with PACKED its 2-bit
// word for the scatter (SAS_ROUTE_PACKED), so the query bytes are read once
template <bool PACKED>
__global__ __launch_bounds__(PACK_BLOCK) void k_route_count(const uint64_t* __restrict__ tw, uint64_t n,
                                                            const uint64_t* __restrict__ sp, uint32_t nsplit,
                                                            const uint8_t* __restrict__ qbytes, uint32_t m, uint64_t nq,
                                                            uint64_t nblk, uint64_t* __restrict__ cnt,
                                                            uint32_t* __restrict__ dest, uint64_t* __restrict__ words) {
    __shared__ uint32_t h[SAS_MAX_SPLIT + 1];
    __shared__ uint64_t sk[SAS_MAX_SPLIT];
    const uint32_t W = nsplit + 1;
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) h[w] = 0;
    stage_split_keys(tw, sp, nsplit, sk);
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * PACK_CHUNK;
    for (int it = 0; it < PACK_ITEMS; it++) {
        const uint64_t i = base + (uint64_t)it * PACK_BLOCK + threadIdx.x;
        if (i >= nq) continue;
        uint32_t lo = 0;
        if (PACKED || nsplit) {
            uint32_t b = 0;
            QueryRegs<PACKED ? 1 : 4> q;
            q.load(qbytes + i * (uint64_t)m, m, &b);
            if (PACKED) words[i] = q.w[0];
            lo = route_of<PACKED ? 1 : 4>(tw, n, sp, sk, nsplit, q);
        }
        dest[i] = lo;
        atomicAdd(&h[lo], 1u);
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) cnt[(uint64_t)w * nblk + blockIdx.x] = h[w];
}

// cap == 0: buckets packed back to back (slot = the exclusive scan); cap > 0: bucket w
// owns slots [w * cap, (w + 1) * cap) and a query past its bucket's cap is not copied (its
// slot is clamped to the last one; the caller sees the overflow in out_counts > cap)
__global__ __launch_bounds__(PACK_BLOCK) void k_pack_scatter(const uint32_t* __restrict__ dest, uint64_t nq,
                                                             uint32_t W, uint64_t nblk,
                                                             const uint64_t* __restrict__ base_slot,
                                                             const uint8_t* __restrict__ qbytes, uint32_t m,
                                                             uint8_t* __restrict__ send,
                                                             uint64_t* __restrict__ slot_of, uint64_t cap,
                                                             bool packed, const uint64_t* __restrict__ words) {
    __shared__ uint32_t h[SAS_MAX_SPLIT + 1];
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) h[w] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * PACK_CHUNK;
    const bool vec = (m & 15) == 0 && ((((uintptr_t)qbytes) | ((uintptr_t)send)) & 15) == 0;
    for (int it = 0; it < PACK_ITEMS; it++) {
        const uint64_t i = base + (uint64_t)it * PACK_BLOCK + threadIdx.x;
        if (i >= nq) continue;
        const uint32_t w = dest[i];
        uint64_t slot = base_slot[(uint64_t)w * nblk + blockIdx.x] + atomicAdd(&h[w], 1u);
        if (cap) {
            const uint64_t r = slot - base_slot[(uint64_t)w * nblk];  // rank inside bucket w
            if (r >= cap) {
                slot_of[i] = (uint64_t)W * cap - 1;
                continue;
            }
            slot = (uint64_t)w * cap + r;
        }
        slot_of[i] = slot;
        const uint8_t* src = qbytes + i * (uint64_t)m;
        if (packed) {  // SAS_ROUTE_PACKED: the query's 2-bit word (m <= 32), 8 B per slot
            uint32_t bad = 0;
            reinterpret_cast<uint64_t*>(send)[slot] = words ? words[i] : pack_query_word(src, m, 0, &bad);
            continue;
        }
        uint8_t* dst = send + slot * (uint64_t)m;
        if (vec) {
            for (uint32_t k = 0; k < m; k += 16)
                *reinterpret_cast<uint4*>(dst + k) = *reinterpret_cast<const uint4*>(src + k);
        } else {
            for (uint32_t k = 0; k < m; k++) dst[k] = src[k];
        }
    }
}

// cap > 0 in one pass over the queries (no dest array, no scan, no second read):
//   1. each thread routes (and with SAS_ROUTE_PACKED packs) its PACK_ITEMS queries; per
//      item, each wave takes one LDS atomic per destination present in it (leader lane,
//      popcount of the ballot), so a lane's rank inside its (block, bucket) share is
//      that share's running offset + the lanes below it with the same destination;
//   2. one global atomic per (block, bucket) claims the share's first rank in bucket w
//      (counts[w], zeroed by the caller of the launch, ends as the bucket's total);
//   3. query i goes to slot w * cap + claimed + rank, or past the cap is clamped as above.
template <bool PACKED, int ITEMS>
__global__ __launch_bounds__(PACK_BLOCK) void k_route_scatter_cap(
    const uint64_t* __restrict__ tw, uint64_t n, const uint64_t* __restrict__ sp, uint32_t nsplit,
    const uint8_t* __restrict__ qbytes, uint32_t m, uint64_t nq, uint64_t cap, unsigned long long* __restrict__ counts,
    uint8_t* __restrict__ send, uint64_t* __restrict__ slot_of) {
    __shared__ uint32_t h[SAS_MAX_SPLIT + 1];
    __shared__ uint64_t claimed[SAS_MAX_SPLIT + 1];
    __shared__ uint64_t sk[SAS_MAX_SPLIT];
    const uint32_t W = nsplit + 1;
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) h[w] = 0;
    stage_split_keys(tw, sp, nsplit, sk);
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * (PACK_BLOCK * ITEMS);
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t dst[ITEMS], rk[ITEMS];
    uint64_t wd[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint64_t i = base + (uint64_t)it * PACK_BLOCK + threadIdx.x;
        const bool valid = i < nq;
        uint32_t lo = 0;
        wd[it] = 0;
        if (valid && (PACKED || nsplit)) {
            uint32_t b = 0;
            QueryRegs<PACKED ? 1 : 4> q;
            q.load(qbytes + i * (uint64_t)m, m, &b);
            wd[it] = q.w[0];
            lo = route_of<PACKED ? 1 : 4>(tw, n, sp, sk, nsplit, q);
        }
        dst[it] = lo;
        rk[it] = 0;
        uint64_t todo = __ballot(valid);
        while (todo) {  // wave-uniform: one pass per distinct destination in the wave
            const int leader = __builtin_ctzll(todo);
            const uint32_t d = (uint32_t)__shfl((int)lo, leader, 64);
            const uint64_t same = __ballot(valid && lo == d);
            uint32_t r0 = 0;
            if (lane == leader) r0 = atomicAdd(&h[d], (uint32_t)__popcll(same));
            r0 = (uint32_t)__shfl((int)r0, leader, 64);
            if (valid && lo == d) rk[it] = r0 + (uint32_t)__popcll(same & below);
            todo &= ~same;
        }
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < W; w += blockDim.x)
        claimed[w] = h[w] ? (uint64_t)atomicAdd(&counts[w], (unsigned long long)h[w]) : 0ull;
    __syncthreads();
    const bool vec = (m & 15) == 0 && ((((uintptr_t)qbytes) | ((uintptr_t)send)) & 15) == 0;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint64_t i = base + (uint64_t)it * PACK_BLOCK + threadIdx.x;
        if (i >= nq) continue;
        const uint32_t w = dst[it];
        const uint64_t r = claimed[w] + rk[it];
        if (r >= cap) {
            slot_of[i] = (uint64_t)W * cap - 1;
            continue;
        }
        const uint64_t slot = (uint64_t)w * cap + r;
        slot_of[i] = slot;
        if (PACKED) {
            reinterpret_cast<uint64_t*>(send)[slot] = wd[it];
            continue;
        }
        const uint8_t* src = qbytes + i * (uint64_t)m;  // read again: the block read it in pass 1
        uint8_t* dp = send + slot * (uint64_t)m;
        if (vec) {
            for (uint32_t k = 0; k < m; k += 16)
                *reinterpret_cast<uint4*>(dp + k) = *reinterpret_cast<const uint4*>(src + k);
        } else {
            for (uint32_t k = 0; k < m; k++) dp[k] = src[k];
        }
    }
}

// The sharded step's receive side: out[i] = back[slot_of[i]] (the positions returned in
// send-slot order, put back in query order); block 0 also raises *overflow (plain store
// of 1, never cleared here) when a bucket's count passed its capacity.
__global__ void k_shard_gather(const uint64_t* __restrict__ back, const uint64_t* __restrict__ slot_of, uint64_t nq,
                               const uint64_t* __restrict__ counts, uint32_t W, uint64_t cap,
                               uint64_t* __restrict__ out, uint32_t* __restrict__ overflow) {
    if (blockIdx.x == 0 && overflow) {
        bool over = false;
        for (uint32_t w = threadIdx.x; w < W; w += blockDim.x) over |= counts[w] > cap;
        if (over) overflow[0] = 1u;
    }
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = back[slot_of[i]];
}

__global__ void k_pack_totals(const uint64_t* __restrict__ base_slot, uint32_t W, uint64_t nblk, uint64_t nq,
                              uint64_t* __restrict__ out_counts) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < W; w += gridDim.x * blockDim.x) {
        const uint64_t lo = base_slot[(uint64_t)w * nblk];
        const uint64_t hi = (w + 1 < W) ? base_slot[(uint64_t)(w + 1) * nblk] : nq;
        out_counts[w] = hi - lo;
    }
}

// The scratch of an exact (variable-size) sharded step comes from a stream-ordered pool
// owned by the index (created on first use, destroyed by sas_free).  Its release threshold
// of "never" keeps freed blocks for the next step; the device's default pool, which other
// libraries in the process share, is left alone.
static int route_pool(const sas_index* x, hipMemPool_t* out) {
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (!x->route_pool) {
        hipMemPoolProps pp{};
        pp.allocType = hipMemAllocationTypePinned;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = x->device;
        hipMemPool_t pool = nullptr;
        HIP_TRY(hipMemPoolCreate(&pool, &pp));
        uint64_t thr = UINT64_MAX;
        HIP_TRY(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
        x->route_pool = pool;
    }
    *out = x->route_pool;
    return 0;
}

static int route_pack_impl(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit,
                           const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t cap, uint64_t* out_counts,
                           uint8_t* out_send, uint64_t* out_slot, void* stream, uint32_t flags) {
    if (!x || (nsplit && !splitter_pos) || !out_counts || (nq && (!qbytes || !out_send || !out_slot)))
        SAS_FAIL(EINVAL, "sas_route_pack: null argument");
    if (!(flags & SAS_DEVICE_PTRS)) SAS_FAIL(EINVAL, "sas_route_pack: device pointers only (SAS_DEVICE_PTRS)");
    if (nsplit > SAS_MAX_SPLIT) SAS_FAIL(EINVAL, "sas_route_pack: too many splitters");
    if ((flags & SAS_ROUTE_PACKED) && m > 32) SAS_FAIL(EINVAL, "sas_route_pack: SAS_ROUTE_PACKED needs m <= 32");
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t W = nsplit + 1;
    if (nq == 0) {
        HIP_TRY(hipMemsetAsync(out_counts, 0, W * 8, st));
        return 0;
    }
    const uint64_t nblk = (nq + PACK_CHUNK - 1) / PACK_CHUNK;
    const bool packed = (flags & SAS_ROUTE_PACKED) != 0;
    if (cap) {  // fixed-capacity buckets: one pass, no scratch
        HIP_TRY(hipMemsetAsync(out_counts, 0, W * 8, st));
        auto* c = reinterpret_cast<unsigned long long*>(out_counts);
        // queries per thread (A/B knob SAS_ROUTE_ITEMS = 2 / 4 / 8)
        static const int items = [] {
            const char* e = getenv("SAS_ROUTE_ITEMS");
            const int v = e ? atoi(e) : SAS_ROUTE_ITEMS;
            return (v == 2 || v == 4 || v == 8) ? v : SAS_ROUTE_ITEMS;
        }();
        const dim3 grid((unsigned)((nq + (uint64_t)PACK_BLOCK * items - 1) / ((uint64_t)PACK_BLOCK * items)));
#define SAS_RSC(P, I)                                                                                              \
    hipLaunchKernelGGL((k_route_scatter_cap<P, I>), grid, dim3(PACK_BLOCK), 0, st, x->text_w, x->n, splitter_pos, \
                       nsplit, qbytes, m, nq, cap, c, out_send, out_slot)
        if (packed) {
            if (items == 2) SAS_RSC(true, 2);
            else if (items == 4) SAS_RSC(true, 4);
            else SAS_RSC(true, 8);
        } else {
            if (items == 2) SAS_RSC(false, 2);
            else if (items == 4) SAS_RSC(false, 4);
            else SAS_RSC(false, 8);
        }
#undef SAS_RSC
        HIP_TRY(hipGetLastError());
        return 0;
    }
    hipMemPool_t pool;
    TRY_RC(route_pool(x, &pool));
    // with splitters the routing reads each query anyway and packs it on the way (words);
    // without (one part) the routing reads nothing and the scatter packs from the bytes
    const bool pack_in_route = packed && nsplit > 0;
    void* dest = nullptr;
    void* cnt = nullptr;
    void* tmp = nullptr;
    void* words = nullptr;
    size_t tbytes = 0;
    HIP_TRY(rocprim::exclusive_scan(nullptr, tbytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0,
                                    (size_t)(nblk * W), rocprim::plus<uint64_t>(), st));
    HIP_TRY(hipMallocFromPoolAsync(&dest, nq * 4, pool, st));
    HIP_TRY(hipMallocFromPoolAsync(&cnt, nblk * W * 8, pool, st));
    HIP_TRY(hipMallocFromPoolAsync(&tmp, tbytes ? tbytes : 8, pool, st));
    if (pack_in_route) HIP_TRY(hipMallocFromPoolAsync(&words, nq * 8, pool, st));
    if (pack_in_route)
        hipLaunchKernelGGL(k_route_count<true>, dim3((unsigned)nblk), dim3(PACK_BLOCK), 0, st, x->text_w, x->n,
                           splitter_pos, nsplit, qbytes, m, nq, nblk, static_cast<uint64_t*>(cnt),
                           static_cast<uint32_t*>(dest), static_cast<uint64_t*>(words));
    else
        hipLaunchKernelGGL(k_route_count<false>, dim3((unsigned)nblk), dim3(PACK_BLOCK), 0, st, x->text_w, x->n,
                           splitter_pos, nsplit, qbytes, m, nq, nblk, static_cast<uint64_t*>(cnt),
                           static_cast<uint32_t*>(dest), (uint64_t*)nullptr);
    HIP_TRY(rocprim::exclusive_scan(tmp, tbytes, static_cast<uint64_t*>(cnt), static_cast<uint64_t*>(cnt),
                                    (uint64_t)0, (size_t)(nblk * W), rocprim::plus<uint64_t>(), st));
    hipLaunchKernelGGL(k_pack_scatter, dim3((unsigned)nblk), dim3(PACK_BLOCK), 0, st, static_cast<uint32_t*>(dest),
                       nq, W, nblk, static_cast<uint64_t*>(cnt), qbytes, m, out_send, out_slot, cap, packed,
                       static_cast<const uint64_t*>(words));
    hipLaunchKernelGGL(k_pack_totals, dim3(1), dim3(256), 0, st, static_cast<uint64_t*>(cnt), W, nblk, nq, out_counts);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(dest, st));
    HIP_TRY(hipFreeAsync(cnt, st));
    HIP_TRY(hipFreeAsync(tmp, st));
    if (words) HIP_TRY(hipFreeAsync(words, st));
    return 0;
}

extern "C" int sas_route_pack(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit,
                              const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t* out_counts,
                              uint8_t* out_send, uint64_t* out_slot, void* stream, uint32_t flags) {
    return route_pack_impl(x, splitter_pos, nsplit, qbytes, m, nq, 0, out_counts, out_send, out_slot, stream, flags);
}

extern "C" int sas_route_pack_cap(const sas_index* x, const uint64_t* splitter_pos, uint32_t nsplit,
                                  const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t cap, uint64_t* out_counts,
                                  uint8_t* out_send, uint64_t* out_slot, void* stream, uint32_t flags) {
    if (cap == 0) SAS_FAIL(EINVAL, "sas_route_pack_cap: cap must be > 0");
    return route_pack_impl(x, splitter_pos, nsplit, qbytes, m, nq, cap, out_counts, out_send, out_slot, stream, flags);
}

extern "C" int sas_shard_gather(const sas_index* x, const uint64_t* back, const uint64_t* slot, uint64_t nq,
                                const uint64_t* counts, uint32_t nparts, uint64_t cap, uint64_t* out,
                                uint32_t* overflow, void* stream, uint32_t flags) {
    if (!x || (nq && (!back || !slot || !out)) || (overflow && (!counts || nparts == 0)))
        SAS_FAIL(EINVAL, "sas_shard_gather: null argument");
    if (!(flags & SAS_DEVICE_PTRS)) SAS_FAIL(EINVAL, "sas_shard_gather: device pointers only (SAS_DEVICE_PTRS)");
    if (nq == 0 && !overflow) return 0;
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t blocks = (nq + 255) / 256;
    const uint64_t capb = (uint64_t)x->num_cus * 8;
    if (blocks > capb) blocks = capb;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_shard_gather, dim3((unsigned)blocks), dim3(256), 0, st, back, slot, nq, counts, nparts, cap,
                       out, overflow);
    HIP_TRY(hipGetLastError());
    return 0;
}

// ------------------------------------------------------------------ occurrence ranges
template <bool KO, int W>
static void launch_quad_range(int qw, dim3 grid, dim3 block, hipStream_t st, const SearchArgs& a, uint64_t* dhi) {
    switch (qw) {
        case 1: hipLaunchKernelGGL((k_sa_quad_range<1, KO, W>), grid, block, 0, st, a, dhi); break;
        case 2: hipLaunchKernelGGL((k_sa_quad_range<2, KO, W>), grid, block, 0, st, a, dhi); break;
        case 4: hipLaunchKernelGGL((k_sa_quad_range<4, KO, W>), grid, block, 0, st, a, dhi); break;
        default: hipLaunchKernelGGL((k_sa_quad_range<8, KO, W>), grid, block, 0, st, a, dhi); break;
    }
}

// Occurrence-range kernel for the index's structures (a.nq queries; lo to a.out_pos, hi to dhi)
static void launch_range(const sas_index* x, const SearchArgs& a, int qw, uint32_t flags, hipStream_t st,
                         uint64_t* dhi) {
    const bool quad = x->quad_leaves != nullptr;
    // the prefix table, when built, replaces the two tree descents (one lane per query;
    // G lanes per query on a G-slot inline table)
    const bool ptab = quad && x->prefix && !(flags & SAS_NO_PREFIX_TABLE);
    const bool pair = ptab && !x->quad_compact && (x->prefix_w == 32 || x->prefix_w == 64) &&
                      !(flags & SAS_RANGE_NO_INLINE);
    const uint64_t per = (quad && !ptab) ? QUAD_G : (pair ? x->prefix_w / 16 : 1);
    uint64_t blocks = (a.nq * per + SEARCH_BLOCK - 1) / SEARCH_BLOCK;
    uint64_t cap = (uint64_t)x->num_cus * BLOCKS_PER_CU;
    if (blocks > cap) blocks = cap;
    dim3 grid((unsigned)blocks), block(SEARCH_BLOCK);
    if (x->tag_lines) {
        switch (qw) {
            case 1: hipLaunchKernelGGL(k_sa_tagged_lines_range<1>, grid, block, 0, st, a, dhi); break;
            case 2: hipLaunchKernelGGL(k_sa_tagged_lines_range<2>, grid, block, 0, st, a, dhi); break;
            case 4: hipLaunchKernelGGL(k_sa_tagged_lines_range<4>, grid, block, 0, st, a, dhi); break;
            default: hipLaunchKernelGGL(k_sa_tagged_lines_range<8>, grid, block, 0, st, a, dhi); break;
        }
    } else if (x->tag_table) {
        switch (qw) {
            case 1: hipLaunchKernelGGL(k_sa_tagged_range<1>, grid, block, 0, st, a, dhi); break;
            case 2: hipLaunchKernelGGL(k_sa_tagged_range<2>, grid, block, 0, st, a, dhi); break;
            case 4: hipLaunchKernelGGL(k_sa_tagged_range<4>, grid, block, 0, st, a, dhi); break;
            default: hipLaunchKernelGGL(k_sa_tagged_range<8>, grid, block, 0, st, a, dhi); break;
        }
    } else if (pair) {
        if (x->prefix_w == 32) launch_prefix2_range<2>(qw, grid, block, st, a, dhi);
        else launch_prefix2_range<4>(qw, grid, block, st, a, dhi);
    } else if (ptab) {
        if (!x->quad_compact) launch_prefix_range<false, 4>(qw, grid, block, st, a, dhi);
        else if (x->sa_w == 5) launch_prefix_range<true, 5>(qw, grid, block, st, a, dhi);
        else launch_prefix_range<true, 4>(qw, grid, block, st, a, dhi);
    } else if (quad && !x->quad_compact) {
        launch_quad_range<false, 4>(qw, grid, block, st, a, dhi);
    } else if (quad) {
        if (x->sa_w == 5) launch_quad_range<true, 5>(qw, grid, block, st, a, dhi);
        else launch_quad_range<true, 4>(qw, grid, block, st, a, dhi);
    } else {
        switch (qw) {
            case 1: hipLaunchKernelGGL(k_sa_sector_range<1>, grid, block, 0, st, a, dhi); break;
            case 2: hipLaunchKernelGGL(k_sa_sector_range<2>, grid, block, 0, st, a, dhi); break;
            case 4: hipLaunchKernelGGL(k_sa_sector_range<4>, grid, block, 0, st, a, dhi); break;
            default: hipLaunchKernelGGL(k_sa_sector_range<8>, grid, block, 0, st, a, dhi); break;
        }
    }
}

// ragged (qoff, qlen) or fixed-length (qoff == nullptr: m_fixed chars per query)
static int range_impl(const sas_index* x, const uint8_t* qbytes, uint32_t m_fixed, const uint64_t* qoff,
                      const uint32_t* qlen, uint64_t nq, uint64_t* out_lo, uint64_t* out_hi, void* stream,
                      uint32_t flags) {
    if (!x) SAS_FAIL(EINVAL, "sas_search_range: null index");
    if (!x->sec_leaves && !x->quad_leaves && !x->tag_table && !x->tag_lines)
        SAS_FAIL(EINVAL, "sas_search_range: needs SAS_BUILD_QUAD, SAS_BUILD_SECTOR or SAS_BUILD_TAGGED");
    const bool ragged = qoff != nullptr || qlen != nullptr;
    if (nq == 0) return 0;
    if (!qbytes || !out_lo || !out_hi || (ragged && (!qoff || !qlen)))
        SAS_FAIL(EINVAL, "sas_search_range: null argument");
    HIP_TRY(hipSetDevice(x->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    bool dev = flags & SAS_DEVICE_PTRS;
    if (!dev) {
        // host arrays: the pinned, chunked pipeline unless one query alone exceeds a chunk
        uint64_t maxlen = m_fixed;
        if (ragged)
            for (uint64_t k = 0; k < nq; k++) maxlen = qlen[k] > maxlen ? qlen[k] : maxlen;
        if (maxlen <= SAS_STAGE_BYTES)
            return host_pipeline(x, ragged ? HM_RAGGED : HM_FIXED, qbytes, qoff, qlen, nullptr, m_fixed, nq, -1,
                                 out_lo, nullptr, st, flags, out_hi);
    }
    SearchArgs a{};
    fill_args(x, a);
    a.nq = nq;
    a.m_fixed = ragged ? 0 : m_fixed;
    a.bad = x->scratch;  // per-call flag when read back (see search_impl)
    bool check_bad = !dev || (flags & SAS_VALIDATE);
    DeviceBuf bflag;
    if (check_bad) {
        HIP_TRY(hipMalloc(&bflag.p, 4));
        HIP_TRY(hipMemsetAsync(bflag.p, 0, 4, st));
        a.bad = static_cast<uint32_t*>(bflag.p);
    }
    DeviceBuf bqb, bqoff, bqlen, blo, bhi;
    uint64_t* dhi = out_hi;
    int qw = ragged ? 4 : qw_for(m_fixed);
    if (dev) {
        a.qbytes = qbytes;
        a.qoff = qoff;
        a.qlen = qlen;
        a.out_pos = out_lo;
    } else {
        uint64_t span = nq * (uint64_t)m_fixed, maxlen = m_fixed;
        if (ragged) {
            span = maxlen = 0;
            for (uint64_t k = 0; k < nq; k++) {
                uint64_t e = qoff[k] + qlen[k];
                if (e > span) span = e;
                if (qlen[k] > maxlen) maxlen = qlen[k];
            }
        }
        qw = qw_for(maxlen);
        a.m_max = maxlen ? (uint32_t)maxlen : 1;
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMalloc(&bqb.p, span + 64));
        if (span) HIP_TRY(hipMemcpy(bqb.p, qbytes, span, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&blo.p, nq * 8));
        HIP_TRY(hipMalloc(&bhi.p, nq * 8));
        a.qbytes = static_cast<const uint8_t*>(bqb.p);
        if (ragged) {
            HIP_TRY(hipMalloc(&bqoff.p, nq * 8));
            HIP_TRY(hipMalloc(&bqlen.p, nq * 4));
            HIP_TRY(hipMemcpy(bqoff.p, qoff, nq * 8, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(bqlen.p, qlen, nq * 4, hipMemcpyHostToDevice));
            a.qoff = static_cast<const uint64_t*>(bqoff.p);
            a.qlen = static_cast<const uint32_t*>(bqlen.p);
        }
        a.out_pos = static_cast<uint64_t*>(blo.p);
        dhi = static_cast<uint64_t*>(bhi.p);
    }
    if (check_bad) {
        uint64_t vb = (nq + 255) / 256;
        if (vb > 65536) vb = 65536;
        hipLaunchKernelGGL(k_validate_queries, dim3((unsigned)vb), dim3(256), 0, st, a.qbytes, a.qoff, a.qlen,
                           a.m_fixed, nq, a.bad);
    }
    launch_range(x, a, qw, flags, st, dhi);
    HIP_TRY(hipGetLastError());
    if (check_bad || !dev) {
        HIP_TRY(hipStreamSynchronize(st));
        uint32_t hbad = 0;
        if (check_bad) HIP_TRY(hipMemcpy(&hbad, a.bad, 4, hipMemcpyDeviceToHost));
        if (!dev) {
            HIP_TRY(hipMemcpy(out_lo, a.out_pos, nq * 8, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(out_hi, dhi, nq * 8, hipMemcpyDeviceToHost));
        }
        if (hbad) SAS_FAIL(EINVAL, "sas_search_range: query bytes must be DNA codes 0..3");
    }
    return 0;
}

extern "C" int sas_search_range(const sas_index* x, const uint8_t* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                                uint64_t nq, uint64_t* out_lo, uint64_t* out_hi, void* stream, uint32_t flags) {
    if (nq && (!qoff || !qlen)) SAS_FAIL(EINVAL, "sas_search_range: null qoff/qlen");
    return range_impl(x, qbytes, 0, qoff, qlen, nq, out_lo, out_hi, stream, flags);
}

extern "C" int sas_search_range_fixed(const sas_index* x, const uint8_t* qbytes, uint32_t m, uint64_t nq,
                                      uint64_t* out_lo, uint64_t* out_hi, void* stream, uint32_t flags) {
    return range_impl(x, qbytes, m, nullptr, nullptr, nq, out_lo, out_hi, stream, flags);
}
