/*
 * sa_oracle.c -- CPU restatement of the reference algorithms on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load it
 * (as oracle/liboracle.so through ctypes).  The product library
 * (suffix-array-searching_amd/libsas_amd.so) never links or calls it.
 *
 * Reference: RagnarGrootKoerkamp/suffix-array-searching @ 2025-07-11
 *   sas/ = suffix-array-searching/src,  sst/ = static-search-tree/src
 * The reference is nightly Rust with a git-only SA builder (libsais-rs); it
 * cannot be compiled in this image (no cargo/rustc, no network), so every
 * function below restates the Rust line by line, citing file:line.
 *
 * Parity pinning: the S-tree / Eytzinger / SortedVec restatements are pinned
 * by the reference's own known-answer tests (tests/golden/reference_kats.json,
 * from sst/eytzinger.rs:183-231, sst/s_tree.rs:841-896).  The SA search is
 * pinned by a definition oracle (Python sorted()/bisect on small texts,
 * tests/golden/make_golden.py).  The ChaCha core is pinned by the RFC 7539
 * ChaCha20 block vector; the rand 0.8.5 sampling on top of it is restated
 * from the published crate and is "parity unpinned" (no Rust here).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <emmintrin.h>

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* rand_chacha 0.3.1 ChaCha8Rng + rand_core 0.6 seed_from_u64 + rand 0.8.5   */
/* (sas/main.rs:38 `ChaCha8Rng::seed_from_u64(31415)`)                        */
/* ------------------------------------------------------------------------ */

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define QR(a, b, c, d)                 \
    a += b; d ^= a; d = rotl32(d, 16); \
    c += d; b ^= c; b = rotl32(b, 12); \
    a += b; d ^= a; d = rotl32(d, 8);  \
    c += d; b ^= c; b = rotl32(b, 7);

/* Raw ChaCha block: words 12..15 given explicitly (djb layout: 64-bit block
 * counter in 12/13, 64-bit stream in 14/15; RFC 7539 layout: 32-bit counter
 * in 12, nonce in 13..15). */
EXPORT void orc_chacha_block(const uint32_t key[8], uint32_t w12, uint32_t w13,
                             uint32_t w14, uint32_t w15, int rounds,
                             uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                      w12, w13, w14, w15};
    uint32_t x[16];
    memcpy(x, s, sizeof x);
    for (int i = 0; i < rounds; i += 2) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
        QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
        QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

/* rand_core 0.6 SeedableRng::seed_from_u64: PCG32 expands the u64 into the
 * 32-byte seed, 4 bytes per step; ChaCha8Rng::from_seed takes it as the key. */
EXPORT void orc_seed_from_u64(uint64_t state, uint32_t key[8]) {
    const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
    for (int i = 0; i < 8; i++) {
        state = state * MUL + INC;
        uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        key[i] = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    }
}

/* Keystream word `w` of ChaCha8Rng (stream 0): BlockRng hands out the words
 * of consecutive 16-word blocks in order, so word w = block w/16, lane w%16. */
typedef struct {
    uint32_t key[8];
    uint64_t blk;      /* block currently cached */
    uint32_t buf[16];
    uint64_t pos;      /* next word index */
} orc_rng;

static void rng_init(orc_rng* r, uint64_t seed, uint64_t word_pos) {
    orc_seed_from_u64(seed, r->key);
    r->blk = UINT64_MAX;
    r->pos = word_pos;
}
static inline uint32_t rng_word(orc_rng* r, uint64_t w) {
    uint64_t b = w >> 4;
    if (b != r->blk) {
        orc_chacha_block(r->key, (uint32_t)b, (uint32_t)(b >> 32), 0, 0, 8, r->buf);
        r->blk = b;
    }
    return r->buf[w & 15];
}
static inline uint32_t rng_next_u32(orc_rng* r) { return rng_word(r, r->pos++); }
/* BlockRng::next_u64: two consecutive words, low word first (also across a
 * buffer refill, rand_core 0.6 block.rs). */
static inline uint64_t rng_next_u64(orc_rng* r) {
    uint64_t lo = rng_word(r, r->pos), hi = rng_word(r, r->pos + 1);
    r->pos += 2;
    return lo | (hi << 32);
}
/* rand 0.8.5 UniformInt<usize>::sample_single(low..high): widening multiply
 * with the "conservative" zone (range << lz) - 1. */
static uint64_t rng_range_u64(orc_rng* r, uint64_t low, uint64_t high) {
    uint64_t range = high - low;
    uint64_t zone = (range << __builtin_clzll(range)) - 1;
    for (;;) {
        uint64_t v = rng_next_u64(r);
        unsigned __int128 p = (unsigned __int128)v * range;
        uint64_t hi = (uint64_t)(p >> 64), lo = (uint64_t)p;
        if (lo <= zone) return low + hi;
    }
}

/* sas/util.rs:9-15 random_string: gen_range(0..4) as u8.  UniformInt<u8>
 * samples a u32 with zone = u32::MAX (no rejection for range 4), result =
 * (v * 4) >> 32 = v >> 30.  Consumes exactly n words. */
EXPORT void orc_random_string(uint64_t seed, uint64_t n, uint8_t* out) {
    orc_rng r;
    rng_init(&r, seed, 0);
    for (uint64_t i = 0; i < n; i++) out[i] = (uint8_t)(rng_next_u32(&r) >> 30);
}

/* sas/util.rs:18-26 random_queries: i = gen_range(0..n - margin),
 * len = gen_range(len_lo..len_hi).  The reference uses margin = 200,
 * len in [30,100).  len_hi == len_lo + 1 means a fixed length and draws no
 * length word (the BASELINE configs use fixed m).  Starts at keystream word
 * `word_pos` (= n after random_string) and returns the next free word. */
EXPORT uint64_t orc_random_queries(uint64_t seed, uint64_t word_pos, uint64_t n,
                                   uint64_t nq, uint64_t margin, uint32_t len_lo,
                                   uint32_t len_hi, uint64_t* off, uint32_t* len) {
    orc_rng r;
    rng_init(&r, seed, word_pos);
    for (uint64_t k = 0; k < nq; k++) {
        off[k] = rng_range_u64(&r, 0, n - margin);
        len[k] = (len_hi == len_lo + 1) ? len_lo : (uint32_t)rng_range_u64(&r, len_lo, len_hi);
    }
    return r.pos;
}

/* ------------------------------------------------------------------------ */
/* Suffix order and suffix-array construction                               */
/* ------------------------------------------------------------------------ */

/* Rust slice Ord (`t[a..] < q`): lexicographic, a proper prefix sorts first. */
static inline int slice_cmp(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
    uint64_t k = la < lb ? la : lb;
    int c = memcmp(a, b, k);
    if (c) return c < 0 ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

typedef struct { int64_t a, b; uint32_t i; } dbl_item;
static int dbl_cmp(const void* x, const void* y) {
    const dbl_item *p = x, *q = y;
    if (p->a != q->a) return p->a < q->a ? -1 : 1;
    if (p->b != q->b) return p->b < q->b ? -1 : 1;
    return 0;
}

/* Suffix array by prefix doubling (Manber-Myers ranks, qsort per round).
 * The reference builds it with libsais (sas/sa_search.rs:30-35) or
 * libdivsufsort (sas/util.rs:121-127); the SA of a text is unique, so any
 * correct builder is bit-identical.  Returns 0 on success. */
EXPORT int orc_build_sa(const uint8_t* t, uint64_t n, uint32_t* sa) {
    if (n == 0) return 0;
    int64_t* rank = malloc(n * sizeof(int64_t));
    int64_t* tmp = malloc(n * sizeof(int64_t));
    dbl_item* it = malloc(n * sizeof(dbl_item));
    if (!rank || !tmp || !it) { free(rank); free(tmp); free(it); return 12; }
    for (uint64_t i = 0; i < n; i++) rank[i] = t[i];
    for (uint64_t h = 1;; h *= 2) {
        for (uint64_t i = 0; i < n; i++) {
            it[i].a = rank[i];
            it[i].b = i + h < n ? rank[i + h] : -1;
            it[i].i = (uint32_t)i;
        }
        qsort(it, n, sizeof(dbl_item), dbl_cmp);
        uint64_t r = 0, distinct = 1;
        tmp[it[0].i] = 0;
        for (uint64_t k = 1; k < n; k++) {
            if (dbl_cmp(&it[k], &it[k - 1])) { r = k; distinct++; }
            tmp[it[k].i] = (int64_t)r;
        }
        memcpy(rank, tmp, n * sizeof(int64_t));
        if (distinct == n || h >= n) break;
    }
    for (uint64_t k = 0; k < n; k++) sa[rank[k]] = (uint32_t)k;
    free(rank); free(tmp); free(it);
    return 0;
}

/* The reference's only SA check (sas/sa_search.rs:36-38): adjacent suffixes
 * strictly increasing; plus the permutation property. 0 = valid. */
EXPORT int orc_check_sa(const uint8_t* t, uint64_t n, const uint32_t* sa) {
    uint8_t* seen = calloc(n ? n : 1, 1);
    if (!seen) return 12;
    int bad = 0;
    for (uint64_t i = 0; i < n && !bad; i++) {
        if (sa[i] >= n || seen[sa[i]]) bad = 1;
        else seen[sa[i]] = 1;
    }
    for (uint64_t i = 1; i < n && !bad; i++)
        if (slice_cmp(t + sa[i - 1], n - sa[i - 1], t + sa[i], n - sa[i]) >= 0) bad = 2;
    free(seen);
    return bad;
}

/* Kasai et al. LCP: lcp[0] = 0, lcp[r] = lcp(suffix SA[r-1], suffix SA[r]).
 * (Absent from the reference: sas/sa_search.rs:344-345 TODO.) */
EXPORT void orc_kasai_lcp(const uint8_t* t, uint64_t n, const uint32_t* sa, uint32_t* lcp) {
    uint32_t* isa = malloc((n ? n : 1) * sizeof(uint32_t));
    for (uint64_t r = 0; r < n; r++) isa[sa[r]] = (uint32_t)r;
    uint64_t h = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t r = isa[i];
        if (r == 0) { lcp[0] = 0; h = 0; continue; }
        uint64_t j = sa[r - 1];
        while (i + h < n && j + h < n && t[i + h] == t[j + h]) h++;
        lcp[r] = (uint32_t)h;
        if (h) h--;
    }
    free(isa);
}

/* ------------------------------------------------------------------------ */
/* Suffix-array search (sas/sa_search.rs)                                   */
/* ------------------------------------------------------------------------ */

/* `sa.suffix(m) < q` with Rust slice order (sas/sa_search.rs:76-81, :105). */
static inline int suffix_lt(const uint8_t* t, uint64_t n, uint32_t p, const uint8_t* q, uint64_t m) {
    return slice_cmp(t + p, n - p, q, m) < 0;
}

/* sas/sa_search.rs:346-374 `cmp`: 16-byte blocks, eq-mask + trailing_ones.
 * Reads up to 16 bytes past both the suffix and q: the caller provides the
 * reference's zero padding after t (sas/main.rs:56-58) and 16 readable bytes
 * after each query.  Differs from slice order only when the suffix runs into
 * the padding. */
static inline int ref_cmp(const uint8_t* tp, const uint8_t* q, uint64_t len) {
    for (;;) {
        __m128i a = _mm_loadu_si128((const __m128i*)tp);
        __m128i b = _mm_loadu_si128((const __m128i*)q);
        uint32_t eq = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(a, b));
        uint32_t cnt = (uint32_t)__builtin_ctz(~eq);   /* trailing_ones */
        if (cnt < 16 && cnt < len) return tp[cnt] < q[cnt];
        if (len < 16) return 0;
        tp += 16; q += 16; len -= 16;
    }
}

/* sas/sa_search.rs:98-112 `binary_search` -- the CANONICAL semantics.
 * prefix_range() is [0, n) because p = 0 is hard-coded (:31, :83-95).
 * Returns sa[l]; l == n (query above every suffix) reads sa[n] out of bounds
 * in the reference, defined here as the sentinel n. */
EXPORT uint64_t orc_binary_search(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                  const uint8_t* q, uint64_t m, uint64_t* cnt) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        (*cnt)++;
        if (suffix_lt(t, n, sa[mid], q, m)) l = mid + 1;
        else r = mid;
    }
    return l < n ? sa[l] : n;
}

/* Lower-bound RANK (not position); used by tests for range/count checks. */
EXPORT uint64_t orc_lower_bound_rank(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                     const uint8_t* q, uint64_t m) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        if (suffix_lt(t, n, sa[mid], q, m)) l = mid + 1;
        else r = mid;
    }
    return l;
}

/* sas/sa_search.rs:121-136 `binary_search_cmp` (A8): A6 with `cmp`. */
EXPORT uint64_t orc_binary_search_cmp(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                      const uint8_t* q, uint64_t m, uint64_t* cnt) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        (*cnt)++;
        if (ref_cmp(t + sa[mid], q, m)) l = mid + 1;
        else r = mid;
    }
    return l < n ? sa[l] : n;
}

/* sas/sa_search.rs:138-155 `branchy_search` (A10): returns the RANK m on
 * full-slice equality -- inconsistent return type, excluded from parity. */
EXPORT uint64_t orc_branchy_search(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                   const uint8_t* q, uint64_t m, uint64_t* cnt) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        (*cnt)++;
        int c = slice_cmp(t + sa[mid], n - sa[mid], q, m);
        if (c < 0) l = mid + 1;
        else if (c > 0) r = mid;
        else return mid;
    }
    return l < n ? sa[l] : n;
}

/* sas/sa_search.rs:241-252 `branchfree_search` (A11): predecessor semantics.
 * Probes index l+half which can equal n (out of bounds in the reference);
 * restated with suffix(n) := the empty suffix.  Excluded from parity. */
EXPORT uint64_t orc_branchfree_search(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                      const uint8_t* q, uint64_t m, uint64_t* cnt) {
    uint64_t l = 0, len = n;
    while (len > 0) {
        uint64_t half = (len + 1) / 2;
        (*cnt)++;
        uint64_t k = l + half;
        int lt = k < n ? suffix_lt(t, n, sa[k], q, m) : (m > 0);
        l = lt ? k : l;
        len -= half;
    }
    return l < n ? sa[l] : n;
}

/* sas/util.rs:76-117 `string_value<K>`: the first K chars as a base-4 number.
 * The K = 16 path (the one main.rs:97 runs) reads 16 bytes with two unaligned
 * u64 loads + pext of each byte's low 2 bits, i.e. it reads past a slice shorter
 * than K: with the zero padding after the text (sas/main.rs:56-58) and after
 * each query (the callers here pad queries with zeros) that is "zero padded". */
static inline uint64_t string_value(const uint8_t* s, int K) {
    uint64_t v = 0;
    for (int i = 0; i < K; i++) v = v * 4 + (s[i] & 3u);
    return v;
}

/* sas/sa_search.rs:376-421 `interpolation_search<K>` (A12).  prefix_range() is
 * [0, n) with no cnt increment (p = 0, :86-95).  Mid = the interpolated rank
 * l + (r-l)(q_val - l_val + 1) / (r_val - l_val + 2) clamped to the
 * [1/16, 15/16] interior (:406-409), exact slice compare (:411).  usize
 * arithmetic wraps in the release profile (Cargo.toml: no overflow-checks), so
 * q_val < l_val - 1 (q below the first suffix) wraps here too: the clamp keeps
 * l <= mid < r, and the result is binary_search's.  The reference asserts
 * r_val * r does not overflow (:389-392): n < 2^32 at K = 16. */
EXPORT uint64_t orc_interpolation_search(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                         const uint8_t* q, uint64_t m, int K, uint64_t* cnt) {
    uint64_t l = 0, r = n;
    uint64_t l_val = string_value(t + sa[l], K);
    uint64_t r_val = r < n ? string_value(t + sa[r], K) : (1ull << (2 * K));
    const uint64_t q_val = string_value(q, K);
    while (l < r) {
        (*cnt)++;
        uint64_t mid = l + ((r - l) * (q_val - l_val + 1)) / (r_val - l_val + 2);
        const uint64_t low = l + (r - l) / 16, high = l + 15 * (r - l) / 16;
        mid = mid < low ? low : (mid > high ? high : mid);
        const uint32_t p = sa[mid];
        const uint64_t m_val = string_value(t + p, K);
        if (suffix_lt(t, n, p, q, m)) {
            l = mid + 1;
            l_val = m_val;
        } else {
            r = mid;
            r_val = m_val;
        }
    }
    return l < n ? sa[l] : n;
}

/* sas/sa_search.rs:157-239 `binary_search_batch<B>` / `_batch_c<B>` (A9):
 * B queries in lockstep for ilog2(n)+1 iterations (:171-172), three passes
 * per iteration (mids + prefetch sa, load sa + prefetch text, compare).
 * cnt += B per iteration (:178).  A lane with l == r == n would probe sa[n];
 * restated as a no-op for that lane. */
EXPORT void orc_binary_search_batch(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                    const uint8_t* const* qs, const uint64_t* ms, int B,
                                    int use_cmp, uint64_t* out, uint64_t* cnt) {
    uint64_t l[64], r[64], mid[64];
    uint32_t idx[64];
    if (B > 64) B = 64;
    for (int i = 0; i < B; i++) { l[i] = 0; r[i] = n; }
    int iters = n ? 64 - __builtin_clzll(n) : 0;   /* ilog2(max_len) + 1 */
    for (int it = 0; it < iters; it++) {
        for (int i = 0; i < B; i++) {
            mid[i] = (l[i] + r[i]) / 2;
            (*cnt)++;
            if (mid[i] < n) __builtin_prefetch(&sa[mid[i]]);
        }
        for (int i = 0; i < B; i++) {
            idx[i] = mid[i] < n ? sa[mid[i]] : (uint32_t)n;
            __builtin_prefetch(t + idx[i]);
            __builtin_prefetch(t + idx[i] + 15);
        }
        for (int i = 0; i < B; i++) {
            if (mid[i] >= n) continue;
            int lt = use_cmp ? ref_cmp(t + idx[i], qs[i], ms[i])
                             : suffix_lt(t, n, idx[i], qs[i], ms[i]);
            if (lt) l[i] = mid[i] + 1;
            else r[i] = mid[i];
        }
    }
    for (int i = 0; i < B; i++) out[i] = l[i] < n ? sa[l[i]] : n;
}

/* Multi-threaded driver, same shape as the reference benches: contiguous
 * query chunks per thread (sst/bin/bench.rs:558-573), one wall clock.
 * algo: 0 binary_search (A6), 1 binary_search_cmp (A8),
 *       2 binary_search_batch_c<16> (A9), 3 binary_search_batch<16>,
 *       4 interpolation_search<16> (A12).
 * Queries are qbytes[qoff[k] .. qoff[k]+qlen[k]]. */
typedef struct {
    const uint8_t* t; uint64_t n; const uint32_t* sa;
    const uint8_t* qb; const uint64_t* qoff; const uint32_t* qlen;
    uint64_t lo, hi; int algo; uint64_t* out; uint64_t cnt;
} search_job;

static void* search_worker(void* arg) {
    search_job* j = arg;
    uint64_t cnt = 0;
    if (j->algo == 2 || j->algo == 3) {
        const int B = 16;
        uint64_t k = j->lo;
        for (; k + B <= j->hi; k += B) {
            const uint8_t* qs[16]; uint64_t ms[16];
            for (int i = 0; i < B; i++) { qs[i] = j->qb + j->qoff[k + i]; ms[i] = j->qlen[k + i]; }
            orc_binary_search_batch(j->t, j->n, j->sa, qs, ms, B, j->algo == 2, j->out + k, &cnt);
        }
        for (; k < j->hi; k++)  /* remainder: the reference drops it (:441); we don't */
            j->out[k] = orc_binary_search_cmp(j->t, j->n, j->sa, j->qb + j->qoff[k], j->qlen[k], &cnt);
    } else if (j->algo == 4) {
        for (uint64_t k = j->lo; k < j->hi; k++)
            j->out[k] = orc_interpolation_search(j->t, j->n, j->sa, j->qb + j->qoff[k], j->qlen[k], 16, &cnt);
    } else {
        for (uint64_t k = j->lo; k < j->hi; k++) {
            const uint8_t* q = j->qb + j->qoff[k];
            j->out[k] = j->algo == 1 ? orc_binary_search_cmp(j->t, j->n, j->sa, q, j->qlen[k], &cnt)
                                     : orc_binary_search(j->t, j->n, j->sa, q, j->qlen[k], &cnt);
        }
    }
    j->cnt = cnt;
    return 0;
}

EXPORT uint64_t orc_search_many(const uint8_t* t, uint64_t n, const uint32_t* sa,
                                const uint8_t* qb, const uint64_t* qoff, const uint32_t* qlen,
                                uint64_t nq, int algo, uint64_t* out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    search_job jobs[256];
    uint64_t chunk = (nq + threads - 1) / threads;
    for (int i = 0; i < threads; i++) {
        uint64_t lo = (uint64_t)i * chunk, hi = lo + chunk;
        if (lo > nq) lo = nq;
        if (hi > nq) hi = nq;
        jobs[i] = (search_job){t, n, sa, qb, qoff, qlen, lo, hi, algo, out, 0};
        pthread_create(&th[i], 0, search_worker, &jobs[i]);
    }
    uint64_t cnt = 0;
    for (int i = 0; i < threads; i++) { pthread_join(th[i], 0); cnt += jobs[i].cnt; }
    return cnt;
}

/* ------------------------------------------------------------------------ */
/* Static search tree over u32 (sst/)                                       */
/* ------------------------------------------------------------------------ */

#define SST_MAX 0x7fffffffu /* sst/node.rs:5  MAX = i32::MAX */

/* sst/node.rs:93-109 find_popcnt: count of keys < q with SIGNED compares
 * (two 8-lane i32 halves, packs + movemask, popcount/2). */
EXPORT uint32_t orc_node_find(const uint32_t* node, uint32_t N, uint32_t q) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < N; i++) c += (int32_t)q > (int32_t)node[i];
    return c;
}

/* sst/s_tree.rs:22-45 TreeBase. */
static uint64_t tb_blocks(uint64_t n, uint64_t B) { return (n + B - 1) / B; }
static uint64_t tb_prev_keys(uint64_t n, uint64_t B) { return (tb_blocks(n, B) + B) / (B + 1) * B; }
static uint64_t tb_height(uint64_t n, uint64_t B) { return n <= B ? 1 : tb_height(tb_prev_keys(n, B), B) + 1; }
static uint64_t tb_layer_size(uint64_t n, uint64_t h, uint64_t height, uint64_t B) {
    for (uint64_t i = h; i + 1 < height; i++) n = tb_prev_keys(n, B);
    return n;
}

/* Layer sizes in nodes (sst/s_tree.rs:90-99); returns height, fills
 * layer_sizes[0..height) (<= 16 entries), *n_blocks = sum. */
EXPORT uint32_t orc_stree_dims(uint64_t n, uint32_t B, int full, uint64_t* layer_sizes, uint64_t* n_blocks) {
    uint64_t height = tb_height(n, B), tot = 0;
    for (uint64_t h = 0; h < height; h++) {
        uint64_t s;
        if (full) { s = 1; for (uint64_t k = 0; k < h; k++) s *= (B + 1); }
        else s = (tb_layer_size(n, h, height, B) + B - 1) / B;
        layer_sizes[h] = s;
        tot += s;
    }
    *n_blocks = tot;
    return (uint32_t)height;
}

/* sst/s_tree.rs:72-176 STree::new_params(vals, left_max, reverse, full).
 * `tree` must hold n_blocks*N u32 and be ZERO-initialised (the reference
 * allocates with vec_on_hugepages: fresh zeroed pages, :125-129).
 * offsets[h] (in nodes) are written for h < height. */
EXPORT int orc_stree_build(const uint32_t* vals, uint64_t n, uint32_t B, uint32_t N,
                           int left_max, int reverse, int full, uint32_t* tree, uint64_t* offsets) {
    if (n == 0) return 22;
    if (full && reverse) return 22;
    for (uint64_t i = 0; i < n; i++) if (vals[i] > SST_MAX) return 22;
    uint64_t ls[64], nb;
    uint32_t height = orc_stree_dims(n, B, full, ls, &nb);
    uint64_t sum = 0;
    for (uint32_t h = 0; h < height; h++) {
        if (!reverse) { offsets[h] = sum; sum += ls[h]; }
        else { sum += ls[h]; offsets[h] = nb - sum; }
    }
    uint64_t ol = offsets[height - 1];
#define NODE(b) (tree + (uint64_t)(b) * N)
    for (uint64_t i = 0; i < n; i++) {
        NODE(ol + i / B)[i % B] = vals[i];
        if (B < N && i % B == 0 && i > 0) NODE(ol + i / B - 1)[B] = vals[i];
    }
    if (n / B < ls[height - 1])
        for (uint64_t j = n % B; j < N; j++) NODE(ol + n / B)[j] = SST_MAX;
    for (int h = (int)height - 2; h >= 0; h--) {
        uint64_t oh = offsets[h];
        for (uint64_t b = 0; b < ls[h]; b++)
            for (uint32_t j = 0; j < N; j++) NODE(oh + b)[j] = SST_MAX;
        for (uint64_t i = 0; i < (uint64_t)B * ls[h]; i++) {
            uint64_t k = i / B, j = i % B;
            k = k * (B + 1) + j + 1;
            for (uint32_t l = (uint32_t)h; l + 2 < height; l++) k *= (B + 1);
            NODE(oh + i / B)[i % B] = k * B < n
                ? (!left_max ? NODE(ol + k)[0] : NODE(ol + k - 1)[B - 1])
                : SST_MAX;
        }
    }
#undef NODE
    return 0;
}

/* sst/s_tree.rs:196-206 STree::search: value of the first key >= q.
 * Also returns the leaf rank k*B + idx through *rank (may be NULL). */
EXPORT uint32_t orc_stree_search(const uint32_t* tree, const uint64_t* offsets, uint32_t height,
                                 uint32_t B, uint32_t N, uint32_t q, uint64_t* rank) {
    uint64_t k = 0;
    for (uint32_t h = 0; h + 1 < height; h++) {
        uint32_t jump = orc_node_find(tree + (offsets[h] + k) * N, N, q);
        k = k * (B + 1) + jump;
    }
    uint64_t o = offsets[height - 1];
    uint32_t idx = orc_node_find(tree + (o + k) * N, N, q);
    if (rank) *rank = k * B + idx;
    return tree[(o + k + idx / N) * N + idx % N];
}

/* sst/eytzinger.rs:37-63 Eytzinger::new: vals[0] = u32::MAX, in-order fill. */
static void eyt_rec(uint32_t* e, uint64_t len, const uint32_t* a, uint64_t* i, uint64_t k) {
    if (k <= len) {   /* k <= a.len() */
        eyt_rec(e, len, a, i, 2 * k);
        e[k] = a[(*i)++];
        eyt_rec(e, len, a, i, 2 * k + 1);
    }
}
EXPORT void orc_eytzinger_build(const uint32_t* vals, uint64_t n, uint32_t* e /* n+1 */) {
    uint64_t i = 0;
    e[0] = UINT32_MAX;
    eyt_rec(e, n, vals, &i, 1);
}

/* sst/eytzinger.rs:5-7 search_result_to_index. */
static inline uint64_t eyt_to_index(uint64_t idx) { return idx >> (__builtin_ctzll(~idx) + 1); }

/* sst/eytzinger.rs:81-88 Eytzinger::search. */
EXPORT uint32_t orc_eytzinger_search(const uint32_t* e, uint64_t n, uint32_t q) {
    uint64_t len = n + 1, idx = 1;
    while (idx < len) idx = 2 * idx + (q > e[idx]);
    return e[eyt_to_index(idx)];
}

/* sst/eytzinger.rs:90-102 + :19-31 search_branchless (num_iters = ilog2(len),
 * then the guarded final step). */
EXPORT uint32_t orc_eytzinger_search_branchless(const uint32_t* e, uint64_t n, uint32_t q) {
    uint64_t len = n + 1, idx = 1;
    uint32_t iters = 63 - __builtin_clzll(len);
    for (uint32_t i = 0; i < iters; i++) idx = 2 * idx + (q > e[idx]);
    int inb = idx < len;
    idx = 2 * idx + ((q > e[inb ? idx : 0]) || !inb);
    return e[eyt_to_index(idx)];
}

/* sst/binary_search.rs:37-49 SortedVec::binary_search -- the oracle all
 * reference tests compare to.  vals[n] (OOB when no key >= q) is defined as
 * u32::MAX here; *rank = lower bound. */
EXPORT uint32_t orc_sorted_search(const uint32_t* vals, uint64_t n, uint32_t q, uint64_t* rank) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t m = (l + r) / 2;
        if (vals[m] < q) l = m + 1;
        else r = m;
    }
    if (rank) *rank = l;
    return l < n ? vals[l] : UINT32_MAX;
}

/* sst/s_tree.rs:303-326 batch_final::<P> (the reference's bench variant, run with
 * P = 128, sst/bin/bench.rs:96): P queries descend layer by layer; after each
 * node a query's next node is prefetched, so P independent loads are in flight.
 * Node compare = find_popcnt with SSE2 signed compares (sst/node.rs:93-109). */
static inline uint32_t node_find16_sse(const uint32_t* node, uint32_t q) {
    const __m128i qv = _mm_set1_epi32((int32_t)q);
    uint32_t c = 0;
    for (int j = 0; j < 4; j++) {
        __m128i v = _mm_loadu_si128((const __m128i*)(node + 4 * j));
        c += (uint32_t)__builtin_popcount(_mm_movemask_ps(_mm_castsi128_ps(_mm_cmpgt_epi32(qv, v))));
    }
    return c;
}

EXPORT void orc_stree_batch(const uint32_t* tree, const uint64_t* offsets, uint32_t height, uint32_t B,
                            const uint32_t* qs, uint64_t nq, uint32_t* out) {
    enum { P = 128 };
    uint64_t k[P];
    for (uint64_t base = 0; base < nq; base += P) {
        const uint64_t cnt = nq - base < P ? nq - base : P;
        for (uint64_t i = 0; i < cnt; i++) k[i] = 0;
        for (uint32_t h = 0; h + 1 < height; h++) {
            const uint32_t* o = tree + offsets[h] * 16;
            const uint32_t* o2 = tree + offsets[h + 1] * 16;
            for (uint64_t i = 0; i < cnt; i++) {
                k[i] = k[i] * (B + 1) + node_find16_sse(o + k[i] * 16, qs[base + i]);
                __builtin_prefetch(o2 + k[i] * 16);
            }
        }
        const uint32_t* o = tree + offsets[height - 1] * 16;
        for (uint64_t i = 0; i < cnt; i++) {
            const uint32_t idx = node_find16_sse(o + k[i] * 16, qs[base + i]);
            out[base + i] = o[k[i] * 16 + idx];
        }
    }
}

struct StreeJob {
    const uint32_t* tree;
    const uint64_t* offsets;
    uint32_t height, B;
    const uint32_t* qs;
    uint64_t nq;
    uint32_t* out;
};
static void* stree_worker(void* arg) {
    struct StreeJob* j = (struct StreeJob*)arg;
    orc_stree_batch(j->tree, j->offsets, j->height, j->B, j->qs, j->nq, j->out);
    return NULL;
}
/* Contiguous query chunks per thread (sst/bin/bench.rs:558-573). */
EXPORT void orc_stree_batch_mt(const uint32_t* tree, const uint64_t* offsets, uint32_t height, uint32_t B,
                               const uint32_t* qs, uint64_t nq, uint32_t* out, uint32_t threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    struct StreeJob jobs[256];
    const uint64_t chunk = (nq + threads - 1) / threads;
    uint32_t started = 0;
    for (uint32_t t = 0; t < threads; t++) {
        const uint64_t lo = t * chunk, hi = lo + chunk < nq ? lo + chunk : nq;
        if (lo >= hi) break;
        jobs[t] = (struct StreeJob){tree, offsets, height, B, qs + lo, hi - lo, out + lo};
        if (pthread_create(&th[t], NULL, stree_worker, &jobs[t]) != 0) {
            stree_worker(&jobs[t]);
            th[t] = 0;
        }
        started = t + 1;
    }
    for (uint32_t t = 0; t < started; t++)
        if (th[t]) pthread_join(th[t], NULL);
}

/* Batch helpers so Python tests do not loop per query. */
EXPORT void orc_stree_query(const uint32_t* tree, const uint64_t* offsets, uint32_t height, uint32_t B,
                            uint32_t N, const uint32_t* qs, uint64_t nq, uint32_t* out, uint64_t* rank) {
    for (uint64_t i = 0; i < nq; i++) out[i] = orc_stree_search(tree, offsets, height, B, N, qs[i], rank ? rank + i : 0);
}
EXPORT void orc_eytzinger_query(const uint32_t* e, uint64_t n, const uint32_t* qs, uint64_t nq,
                                int branchless, uint32_t* out) {
    for (uint64_t i = 0; i < nq; i++)
        out[i] = branchless ? orc_eytzinger_search_branchless(e, n, qs[i]) : orc_eytzinger_search(e, n, qs[i]);
}
EXPORT void orc_sorted_query(const uint32_t* vals, uint64_t n, const uint32_t* qs, uint64_t nq,
                             uint32_t* out, uint64_t* rank) {
    for (uint64_t i = 0; i < nq; i++) out[i] = orc_sorted_search(vals, n, qs[i], rank ? rank + i : 0);
}

/* ------------------------------------------------------------------------ */
/* Occurrence range (sas/util.rs:36-46 Search::search_prefix, declared but   */
/* unimplemented!() in the reference): ranks [lo, hi) of the suffixes that   */
/* start with q.  lo = lower bound (A6); hi = first rank whose first         */
/* min(m, len) chars compare > q.                                            */
/* ------------------------------------------------------------------------ */
EXPORT void orc_prefix_range(const uint8_t* t, uint64_t n, const uint32_t* sa, const uint8_t* q, uint64_t m,
                             uint64_t* lo_out, uint64_t* hi_out) {
    uint64_t l = 0, r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        if (suffix_lt(t, n, sa[mid], q, m)) l = mid + 1;
        else r = mid;
    }
    *lo_out = l;
    r = n;
    while (l < r) {
        uint64_t mid = (l + r) / 2;
        uint64_t p = sa[mid], len = n - p, k = len < m ? len : m;
        int c = memcmp(t + p, q, k);
        int gt = c > 0;  /* equal on k chars: starts with q (k == m) or is shorter (< q) */
        if (!gt) l = mid + 1;
        else r = mid;
    }
    *hi_out = l;
}
