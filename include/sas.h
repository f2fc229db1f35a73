/*
 * sas.h -- C ABI of the MI355X suffix-array search engine (libsas_amd.so).
 *
 * Drop-in boundary for the reference's Rust SA query API
 * (RagnarGrootKoerkamp/suffix-array-searching, sas/ = suffix-array-searching/src):
 *
 *   sas_build          replaces SaNaive::build(t: &Seq) -> SaNaive      sas/sa_search.rs:30-57
 *                      and Search::build                                  sas/util.rs:31
 *   sas_search_batch   replaces the batch type F<B>                       sas/sa_search.rs:454
 *                        fn(&SaNaive, [&[u8]; B], &mut usize) -> [usize; B]
 *                      and the single-query type F1                       sas/sa_search.rs:453
 *                        fn(&SaNaive, &[u8], &mut usize) -> usize   (nq = 1)
 *                      Semantics of every algo = binary_search            sas/sa_search.rs:98-112
 *                        position SA[lower_bound(q)] under Rust slice order.
 *   sas_search_fixed   the same for a contiguous block of fixed-length queries
 *   sas_gen_text       random_string(n, ChaCha8Rng::seed_from_u64(seed))  sas/util.rs:9-15, sas/main.rs:38
 *   sas_gen_queries    random_queries(t, q, rng)                          sas/util.rs:18-26
 *
 * Conventions (no C++ exceptions cross this ABI; sas/Cargo.toml panics instead):
 *   - every function returns 0 on success or a positive errno value
 *     (EINVAL bad argument, ENOMEM device memory, ENOTSUP unsupported size,
 *     EIO HIP runtime failure); sas_last_error() gives a thread-local message.
 *   - text and query bytes are DNA codes 0..3 (the reference's random_string
 *     and FASTA loader only produce these, sas/util.rs:9-15,144-169).
 *   - a query above every suffix gets the sentinel position n (the reference
 *     reads sa[n] out of bounds there).
 *   - pointers are host pointers unless SAS_DEVICE_PTRS is set, in which case
 *     every input/output array of the call is device (HBM) memory.
 *   - a built index is immutable and thread-safe; concurrent searches on
 *     different streams are allowed.
 */
#ifndef SAS_H
#define SAS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sas_index sas_index;

/* flags */
#define SAS_DEVICE_PTRS   (1u << 0)  /* all array arguments are device pointers          */
#define SAS_BUILD_LCP     (1u << 1)  /* also build the LCP array (Kasai semantics)       */
#define SAS_BUILD_STREE   (1u << 2)  /* also build the S-tree over 16-char SA keys       */
#define SAS_BUILD_VERIFY  (1u << 3)  /* run the adjacency + permutation check on the SA  */
#define SAS_NO_LDS_TOP    (1u << 4)  /* search: do not serve the top levels from LDS     */
#define SAS_VALIDATE      (1u << 5)  /* search: reject query bytes > 3 (synchronises)    */
#define SAS_ROUTE_PACKED  (1u << 26)  /* sas_route_pack(_cap): write each query as one 2-bit
                                         packed word (m <= 32, 8 B per send slot, the
                                         sas_search_packed format) instead of its m bytes */
#define SAS_NO_PREFIX_TABLE (1u << 25) /* sas_search_range: use the tree descents even when
                                        the index has a prefix table                      */
#define SAS_QUERIES_ARE_SLICES (1u << 28) /* sas_search_batch, SAS_ALGO_TAGGED, device pointers:
                                        query k is the slice t[qoff[k] .. qoff[k] + qlen[k])
                                        of the indexed text itself (the reference's borrowed
                                        &t[i..i+len] queries, sas/util.rs:18-26); qbytes is
                                        ignored (may be NULL), the chars come from the index's
                                        packed text, and a lookup whose candidate suffix is
                                        the query's own start skips its text compare.  The
                                        call checks every slice lies inside the text (EINVAL)
                                        and synchronises on the stream to do so            */
#define SAS_RANGE_NO_INLINE (1u << 27) /* sas_search_range(_fixed): on a two/four-suffix inline
                                        prefix table, bisect both bounds from the table's rank
                                        range instead of testing the inline slots first     */
#define SAS_PREFIX_RANGE  (1u << 24) /* search, PLAIN / LCP: start binary_search from the
                                        prefix table's range of q's first p chars, as the
                                        reference's binary_search does (sas/sa_search.rs:
                                        98-101); needs SAS_BUILD_PREFIX                    */
#define SAS_BUILD_WIDE    (1u << 6)  /* build: use the n >= 2^31 two-pass doubling rounds
                                        at any n (test hook for that path)               */
#define SAS_BUILD_SECTOR  (1u << 7)  /* also build the sector tree (SAS_ALGO_SECTOR)     */
#define SAS_BUILD_SA40    (1u << 8)  /* store the SA as packed 40-bit entries and use the
                                        bucketed 64-bit builder at any n (automatic for
                                        n >= 2^32 - 64; test hook below that)             */
#define SAS_BUILD_QUAD    (1u << 9)  /* also build the quad tree (SAS_ALGO_QUAD)         */
#define SAS_BUILD_QUAD_COMPACT (1u << 10) /* build the quad tree with key-only leaves: 8 B
                                        per suffix (eight 32-char keys per 64-B leaf) instead
                                        of 16, SA values read from the SA array.  Fits next to
                                        a 40-bit SA at n = 2^34 in one GPU's HBM.  Implies
                                        SAS_BUILD_QUAD                                     */
#define SAS_BUILD_QUAD_ABS (1u << 11) /* quad tree inner nodes in the absolute layout: 16 u32
                                        16-char separators, 17-ary                        */
#define SAS_BUILD_QUAD_REL (1u << 12) /* quad tree inner nodes in the prefix-relative layout:
                                        the node's shared d-char prefix + 30 u16 separators
                                        over the next 8 chars, 31-ary.  Neither flag: the
                                        layout with fewer levels larger than the 256 MiB
                                        Infinity Cache (absolute on a tie; n = 2^30 builds
                                        absolute, n = 2^34 compact builds relative)        */
#define SAS_BUILD_PREFIX  (1u << 14) /* also build the prefix table for SAS_ALGO_PREFIX (the
                                        reference's fill_prefix_table, sas/sa_search.rs:59-95):
                                        u32[4^p + 1], entry x = first SA rank whose p-char
                                        key is >= x.  p = SAS_BUILD_PREFIX_P(p) (1..17) or,
                                        if 0, ceil(log4(n)) + 1 capped at 16 (16 at n = 2^30:
                                        16 GiB).  Needs SAS_BUILD_QUAD.  u32 entries, or
                                        packed 40-bit ones beside a 40-bit SA             */
#define SAS_BUILD_PREFIX_INLINE (1u << 15) /* the prefix table with 16-B entries: the first
                                        suffix of each key's range inlined as {32-char key,
                                        rank, SA}, so a lookup answered by that suffix is
                                        one read.  Fused quad leaves, u32 SA only         */
#define SAS_BUILD_PREFIX_INLINE2 (1u << 21) /* the prefix table with 32-B entries: the first
                                        TWO suffixes of each key's range (ranks r, r + 1)
                                        inlined, read by a lane pair as one request       */
#define SAS_BUILD_PREFIX_INLINE4 (1u << 22) /* 64-B entries: the first FOUR suffixes of each
                                        range, read by a 4-lane group as one request      */
#define SAS_BUILD_PREFIX_P(p) ((uint32_t)(p) << 16)  /* bits 16..20: prefix chars       */
#define SAS_BUILD_TAGGED  (1u << 23) /* store the SA as 8-B tagged entries {SA 40 bits | the
                                        suffix's chars [p, p+12) in the high 24 bits} plus a
                                        u64 bucket table over the first p chars {first rank
                                        40 bits | rank count 24 bits} (the reference's prefix
                                        table, sas/sa_search.rs:59-95, live) for
                                        SAS_ALGO_TAGGED: an entry holds a suffix's (p+12)-char
                                        key AND its position, so a lookup is the bucket
                                        entry, one window of consecutive entries and (for
                                        m > p + 12) one text window.  p = SAS_BUILD_PREFIX_P
                                        or ceil(log4 n) capped at 16 (16 at n = 2^34: 32 GiB
                                        table beside 128 GiB of entries).  The entries
                                        replace the SA (sa_width 8).  Combines with LCP;
                                        not with the trees, LLCP or SAS_BUILD_PREFIX*  */
#define SAS_BUILD_TOP2_LEVELS(L) ((uint32_t)(L) << 27) /* bits 27..31: depth L (1..31) of
                                        the binary-search pivots (PLAIN / LCP / LLCP / INLINE):
                                        prefix-relative blocks of up to 4 levels (32 B each:
                                        the lcp P of the block's bounds and the 8 chars after
                                        P of 15 pivots); levels 1-15 (72.5 KiB) are staged in
                                        each workgroup's LDS, the rest cost one request per
                                        block instead of an SA word and a text window per
                                        level.  L is rounded up to the 4-level grid past the
                                        LDS levels (19, 23, 27, 31).  0 = the default, 27
                                        levels (273 MiB); 31 levels cost 4.3 GiB at n = 2^30.
                                        Clamped to the iteration count; results never depend
                                        on L                                               */
#define SAS_BUILD_TAG_LINES (1u << 24) /* with SAS_BUILD_TAGGED: the tagged entries as one
                                        128-B line per p-char bucket {overflow offset 40 bits
                                        | count 24 bits, the 20 entries of ranks first ..
                                        first + 19 as 48-bit {SA | tag} split into u16 high and
                                        u32 low halves} (slots past the bucket's count hold the
                                        next buckets' first suffixes, so the line ends with
                                        the answer to "every suffix of the bucket is < q") plus
                                        an overflow array with ranks first + 20 .. first + count
                                        of the larger buckets, the buckets' first ranks and a
                                        second text copy 64 B off the 128-B line grid.  A
                                        lookup reads its line as one request of an 8-lane
                                        group: bucket and first entries together.  p =
                                        SAS_BUILD_PREFIX_P or ceil(log4 n) - 2 (15 at n = 2^34:
                                        128 GiB of lines, ~16 suffixes each).  No SA array:
                                        TAGGED lookups, ranges and sas_copy_sa64          */
#define SAS_BUILD_LLCP    (1u << 13) /* also build the Manber-Myers accelerant for
                                        SAS_ALGO_LLCP: per SA rank m, one 16-B entry
                                        {SA[m] 40 bits, Llcp 12 bits, Rlcp 12 bits, 16 chars
                                        of SA[m] after each} of the binary-search interval
                                        whose mid is m, derived from the LCP array (built
                                        too).  16 B per suffix                           */

/* search algorithms; all return bit-identical positions */
enum sas_algo {
    SAS_ALGO_PLAIN = 0, /* lockstep lower-bound binary search over SA (A6/A9)              */
    SAS_ALGO_LCP   = 1, /* same probes, Manber-Myers mlr LCP skipping of known chars (A21) */
    SAS_ALGO_STREE = 2, /* S-tree over 16-char SA keys + exact tail search (K2+K3)         */
    SAS_ALGO_SECTOR = 3, /* sector tree: 32-B nodes (one HBM sector), 9-ary on 16-char keys,
                           leaves fuse (32-char key, SA value) pairs: no text/SA reads for m<=32 */
    SAS_ALGO_QUAD = 4,  /* quad tree: 4 lanes per query load each 64-B node in one request;
                           31-ary on the 8 chars after each node's shared prefix (17-ary on
                           16-char keys with SAS_BUILD_QUAD_ABS), leaves = 4 fused (32-char
                           key, SA) entries                                                  */
    SAS_ALGO_INLINE = 5, /* PLAIN's probe sequence (binary_search_batch) over the quad tree's
                           fused (32-char key, SA) entries: one 16-B read per probe instead of
                           an SA word + text words ("inlining values", todo.org:18-19)     */
    SAS_ALGO_LLCP = 6,  /* PLAIN's probe sequence with Manber-Myers LLCP/RLCP skipping: a probe
                           reads one 16-B {SA, Llcp, Rlcp, chars} entry and decides from the
                           lcp values alone unless they tie llcp/rlcp; a tie compares the
                           entry's 16 chars before any text (needs SAS_BUILD_LLCP; the LCP
                           array at work, A21)                                              */
    SAS_ALGO_PREFIX = 7, /* prefix table lookup (the rank range of q's first p chars, one 8-B
                           read; sas/sa_search.rs:59-95) + binary search over that range on
                           the quad tree's leaf entries: ~2 memory requests per lookup
                           (needs SAS_BUILD_PREFIX)                                          */
    SAS_ALGO_INTERP = 8, /* interpolation_search<16> (sas/sa_search.rs:376-421): the mid is
                           interpolated from string_value<16> of the bounds and the query
                           (sas/util.rs:76-117), clamped to [1/16, 15/16] of the range, exact
                           compares; out_probes = its cnt.  Reads the fused quad leaves'
                           {32-char key, SA} entries when built (one request per probe),
                           else SA + text.  With SAS_PREFIX_RANGE it starts from the prefix
                           table's range.  n < 2^32 (the reference asserts r_val * r fits a
                           usize, :389-392); ENOTSUP above                                   */
    SAS_ALGO_TAGGED = 9, /* bucket table + tagged SA entries (needs SAS_BUILD_TAGGED): the
                           configs[3] shape's lookup, ~4-5 memory requests for a long query  */
    SAS_ALGO_STREE_LLCP = 10, /* configs[2]'s combination: the STREE descent over the 16-char SA keys
                           (LDS-staged top layers) gives the run of suffixes sharing q's key,
                           then Manber-Myers LLCP skipping finishes inside it (the LLCP entries'
                           binary-search tree walked from its root, mids outside the run decided
                           with no read); needs SAS_BUILD_STREE and SAS_BUILD_LLCP          */
    SAS_ALGO_QUAD_LLCP = 11 /* configs[2] as one kernel: QUAD's descent over the fused 32-char
                           keys (LDS-staged top layers); a query the routed leaf does not settle
                           (q's 32-char key shared by several suffixes: long queries on
                           repetitive text) continues with LLCP skipping inside the run of
                           suffixes sharing its key, whose far end comes from where the path of
                           the next 16-char key parts from q's.  m <= 32: QUAD itself.  Needs
                           SAS_BUILD_QUAD with fused leaves in the absolute layout (the default
                           below 2^31 suffixes; SAS_BUILD_QUAD_ABS) and SAS_BUILD_LLCP        */
};

typedef struct sas_stats {
    uint64_t n;              /* text length (chars)                               */
    uint64_t text_bytes;     /* packed 2-bit text in HBM                          */
    uint64_t sa_bytes;       /* suffix array (sa_width bytes per entry)           */
    uint64_t lcp_bytes;      /* LCP array (u32), 0 if not built                   */
    uint64_t stree_bytes;    /* S-tree incl. 16-char key leaves, 0 if not built   */
    uint32_t stree_layers;   /* S-tree height (layers incl. leaves)               */
    uint32_t stree_lds_layers; /* layers served from LDS                          */
    uint32_t top_levels;     /* binary-search levels served from LDS (15, fewer for a
                                shallow search)                                       */
    uint32_t iterations;     /* ilog2(n)+1 lockstep iterations (sa_search.rs:171) */
    uint64_t build_sa_ns;    /* wall time of the SA construction (0 if supplied)  */
    uint64_t build_total_ns; /* wall time of sas_build                            */
    uint32_t sa_rounds;      /* prefix-doubling rounds after the 32-char sort     */
    uint32_t sa_width;       /* bytes per stored SA entry: 4 (u32) or 5 (40-bit)  */
    uint64_t rank_lo;        /* global SA rank of this index's first entry         */
    uint64_t sa_entries;     /* SA entries held (n, or a shard's rank range)       */
    uint64_t next_pos;       /* SA[rank_lo + sa_entries] (n if none)               */
    uint64_t sector_bytes;   /* sector tree (inner nodes + fused leaves), 0 if not built */
    uint32_t sector_layers;  /* sector tree height incl. the leaf layer           */
    uint32_t sector_lds_layers; /* its layers served from LDS                     */
    uint64_t quad_bytes;     /* quad tree (inner nodes + leaves), 0 if not built   */
    uint32_t quad_layers;    /* quad tree height incl. the leaf layer              */
    uint32_t quad_lds_layers; /* its layers served from LDS                       */
    uint32_t quad_entry_bytes; /* quad leaf bytes per suffix: 16 (fused key + SA),
                                  8 (SAS_BUILD_QUAD_COMPACT), 0 if not built        */
    uint32_t quad_fan;       /* quad inner-node fan-out: 31 (prefix-relative nodes) or
                                17 (SAS_BUILD_QUAD_ABS), 0 if not built              */
    uint32_t top2_levels;    /* binary-search levels whose pivots come from LDS or the
                                prefix-relative blocks (PLAIN/LCP/LLCP/INLINE)       */
    uint64_t llcp_bytes;     /* SAS_BUILD_LLCP entries (16 B per suffix), 0 if not built */
    uint64_t prefix_bytes;   /* SAS_BUILD_PREFIX table, 0 if not built                */
    uint32_t prefix_chars;   /* its p (chars per table key)                           */
    uint32_t tag_chars;      /* SAS_BUILD_TAGGED: p of the bucket table (0 if not built);
                                sa_width is then 8 (tagged entries)                   */
    uint64_t tag_table_bytes; /* SAS_BUILD_TAGGED bucket table, (4^p + 1) x 8 B       */
    uint64_t index_bytes;    /* every HBM array of the index together (text, SA or tagged
                                entries, LCP, LLCP, trees, tables, top2)              */
    uint32_t tag_line_slots; /* SAS_BUILD_TAG_LINES: entries per 128-B bucket line (20), else 0;
                                tag_table_bytes is then the lines and the first-rank
                                table, sa_bytes the overflow                          */
    uint32_t tag_line_tag_bits; /* SAS_BUILD_TAG_LINES: tag bits of a line entry (48 minus
                                the SA bits: 16 below n = 2^32, 13 at n = 2^34)       */
    uint64_t tag_overflow_entries; /* SAS_BUILD_TAG_LINES: entries in the overflow array */
    uint64_t text2_bytes;    /* SAS_BUILD_TAG_LINES: the second packed-text copy (64 B off
                                the 128-B line grid, so a tie's compare reads one line) */
    uint64_t top2_bytes;     /* 0 since round 4: every pivot level is in the rel blocks */
    uint32_t rel_levels;     /* the prefix-relative pivot blocks: the levels they reach
                                (the pivot depth rounded up to 4-level blocks past the
                                15 LDS levels, clamped to the iterations; 0 if none) */
    uint32_t rel_pad;        /* 0 */
    uint64_t rel_bytes;      /* their array: one 32-B block {lcp of the block's bounds, the
                                8 chars after it of each of 15 pivots} per 4-level subtree
                                (16 B for a shorter one), the LDS levels' first    */
    uint64_t prefix_key_lo;  /* SAS_BUILD_PREFIX: the first p-char key the table holds an entry
                                for: 0 for a whole index; for a part / shard (a contiguous SA
                                rank range) the key of its first suffix                */
    uint64_t prefix_entries; /* its entries: 4^p + 1 for a whole index; for a part, its first
                                suffix's key .. its last one's + 2 (1/8 of the keys each at 8
                                parts of a random text); prefix_bytes = entries x entry bytes */
} sas_stats;

const char* sas_last_error(void);

/* Build an index over text[0..n).  sa_or_null: caller's suffix array with
 * sa_width = 4 (u32, n < 2^32), 5 (packed 40-bit little-endian) or 8 (u64),
 * or NULL to construct it on the GPU (prefix doubling on 32-char packed keys).
 * n < 2^32 - 64 keeps a u32 SA; larger n (up to 2^40, as HBM allows) or
 * SAS_BUILD_SA40 store a packed 40-bit SA, built by the bucketed builder
 * (32-char-key buckets sorted one at a time, then doubling rounds over the
 * tied suffixes only).  The library copies everything into HBM. */
int sas_build(const uint8_t* text, uint64_t n, const void* sa_or_null, int sa_width,
              uint32_t flags, sas_index** out);
int sas_free(sas_index* index);

/* Sharded-text mode: the index holds only global SA ranks
 * [rank_lo, rank_hi) (the packed text stays whole: compares need any suffix).
 * sa_or_null is the FULL suffix array, or NULL to construct it here.  A
 * search on a shard returns SA[global lower bound] when that rank lies in
 * (rank_lo, rank_hi], i.e. for every query routed to it by sas_route. */
int sas_build_shard(const uint8_t* text, uint64_t n, const void* sa_or_null, int sa_width,
                    uint64_t rank_lo, uint64_t rank_hi, uint32_t flags, sas_index** out);

/* Sharded-text mode without any whole-SA step: part `part` of `parts` builds ONLY
 * its own SA rank range, so the text size is not capped by one GPU's memory for
 * a full SA.  Every part takes the same contiguous range of
 * 7-char-prefix bins from the text's histogram (balanced to bin granularity, so
 * the range is chosen by the library: sas_get_stats -> rank_lo, sa_entries,
 * next_pos), ties on 32-char keys are resolved inside the part by text windows.
 * The SA is stored 40-bit.  ENOTSUP for a text whose repeated prefixes exceed
 * 2^21 chars (use sas_build_shard), EINVAL for an empty part. */
int sas_build_part(const uint8_t* text, uint64_t n, uint32_t part, uint32_t parts, uint32_t flags,
                   sas_index** out);

/* sas_build / sas_build_part over the text random_string(n) draws from
 * ChaCha8Rng::seed_from_u64(seed) (sas/util.rs:9-15, sas/main.rs:38 -- the same
 * chars sas_gen_text writes), generated on the GPU straight into the index's 2-bit
 * packed text: no n-byte copy exists on the host or the device (a sharded rank of
 * configs[4] holds the whole text packed, n/4 bytes, and never its bytes).  Replaces
 * `SaNaive::build(&random_string(n))` of sas/main.rs:53-65. */
int sas_build_gen(uint64_t seed, uint64_t n, uint32_t flags, sas_index** out);
int sas_build_part_gen(uint64_t seed, uint64_t n, uint32_t part, uint32_t parts, uint32_t flags,
                       sas_index** out);

/* Query routing for the sharded mode: out_shard[k] = number of splitter
 * suffixes (text positions splitter_pos[0..nsplit), in increasing suffix
 * order: the first suffix of shards 1..W-1) that are < query k.  Fixed-length
 * queries qbytes[k*m .. (k+1)*m).  Device pointers with SAS_DEVICE_PTRS. */
int sas_route(const sas_index* index, const uint64_t* splitter_pos, uint32_t nsplit,
              const uint8_t* qbytes, uint32_t m, uint64_t nq, uint32_t* out_shard,
              void* stream, uint32_t flags);

/* sas_route for ragged queries: query k = qbytes[qoff[k] .. qoff[k] + qlen[k]). */
int sas_route_batch(const sas_index* index, const uint64_t* splitter_pos, uint32_t nsplit,
                    const uint8_t* qbytes, const uint64_t* qoff, const uint32_t* qlen, uint64_t nq,
                    uint32_t* out_shard, void* stream, uint32_t flags);

/* One sharded step's send side, fused on the GPU (device pointers only,
 * SAS_DEVICE_PTRS): route each fixed-length query (as sas_route), group the
 * queries by destination shard (counting sort) and copy their bytes into
 * out_send, bucket after bucket.  out_counts[w] = queries for shard w
 * (w < nsplit + 1); out_slot[k] = send position of query k, so the positions
 * that come back in send order are gathered with it.  Order inside a bucket is
 * unspecified. */
int sas_route_pack(const sas_index* index, const uint64_t* splitter_pos, uint32_t nsplit,
                   const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t* out_counts,
                   uint8_t* out_send, uint64_t* out_slot, void* stream, uint32_t flags);

/* (SAS_ROUTE_PACKED in flags: out_send holds one u64 packed word per slot.) */
/* sas_route_pack with fixed-capacity buckets: bucket w owns send slots [w*cap, (w+1)*cap)
 * (out_send holds (nsplit + 1) * cap * m bytes), so every rank's all-to-all uses equal splits
 * and needs no host-side counts.  out_counts[w] is the true count; a query past its bucket's
 * cap is not copied and its out_slot is (nsplit + 1) * cap - 1: the caller checks
 * out_counts[w] <= cap on the device and redoes an overflowing step exactly.  Send slots a
 * bucket does not fill keep their old bytes.  EINVAL if cap == 0.  One pass over the
 * queries: out_counts is zeroed and accumulated on the stream. */
int sas_route_pack_cap(const sas_index* index, const uint64_t* splitter_pos, uint32_t nsplit,
                       const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t cap, uint64_t* out_counts,
                       uint8_t* out_send, uint64_t* out_slot, void* stream, uint32_t flags);

/* The sharded step's receive side (device pointers only, SAS_DEVICE_PTRS): out[k] =
 * back[slot[k]], the positions that came back in send-slot order put in query order; with
 * overflow non-null, *overflow is set to 1 (never cleared) when some counts[w] > cap,
 * w < nparts (the out_counts of sas_route_pack_cap), so a caller can defer that check. */
int sas_shard_gather(const sas_index* index, const uint64_t* back, const uint64_t* slot, uint64_t nq,
                     const uint64_t* counts, uint32_t nparts, uint64_t cap, uint64_t* out,
                     uint32_t* overflow, void* stream, uint32_t flags);

/* The sharded step's local lookup over the received slots (device pointers only,
 * SAS_DEVICE_PTRS): slot b*cap + j (b < nbuckets, j < cap) holds a query iff
 * j < counts[b] (the counts each source rank sent, e.g. sas_route_pack_cap's out_counts
 * after a count exchange); only those slots are searched and written, the others are
 * skipped without a read.  queries: m bytes per slot, or with SAS_ROUTE_PACKED one u64
 * 2-bit word per slot (SAS_ALGO_PREFIX, m <= 32).  Algorithms: PLAIN, LCP, LLCP, PREFIX,
 * and QUAD for m <= 32 (ENOTSUP otherwise: search every slot with sas_search_fixed).
 * EINVAL if nbuckets * cap >= 2^32.  Asynchronous on `stream`. */
int sas_search_buckets(const sas_index* index, const void* queries, uint32_t m, uint32_t nbuckets,
                       uint64_t cap, const uint64_t* counts, int algo, uint64_t* out_pos, void* stream,
                       uint32_t flags);

/* The source hash the library was built from (the Makefile's sha256 over csrc/ and
 * include/, 16 hex digits): profiles record it, so counters collected on one build are
 * never attached to another. */
const char* sas_source_hash(void);

int sas_get_stats(const sas_index* index, sas_stats* out);

/* Copy the suffix array / LCP array out (dst host or device per flags).
 * sas_copy_sa needs a u32 SA (sa_width 4, EINVAL otherwise); sas_copy_sa64
 * copies global ranks [start, start+count) of either width as u64.  LCP values
 * are u32 (capped at 2^32-1). */
int sas_copy_sa(const sas_index* index, uint32_t* dst, uint64_t count, uint32_t flags);
int sas_copy_sa64(const sas_index* index, uint64_t start, uint64_t count, uint64_t* dst, uint32_t flags);
int sas_copy_lcp(const sas_index* index, uint32_t* dst, uint64_t count, uint32_t flags);

/* 2-bit packed fixed-length queries, m <= 32: word i holds query i's chars, the first in
 * bits 63..62, zero padded (how the reference packs DNA for its interpolation search,
 * string_value<K>, sas/util.rs:76-117).  A lookup then reads 8 B of query instead of m.
 * sas_pack_queries: device pointers (SAS_DEVICE_PTRS: a kernel on `stream`) or host arrays
 * (packed on the host's worker pool, AVX2 or BMI2 where the CPU has them); EINVAL on codes > 3.
 * sas_search_packed: SAS_ALGO_PREFIX only; host or device pointers per flags. */
int sas_pack_queries(const uint8_t* qbytes, uint32_t m, uint64_t nq, uint64_t* out_words, void* stream,
                     uint32_t flags);
int sas_search_packed(const sas_index* index, const uint64_t* qwords, uint32_t m, uint64_t nq, int algo,
                      uint64_t* out_pos, uint32_t* out_probes, void* stream, uint32_t flags);

/* Substrings of the indexed text as byte codes 0..3: out[out_off[i] .. out_off[i] + len[i])
 * = text[pos[i] .. pos[i] + len[i]) (0 past the text end), from the index's packed copy,
 * so a caller can drop its own byte copy of a large text after sas_build.  Device
 * pointers only (SAS_DEVICE_PTRS), stream-ordered on `stream`. */
int sas_extract(const sas_index* index, const uint64_t* pos, const uint32_t* len, const uint64_t* out_off,
                uint64_t count, uint8_t* out, void* stream, uint32_t flags);

/* GPU check of the SA: strictly increasing adjacent suffixes (the
 * reference's build assertion, sas/sa_search.rs:36-38) + permutation.
 * Returns 0 if valid, EINVAL (with message) if not. */
int sas_verify(const sas_index* index);

/* Ragged batch: query k = qbytes[qoff[k] .. qoff[k] + qlen[k]).
 * out_pos[k] = SA[lower_bound(q_k)] (or n).  out_probes (optional): for PLAIN, LCP,
 * LLCP and INTERP the number of probes of query k, the reference's `cnt` counter
 * (sas/sa_search.rs:104,178); for the tree algorithms the memory reads of the lookup
 * (tree nodes and leaves; STREE_LLCP / QUAD_LLCP: + the LLCP entries read, QUAD_LLCP: + the
 * text compare of the leaf's candidate), which have no reference counterpart.
 * stream: hipStream_t or NULL.
 * With host pointers the call is synchronous; with SAS_DEVICE_PTRS it is
 * asynchronous on `stream`. */
int sas_search_batch(const sas_index* index, const uint8_t* qbytes, const uint64_t* qoff,
                     const uint32_t* qlen, uint64_t nq, int algo, uint64_t* out_pos,
                     uint32_t* out_probes, void* stream, uint32_t flags);

/* Fixed-length batch: query k = qbytes[k*m .. (k+1)*m). */
int sas_search_fixed(const sas_index* index, const uint8_t* qbytes, uint32_t m, uint64_t nq,
                     int algo, uint64_t* out_pos, uint32_t* out_probes, void* stream,
                     uint32_t flags);

/* Occurrence ranges (Search::search_prefix / search_range, sas/util.rs:36-46,
 * declared but unimplemented!() in the reference): global SA ranks
 * [out_lo[k], out_hi[k]) of the suffixes that start with query k; the count
 * is out_hi - out_lo and the positions are SA[out_lo .. out_hi)
 * (sas_copy_sa_range).  Needs SAS_BUILD_TAGGED, SAS_BUILD_QUAD or SAS_BUILD_SECTOR: the
 * tagged index uses its bucket table; otherwise the prefix table when built beside the quad
 * tree (unless SAS_NO_PREFIX_TABLE), else the quad tree, else the sector tree.  On a
 * two/four-suffix inline prefix table a query's lane group tests both bounds on the entry's
 * slots first (one request answers most queries); bounds not found there are bisected in
 * lock step.  No probe counts are reported (the reference has no range search to count
 * against).  Ragged queries as in sas_search_batch. */
int sas_search_range(const sas_index* index, const uint8_t* qbytes, const uint64_t* qoff,
                     const uint32_t* qlen, uint64_t nq, uint64_t* out_lo, uint64_t* out_hi,
                     void* stream, uint32_t flags);
/* sas_search_range for fixed-length queries qbytes[k*m .. (k+1)*m). */
int sas_search_range_fixed(const sas_index* index, const uint8_t* qbytes, uint32_t m, uint64_t nq,
                           uint64_t* out_lo, uint64_t* out_hi, void* stream, uint32_t flags);
/* Copy SA[start .. start+count) (global ranks) out: the text positions of a range. */
int sas_copy_sa_range(const sas_index* index, uint64_t start, uint64_t count, uint32_t* dst,
                      uint32_t flags);

/* Timing helper for benches: run `reps` back-to-back fixed-length searches on
 * device buffers and report the average duration of the search kernel itself
 * (HIP events on `stream`) in *kernel_ns and of the whole call in *call_ns. */
int sas_time_fixed(const sas_index* index, const uint8_t* d_qbytes, uint32_t m, uint64_t nq,
                   int algo, uint64_t* d_out_pos, int reps, void* stream, uint32_t flags,
                   double* kernel_ns, double* call_ns);

/* Generators (bit-exact restatements of the reference's seeded inputs). */
int sas_gen_text(uint64_t seed, uint64_t n, uint8_t* out, uint32_t flags);
/* Offsets i = gen_range(0..n - margin) and lengths gen_range(len_lo..len_hi)
 * (fixed when len_hi == len_lo + 1), continuing the ChaCha8 stream at
 * keystream word `word_pos` (= n after sas_gen_text).  Host arrays only.
 * Returns the next free keystream word through *next_word (may be NULL). */
int sas_gen_queries(uint64_t seed, uint64_t word_pos, uint64_t n, uint64_t nq, uint64_t margin,
                    uint32_t len_lo, uint32_t len_hi, uint64_t* off, uint32_t* len,
                    uint64_t* next_word);

/* One process, several GPUs (SURVEY §8b sas_build_multi).  mode
 * SAS_MULTI_REPLICATE: every device builds the whole index (sas_build) and a
 * batch is cut into contiguous query chunks, one per device, run concurrently.
 * SAS_MULTI_SHARD: device g builds only part g of the SA rank space
 * (sas_build_part, balanced to 7-char-prefix bins); queries are routed on the
 * first device against the parts' first suffixes (sas_route_batch) and each part
 * answers its own.  Results are identical to one sas_build index.  `devices`
 * lists ngpu device ordinals (repeats allowed: several parts on one GPU).  Host
 * pointers only; the text stays with the caller.  The one-process-per-GPU path
 * over RCCL is bench.py --mode shard / sas_amd.shard. */
typedef struct sas_multi sas_multi;
#define SAS_MULTI_REPLICATE 0
#define SAS_MULTI_SHARD     1
int sas_build_multi(const uint8_t* text, uint64_t n, const int* devices, int ngpu, int mode,
                    uint32_t flags, sas_multi** out);
int sas_multi_free(sas_multi* multi);
int sas_multi_parts(const sas_multi* multi);
int sas_multi_get_stats(const sas_multi* multi, int part, sas_stats* out);
/* Ragged batch as sas_search_batch (synchronous, host pointers). */
int sas_search_multi(const sas_multi* multi, const uint8_t* qbytes, const uint64_t* qoff,
                     const uint32_t* qlen, uint64_t nq, int algo, uint64_t* out_pos, uint32_t flags);

/* Real-data inputs.
 * sas_read_fasta: read_fasta_file (sas/util.rs:144-169) -- records concatenated,
 * A/C/G/T/a/c/g/t -> 0..3, every other byte -> 0; FASTA and FASTQ, no gzip.
 * out == NULL -> only *len is computed (size the buffer, then call again). */
int sas_read_fasta(const char* path, uint8_t* out, uint64_t cap, uint64_t* len);
/* sas_kmer_keys: the --human u32 keys of sst/bin/bench.rs:58-76 for the S-tree:
 * out[j] = packed chars [j, j+k) & i32::MAX, j < min(n, limit+k-1) - (k-1),
 * out[0] = i32::MAX.  out == NULL -> only *count.  k in 1..16. */
int sas_kmer_keys(const uint8_t* text, uint64_t n, uint32_t k, uint64_t limit, uint32_t* out,
                  uint64_t* count, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* SAS_H */
