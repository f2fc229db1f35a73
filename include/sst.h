/*
 * sst.h -- C ABI of the MI355X static-search-tree engine over sorted u32 keys
 * (part of libsas_amd.so).
 *
 * Drop-in boundary for the reference's u32 search API
 * (static-search-tree/src = sst/):
 *
 *   sst_build   replaces SearchIndex::new(&[u32])                 sst/lib.rs:30-33
 *               and STree::new_params(vals, left_max, reverse, full)  sst/s_tree.rs:72-176
 *               (layouts: SortedVec sst/binary_search.rs:19-27, Eytzinger
 *               sst/eytzinger.rs:37-63, STree16/STree15 sst/s_tree.rs:19-20)
 *   sst_size    replaces SearchIndex::size()                      sst/lib.rs:35-36
 *   sst_layers  replaces SearchIndex::layers()                    sst/lib.rs:38-39
 *   sst_query   replaces SearchScheme::query(&I, &[u32]) -> Vec<u32>  sst/lib.rs:55-57
 *               (all schemes of one index give identical results, sst/test.rs:185-196)
 *
 * Result semantics: the VALUE of the first key >= q (STree::search,
 * sst/s_tree.rs:196-206).  Keys must be sorted and, for the S-tree layouts,
 * <= i32::MAX (sst/node.rs:5, compares are signed as in find_popcnt
 * sst/node.rs:93-109) -> EINVAL otherwise (the reference asserts).  As in the
 * reference, the caller includes a MAX sentinel (sst/util.rs:37) so every
 * query has an answer.  SortedVec without an answer returns u32::MAX (the
 * reference reads vals[n] out of bounds); Eytzinger returns u32::MAX
 * (sst/eytzinger.rs:224-230).  out_rank (optional, S-tree and SortedVec only)
 * = leaf slot k*B + idx = index of the answer in the sorted keys.
 *
 * Errors: 0 / errno as in sas.h; sas_last_error() gives the message.
 */
#ifndef SST_H
#define SST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sst_index sst_index;

enum sst_layout {
    SST_SORTED    = 0, /* SortedVec: plain sorted array, binary search              */
    SST_EYTZINGER = 1, /* Eytzinger BFS layout, vals[0] = u32::MAX                  */
    SST_STREE16   = 2, /* STree<16,16>: B+ tree, 64-B nodes                          */
    SST_STREE15   = 3, /* STree<15,16>: 15 keys + copy of the next node's first key */
    SST_PARTITIONED_MAP = 4, /* PartitionedSTree16M: prefix map on the top b key bits
                               + S-tree (sst/partitioned_s_tree.rs:111-190,364-648);
                               b = SST_PART_BITS(b) in flags                         */
    SST_DIRECT_MAP = 5, /* the prefix map taken to its limit: a direct-address table on
                          the top b of the 31 key bits (b = SST_PART_BITS(b), 0 = ceil(
                          log2 n) + 1, at most 30), 16-B entries {first index whose key
                          is >= the bucket start, that key and the next two}: a lookup
                          is one read unless three keys of its bucket are < q (then a
                          binary search over the sorted keys of the bucket)          */
    /* PartitionedSTree<16,16,Tp>::new(vals, b) (sst/partitioned_s_tree.rs:111-648,
       searches :654-831) for the other four markers the reference's differential test
       runs (sst/test.rs:222-246); b = SST_PART_BITS(b).  Leaves are padded per part, so
       these layouts return values only (out_rank: EINVAL) */
    SST_PARTITIONED = 6,         /* Simple: (B+1)^h-node layers per part, layer by layer  */
    SST_PARTITIONED_COMPACT = 7, /* Compact: one packed tree per part (bpp nodes each)   */
    SST_PARTITIONED_L1 = 8,      /* L1: the root's fan-out cut to what the parts need    */
    SST_PARTITIONED_OVERLAP = 9  /* Overlapping: parts share root windows (16 - overlap
                                    new subtrees per part)                               */
};

/* layout flags (STree::new_params arguments) */
#define SST_LEFT_MAX   (1u << 0)  /* internal key = max of left subtree              */
#define SST_REVERSE    (1u << 1)  /* layers stored leaves-first                      */
#define SST_FULL       (1u << 2)  /* (B+1)^h-sized layers                            */
#define SST_DEVICE_PTRS (1u << 8) /* sst_query: qs/out_val/out_rank are device ptrs  */
#define SST_NO_LDS_TOP (1u << 9)  /* sst_query: do not stage top layers in LDS       */
#define SST_PART_BITS(b) (((uint32_t)(b) & 0xFFu) << 16) /* PartitionedSTree16M::new(vals, b) */
#define SST_PART_BITS_OF(flags) (((flags) >> 16) & 0xFFu)

int sst_build(const uint32_t* sorted_vals, uint64_t n, int layout, uint32_t flags, sst_index** out);
int sst_free(sst_index* index);
uint64_t sst_size(const sst_index* index);
uint64_t sst_layers(const sst_index* index);
int sst_query(const sst_index* index, const uint32_t* qs, uint64_t nq, uint32_t* out_val,
              uint64_t* out_rank, void* stream, uint32_t flags);
/* Copy the built node array (host) for layout checks: count = u32 words. */
int sst_copy_nodes(const sst_index* index, uint32_t* dst, uint64_t count);
/* Average kernel time of `reps` back-to-back queries on device buffers. */
int sst_time_query(const sst_index* index, const uint32_t* d_qs, uint64_t nq, uint32_t* d_out,
                   int reps, void* stream, uint32_t flags, double* kernel_ns);

#ifdef __cplusplus
}
#endif
#endif /* SST_H */
