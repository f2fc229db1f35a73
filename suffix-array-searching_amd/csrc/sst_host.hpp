// sst_host.hpp -- the host builders of the u32 static-search-tree layouts (sst.hip):
// each restates the reference's constructor line by line and fills a node array that
// sst_build then moves to HBM.  Host-only code: tests/cpp/sst_host_check.cpp also compiles
// it on the CPU and walks the arrays with the kernels' index arithmetic.
#pragma once
#include "common.hpp"

#include <algorithm>
#include <vector>

static constexpr uint32_t SST_MAX = 0x7fffffffu;  // sst/node.rs:5

// ------------------------------------------------------------------ host builders
// TreeBase<B> (sst/s_tree.rs:22-45)
static uint64_t blocks_of(uint64_t n, uint64_t B) { return (n + B - 1) / B; }
static uint64_t prev_keys(uint64_t n, uint64_t B) { return (blocks_of(n, B) + B) / (B + 1) * B; }
static uint32_t height_of(uint64_t n, uint64_t B) { return n <= B ? 1 : height_of(prev_keys(n, B), B) + 1; }
static uint64_t layer_size(uint64_t n, uint32_t h, uint32_t height, uint64_t B) {
    for (uint32_t i = h; i + 1 < height; i++) n = prev_keys(n, B);
    return n;
}

// STree::new_params (sst/s_tree.rs:72-176).  The node array starts zeroed
// like the reference's fresh hugepage allocation (:125-129).
static int build_stree_host(const uint32_t* vals, uint64_t n, uint32_t B, bool left_max, bool reverse, bool full,
                            std::vector<uint32_t>& tree, sst_index* x) {
    const uint32_t N = 16;
    if (full && reverse) SAS_FAIL(EINVAL, "sst_build: full array only makes sense in forward layout");
    for (uint64_t i = 0; i < n; i++)
        if (vals[i] > SST_MAX) SAS_FAIL(EINVAL, "sst_build: S-tree keys must be <= i32::MAX (sst/node.rs:5)");
    uint32_t height = height_of(n, B);
    if (height > SAS_STREE_MAX_LAYERS) SAS_FAIL(ENOTSUP, "sst_build: tree too high");
    uint64_t ls[SAS_STREE_MAX_LAYERS], nb = 0;
    for (uint32_t h = 0; h < height; h++) {
        if (full) {
            uint64_t s = 1;
            for (uint32_t k = 0; k < h; k++) s *= (B + 1);
            ls[h] = s;
        } else {
            ls[h] = (layer_size(n, h, height, B) + B - 1) / B;
        }
        nb += ls[h];
    }
    uint64_t sum = 0;
    for (uint32_t h = 0; h < height; h++) {
        if (!reverse) { x->off[h] = sum; sum += ls[h]; }
        else { sum += ls[h]; x->off[h] = nb - sum; }
        x->layer_nodes[h] = ls[h];
    }
    tree.assign(nb * N, 0u);
    auto node = [&](uint64_t b) { return tree.data() + b * N; };
    uint64_t ol = x->off[height - 1];
    for (uint64_t i = 0; i < n; i++) {
        node(ol + i / B)[i % B] = vals[i];
        if (B < N && i % B == 0 && i > 0) node(ol + i / B - 1)[B] = vals[i];
    }
    if (n / B < ls[height - 1])
        for (uint64_t j = n % B; j < N; j++) node(ol + n / B)[j] = SST_MAX;
    for (int h = (int)height - 2; h >= 0; h--) {
        uint64_t oh = x->off[h];
        std::fill(tree.begin() + oh * N, tree.begin() + (oh + ls[h]) * N, SST_MAX);
        for (uint64_t i = 0; i < (uint64_t)B * ls[h]; i++) {
            uint64_t k = i / B, j = i % B;
            k = k * (B + 1) + j + 1;
            for (uint32_t l = (uint32_t)h; l + 2 < height; l++) k *= (B + 1);
            node(oh + i / B)[i % B] =
                k * B < n ? (!left_max ? node(ol + k)[0] : node(ol + k - 1)[B - 1]) : SST_MAX;
        }
    }
    x->height = height;
    x->B = B;
    x->N = N;
    // LDS-staged top layers
    uint32_t L = 0, nodes = 0;
    for (uint32_t h = 0; h + 1 < height; h++) {
        if (nodes + ls[h] > SAS_STREE_LDS_NODES) break;
        nodes += (uint32_t)ls[h];
        L++;
    }
    x->lds_layers = L;
    x->lds_nodes = nodes;
    return 0;
}

// PartitionedSTree<16,16,Map>::get_part_size + try_new
// (sst/partitioned_s_tree.rs:111-190, 364-648 with Tp = Map: not compact, L1,
// overlap Some(0), prefix map).
static int build_pmap_host(const uint32_t* vals, uint64_t n, uint32_t b, std::vector<uint32_t>& tree,
                           std::vector<uint32_t>& pmap, sst_index* x) {
    const uint64_t B = 16;
    if (vals[n - 1] > SST_MAX) SAS_FAIL(EINVAL, "sst_build: keys must be <= i32::MAX (sst/node.rs:5)");
    // get_part_size (:111-190)
    uint32_t bits = 1 + (31 - __builtin_clz(vals[n - 1] ? vals[n - 1] : 1));
    if (vals[n - 1] == 0) bits = 1;  // ilog2(0) panics in the reference; treat as 1 bit
    auto part_sizes = [&](uint32_t shift, uint64_t parts, uint64_t* maxb) {
        std::vector<uint64_t> bs(parts, 0);
        for (uint64_t i = 0; i < n; i++) bs[vals[i] >> shift]++;
        uint64_t m = 0;
        for (uint64_t v : bs) m = v > m ? v : m;
        *maxb = m;
    };
    auto get_height = [&](uint64_t xx) { return height_of((xx * 17 + 15) / 16, B); };  // MAP: x*17/16
    uint32_t shift = bits > b ? bits - b : 0;
    uint64_t parts = 1ull << (bits - shift);
    uint64_t max_bucket;
    part_sizes(shift, parts, &max_bucket);
    uint32_t height = get_height(max_bucket);
    uint32_t b2 = b;
    for (;;) {
        if (b2 == 0) break;
        b2 -= 1;
        if (b2 > bits) break;
        uint32_t shift2 = bits > b2 ? bits - b2 : 0;
        uint64_t parts2 = 1ull << (bits - shift2);
        uint64_t mb2;
        part_sizes(shift2, parts2, &mb2);
        uint32_t h2 = get_height(mb2);
        if (h2 > height) break;
        shift = shift2;
        parts = parts2;
        max_bucket = mb2;
        height = h2;
    }
    // try_new (:364-648), Map
    uint64_t ls[SAS_STREE_MAX_LAYERS];
    if (height > SAS_STREE_MAX_LAYERS) SAS_FAIL(ENOTSUP, "sst_build: tree too high");
    for (uint32_t h = 0; h < height; h++) ls[h] = (layer_size(n, h, height, B) + B - 1) / B;
    if (height > 1) ls[0] = ((layer_size(n, 1, height, B) + B - 1) / B + B - 1) / B;
    uint64_t nb = 0;
    for (uint32_t h = 0; h < height; h++) {
        x->off[h] = nb;
        x->layer_nodes[h] = ls[h];
        nb += ls[h];
    }
    if (nb * 64 > (32ull << 30)) SAS_FAIL(ENOMEM, "sst_build: PartitionedSTree16M overhead too large (try_new -> None)");
    tree.assign(nb * 16, SST_MAX);
    uint64_t ol = x->off[height - 1];
    for (uint64_t i = 0; i < n; i++) tree[(ol + i / B) * 16 + i % B] = vals[i];
    uint64_t subtree = height == 1 ? 1 : B;
    for (uint32_t k = 0; k + 2 < height; k++) subtree *= (B + 1);
    for (int h = (int)height - 2; h >= 0; h--) {
        uint64_t oh = x->off[h];
        if (h == 0) {  // overlap Some(0): layer 0 holds the max of every layer-1 subtree
            for (uint64_t i = 0; i + 1 < ls[1]; i++) {
                uint64_t j = (i + 1) * subtree - 1;
                tree[(oh + i / B) * 16 + i % B] = tree[(ol + j / B) * 16 + j % B];
            }
            break;
        }
        for (uint64_t i = 0; i < B * ls[h]; i++) {
            uint64_t k = i / B, j = i % B;
            k = k * (B + 1) + j + 1;
            for (uint32_t l = (uint32_t)h; l + 2 < height; l++) k *= (B + 1);
            tree[(oh + i / B) * 16 + i % B] = k * B < n ? tree[(ol + k - 1) * 16 + B - 1] : SST_MAX;
        }
    }
    // prefix map (:605-627)
    pmap.assign(parts, 0);
    uint64_t max_idx = ls[0] * B - B;
    uint64_t p = 0;
    for (uint64_t i = 0; i < ls[0] * B; i++) {
        uint64_t pi = tree[x->off[0] * 16 + i] >> shift;
        while (p < pi && p + 1 < parts) {
            p++;
            pmap[p] = (uint32_t)(i < max_idx ? i : max_idx);
        }
    }
    while (p + 1 < parts) {
        p++;
        pmap[p] = (uint32_t)max_idx;
    }
    x->height = height;
    x->B = 16;
    x->N = 16;
    x->shift = shift;
    x->parts = (uint32_t)parts;
    return 0;
}

// PartitionedSTree<16,16,Tp>::get_part_size + try_new (sst/partitioned_s_tree.rs:111-227
// max_overlap, 229-345 Compact, 347-648 the others) for Tp = Simple, Compact, L1,
// Overlapping.  MAX-filled node array; a build the reference refuses (try_new -> None, more
// than 32 GiB of nodes) is ENOMEM, one it asserts against is EINVAL.
static int build_part_host(const uint32_t* vals, uint64_t n, uint32_t b, int layout, std::vector<uint32_t>& tree,
                           sst_index* x) {
    const uint64_t B = 16, N = 16;
    const bool COMPACT = layout == SST_PARTITIONED_COMPACT;
    const bool L1 = layout == SST_PARTITIONED_L1 || layout == SST_PARTITIONED_OVERLAP;
    const bool OL = layout == SST_PARTITIONED_OVERLAP;
    if (vals[n - 1] > SST_MAX) SAS_FAIL(EINVAL, "sst_build: keys must be <= i32::MAX (sst/node.rs:5)");
    uint32_t bits = vals[n - 1] ? 1 + (31 - __builtin_clz(vals[n - 1])) : 1;
    auto bucket_sizes = [&](uint32_t shift, uint64_t parts) {
        std::vector<uint64_t> bs(parts, COMPACT ? 1 : 0);  // Compact: one sentinel per part
        for (uint64_t i = 0; i < n; i++) bs[vals[i] >> shift]++;
        return bs;
    };
    auto maxof = [](const std::vector<uint64_t>& v) {
        uint64_t m = 0;
        for (uint64_t y : v) m = y > m ? y : m;
        return m;
    };
    uint32_t shift = bits > b ? bits - b : 0;
    uint64_t parts = 1ull << (bits - shift);
    std::vector<uint64_t> bs = bucket_sizes(shift, parts);
    uint64_t max_bucket = maxof(bs);
    uint32_t height = height_of(max_bucket, B);
    for (uint32_t b2 = b;;) {  // fewer parts while the height stays (:136-170)
        if (b2 == 0) break;
        b2 -= 1;
        if (b2 > bits) break;
        const uint32_t shift2 = bits > b2 ? bits - b2 : 0;
        const uint64_t parts2 = 1ull << (bits - shift2);
        std::vector<uint64_t> bs2 = bucket_sizes(shift2, parts2);
        const uint64_t mb2 = maxof(bs2);
        const uint32_t h2 = height_of(mb2, B);
        if (h2 > height) break;
        shift = shift2;
        parts = parts2;
        max_bucket = mb2;
        bs.swap(bs2);
        height = h2;
    }
    if (height > SAS_STREE_MAX_LAYERS) SAS_FAIL(ENOTSUP, "sst_build: tree too high");
    uint64_t p17[SAS_STREE_MAX_LAYERS + 1];
    p17[0] = 1;
    for (uint32_t h = 1; h <= SAS_STREE_MAX_LAYERS; h++) p17[h] = p17[h - 1] * (B + 1);
    const uint64_t subtree = height == 1 ? 1 : B * p17[height - 2];
    int64_t overlap = -1;  // None
    if (OL) {  // max_overlap (:199-227)
        if (bs.size() == 1) {
            overlap = bs[0] <= subtree ? 0 : -1;
        } else {
            const uint64_t capacity = 16 * subtree;
            for (int o = 15; o >= 0 && overlap < 0; o--) {
                uint64_t acc = 0;
                bool ok = true;
                for (uint64_t v : bs) {
                    acc += v;
                    if (acc > capacity) { ok = false; break; }
                    const uint64_t d = (16 - (uint64_t)o) * subtree;
                    acc = acc > d ? acc - d : 0;
                }
                if (ok) overlap = o;
            }
        }
    }
    uint64_t ls[SAS_STREE_MAX_LAYERS];
    uint64_t l1 = 0;
    if (COMPACT) {
        for (uint32_t h = 0; h < height; h++) ls[h] = (layer_size(max_bucket, h, height, B) + B - 1) / B;
    } else if (!L1) {
        for (uint32_t h = 0; h < height; h++) ls[h] = p17[h];
    } else {
        l1 = OL ? (overlap < 0 ? N + 1 : N - (uint64_t)overlap) : (layer_size(max_bucket, 1, height, B) + B - 1) / B;
        for (uint32_t h = 0; h < height; h++) ls[h] = (p17[h] * l1 + B) / (B + 1);
    }
    if (ls[0] != 1) SAS_FAIL(EINVAL, "sst_build: partitioned root of more than one node (the reference asserts)");
    uint64_t nb = 0, bpp = 0, extra = 0;
    if (COMPACT) {
        for (uint32_t h = 0; h < height; h++) {
            x->off[h] = bpp;
            x->layer_nodes[h] = ls[h];
            bpp += ls[h];
        }
        nb = parts * bpp;
    } else {
        extra = l1 == 0 ? 0 : ((overlap < 0 ? 0 : (uint64_t)overlap) + l1 - 1) / l1;
        for (uint32_t h = 0; h < height; h++) {
            uint64_t lb = ls[h] * (parts + extra);
            if (h == 0 && overlap >= 0) lb = (parts * (16 - (uint64_t)overlap) + (uint64_t)overlap + 15) / 16;
            x->off[h] = nb;
            x->layer_nodes[h] = lb;
            nb += lb;
        }
    }
    if (nb * 64 > (32ull << 30)) SAS_FAIL(ENOMEM, "sst_build: partitioned tree overhead too large (try_new -> None)");
    tree.assign(nb * N, SST_MAX);
    auto at = [&](uint64_t node, uint64_t j) -> uint32_t& { return tree[node * N + j]; };
    const uint32_t H = height - 1;
    const uint64_t ol = x->off[H];
    uint64_t prev = 0, idx = 0;
    if (COMPACT) {  // :274-299
        for (uint64_t v = 0; v < n; v++) {
            const uint32_t val = vals[v];
            const uint64_t part = val >> shift;
            while (prev < part) {
                if (idx / B < ls[H])
                    for (uint64_t j = idx % B; j < N; j++) at(prev * bpp + ol + idx / B, j) = val;
                prev++;
                idx = 0;
            }
            at(part * bpp + ol + idx / B, idx % B) = val;
            idx++;
        }
        for (int h = (int)height - 2; h >= 0; h--) {  // :302-322
            const uint64_t oh = x->off[h];
            for (uint64_t part = 0; part < parts; part++)
                for (uint64_t i = 0; i < B * ls[h]; i++) {
                    uint64_t k = i / B, j = i % B;
                    k = k * (B + 1) + j + 1;
                    for (uint32_t l = (uint32_t)h; l + 2 < height; l++) k *= (B + 1);
                    at(part * bpp + oh + i / B, i % B) = k * B < max_bucket ? at(part * bpp + ol + k - 1, B - 1) : SST_MAX;
                }
        }
    } else {
        const uint64_t part_size = OL ? l1 * subtree : B * ls[H];  // :498-513
        for (uint64_t v = 0; v < n; v++) {  // :516-541
            const uint32_t val = vals[v];
            const uint64_t part = val >> shift;
            while (prev < part) {
                prev++;
                while (idx < prev * part_size) {
                    at(ol + idx / B, idx % B) = val;
                    idx++;
                }
            }
            at(ol + idx / B, idx % B) = val;
            idx++;
        }
        for (int h = (int)height - 2; h >= 0; h--) {  // :545-600
            const uint64_t oh = x->off[h];
            if (h == 0 && overlap >= 0) {  // the root windows: every layer-1 subtree's max
                for (uint64_t i = 0; i < parts * l1 + (uint64_t)overlap; i++) {
                    const uint64_t j = (i + 1) * subtree - 1;
                    at(oh + i / B, i % B) = at(ol + j / B, j % B);
                }
                break;
            }
            const uint64_t l = ls[h], ll = ls[H];
            for (uint64_t p = 0; p < parts + extra; p++)
                for (uint64_t i = 0; i < B * ls[h]; i++) {
                    uint64_t k = i / B, j = i % B;
                    k = k * (B + 1) + j + 1;
                    for (uint32_t q = (uint32_t)h; q + 2 < height; q++) k *= (B + 1);
                    at(oh + l * p + i / B, i % B) = k * B < max_bucket ? at(ol + ll * p + k - 1, B - 1) : SST_MAX;
                }
        }
    }
    x->height = height;
    x->B = 16;
    x->N = 16;
    x->shift = shift;
    x->parts = (uint32_t)parts;
    x->bpp = COMPACT ? bpp : 0;
    // the search's root stride and first multiplier (:654-831): self.l1 = max(l1, 16) when OL
    x->root_stride = COMPACT ? bpp * 16 : OL ? (uint64_t)(16 - (overlap < 0 ? 0 : overlap)) : 16;
    x->l1_mul = COMPACT ? 0 : OL ? (l1 > 16 ? l1 : 16) : L1 ? l1 : 17;
    return 0;
}

// Eytzinger::new (sst/eytzinger.rs:37-63), iterative in-order fill.
static void build_eytzinger_host(const uint32_t* vals, uint64_t n, std::vector<uint32_t>& e) {
    e.assign(n + 1, 0);
    e[0] = 0xFFFFFFFFu;
    uint64_t i = 0, k = 1;
    std::vector<uint64_t> stack;
    while (k <= n || !stack.empty()) {
        while (k <= n) { stack.push_back(k); k *= 2; }
        k = stack.back();
        stack.pop_back();
        e[k] = vals[i++];
        k = 2 * k + 1;
    }
}

