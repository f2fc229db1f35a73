/* sas.hpp -- C++17 host-side mirror of the reference's Rust query API over the C ABI
 * (sas.h, sst.h).  Header only; link libsas_amd.so.  The reference is compiled Rust, so the
 * host side above the ABI is compiled C++ with the reference's names and argument meaning:
 *
 *   sas::SaNaive::build(t)                SaNaive::build              sas/sa_search.rs:30-57
 *   sas::binary_search(sa, q, cnt)        binary_search (type F1)     sas/sa_search.rs:98-112, :453
 *   sas::binary_search_batch<B>(sa,qs,cnt) binary_search_batch<B> (F<B>) sas/sa_search.rs:157-196, :454
 *   sas::interpolation_search<16>(sa,q,cnt) interpolation_search<K>   sas/sa_search.rs:376-421
 *   sas::bench / sas::bench_batch         bench / bench_batch         sas/sa_search.rs:423-451
 *   SaNaive::search / search_prefix       Search::search/_prefix      sas/util.rs:29-47
 *   sas::random_string / random_queries   util.rs:9-26 (ChaCha8Rng::seed_from_u64(31415), main.rs:38)
 *   sas::read_fasta_file                  util.rs:144-169
 *   sst::SortedVec / Eytzinger / STree16 / STree15 / PartitionedSTree16M / DirectMap /
 *   PartitionedSTree16 / 16C / 16L / 16O
 *                                         SearchIndex::new/size/layers + SearchScheme::query
 *                                         sst/lib.rs:30-57, s_tree.rs:72-176, eytzinger.rs, binary_search.rs
 *
 * Every lookup runs on the GPU: host slices go through the library's pinned staging
 * pipeline.  Differences that the GPU makes worth having: `search_many` takes any number of
 * queries (no `array_chunks` remainder is dropped, sas/sa_search.rs:441), and a lower bound
 * of n returns the sentinel position n where the reference reads sa[n] out of bounds.
 *
 * Error behaviour: the reference panics with panic = "abort" (Cargo.toml:12).  Here a
 * non-zero status throws sas::Panic (a std::runtime_error carrying sas_last_error()); left
 * uncaught it terminates the process as the reference's panic does.
 */
#ifndef SAS_HPP
#define SAS_HPP

#include <array>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sas.h"
#include "sst.h"

namespace sas {

/* &[u8]: byte codes 0..3 (the reference's Seq = [u8], sas/util.rs:5-6) */
struct Seq {
    const uint8_t* ptr = nullptr;
    size_t len = 0;
    Seq() = default;
    Seq(const uint8_t* p, size_t n) : ptr(p), len(n) {}
    Seq(const std::vector<uint8_t>& v) : ptr(v.data()), len(v.size()) {}  // NOLINT: as &v[..]
    Seq slice(size_t a, size_t b) const { return Seq(ptr + a, b - a); }   // &t[a..b]
    size_t size() const { return len; }
};

struct Panic : std::runtime_error {
    int code;
    Panic(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc) {
    if (rc != 0) throw Panic(rc, std::string("libsas_amd: ") + sas_last_error());
}

enum class Algo : int {
    Plain = SAS_ALGO_PLAIN,
    Lcp = SAS_ALGO_LCP,
    STree = SAS_ALGO_STREE,
    Sector = SAS_ALGO_SECTOR,
    Quad = SAS_ALGO_QUAD,
    Inline = SAS_ALGO_INLINE,
    Llcp = SAS_ALGO_LLCP,
    Prefix = SAS_ALGO_PREFIX,
    Interp = SAS_ALGO_INTERP,
    Tagged = SAS_ALGO_TAGGED,
    StreeLlcp = SAS_ALGO_STREE_LLCP,
    QuadLlcp = SAS_ALGO_QUAD_LLCP,
};

/* build flags of SaNaive::build: the LCP array, the fused quad tree and the p = 16 prefix
 * table with two-suffix inline entries (the fastest lookup at n = 2^30) */
constexpr uint32_t kDefaultBuild = SAS_BUILD_LCP | SAS_BUILD_QUAD | SAS_BUILD_PREFIX | SAS_BUILD_PREFIX_INLINE2;
/* the configs[3] index (long texts, long ragged queries): tagged entries in 128-B bucket
 * lines, no SA array; it answers Algo::Tagged lookups, ranges and sa(rank) */
constexpr uint32_t kLinesBuild = SAS_BUILD_TAGGED | SAS_BUILD_TAG_LINES;

/* GPU-resident replacement for SaNaive<'t> (sas/sa_search.rs:11-19): the packed text, the
 * SA and the search structures live in HBM; the caller keeps its text. */
class SaNaive {
   public:
    /* SaNaive::build(t) (sas/sa_search.rs:30-57): SA built and verified on the GPU */
    static SaNaive build(Seq t, uint32_t flags = kDefaultBuild) {
        sas_index* h = nullptr;
        if (t.len >= 0xFFFFFFFFull) flags &= ~(uint32_t)SAS_BUILD_PREFIX_INLINE2;  // 40-bit SA: rank table
        check(sas_build(t.ptr, t.len, nullptr, 4, flags | SAS_BUILD_VERIFY, &h));
        const Algo a = (flags & SAS_BUILD_TAGGED) ? Algo::Tagged : (flags & SAS_BUILD_PREFIX) ? Algo::Prefix : Algo::Plain;
        return SaNaive(h, t.len, a);
    }
    SaNaive(SaNaive&& o) noexcept : h_(o.h_), n_(o.n_), algo_(o.algo_) { o.h_ = nullptr; }
    SaNaive& operator=(SaNaive&& o) noexcept {
        std::swap(h_, o.h_);
        std::swap(n_, o.n_);
        std::swap(algo_, o.algo_);
        return *this;
    }
    SaNaive(const SaNaive&) = delete;
    SaNaive& operator=(const SaNaive&) = delete;
    ~SaNaive() {
        if (h_) sas_free(h_);
    }

    size_t n() const { return n_; }
    /* the fastest lookup the build flags made possible: Tagged (SAS_BUILD_TAGGED), Prefix
     * (SAS_BUILD_PREFIX), else Plain; Search::search uses it */
    Algo default_algo() const { return algo_; }
    const sas_index* raw() const { return h_; }
    sas_stats stats() const {
        sas_stats s{};
        check(sas_get_stats(h_, &s));
        return s;
    }

    /* sa[rank] (SaNaive::suffix_at's position, sas/sa_search.rs:79-81) */
    uint64_t sa(uint64_t rank) const {
        uint64_t v = 0;
        check(sas_copy_sa64(h_, rank, 1, &v, 0));
        return v;
    }

    /* one batched lookup of any number of queries; cnt += the reference's probe counter */
    std::vector<size_t> search_many(const std::vector<Seq>& qs, Algo algo, size_t* cnt = nullptr,
                                    uint32_t flags = 0) const {
        std::vector<uint8_t> bytes;
        std::vector<uint64_t> off(qs.size());
        std::vector<uint32_t> len(qs.size());
        size_t total = 0;
        for (size_t i = 0; i < qs.size(); i++) total += qs[i].len;
        bytes.reserve(total + 64);
        for (size_t i = 0; i < qs.size(); i++) {
            off[i] = bytes.size();
            len[i] = (uint32_t)qs[i].len;
            bytes.insert(bytes.end(), qs[i].ptr, qs[i].ptr + qs[i].len);
        }
        bytes.resize(total + 64, 0);
        std::vector<uint64_t> pos(qs.size());
        std::vector<uint32_t> probes(cnt ? qs.size() : 0);
        if (!qs.empty())
            check(sas_search_batch(h_, bytes.data(), off.data(), len.data(), qs.size(), (int)algo, pos.data(),
                                   cnt ? probes.data() : nullptr, nullptr, flags));
        if (cnt)
            for (uint32_t p : probes) *cnt += p;
        return std::vector<size_t>(pos.begin(), pos.end());
    }

    /* Search::search (sas/util.rs:34): position of the smallest suffix >= q (n if none) */
    size_t search(Seq q) const {
        size_t c = 0;
        return search_many({q}, algo_, &c)[0];
    }

    /* occurrence range: global SA ranks [lo, hi) of the suffixes starting with q */
    std::pair<uint64_t, uint64_t> search_range(Seq q) const {
        const std::vector<uint8_t> b = padded(q);
        const uint64_t off = 0;
        const uint32_t len = (uint32_t)q.len;
        uint64_t lo = 0, hi = 0;
        check(sas_search_range(h_, b.data(), &off, &len, 1, &lo, &hi, nullptr, 0));
        return {lo, hi};
    }

    /* occurrence ranges of many queries in one call (the staged host pipeline) */
    std::vector<std::pair<uint64_t, uint64_t>> search_ranges(const std::vector<Seq>& qs, uint32_t flags = 0) const {
        std::vector<uint8_t> bytes;
        std::vector<uint64_t> off(qs.size()), lo(qs.size()), hi(qs.size());
        std::vector<uint32_t> len(qs.size());
        for (size_t i = 0; i < qs.size(); i++) {
            off[i] = bytes.size();
            len[i] = (uint32_t)qs[i].len;
            bytes.insert(bytes.end(), qs[i].ptr, qs[i].ptr + qs[i].len);
        }
        bytes.resize(bytes.size() + 64, 0);
        if (!qs.empty())
            check(sas_search_range(h_, bytes.data(), off.data(), len.data(), qs.size(), lo.data(), hi.data(), nullptr,
                                   flags));
        std::vector<std::pair<uint64_t, uint64_t>> r(qs.size());
        for (size_t i = 0; i < qs.size(); i++) r[i] = {lo[i], hi[i]};
        return r;
    }

    /* Search::search_prefix (sas/util.rs:36-40, unimplemented!() upstream): every text
     * position where q occurs, in SA order */
    std::vector<size_t> search_prefix(Seq q) const {
        const auto r = search_range(q);
        std::vector<uint64_t> v(r.second - r.first);
        if (!v.empty()) check(sas_copy_sa64(h_, r.first, v.size(), v.data(), 0));
        return std::vector<size_t>(v.begin(), v.end());
    }

   private:
    SaNaive(sas_index* h, size_t n, Algo a) : h_(h), n_(n), algo_(a) {}
    static std::vector<uint8_t> padded(Seq q) {
        std::vector<uint8_t> b(q.ptr, q.ptr + q.len);
        b.resize(q.len + 64, 0);
        return b;
    }
    sas_index* h_ = nullptr;
    size_t n_ = 0;
    Algo algo_ = Algo::Prefix;
};

/* type F1 (sas/sa_search.rs:453): binary_search (:98-112), the canonical lookup: the
 * position of the lower bound of q under slice order; cnt counts loop iterations */
inline size_t binary_search(const SaNaive& sa, Seq q, size_t& cnt) { return sa.search_many({q}, Algo::Plain, &cnt)[0]; }

/* the same positions from the fastest GPU structure (PREFIX: the prefix table made live);
 * cnt counts as binary_search's does from the table's range (1 + iterations) */
inline size_t prefix_search(const SaNaive& sa, Seq q, size_t& cnt) { return sa.search_many({q}, Algo::Prefix, &cnt)[0]; }

/* interpolation_search<K> (sas/sa_search.rs:376-421), K = 16 as main.rs:97 runs it */
template <size_t K = 16>
inline size_t interpolation_search(const SaNaive& sa, Seq q, size_t& cnt) {
    static_assert(K == 16, "the GPU kernel restates interpolation_search<16>");
    return sa.search_many({q}, Algo::Interp, &cnt)[0];
}

/* type F<B> (sas/sa_search.rs:454): binary_search_batch<B> (:157-196) */
template <size_t B>
inline std::array<size_t, B> binary_search_batch(const SaNaive& sa, const std::array<Seq, B>& qs, size_t& cnt) {
    const auto v = sa.search_many(std::vector<Seq>(qs.begin(), qs.end()), Algo::Plain, &cnt);
    std::array<size_t, B> out{};
    for (size_t i = 0; i < B; i++) out[i] = v[i];
    return out;
}

using F1 = size_t (*)(const SaNaive&, Seq, size_t&);

/* bench (sas/sa_search.rs:423-436): time f over the queries, print name, total, per query,
 * per probe, probes per query to stderr; returns the elapsed seconds */
inline double bench(const SaNaive& sa, const std::vector<Seq>& queries, const char* name, F1 f) {
    const auto t0 = std::chrono::steady_clock::now();
    size_t cnt = 0;
    for (const Seq& q : queries) f(sa, q, cnt);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "%-20s: %8.2fs %6.0fns %6.0fns %5.2f\n", name, s, s * 1e9 / queries.size(),
                 s * 1e9 / (cnt ? cnt : 1), (double)cnt / queries.size());
    return s;
}

/* bench_batch (sas/sa_search.rs:438-451), except that the whole query list is one GPU
 * batch (the reference's array_chunks::<B> drops the remainder) */
inline double bench_batch(const SaNaive& sa, const std::vector<Seq>& queries, const char* name,
                          Algo algo = Algo::Prefix) {
    const auto t0 = std::chrono::steady_clock::now();
    size_t cnt = 0;
    sa.search_many(queries, algo, &cnt);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "%-20s: %8.2fs %6.0fns %6.0fns %5.2f\n", name, s, s * 1e9 / queries.size(),
                 s * 1e9 / (cnt ? cnt : 1), (double)cnt / queries.size());
    return s;
}

/* random_string (sas/util.rs:9-15) with ChaCha8Rng::seed_from_u64(seed) */
inline std::vector<uint8_t> random_string(size_t n, uint64_t seed = 31415) {
    std::vector<uint8_t> t(n);
    if (n) check(sas_gen_text(seed, n, t.data(), 0));
    return t;
}

/* random_queries (sas/util.rs:18-26): substrings t[i..i+len], i < n - margin, len in
 * [len_lo, len_hi); the ChaCha8 stream continues after the text's n words */
inline std::vector<Seq> random_queries(Seq t, size_t nq, uint64_t seed = 31415, uint32_t len_lo = 30,
                                       uint32_t len_hi = 100, uint64_t margin = 200) {
    std::vector<uint64_t> off(nq);
    std::vector<uint32_t> len(nq);
    if (nq) check(sas_gen_queries(seed, t.len, t.len, nq, margin, len_lo, len_hi, off.data(), len.data(), nullptr));
    std::vector<Seq> qs(nq);
    for (size_t i = 0; i < nq; i++) qs[i] = t.slice(off[i], off[i] + len[i]);
    return qs;
}

/* read_fasta_file (sas/util.rs:144-169): A/C/G/T/a/c/g/t -> 0..3, every other byte -> 0 */
inline std::vector<uint8_t> read_fasta_file(const std::string& path) {
    uint64_t n = 0;
    check(sas_read_fasta(path.c_str(), nullptr, 0, &n));
    std::vector<uint8_t> v(n);
    check(sas_read_fasta(path.c_str(), v.data(), n, &n));
    v.resize(n);
    return v;
}

}  // namespace sas

namespace sst {

using sas::check;

/* SearchIndex (sst/lib.rs:30-48) over sorted u32 keys: new / size / layers, and query
 * (SearchScheme::query, :55-57): the first key >= q for every query (u32::MAX if none for
 * Eytzinger and SortedVec, as upstream; the S-trees need the MAX sentinel the reference's
 * tests push, sst/s_tree.rs:864) */
class SearchIndex {
   public:
    SearchIndex(SearchIndex&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    SearchIndex& operator=(SearchIndex&& o) noexcept {
        std::swap(h_, o.h_);
        return *this;
    }
    SearchIndex(const SearchIndex&) = delete;
    ~SearchIndex() {
        if (h_) sst_free(h_);
    }
    size_t size() const { return (size_t)sst_size(h_); }
    size_t layers() const { return (size_t)sst_layers(h_); }
    std::vector<uint32_t> query(const std::vector<uint32_t>& qs) const {
        std::vector<uint32_t> out(qs.size());
        if (!qs.empty()) check(sst_query(h_, qs.data(), qs.size(), out.data(), nullptr, nullptr, 0));
        return out;
    }
    uint32_t query_one(uint32_t q) const { return query({q})[0]; }
    /* the leaf slot of each answer (the rank the SA use of the tree needs) */
    std::vector<uint64_t> ranks(const std::vector<uint32_t>& qs) const {
        std::vector<uint32_t> v(qs.size());
        std::vector<uint64_t> r(qs.size());
        if (!qs.empty()) check(sst_query(h_, qs.data(), qs.size(), v.data(), r.data(), nullptr, 0));
        return r;
    }

   protected:
    static sst_index* make(const std::vector<uint32_t>& vals, int layout, uint32_t flags) {
        sst_index* h = nullptr;
        check(sst_build(vals.data(), vals.size(), layout, flags, &h));
        return h;
    }
    explicit SearchIndex(sst_index* h) : h_(h) {}
    sst_index* h_ = nullptr;
};

struct SortedVec : SearchIndex {  // sst/binary_search.rs:8-49
    static SortedVec new_(const std::vector<uint32_t>& v) { return SortedVec(make(v, SST_SORTED, 0)); }
    using SearchIndex::SearchIndex;
};
struct Eytzinger : SearchIndex {  // sst/eytzinger.rs:9-180
    static Eytzinger new_(const std::vector<uint32_t>& v) { return Eytzinger(make(v, SST_EYTZINGER, 0)); }
    using SearchIndex::SearchIndex;
};
template <int LAYOUT>
struct STree : SearchIndex {  // sst/s_tree.rs:14-20: STree16 = STree<16,16>, STree15 = STree<15,16>
    /* SearchIndex::new = new_params(vals, false, false, false) (s_tree.rs:48-50) */
    static STree new_(const std::vector<uint32_t>& v) { return new_params(v, false, false, false); }
    /* STree::new_params (s_tree.rs:72-176) */
    static STree new_params(const std::vector<uint32_t>& v, bool left_max, bool reverse, bool full) {
        const uint32_t f = (left_max ? SST_LEFT_MAX : 0) | (reverse ? SST_REVERSE : 0) | (full ? SST_FULL : 0);
        return STree(make(v, LAYOUT, f));
    }
    using SearchIndex::SearchIndex;
};
using STree16 = STree<SST_STREE16>;
using STree15 = STree<SST_STREE15>;
struct PartitionedSTree16M : SearchIndex {  // sst/partitioned_s_tree.rs:98
    static PartitionedSTree16M new_(const std::vector<uint32_t>& v, uint32_t b) {
        return PartitionedSTree16M(make(v, SST_PARTITIONED_MAP, SST_PART_BITS(b)));
    }
    using SearchIndex::SearchIndex;
};
/* PartitionedSTree<16,16,Tp>::new(vals, b) for Tp = Simple, Compact, L1, Overlapping
   (sst/partitioned_s_tree.rs:86-94 type aliases; values only: the leaves are padded) */
template <int LAYOUT>
struct PartitionedSTree : SearchIndex {
    static PartitionedSTree new_(const std::vector<uint32_t>& v, uint32_t b) {
        return PartitionedSTree(make(v, LAYOUT, SST_PART_BITS(b)));
    }
    using SearchIndex::SearchIndex;
};
using PartitionedSTree16 = PartitionedSTree<SST_PARTITIONED>;
using PartitionedSTree16C = PartitionedSTree<SST_PARTITIONED_COMPACT>;
using PartitionedSTree16L = PartitionedSTree<SST_PARTITIONED_L1>;
using PartitionedSTree16O = PartitionedSTree<SST_PARTITIONED_OVERLAP>;
struct DirectMap : SearchIndex {  // the prefix map taken to its limit (sst.h SST_DIRECT_MAP)
    static DirectMap new_(const std::vector<uint32_t>& v) { return DirectMap(make(v, SST_DIRECT_MAP, 0)); }
    using SearchIndex::SearchIndex;
};

}  // namespace sst

#endif /* SAS_HPP */
