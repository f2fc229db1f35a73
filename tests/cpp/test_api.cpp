// C++ host API (include/sas.hpp) against the CPU oracle, in the shape of the reference's own
// tests: sst/src/test.rs (every layout equals SortedVec over sizes and queries), the
// s_tree.rs KAT (1..2000 ++ [MAX]), and the SA lookups of sas/src/main.rs's lineup
// (binary_search, binary_search_batch<B>, interpolation_search<16>) query by query with
// their `cnt`.  The oracle (oracle/liboracle.so) is test infrastructure: it is the checker,
// never the thing run.  Exit status 0 = every check passed.  Built by the Makefile in this
// directory; run by tests/test_cpp_api.py on the GPU.
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "sas.hpp"

extern "C" {
void orc_random_string(uint64_t seed, uint64_t n, uint8_t* out);
int orc_build_sa(const uint8_t* t, uint64_t n, uint32_t* sa);
uint64_t orc_binary_search(const uint8_t* t, uint64_t n, const uint32_t* sa, const uint8_t* q, uint64_t m,
                           uint64_t* cnt);
uint64_t orc_interpolation_search(const uint8_t* t, uint64_t n, const uint32_t* sa, const uint8_t* q, uint64_t m,
                                  int K, uint64_t* cnt);
}

static int failures = 0;
#define EXPECT(cond, ...)                                  \
    do {                                                   \
        if (!(cond)) {                                     \
            failures++;                                    \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);             \
            std::fprintf(stderr, "\n");                    \
        }                                                  \
    } while (0)

static std::vector<uint8_t> pad(const uint8_t* p, size_t n, size_t extra = 256) {
    std::vector<uint8_t> v(p, p + n);
    v.resize(n + extra, 0);
    return v;
}

static void test_sa() {
    const size_t n = (1u << 18) + 77;
    const std::vector<uint8_t> t = sas::random_string(n);
    {  // the generator equals the oracle's restatement of random_string
        std::vector<uint8_t> o(n);
        orc_random_string(31415, n, o.data());
        EXPECT(o == t, "random_string differs from the oracle");
    }
    std::vector<uint32_t> osa(n);
    EXPECT(orc_build_sa(t.data(), n, osa.data()) == 0, "oracle SA");
    const std::vector<uint8_t> tp = pad(t.data(), n);
    const sas::SaNaive sa = sas::SaNaive::build(t);
    EXPECT(sa.n() == n, "n");
    for (size_t r : {size_t(0), size_t(1), n / 2, n - 1}) EXPECT(sa.sa(r) == osa[r], "sa[%zu]", r);

    // queries: main.rs's random_queries (len 30..100) + misses + edge cases
    std::vector<sas::Seq> qs = sas::random_queries(t, 3000);
    std::mt19937_64 rng(5);
    std::vector<std::vector<uint8_t>> own;
    for (int i = 0; i < 500; i++) {
        std::vector<uint8_t> q(rng() % 60);
        for (auto& c : q) c = rng() & 3;
        own.push_back(q);
    }
    own.push_back(std::vector<uint8_t>(40, 3));                            // above every suffix
    own.push_back({});                                                     // empty
    own.push_back(std::vector<uint8_t>(t.end() - 13, t.end()));            // a text-end suffix
    std::vector<uint8_t> tail(t.end() - 13, t.end());
    tail.push_back(0);
    tail.push_back(0);
    own.push_back(tail);  // the same + zeros (the A7 cmp edge case: slice order, as binary_search)
    for (auto& q : own) qs.emplace_back(q.data(), q.size());

    size_t cnt_plain = 0, cnt_oracle = 0, cnt_interp = 0, cnt_ointerp = 0, cnt_prefix = 0;
    for (const sas::Seq& q : qs) {
        const std::vector<uint8_t> qp = pad(q.ptr, q.len, 64);
        uint64_t c = 0, ci = 0;
        const uint64_t e = orc_binary_search(tp.data(), n, osa.data(), qp.data(), q.len, &c);
        const uint64_t ei = orc_interpolation_search(tp.data(), n, osa.data(), qp.data(), q.len, 16, &ci);
        cnt_oracle += c;
        cnt_ointerp += ci;
        size_t gc = 0, gi = 0;
        EXPECT(sas::binary_search(sa, q, gc) == e, "binary_search len %zu", q.len);
        EXPECT(gc == c, "binary_search cnt %zu vs %llu", gc, (unsigned long long)c);
        EXPECT(sas::interpolation_search<16>(sa, q, gi) == ei, "interpolation_search");
        EXPECT(gi == ci, "interpolation_search cnt %zu vs %llu", gi, (unsigned long long)ci);
        EXPECT(ei == e, "interpolation_search != binary_search");
        cnt_plain += gc;
        cnt_interp += gi;
    }
    // one batch of everything, and the reference's fixed-width batches
    std::vector<size_t> all = sa.search_many(qs, sas::Algo::Prefix, &cnt_prefix);
    for (size_t i = 0; i < 64; i++) {
        uint64_t c = 0;
        const std::vector<uint8_t> qp = pad(qs[i].ptr, qs[i].len, 64);
        EXPECT(all[i] == orc_binary_search(tp.data(), n, osa.data(), qp.data(), qs[i].len, &c), "prefix %zu", i);
    }
    std::array<sas::Seq, 64> b{};
    for (size_t i = 0; i < 64; i++) b[i] = qs[100 + i];
    size_t bc = 0;
    const auto got = sas::binary_search_batch<64>(sa, b, bc);
    for (size_t i = 0; i < 64; i++) EXPECT(got[i] == all[100 + i], "binary_search_batch %zu", i);
    // Search::search_prefix: every occurrence, checked by a scan of the text
    for (size_t i = 0; i < 20; i++) {
        const sas::Seq q = qs[i];
        std::vector<size_t> occ = sa.search_prefix(q);
        std::vector<size_t> scan;
        for (size_t p = 0; p + q.len <= n; p++)
            if (std::equal(q.ptr, q.ptr + q.len, t.begin() + p)) scan.push_back(p);
        std::sort(occ.begin(), occ.end());
        EXPECT(occ == scan, "search_prefix %zu: %zu vs %zu occurrences", i, occ.size(), scan.size());
    }
    {  // many ranges in one call equal the one-query calls
        const std::vector<sas::Seq> some(qs.begin(), qs.begin() + 300);
        const auto rs = sa.search_ranges(some);
        for (size_t i = 0; i < some.size(); i += 7) EXPECT(rs[i] == sa.search_range(some[i]), "search_ranges %zu", i);
        for (size_t i = 0; i < some.size(); i++) EXPECT(rs[i].second >= rs[i].first, "range order %zu", i);
    }
    EXPECT(sa.search(qs[0]) == all[0], "Search::search");
    {  // the configs[3] index (bucket lines, no SA array): the same positions, ranges and SA
        const sas::SaNaive lines = sas::SaNaive::build(t, sas::kLinesBuild);
        EXPECT(lines.default_algo() == sas::Algo::Tagged, "bucket lines default to TAGGED");
        EXPECT(lines.stats().tag_line_slots == 20, "20 slots a line");
        const std::vector<size_t> plain = sa.search_many(qs, sas::Algo::Plain);
        size_t lc = 0;
        EXPECT(lines.search_many(qs, sas::Algo::Tagged, &lc) == plain, "TAGGED on bucket lines != PLAIN");
        EXPECT(lines.search(qs[1]) == plain[1], "Search::search on bucket lines");
        const std::vector<sas::Seq> some(qs.begin(), qs.begin() + 300);
        EXPECT(lines.search_ranges(some) == sa.search_ranges(some), "bucket-line ranges");
        for (size_t r : {size_t(0), size_t(1), n / 3, n - 1}) EXPECT(lines.sa(r) == osa[r], "lines sa[%zu]", r);
        bool threw = false;
        try {
            lines.search_many(some, sas::Algo::Plain);
        } catch (const sas::Panic& e) {
            threw = e.code == ENOTSUP;
        }
        EXPECT(threw, "PLAIN on an index without an SA array must panic with ENOTSUP");
    }
    std::fprintf(stderr, "SA: %zu queries, cnt plain %zu (oracle %zu), interp %zu (oracle %zu), prefix %zu\n",
                 qs.size(), cnt_plain, cnt_oracle, cnt_interp, cnt_ointerp, cnt_prefix);
    sas::bench(sa, std::vector<sas::Seq>(qs.begin(), qs.begin() + 200), "binary_search (GPU)", sas::binary_search);
    sas::bench_batch(sa, qs, "search_many PREFIX");

    // error behaviour: the reference panics; here sas::Panic (EINVAL for a code > 3)
    bool threw = false;
    try {
        std::vector<uint8_t> bad = t;
        bad[10] = 7;
        sas::SaNaive::build(bad);
    } catch (const sas::Panic& e) {
        threw = e.code == EINVAL;
    }
    EXPECT(threw, "a text byte > 3 must panic with EINVAL");
}

template <class I>
static void same(const I& idx, const std::vector<uint32_t>& qs, const std::vector<uint32_t>& expect,
                 const char* name, size_t n) {
    EXPECT(idx.query(qs) == expect, "%s at n = %zu", name, n);
}

static void test_sst() {
    // sst/src/test.rs: sizes 2^6 .. 2^20 x {1, 5/4, 3/2, 7/4}, keys < i32::MAX with the MAX
    // sentinel, queries uniform; every layout returns SortedVec's values
    std::mt19937_64 rng(7);
    const uint32_t MAX = 0x7FFFFFFFu;
    for (size_t e = 6; e <= 20; e += 2) {
        for (size_t f : {4, 5, 6, 7}) {
            const size_t n = (size_t(1) << e) * f / 4;
            std::vector<uint32_t> vals(n);
            for (auto& v : vals) v = (uint32_t)(rng() % MAX);
            vals[0] = MAX;
            std::sort(vals.begin(), vals.end());
            std::vector<uint32_t> qs(1024);
            for (auto& q : qs) q = (uint32_t)(rng() % MAX);
            std::vector<uint32_t> expect(qs.size());
            for (size_t i = 0; i < qs.size(); i++) expect[i] = *std::lower_bound(vals.begin(), vals.end(), qs[i]);
            same(sst::SortedVec::new_(vals), qs, expect, "SortedVec", n);
            same(sst::Eytzinger::new_(vals), qs, expect, "Eytzinger", n);
            same(sst::STree16::new_(vals), qs, expect, "STree16", n);
            same(sst::STree16::new_params(vals, true, false, false), qs, expect, "STree16 left_max", n);
            same(sst::STree16::new_params(vals, false, true, false), qs, expect, "STree16 reverse", n);
            same(sst::STree16::new_params(vals, false, false, true), qs, expect, "STree16 full", n);
            same(sst::STree15::new_(vals), qs, expect, "STree15", n);
            if (n >= 4096) same(sst::PartitionedSTree16M::new_(vals, 8), qs, expect, "PartitionedSTree16M", n);
            // sst/test.rs:222-246: the other partitioned markers
            for (uint32_t b : {0u, 8u, 16u}) {
                same(sst::PartitionedSTree16::new_(vals, b), qs, expect, "PartitionedSTree16", n);
                same(sst::PartitionedSTree16C::new_(vals, b), qs, expect, "PartitionedSTree16C", n);
                same(sst::PartitionedSTree16L::new_(vals, b), qs, expect, "PartitionedSTree16L", n);
                same(sst::PartitionedSTree16O::new_(vals, b), qs, expect, "PartitionedSTree16O", n);
            }
            same(sst::DirectMap::new_(vals), qs, expect, "DirectMap", n);
        }
    }
    // s_tree.rs:861-885: STree over 1..2000 ++ [MAX]: the first key >= q
    std::vector<uint32_t> vals;
    for (uint32_t i = 1; i < 2000; i++) vals.push_back(i);
    vals.push_back(MAX);
    const auto st = sst::STree16::new_(vals);
    for (uint32_t q : {0u, 1u, 2u, 1000u, 1999u, 2000u, 2001u, 5000u}) {
        const uint32_t e = q == 0 ? 1 : (q < 2000 ? q : MAX);
        EXPECT(st.query_one(q) == e, "STree16 KAT q = %u", q);
    }
    EXPECT(st.layers() >= 2 && st.size() > vals.size() * 4, "STree16 size/layers");
}

int main() {
    test_sa();
    test_sst();
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("cpp api ok\n");
    return 0;
}
