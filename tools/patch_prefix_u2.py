# A/B patch (not kept): two queries per lane pair and iteration in k_sa_prefix2; applied to a
# package copy by: python3 tools/patch_prefix_u2.py <copy>/csrc/sas_search.hip, built with -DSAS_PREFIX_U2=1
# (tools/gpu_ab_u2.sh; profiles/r3/ab_prefix_u2/: 0.305-0.307 against 0.293-0.300 ms per 10^7)
import sys
p=sys.argv[1]
s=open(p).read()
anchor='''template <int QW, int G, bool HI40 = false>
__global__ __launch_bounds__(SEARCH_BLOCK, 8) void k_sa_prefix2(SearchArgs a) {'''
assert anchor in s
u2='''#ifndef SAS_PREFIX_U2
#define SAS_PREFIX_U2 0
#endif
// the headline shape (fixed 32-char byte queries, 16-B aligned, a lane pair per query, no
// HI40): two queries per pair and iteration, their table entries loaded back to back, so a
// wave keeps twice the random requests in flight
template <int G>
__device__ __forceinline__ void prefix2_u2(const SearchArgs& a, uint32_t* bad_out) {
    uint32_t bad = 0;
    const uint32_t sh = 64 - 2 * a.prefix_chars;
    const uint64_t sa_n = a.sa_n;
    const uint32_t sub = threadIdx.x & (G - 1);
    const int lane0 = (int)((threadIdx.x & 63) & ~(uint32_t)(G - 1));
    const uint4* pt = reinterpret_cast<const uint4*>(a.prefix);
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) / G;
    auto qload = [&](uint64_t k) -> uint4 {
        const uint4* p = reinterpret_cast<const uint4*>(a.qbytes + k * 32) + sub;
        return SAS_QUAD_NT_IO ? nt_load4(p) : *p;
    };
    auto key_of = [&](uint4 v) -> uint64_t {
        bad |= (v.x | v.y | v.z | v.w) & 0xFCFCFCFCu;
        const uint32_t part = (pack4(v.x) << 24) | (pack4(v.y) << 16) | (pack4(v.z) << 8) | pack4(v.w);
        const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)part, 0xB1, 0xF, 0xF, false);
        return sub ? (((uint64_t)other << 32) | part) : (((uint64_t)part << 32) | other);
    };
    auto finish = [&](uint64_t i, uint4 e, uint64_t K64) {
        QueryRegs<1> q;
        q.bytes = a.qbytes + i * 32;
        q.m = 32;
        q.w[0] = K64;
        const uint64_t K = K64 >> sh;
        const uint64_t r0 = (uint32_t)__shfl((int)e.z, lane0, 64);
        const uint64_t rank = r0 + sub;
        const bool ok = rank >= sa_n || sector_ge<1>((uint64_t)e.x | ((uint64_t)e.y << 32), (uint64_t)e.w, K64, a, q);
        const uint32_t grp = (uint32_t)(__ballot(ok) >> lane0) & ((1u << G) - 1u);
        const uint32_t j = grp ? (uint32_t)__builtin_ctz(grp) : 0u;
        const uint32_t pw = (uint32_t)__shfl((int)e.w, lane0 + (int)j, 64);
        uint64_t ans, pos;
        if (grp) {
            ans = r0 + j;
            pos = ans >= sa_n ? a.next_pos : pw;
        } else {
            uint64_t lo = r0 + G, hi = pt[G * (K + 1)].z, pr = QUAD_NO_SA;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                const uint4 f = SAS_PREFIX_NT ? nt_load4(a.quad_leaves + mid) : a.quad_leaves[mid];
                const uint64_t pp = (uint64_t)f.z | ((uint64_t)(f.w & 0xFFu) << 32);
                if (sector_ge<1>((uint64_t)f.x | ((uint64_t)f.y << 32), pp, K64, a, q)) {
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
            a.out_pos[i] = pos;
            if (a.out_probes) {
                uint32_t probes = 1;
                for (uint64_t l2 = r0, h2 = pt[G * (K + 1)].z; l2 < h2; probes++) {
                    const uint64_t mid = (l2 + h2) >> 1;
                    if (mid < ans) l2 = mid + 1;
                    else h2 = mid;
                }
                a.out_probes[i] = probes;
            }
        }
    };
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; i < a.nq; i += 2 * stride) {
        const uint64_t i1 = i + stride;
        const bool has1 = i1 < a.nq;  // uniform over the pair
        const uint4 v0 = qload(i);
        const uint4 v1 = has1 ? qload(i1) : make_uint4(0, 0, 0, 0);
        const uint64_t k0 = key_of(v0), k1 = key_of(v1);
        const uint4 e0 = SAS_PREFIX_NT ? nt_load4(pt + G * (k0 >> sh) + sub) : pt[G * (k0 >> sh) + sub];
        uint4 e1 = make_uint4(0, 0, 0, 0);
        if (has1) e1 = SAS_PREFIX_NT ? nt_load4(pt + G * (k1 >> sh) + sub) : pt[G * (k1 >> sh) + sub];
        finish(i, e0, k0);
        if (has1) finish(i1, e1, k1);
    }
    *bad_out |= bad;
}

'''
s=s.replace(anchor,u2+anchor)
old='''    const bool split = SAS_PREFIX_SPLITQ && G == 2 && QW == 1 && a.qoff == nullptr && a.qwords == nullptr &&
                       a.m_fixed == 32 && a.bcounts == nullptr &&
                       (((uintptr_t)a.qbytes) & 15) == 0;'''
assert old in s
s=s.replace(old,old+'''
    if (SAS_PREFIX_U2 && split && !HI40) {
        prefix2_u2<G>(a, &bad);
        if (bad) atomicOr(a.bad, 1u);
        return;
    }''')
open(p,'w').write(s)
