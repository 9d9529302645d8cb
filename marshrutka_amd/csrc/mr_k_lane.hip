// mr_k_lane.hip — the hub solver with one source per lane (hub_lane_kernel, mr_hub_lane.hpp)
// for the six comparator permutations; host-side launch helpers called from mr_host.cpp.
#include "mr_hub_lane.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mr {

// the kernel of each comparator permutation, per table size: 22 here, 24 and 32 in
// mr_k_lane24.hip / mr_k_lane32.hip
template <uint32_t TM>
const void *lane_fn_tm(uint32_t perm);
template <>
const void *lane_fn_tm<24>(uint32_t perm);
template <>
const void *lane_fn_tm<32>(uint32_t perm);
// Fleetfoot 1..3 (hub_lane_kernel<PERM, TM, true>): mr_k_lane_nl.hip, mr_k_lane_nl2.hip
template <uint32_t TM>
const void *lane_nl_fn_tm(uint32_t perm);
template <>
const void *lane_nl_fn_tm<22>(uint32_t perm);
template <>
const void *lane_nl_fn_tm<24>(uint32_t perm);
template <>
const void *lane_nl_fn_tm<32>(uint32_t perm);

template <>
const void *lane_fn_tm<22>(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_lane_kernel<5, 22>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_lane_kernel<7, 22>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_lane_kernel<11, 22>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_lane_kernel<15, 22>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_lane_kernel<19, 22>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_lane_kernel<21, 22>);  // time money legs
        default: return nullptr;
    }
}


// table entries (NS + 1) the lane kernel holds in registers; 0 = not applicable.  22
// entries (Center, 4 border-1 cells, 16 campfires + HQ or 17 campfires) run at two
// waves per SIMD, 24 and 32 at one (lane_waves)
uint32_t hub_lane_entries(uint32_t NS) { return NS + 1 <= 22 ? 22u : (NS + 1 <= 24 ? 24u : (NS + 1 <= 32 ? 32u : 0u)); }

static const void *lane_fn(const uint32_t perm[3], uint32_t NS, bool nonlin) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    switch (hub_lane_entries(NS)) {
        case 22: return nonlin ? lane_nl_fn_tm<22>(k) : lane_fn_tm<22>(k);
        case 24: return nonlin ? lane_nl_fn_tm<24>(k) : lane_fn_tm<24>(k);
        case 32: return nonlin ? lane_nl_fn_tm<32>(k) : lane_fn_tm<32>(k);
        default: return nullptr;
    }
}

// The lane and group kernels' per-plan LDS block for a table of TM entries (layout:
// lane_off_* in mr_hub_lane.hpp): the specials' records, their rows of the grid's region
// table, the pair table of walks / caravans / SoE-region candidates and its row masks
// (LaneHub::from_s), the specials' cells by hash, and the header words.  near_sp holds the
// specials' rows of the grid's region table ({distance, rank} per special t and region, at
// 2 * (t * nreg + r)).  Walk times are the Fleetfoot ceil of 180 s a leg (ff_num / ff_den;
// 1 / 1 without).  Returns the byte size.
uint32_t lane_blob_build(const SpecialStatic *sp, uint32_t NS, uint32_t nreg, uint32_t TM, uint32_t rgt,
                         uint32_t ff_num, uint32_t ff_den, const uint32_t *near_sp, std::vector<uint32_t> &blob) {
    auto run_time = [&](uint32_t k) { return uint32_t((180ull * k * ff_num + ff_den - 1) / ff_den); };
    const uint32_t bytes = lane_blob_bytes(NS, nreg, TM);
    blob.assign(bytes / 4, 0u);
    char *base = reinterpret_cast<char *>(blob.data());
    std::memcpy(base, sp, (NS + 1) * sizeof(SpecialStatic));
    uint2 *nearl = reinterpret_cast<uint2 *>(base + lane_off_near(NS));
    for (uint32_t t = 1; t <= NS; ++t)
        for (uint32_t r = 0; r < nreg; ++r) {
            const uint32_t *e = near_sp + 2ull * ((unsigned long long)t * nreg + r);
            nearl[t * nreg + r] = make_uint2(e[0], e[1]);
        }
    uint4 *pa = reinterpret_cast<uint4 *>(base + lane_off_pt(NS, nreg));
    uint2 *pb = reinterpret_cast<uint2 *>(base + lane_off_pb(NS, nreg, TM));
    uint32_t *rm = reinterpret_cast<uint32_t *>(base + lane_off_rm(NS, nreg, TM));
    for (uint32_t s = 1; s <= NS && s < TM; ++s)
        for (uint32_t t = 1; t <= NS && t < TM; ++t) {
            const SpecialStatic &ss = sp[s], &st = sp[t];
            const uint32_t wd = walk_dist(ss.x, ss.y, st.x, st.y);
            const uint32_t md = uint32_t(std::abs(ss.x - st.x) + std::abs(ss.y - st.y));
            pa[s * TM + t] = make_uint4(wd, run_time(wd), (st.coef5 ? 5u : 2u) * md, rgt * md);
            if (st.rid != kNone10) {
                const uint32_t d = nearl[s * nreg + st.rid].x;
                if (d != kNone32) {
                    pb[s * TM + t] = make_uint2(d, run_time(d));
                    if (d != 0) rm[s] |= 1u << t;
                }
            }
        }
    uint2 *ht = reinterpret_cast<uint2 *>(base + lane_off_hash(NS, nreg, TM));
    for (uint32_t h = 0; h < kLaneHash; ++h) ht[h] = make_uint2(kNone32, kNone10);
    uint32_t probes = 1, hubm = 0, c5m = 0, regm = 0;
    for (uint32_t t = 1; t <= NS && t < TM; ++t) {
        uint32_t h = lane_hash(sp[t].v), k = 1;
        while (ht[h].x != kNone32) {
            h = (h + 1u) & (kLaneHash - 1u);
            ++k;
        }
        ht[h] = make_uint2(sp[t].v, t);
        probes = std::max(probes, k);
        hubm |= (sp[t].flags & kSpHub) ? (1u << t) : 0u;
        c5m |= sp[t].coef5 ? (1u << t) : 0u;
        regm |= sp[t].rid != kNone10 ? (1u << t) : 0u;
    }
    *reinterpret_cast<uint4 *>(base + lane_off_hdr(NS, nreg, TM)) = make_uint4(probes, hubm, c5m, regm);
    return bytes;
}

// (the lane kernel's LDS: the lane kernels' block and meta copy, then its per-wave
// candidate metas, LaneHub::MC)
uint32_t hub_lane_lds_bytes(uint32_t NS, uint32_t nreg) {
    const uint32_t TM = hub_lane_entries(NS);
    return lane_lds_total(NS, nreg, TM) + (kBS / 64) * TM * 64u * 4u;
}

hipError_t launch_hub_lane(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t n_lane,
                           bool nonlin, hipStream_t stream) {
    const void *fn = lane_fn(perm, NS, nonlin);
    if (!fn) return hipErrorInvalidValue;
    const uint32_t bytes = hub_lane_lds_bytes(NS, nreg);
    if (bytes > 64u * 1024u) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    const uint32_t waves = (n_lane + 63u) / 64u, blocks = (waves + 3u) / 4u;
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks ? blocks : 1u), dim3(kBS), args, bytes, stream);
}

}  // namespace mr
