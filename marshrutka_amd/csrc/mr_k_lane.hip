// mr_k_lane.hip — the hub solver with one source per lane (hub_lane_kernel, mr_hub_lane.hpp)
// for the six comparator permutations; host-side launch helpers called from mr_host.cpp.
#include "mr_hub_lane.hpp"

namespace mr {

template <uint32_t TM>
static const void *lane_fn_tm(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_lane_kernel<5, TM>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_lane_kernel<7, TM>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_lane_kernel<11, TM>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_lane_kernel<15, TM>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_lane_kernel<19, TM>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_lane_kernel<21, TM>);  // time money legs
        default: return nullptr;
    }
}

// table entries (NS + 1) the lane kernel holds in registers; 0 = not applicable.  One
// size: 22 entries (Center, 4 border-1 cells, 16 campfires + HQ or 17 campfires) fit
// the 256-VGPR budget of two waves per SIMD; a 24- or 32-entry table spills (17 /
// 205 VGPRs with the current loop), so those plans stay on hub_kernel.
uint32_t hub_lane_entries(uint32_t NS) { return NS + 1 <= 22 ? 22u : 0u; }

static const void *lane_fn(const uint32_t perm[3], uint32_t NS) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    return hub_lane_entries(NS) == 22 ? lane_fn_tm<22>(k) : nullptr;
}

uint32_t hub_lane_lds_bytes(uint32_t NS, uint32_t nreg) {
    return lane_lds_total(NS, nreg, hub_lane_entries(NS));
}

hipError_t launch_hub_lane(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t n_lane,
                           hipStream_t stream) {
    const void *fn = lane_fn(perm, NS);
    if (!fn) return hipErrorInvalidValue;
    const uint32_t bytes = hub_lane_lds_bytes(NS, nreg);
    const uint32_t waves = (n_lane + 63u) / 64u, blocks = (waves + 3u) / 4u;
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks ? blocks : 1u), dim3(kBS), args, bytes, stream);
}

}  // namespace mr
