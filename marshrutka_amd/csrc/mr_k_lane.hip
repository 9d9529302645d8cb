// mr_k_lane.hip — the hub solver with one source per lane (hub_lane_kernel, mr_hub_lane.hpp)
// for the six comparator permutations; host-side launch helpers called from mr_host.cpp.
#include "mr_hub_lane.hpp"

namespace mr {

// the kernel of each comparator permutation, per table size: 22 here, 24 and 32 in
// mr_k_lane24.hip / mr_k_lane32.hip
template <uint32_t TM>
const void *lane_fn_tm(uint32_t perm);
template <>
const void *lane_fn_tm<24>(uint32_t perm);
template <>
const void *lane_fn_tm<32>(uint32_t perm);

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

static const void *lane_fn(const uint32_t perm[3], uint32_t NS) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    switch (hub_lane_entries(NS)) {
        case 22: return lane_fn_tm<22>(k);
        case 24: return lane_fn_tm<24>(k);
        case 32: return lane_fn_tm<32>(k);
        default: return nullptr;
    }
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
