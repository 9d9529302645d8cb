// mr_k_lane_nl.hip — hub_lane_kernel with Fleetfoot 1..3 run times (NL: the walk
// certification of mr_hub_lane.hpp) for a 22-entry table, a translation unit of its own so it
// compiles in parallel with the linear kernels (launch: mr_k_lane.hip).
#include "mr_hub_lane.hpp"

namespace mr {

template <uint32_t TM>
const void *lane_nl_fn_tm(uint32_t perm);

template <>
const void *lane_nl_fn_tm<22>(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_lane_kernel<5, 22, true>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_lane_kernel<7, 22, true>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_lane_kernel<11, 22, true>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_lane_kernel<15, 22, true>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_lane_kernel<19, 22, true>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_lane_kernel<21, 22, true>);  // time money legs
        default: return nullptr;
    }
}

}  // namespace mr
