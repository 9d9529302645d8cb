// mr_k_lane24.hip — hub_lane_kernel with a 24-entry table (one wave per SIMD), its own
// translation unit so the three table sizes compile in parallel (launch: mr_k_lane.hip).
#include "mr_hub_lane.hpp"

namespace mr {

template <uint32_t TM>
const void *lane_fn_tm(uint32_t perm);

template <>
const void *lane_fn_tm<24>(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_lane_kernel<5, 24>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_lane_kernel<7, 24>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_lane_kernel<11, 24>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_lane_kernel<15, 24>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_lane_kernel<19, 24>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_lane_kernel<21, 24>);  // time money legs
        default: return nullptr;
    }
}

}  // namespace mr
