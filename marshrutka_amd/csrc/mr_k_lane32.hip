// mr_k_lane32.hip — hub_lane_kernel with a 32-entry table (one wave per SIMD), its own
// translation unit so the three table sizes compile in parallel (launch: mr_k_lane.hip).
#include "mr_hub_lane.hpp"

namespace mr {

template <uint32_t TM>
const void *lane_fn_tm(uint32_t perm);

template <>
const void *lane_fn_tm<32>(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_lane_kernel<5, 32>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_lane_kernel<7, 32>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_lane_kernel<11, 32>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_lane_kernel<15, 32>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_lane_kernel<19, 32>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_lane_kernel<21, 32>);  // time money legs
        default: return nullptr;
    }
}

}  // namespace mr
