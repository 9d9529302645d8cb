// mr_k_group_nl.hip — hub_group_kernel with Fleetfoot 1..3 run times (NL: the walk
// certification of mr_hub_lane.hpp shared by the group's lanes, mr_hub_group.hpp), a
// translation unit of its own so it compiles in parallel (launch: mr_k_group.hip).
#include "mr_hub_group.hpp"

namespace mr {

template <uint32_t G, uint32_t E>
static const void *group_nl_ge(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_group_kernel<5, G, E, true>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_group_kernel<7, G, E, true>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_group_kernel<11, G, E, true>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_group_kernel<15, G, E, true>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_group_kernel<19, G, E, true>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_group_kernel<21, G, E, true>);  // time money legs
        default: return nullptr;
    }
}

const void *group_nl_fn(uint32_t G, uint32_t E, uint32_t perm) {
    if (G == 8 && E == 3) return group_nl_ge<8, 3>(perm);
    if (G == 8 && E == 4) return group_nl_ge<8, 4>(perm);
    if (G == 16 && E == 2) return group_nl_ge<16, 2>(perm);
    if (G == 32 && E == 1) return group_nl_ge<32, 1>(perm);
    return nullptr;
}

}  // namespace mr
