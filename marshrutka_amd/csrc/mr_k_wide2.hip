// mr_k_wide2.hip — wide hub solver kernels with 2 specials per lane
// (hub_wide_kernel<PERM, 2> for the six comparator permutations)
#include "mr_device.hpp"

namespace mr {

const void *wide_fn_spl2(uint32_t perm) {
    constexpr uint32_t SPL = 2;
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_wide_kernel<5, SPL>);
        case 7: return reinterpret_cast<const void *>(&hub_wide_kernel<7, SPL>);
        case 11: return reinterpret_cast<const void *>(&hub_wide_kernel<11, SPL>);
        case 15: return reinterpret_cast<const void *>(&hub_wide_kernel<15, SPL>);
        case 19: return reinterpret_cast<const void *>(&hub_wide_kernel<19, SPL>);
        case 21: return reinterpret_cast<const void *>(&hub_wide_kernel<21, SPL>);
        default: return nullptr;
    }
}

}  // namespace mr
