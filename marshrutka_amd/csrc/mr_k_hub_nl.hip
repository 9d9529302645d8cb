// mr_k_hub_nl.hip — hub solver kernels, non-linear run time (Fleetfoot 1..3) with near-tie certification
// (hub_kernel<PERM, SPW, true> for the six comparator permutations, one or two sources per wave)
#include "mr_device.hpp"

namespace mr {

template <uint32_t SPW>
static const void *hub_fn_spw_nl(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_kernel<5, SPW, true>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_kernel<7, SPW, true>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_kernel<11, SPW, true>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_kernel<15, SPW, true>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_kernel<19, SPW, true>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_kernel<21, SPW, true>);  // time money legs
        default: return nullptr;
    }
}
const void *hub_fn_nl(uint32_t perm, uint32_t spw) { return spw == 2 ? hub_fn_spw_nl<2>(perm) : hub_fn_spw_nl<1>(perm); }

}  // namespace mr
