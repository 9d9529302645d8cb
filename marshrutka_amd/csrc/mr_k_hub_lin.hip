// mr_k_hub_lin.hip — hub solver kernels, linear StandardMove run time (Fleetfoot 0 or out of range)
// (hub_kernel<PERM, SPW, false> for the six comparator permutations, one or two sources per wave)
#include "mr_device.hpp"

namespace mr {

template <uint32_t SPW>
static const void *hub_fn_spw_lin(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_kernel<5, SPW, false>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_kernel<7, SPW, false>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_kernel<11, SPW, false>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_kernel<15, SPW, false>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_kernel<19, SPW, false>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_kernel<21, SPW, false>);  // time money legs
        default: return nullptr;
    }
}
const void *hub_fn_lin(uint32_t perm, uint32_t spw) { return spw == 2 ? hub_fn_spw_lin<2>(perm) : hub_fn_spw_lin<1>(perm); }

}  // namespace mr
