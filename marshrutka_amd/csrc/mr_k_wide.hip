// mr_k_wide.hip — wide hub solver kernels (hub_wide_kernel, 64-511 specials)
// (host-side launch helpers called from mr_host.cpp; device code in mr_device.hpp)
#include "mr_device.hpp"

namespace mr {

uint32_t hub_wide_lds_bytes(uint32_t NS, uint32_t nreg) { return wide_layout(NS, nreg).total; }

// one translation unit per SPL (mr_k_wide_spl.hip built with -DMR_WIDE_SPL=2/5/8)
const void *wide_fn_spl2(uint32_t perm);
const void *wide_fn_spl5(uint32_t perm);
const void *wide_fn_spl8(uint32_t perm);

// specials per lane for a table of NS + 1 entries: 2, 5 or 8 (0 if too many)
uint32_t hub_wide_spl(uint32_t NS) {
    const uint32_t T = NS + 1;
    return T <= 128 ? 2u : (T <= 320 ? 5u : (T <= 512 ? 8u : 0u));
}
static const void *wide_fn(const uint32_t perm[3], uint32_t NS) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    switch (hub_wide_spl(NS)) {
        case 2: return wide_fn_spl2(k);
        case 5: return wide_fn_spl5(k);
        case 8: return wide_fn_spl8(k);
        default: return nullptr;
    }
}
hipError_t launch_hub_wide(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t blocks,
                           hipStream_t stream) {
    const uint32_t bytes = hub_wide_lds_bytes(NS, nreg);
    const void *fn = wide_fn(perm, NS);
    if (!fn) return hipErrorInvalidValue;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks), dim3(kBS), args, bytes, stream);
}
int hub_wide_blocks_per_cu(const uint32_t perm[3], uint32_t NS, uint32_t bytes) {
    int n = 0;
    const void *fn = wide_fn(perm, NS);
    if (fn) n = occupancy_cached(fn, kBS, bytes);
    return n;
}

}  // namespace mr
