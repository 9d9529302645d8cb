// mr_k_hub.hip — hub solver kernels (hub_kernel, one or two sources per wave)
// (host-side launch helpers called from mr_host.cpp; device code in mr_device.hpp)
#include "mr_device.hpp"

namespace mr {

uint32_t hub_lds_bytes(uint32_t NS, uint32_t nreg, uint32_t spw) { return hub_layout(NS, nreg, spw).total; }

template <uint32_t SPW>
static const void *hub_fn_spw(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_kernel<5, SPW>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_kernel<7, SPW>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_kernel<11, SPW>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_kernel<15, SPW>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_kernel<19, SPW>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_kernel<21, SPW>);  // time money legs
        default: return nullptr;
    }
}
static const void *hub_fn(const uint32_t perm[3], uint32_t spw) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    return spw == 2 ? hub_fn_spw<2>(k) : hub_fn_spw<1>(k);
}

hipError_t launch_hub(const KArgs *d_args, const uint32_t perm[3], uint32_t spw, uint32_t NS, uint32_t nreg,
                      uint32_t blocks, hipStream_t stream) {
    const uint32_t bytes = hub_lds_bytes(NS, nreg, spw);
    const void *fn = hub_fn(perm, spw);
    if (!fn) return hipErrorInvalidValue;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks), dim3(kBS), args, bytes, stream);
}

int hub_blocks_per_cu(const uint32_t perm[3], uint32_t spw, uint32_t bytes) {
    int n = 0;
    const void *fn = hub_fn(perm, spw);
    if (fn) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBS, bytes);
    return n;
}

}  // namespace mr
