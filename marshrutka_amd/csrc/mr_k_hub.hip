// mr_k_hub.hip — hub solver kernels (hub_kernel, one or two sources per wave)
// (host-side launch helpers called from mr_host.cpp; device code in mr_device.hpp)
#include "mr_device.hpp"

namespace mr {

uint32_t hub_lds_bytes(uint32_t NS, uint32_t nreg, uint32_t spw) { return hub_layout(NS, nreg, spw).total; }

// the kernels live in mr_k_hub_lin.hip / mr_k_hub_nl.hip (compiled in parallel)
const void *hub_fn_lin(uint32_t perm, uint32_t spw);
const void *hub_fn_nl(uint32_t perm, uint32_t spw);
static const void *hub_fn(const uint32_t perm[3], uint32_t spw, bool nonlin) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    return nonlin ? hub_fn_nl(k, spw) : hub_fn_lin(k, spw);
}

hipError_t launch_hub(const KArgs *d_args, const uint32_t perm[3], uint32_t spw, bool nonlin, uint32_t NS,
                      uint32_t nreg, uint32_t blocks, hipStream_t stream) {
    const uint32_t bytes = hub_lds_bytes(NS, nreg, spw);
    const void *fn = hub_fn(perm, spw, nonlin);
    if (!fn) return hipErrorInvalidValue;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks), dim3(kBS), args, bytes, stream);
}

int hub_blocks_per_cu(const uint32_t perm[3], uint32_t spw, bool nonlin, uint32_t bytes) {
    int n = 0;
    const void *fn = hub_fn(perm, spw, nonlin);
    if (fn) n = occupancy_cached(fn, kBS, bytes);
    return n;
}

}  // namespace mr
