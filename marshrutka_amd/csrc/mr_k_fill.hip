// mr_k_fill.hip — all-destinations fill kernels (fill_kernel)
// (host-side launch helpers called from mr_host.cpp; device code in mr_device.hpp)
#include "mr_device.hpp"

namespace mr {

static const void *fill_fn(const uint32_t perm[3]) {
    switch (perm[0] * 9 + perm[1] * 3 + perm[2]) {
        case 5: return (const void *)&fill_kernel<5>;
        case 7: return (const void *)&fill_kernel<7>;
        case 11: return (const void *)&fill_kernel<11>;
        case 15: return (const void *)&fill_kernel<15>;
        case 19: return (const void *)&fill_kernel<19>;
        case 21: return (const void *)&fill_kernel<21>;
        default: return nullptr;
    }
}

hipError_t launch_fill(const KArgs *d_args, const uint32_t perm[3], uint32_t gx, uint32_t gy, hipStream_t stream) {
    const void *fn = fill_fn(perm);
    if (!fn) return hipErrorInvalidValue;
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(gx, gy), dim3(kBS), args, 0, stream);
}

// resident fill workgroups per CU: the grid is one round of them (each wave then
// takes an equal run of items)
int fill_blocks_per_cu(const uint32_t perm[3]) {
    const void *fn = fill_fn(perm);
    int n = 0;
    if (fn) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBS, 0);
    return n;
}

}  // namespace mr
