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
    if (fn) n = occupancy_cached(fn, kBS, 0);
    return n;
}

template <uint32_t SPW>
static const void *hub_fill_fn_spw(const uint32_t perm[3]) {
    switch (perm[0] * 9 + perm[1] * 3 + perm[2]) {
        case 5: return (const void *)&hub_fill_kernel<5, SPW>;
        case 7: return (const void *)&hub_fill_kernel<7, SPW>;
        case 11: return (const void *)&hub_fill_kernel<11, SPW>;
        case 15: return (const void *)&hub_fill_kernel<15, SPW>;
        case 19: return (const void *)&hub_fill_kernel<19, SPW>;
        case 21: return (const void *)&hub_fill_kernel<21, SPW>;
        default: return nullptr;
    }
}
static const void *hub_fill_fn(const uint32_t perm[3], uint32_t spw) {
    return spw == 2 ? hub_fill_fn_spw<2>(perm) : hub_fill_fn_spw<1>(perm);
}

// one launch: hub_blocks workgroups of the next pass's specials' solve (hub_args), then
// fill_blocks workgroups of this pass's fill (fill_args); lds_bytes = the hub's layout
hipError_t launch_hub_fill(const KArgs *hub_args, const KArgs *fill_args, const uint32_t perm[3], uint32_t spw,
                           uint32_t hub_blocks, uint32_t fill_blocks, uint32_t lds_bytes, hipStream_t stream) {
    const void *fn = hub_fill_fn(perm, spw);
    if (!fn) return hipErrorInvalidValue;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_bytes));
    void *args[] = {const_cast<KArgs **>(&hub_args), const_cast<KArgs **>(&fill_args), &hub_blocks};
    return hipLaunchKernel(fn, dim3(hub_blocks + fill_blocks), dim3(kBS), args, lds_bytes, stream);
}

int hub_fill_blocks_per_cu(const uint32_t perm[3], uint32_t spw, uint32_t lds_bytes) {
    const void *fn = hub_fill_fn(perm, spw);
    int n = 0;
    if (fn) n = occupancy_cached(fn, kBS, lds_bytes);
    return n;
}

}  // namespace mr
