// mr_k_solve.hip — SSSP kernels (solve_kernel): launch and occupancy
// (host-side launch helpers called from mr_host.cpp; device code in mr_device.hpp)
#include "mr_device.hpp"

namespace mr {

uint32_t lds_bytes(uint32_t NS, uint32_t V, bool grid_in_lds, uint32_t algo) {
    return lds_layout(NS, V, grid_in_lds, algo).total;
}

template <bool G, class IdxT, uint32_t ALGO>
static const void *kfn() {
    return reinterpret_cast<const void *>(&solve_kernel<G, IdxT, ALGO>);
}

static const void *select_kernel(bool grid_in_lds, uint32_t algo) {
    if (grid_in_lds) return algo == kAlgoLegs ? kfn<false, uint16_t, kAlgoLegs>() : kfn<false, uint16_t, kAlgoGeneric>();
    return algo == kAlgoLegs ? kfn<true, uint32_t, kAlgoLegs>() : kfn<true, uint32_t, kAlgoGeneric>();
}

hipError_t launch_solve(const KArgs *d_args, bool grid_in_lds, uint32_t algo, uint32_t NS, uint32_t V,
                        uint32_t blocks, hipStream_t stream) {
    const uint32_t bytes = lds_bytes(NS, V, grid_in_lds, algo);
    const void *fn = select_kernel(grid_in_lds, algo);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks), dim3(kBS), args, bytes, stream);
}

int max_blocks_per_cu(bool grid_in_lds, uint32_t algo, uint32_t bytes) {
    int n = 0;
    n = occupancy_cached(select_kernel(grid_in_lds, algo), kBS, bytes);
    return n;
}

}  // namespace mr
