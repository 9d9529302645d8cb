// mr_k_cert.hip — certified fallback kernels (cert_select_kernel, cert_check_kernel, cert_window_kernel,
// cert_tile_kernel, cert_sweep_kernel)
// (host-side launch helpers called from mr_host.cpp; device code in mr_cert.hpp)
#include "mr_cert_tile.hpp"

namespace mr {

// the slots' deterministic assignment (one workgroup)
hipError_t launch_cert_select(const KArgs *d_args, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel((const void *)&cert_select_kernel, dim3(1), dim3(kSelectBS), args, 0, stream);
}

// the check over every slot's cells: gx workgroups per slot, `slots` slots
hipError_t launch_cert_check(const KArgs *d_args, uint32_t gx, uint32_t slots, uint32_t mark, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args), &mark};
    return hipLaunchKernel((const void *)&cert_check_kernel, dim3(gx, slots), dim3(kBS), args, 0, stream);
}

// the repair sweep: one workgroup per slot
hipError_t launch_cert_sweep(const KArgs *d_args, uint32_t slots, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel((const void *)&cert_sweep_kernel, dim3(slots), dim3(kSweepBS), args, 0, stream);
}

// the repair windows: one workgroup per slot
hipError_t launch_cert_window(const KArgs *d_args, uint32_t slots, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel((const void *)&cert_window_kernel, dim3(slots), dim3(256), args, 0, stream);
}

// the tile sweep: a persistent grid of `wgs` workgroups, one a CU (its LDS block admits
// no second), so a team's workgroups are resident together
hipError_t launch_cert_tile(const KArgs *d_args, uint32_t wgs, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel((const void *)&cert_tile_kernel, dim3(wgs), dim3(kTileBS), args, 0, stream);
}

// between the certificate's two rounds: one wave per slot
hipError_t launch_cert_promote(const KArgs *d_args, uint32_t slots, uint32_t *redo, hipStream_t stream) {
    void *args[] = {const_cast<KArgs **>(&d_args), &redo};
    return hipLaunchKernel((const void *)&cert_promote_kernel, dim3(slots), dim3(64), args, 0, stream);
}

// resident workgroups of the tile sweep per CU (1 expected)
int cert_tile_occupancy() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void *)&cert_tile_kernel, kTileBS, 0) != hipSuccess) return 0;
    return n;
}

}  // namespace mr
