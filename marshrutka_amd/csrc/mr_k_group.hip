// mr_k_group.hip — the hub solver with one source per group of G lanes (hub_group_kernel,
// mr_hub_group.hpp) for the six comparator permutations; launch helpers for mr_host.cpp.
#include "mr_hub_group.hpp"

namespace mr {

// Fleetfoot 1..3 (hub_group_kernel<PERM, G, E, true>): mr_k_group_nl.hip
const void *group_nl_fn(uint32_t G, uint32_t E, uint32_t perm);

template <uint32_t G, uint32_t E>
static const void *group_fn_ge(uint32_t perm) {
    switch (perm) {
        case 5: return reinterpret_cast<const void *>(&hub_group_kernel<5, G, E>);    // legs money time
        case 7: return reinterpret_cast<const void *>(&hub_group_kernel<7, G, E>);    // legs time money
        case 11: return reinterpret_cast<const void *>(&hub_group_kernel<11, G, E>);  // money legs time
        case 15: return reinterpret_cast<const void *>(&hub_group_kernel<15, G, E>);  // money time legs
        case 19: return reinterpret_cast<const void *>(&hub_group_kernel<19, G, E>);  // time legs money
        case 21: return reinterpret_cast<const void *>(&hub_group_kernel<21, G, E>);  // time money legs
        default: return nullptr;
    }
}

// slots per lane for a table of NS + 1 entries in groups of G lanes (0: not applicable)
uint32_t hub_group_slots(uint32_t NS, uint32_t G) {
    if (G == 8) return NS + 1 <= 24 ? 3u : (NS + 1 <= 32 ? 4u : 0u);
    if (G == 16) return NS + 1 <= 32 ? 2u : 0u;
    if (G == 32) return NS + 1 <= 32 ? 1u : 0u;
    return 0u;
}

uint32_t hub_group_lds_bytes(uint32_t NS, uint32_t nreg, uint32_t G) {
    const uint32_t E = hub_group_slots(NS, G);
    return E ? group_lds_total(NS, nreg, G, E) : 0u;
}

hipError_t launch_hub_group(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t n,
                            uint32_t G, bool nonlin, hipStream_t stream) {
    const uint32_t k = perm[0] * 9 + perm[1] * 3 + perm[2];
    const uint32_t E = hub_group_slots(NS, G);
    const void *fn = nullptr;
    if (nonlin) fn = E ? group_nl_fn(G, E, k) : nullptr;
    else if (G == 8 && E == 3) fn = group_fn_ge<8, 3>(k);
    else if (G == 8 && E == 4) fn = group_fn_ge<8, 4>(k);
    else if (G == 16 && E == 2) fn = group_fn_ge<16, 2>(k);
    else if (G == 32 && E == 1) fn = group_fn_ge<32, 1>(k);
    if (!fn) return hipErrorInvalidValue;
    const uint32_t bytes = group_lds_total(NS, nreg, G, E);
    if (bytes > 64u * 1024u) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    const uint32_t per_block = kBS / G, blocks = (n + per_block - 1u) / per_block;
    void *args[] = {const_cast<KArgs **>(&d_args)};
    return hipLaunchKernel(fn, dim3(blocks ? blocks : 1u), dim3(kBS), args, bytes, stream);
}

}  // namespace mr
