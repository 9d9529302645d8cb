// group_min variants (round 4: V1 is what mr_hub_group.hpp uses; V2 and V3 put the DPP
// operand on the carry ops themselves and compute wrong minima on gfx950): every lane of each 8-lane group must end with the group's least
// (c1, c2, c3, k) and the m word riding along with it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I marshrutka_amd/csrc tools/micro/group_min.hip -o tools/micro/group_min
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "mr_hub_group.hpp"

// V1: partner words copied by v_mov_b32_dpp, then the plain VCC chain and VOP2 selects
#define V1_ROUND(DPP)                                                                         \
    asm("s_nop 1\n\t"                                                                         \
        "v_mov_b32_dpp %6, %1 " DPP " row_mask:0xf bank_mask:0xf\n\t"                         \
        "v_mov_b32_dpp %7, %2 " DPP " row_mask:0xf bank_mask:0xf\n\t"                         \
        "v_mov_b32_dpp %8, %3 " DPP " row_mask:0xf bank_mask:0xf\n\t"                         \
        "v_mov_b32_dpp %9, %4 " DPP " row_mask:0xf bank_mask:0xf\n\t"                         \
        "v_mov_b32_dpp %10, %5 " DPP " row_mask:0xf bank_mask:0xf\n\t"                        \
        "v_sub_co_u32_e32 %0, vcc, %5, %10\n\t"                                               \
        "v_subb_co_u32_e32 %0, vcc, %3, %8, vcc\n\t"                                          \
        "v_subb_co_u32_e32 %0, vcc, %2, %7, vcc\n\t"                                          \
        "v_subb_co_u32_e32 %0, vcc, %1, %6, vcc\n\t"                                          \
        "v_cndmask_b32_e32 %1, %6, %1, vcc\n\t"                                               \
        "v_cndmask_b32_e32 %2, %7, %2, vcc\n\t"                                               \
        "v_cndmask_b32_e32 %3, %8, %3, vcc\n\t"                                               \
        "v_cndmask_b32_e32 %4, %9, %4, vcc\n\t"                                               \
        "v_cndmask_b32_e32 %5, %10, %5, vcc"                                                  \
        : "=&v"(t_), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(m), "+v"(k), "=&v"(p1), "=&v"(p2),      \
          "=&v"(p3), "=&v"(pm), "=&v"(pk)                                                     \
        :                                                                                     \
        : "vcc")
// V3: DPP in the chain only, plain movs + selects
#define V3_ROUND(DPP)                                                                         \
    asm("s_nop 1\n\t"                                                                         \
        "v_subrev_co_u32_dpp %0, vcc, %5, %5 " DPP " row_mask:0xf bank_mask:0xf\n\t"          \
        "v_subbrev_co_u32_dpp %0, vcc, %3, %3, vcc " DPP " row_mask:0xf bank_mask:0xf\n\t"    \
        "v_subbrev_co_u32_dpp %0, vcc, %2, %2, vcc " DPP " row_mask:0xf bank_mask:0xf\n\t"    \
        "v_subbrev_co_u32_dpp %0, vcc, %1, %1, vcc " DPP " row_mask:0xf bank_mask:0xf\n\t"    \
        "v_cndmask_b32_e64 %0, 0, -1, vcc"                                                    \
        : "=&v"(t_), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(m), "+v"(k)                          \
        :                                                                                     \
        : "vcc")

__device__ inline uint32_t dppmov(uint32_t v, int ctrl) { return v; }

template <int V>
__global__ void k_group_min(const uint32_t *in, uint32_t *out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    uint32_t c1 = in[i * 5 + 0], c2 = in[i * 5 + 1], c3 = in[i * 5 + 2], m = in[i * 5 + 3], k = in[i * 5 + 4];
    if constexpr (V == 2) {
        mr::group_min<8>(c1, c2, c3, m, k);
    } else if constexpr (V == 1) {
        uint32_t t_, p1, p2, p3, pm, pk;
        V1_ROUND("quad_perm:[1,0,3,2]");
        V1_ROUND("quad_perm:[2,3,0,1]");
        V1_ROUND("row_half_mirror");
    } else {
        // V3: the chain's mask (mine < partner) in t_, then selects from DPP'd copies in C
        uint32_t t_;
        V3_ROUND("quad_perm:[1,0,3,2]");
        {
            const uint32_t q1 = __builtin_amdgcn_mov_dpp(c1, 0xB1, 0xF, 0xF, false), q2 = __builtin_amdgcn_mov_dpp(c2, 0xB1, 0xF, 0xF, false),
                           q3 = __builtin_amdgcn_mov_dpp(c3, 0xB1, 0xF, 0xF, false), qm = __builtin_amdgcn_mov_dpp(m, 0xB1, 0xF, 0xF, false),
                           qk = __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, false);
            c1 = t_ ? c1 : q1; c2 = t_ ? c2 : q2; c3 = t_ ? c3 : q3; m = t_ ? m : qm; k = t_ ? k : qk;
        }
    }
    out[i * 5 + 0] = c1;
    out[i * 5 + 1] = c2;
    out[i * 5 + 2] = c3;
    out[i * 5 + 3] = m;
    out[i * 5 + 4] = k;
}

template <int V>
static int run(uint32_t waves, uint32_t seed, uint32_t G, uint32_t rounds_g) {
    const uint32_t n = waves * 64;
    std::vector<uint32_t> h(n * 5), o(n * 5);
    srand(seed);
    for (uint32_t i = 0; i < n; ++i) {
        h[i * 5 + 0] = rand() % 3;
        h[i * 5 + 1] = rand() % 3;
        h[i * 5 + 2] = rand() % 3;
        h[i * 5 + 3] = rand();
        h[i * 5 + 4] = ((rand() % 3) << 24) | (i % 8);
    }
    uint32_t *din, *dout;
    (void)hipMalloc(&din, n * 20);
    (void)hipMalloc(&dout, n * 20);
    (void)hipMemcpy(din, h.data(), n * 20, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_group_min<V>, dim3(waves), dim3(64), 0, 0, din, dout);
    (void)hipMemcpy(o.data(), dout, n * 20, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t g0 = 0; g0 < n; g0 += rounds_g) {
        uint32_t best = g0;
        for (uint32_t j = g0 + 1; j < g0 + rounds_g; ++j) {
            const uint32_t *a = &h[j * 5], *b = &h[best * 5];
            bool lt = a[0] != b[0] ? a[0] < b[0] : a[1] != b[1] ? a[1] < b[1] : a[2] != b[2] ? a[2] < b[2] : a[4] < b[4];
            if (lt) best = j;
        }
        for (uint32_t j = g0; j < g0 + rounds_g; ++j)
            for (int w = 0; w < 5; ++w)
                if (o[j * 5 + w] != h[best * 5 + w]) {
                    if (bad < 3) printf("V%d lane %u word %d: got %u want %u (in %u)\n", V, j, w, o[j * 5 + w], h[best * 5 + w], h[j*5+w]);
                    ++bad;
                }
    }
    printf("variant %d (groups of %u): %u groups, %d wrong words\n", V, rounds_g, n / rounds_g, bad);
    (void)hipFree(din);
    (void)hipFree(dout);
    return bad;
}

int main() {
    int bad = run<1>(64, 1, 8, 8);
    bad += run<2>(64, 1, 8, 8);
    (void)run<3>(64, 1, 8, 2);  // (known wrong: the DPP operand on the carry ops)
    return bad ? 1 : 0;
}
