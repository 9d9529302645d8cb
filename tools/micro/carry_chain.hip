// Micro-benchmark: issue cost of the lane kernel's instruction patterns on gfx950
// (dependent VGPR ops, borrow chains through VCC, two interleaved borrow chains via
// VCC and an SGPR pair, v_cndmask on VCC), one or two waves per SIMD; s_memtime cycles
// per instruction.  Build: hipcc --offload-arch=gfx950 -O3 carry_chain.hip -o carry_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP16(x) x x x x x x x x x x x x x x x x
template <int K>
__global__ void bench(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u, c = a + 7u, d = b ^ 5u, e = 0, f = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; ++it) {
        if constexpr (K == 0) {  // dependent v_add_u32
            asm volatile(REP16("v_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        } else if constexpr (K == 1) {  // independent v_add_u32 (4 chains)
            asm volatile(REP16("v_add_u32 %0, %0, %4\n\t v_add_u32 %1, %1, %4\n\t v_add_u32 %2, %2, %4\n\t v_add_u32 %3, %3, %4\n\t")
                         : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(b));
        } else if constexpr (K == 2) {  // borrow chain through vcc
            asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\t" REP16("v_subb_co_u32 %0, vcc, %0, %1, vcc\n\t")
                         : "+v"(a) : "v"(b) : "vcc");
        } else if constexpr (K == 3) {  // two interleaved borrow chains, vcc and an sgpr pair
            uint64_t s;
            asm volatile("v_sub_co_u32 %0, vcc, %0, %3\n\t v_sub_co_u32_e64 %1, %2, %1, %3\n\t"
                         REP16("v_subb_co_u32 %0, vcc, %0, %3, vcc\n\t v_subb_co_u32_e64 %1, %2, %1, %3, %2\n\t")
                         : "+v"(a), "+v"(c), "=&s"(s) : "v"(b) : "vcc");
        } else if constexpr (K == 4) {  // chain step + cndmask on vcc (the mask materialization)
            asm volatile(REP16("v_sub_co_u32 %0, vcc, %0, %2\n\t v_cndmask_b32_e64 %1, 0, -1, vcc\n\t")
                         : "+v"(a), "+v"(c) : "v"(b) : "vcc");
        } else if constexpr (K == 5) {  // dependent v_bfi_b32 (the selects)
            asm volatile(REP16("v_bfi_b32 %0, %1, %0, %2\n\t") : "+v"(a) : "v"(b), "v"(c));
        } else if constexpr (K == 6) {  // v_cmp + v_cndmask through an sgpr pair (v3 style)
            uint64_t s;
            asm volatile(REP16("v_cmp_lt_u32_e64 %2, %0, %3\n\t v_cndmask_b32_e64 %1, %1, %0, %2\n\t")
                         : "+v"(a), "+v"(c), "=&s"(s) : "v"(b));
        } else if constexpr (K == 7) {  // s_nop 0
            asm volatile(REP16("s_nop 0\n\t"));
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + c + d + e + f;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int K>
static void run(const char *name, int per_inst, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, threads = 256;  // 4 waves per block = 1 per SIMD
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, blocks * threads / 64 * 8);
    bench<K><<<blocks, threads>>>(out, cyc, 1);
    hipDeviceSynchronize();
    bench<K><<<blocks, threads>>>(out, cyc, 2);
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    uint64_t *h = new uint64_t[nw];
    hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nw; ++i) s += double(h[i]);
    // s_memtime ticks at the shader clock here? report raw ticks per instruction
    printf("%-44s waves/SIMD %d : %.2f ticks per instruction\n", name, waves_per_simd, s / nw / (64.0 * per_inst));
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<0>("dependent v_add_u32", 16, w);
        run<1>("independent v_add_u32 (4 chains)", 64, w);
        run<2>("borrow chain via vcc (v_subb_co)", 17, w);
        run<3>("two borrow chains (vcc + sgpr pair)", 34, w);
        run<4>("v_sub_co + v_cndmask on vcc", 32, w);
        run<5>("dependent v_bfi_b32", 16, w);
        run<6>("v_cmp_e64 -> sgpr pair -> v_cndmask", 32, w);
        run<7>("s_nop 0", 16, w);
    }
    return 0;
}
