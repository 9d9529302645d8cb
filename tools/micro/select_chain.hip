// Micro-benchmark: compare-and-select patterns of the lane kernel (mr_hub_lane.hpp) at
// one and two waves per SIMD on every SIMD, s_memtime ticks per instruction per wave.
// A "step" folds a candidate label (c1, c2, c3, m) into a running best, as the scan and
// relax loops do: a borrow chain over (len byte, c3, c2, c1), then a 4-word select.
//   A  the kernel's form: VCC chain, v_cndmask_e64 mask, 4 x v_bfi_b32 (separate asm)
//   B  VCC chain, then 4 x v_cndmask_b32_e32 on VCC directly (one asm block)
//   C  two independent steps interleaved, carries in VCC and an SGPR pair, e64 selects
//   D  form A with the s_nop 0 the compiler puts between asm blocks
// Build: hipcc --offload-arch=gfx950 -O3 select_chain.hip -o select_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
struct L4 { uint32_t a, b, c, m; };

template <int K>
__global__ void bench(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    const uint32_t l = threadIdx.x;
    // candidates that vary per step (registers; the chain's dependence is on the best)
    L4 x{l * 3u + seed, l ^ seed, l + 11u, l & 7u}, y{l * 5u, seed * 7u, l + 3u, (l >> 2) & 7u};
    L4 bx{~0u, 0u, 0u, 0u}, by{~0u, 0u, 0u, 0u};
    uint32_t k = 0, t = 0;
    uint64_t s;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; ++it) {
        if constexpr (K == 0 || K == 3) {
            REP8({
                asm volatile(
                    "v_sub_co_u32_sdwa %0, vcc, %2, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %4, %5, vcc\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %6, %7, vcc\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %8, %9, vcc\n\t"
                    "v_cndmask_b32_e64 %1, 0, -1, vcc"
                    : "=&v"(t), "=v"(k)
                    : "v"(x.m), "v"(bx.m), "v"(x.c), "v"(bx.c), "v"(x.b), "v"(bx.b), "v"(x.a), "v"(bx.a)
                    : "vcc");
                if (K == 3) asm volatile("s_nop 0");
                asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(bx.a) : "v"(k), "v"(x.a));
                asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(bx.b) : "v"(k), "v"(x.b));
                asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(bx.c) : "v"(k), "v"(x.c));
                asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(bx.m) : "v"(k), "v"(x.m));
                if (K == 3) asm volatile("s_nop 0");
                x.a += 1u;
            })
        } else if constexpr (K == 1) {
            REP8({
                asm volatile(
                    "v_sub_co_u32_sdwa %0, vcc, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %3, %4, vcc\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %5, %6, vcc\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %7, %8, vcc\n\t"
                    "v_cndmask_b32_e32 %8, %8, %7, vcc\n\t"
                    "v_cndmask_b32_e32 %6, %6, %5, vcc\n\t"
                    "v_cndmask_b32_e32 %4, %4, %3, vcc\n\t"
                    "v_cndmask_b32_e32 %2, %2, %1, vcc"
                    : "=&v"(t), "+v"(x.m), "+v"(bx.m), "+v"(x.c), "+v"(bx.c), "+v"(x.b), "+v"(bx.b), "+v"(x.a), "+v"(bx.a)
                    :
                    : "vcc");
                x.a += 1u;
            })
        } else if constexpr (K == 2) {
            REP8({
                uint32_t u;
                asm volatile(
                    "v_sub_co_u32_sdwa %0, vcc, %3, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                    "v_cmp_lt_u32_sdwa %2, %11, %12 src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %5, %6, vcc\n\t"
                    "v_subb_co_u32_e64 %1, %2, %13, %14, %2\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %7, %8, vcc\n\t"
                    "v_subb_co_u32_e64 %1, %2, %15, %16, %2\n\t"
                    "v_subb_co_u32_e32 %0, vcc, %9, %10, vcc\n\t"
                    "v_subb_co_u32_e64 %1, %2, %17, %18, %2\n\t"
                    "v_cndmask_b32_e32 %10, %10, %9, vcc\n\t"
                    "v_cndmask_b32_e64 %18, %18, %17, %2\n\t"
                    "v_cndmask_b32_e32 %8, %8, %7, vcc\n\t"
                    "v_cndmask_b32_e64 %16, %16, %15, %2\n\t"
                    "v_cndmask_b32_e32 %6, %6, %5, vcc\n\t"
                    "v_cndmask_b32_e64 %14, %14, %13, %2\n\t"
                    "v_cndmask_b32_e32 %4, %4, %3, vcc\n\t"
                    "v_cndmask_b32_e64 %12, %12, %11, %2"
                    : "=&v"(t), "=&v"(u), "=&s"(s), "+v"(x.m), "+v"(bx.m), "+v"(x.c), "+v"(bx.c), "+v"(x.b), "+v"(bx.b),
                      "+v"(x.a), "+v"(bx.a), "+v"(y.m), "+v"(by.m), "+v"(y.c), "+v"(by.c), "+v"(y.b), "+v"(by.b), "+v"(y.a),
                      "+v"(by.a)
                    :
                    : "vcc");
                x.a += 1u;
                y.a += 1u;
                t += u;
            })
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + l] = bx.a + bx.b + bx.c + bx.m + by.a + by.b + by.c + by.m + k + t;
    if (l % 64 == 0) cyc[(blockIdx.x * blockDim.x + l) / 64] = t1 - t0;
}

template <int K>
static void run(const char *name, double per_step, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, threads = 256;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, blocks * threads * 4);
    (void)hipMalloc(&cyc, blocks * threads / 64 * 8);
    bench<K><<<blocks, threads>>>(out, cyc, 1);
    (void)hipDeviceSynchronize();
    bench<K><<<blocks, threads>>>(out, cyc, 2);
    (void)hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    uint64_t *h = new uint64_t[nw];
    (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nw; ++i) s += double(h[i]);
    const double steps = 64.0 * 8.0;
    printf("%-62s waves/SIMD %d : %.1f ticks per step, %.2f per VALU\n", name, waves_per_simd, s / nw / steps,
           s / nw / steps / per_step);
    delete[] h;
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 3; ++w) {
        run<0>("A: vcc chain, cndmask_e64 mask, 4 bfi (+1 add)", 10, w);
        run<3>("D: A with s_nop 0 around the selects", 10, w);
        run<1>("B: vcc chain, 4 cndmask_e32 on vcc (+1 add)", 9, w);
        run<2>("C: two steps interleaved (vcc + sgpr pair) (+2 add)", 18, w);
    }
    return 0;
}
