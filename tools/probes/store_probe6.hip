// Store-bandwidth probe for the fill's 4 B cell words (not product code): nsrc
// sources x S rows of P cells (P = S: dense rows; P = S rounded up to 64: every
// 64-cell tile row is one aligned 256 B run), 64x16 tiles, lane = column, each
// source's tiles interleaved over its group of waves (the fill's schedule).
// FULL: tiles at the right edge store all 64 columns (the pad) instead of masking.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <bool NT, bool FULL>
__global__ __launch_bounds__(256) void tiles(uint32_t *out, uint32_t S, uint32_t P, uint32_t nsrc) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tpx = (S + 63) / 64, tpy = (S + 15) / 16, ntile = tpx * tpy;
    const uint32_t nw = gridDim.x * 4, gw = blockIdx.x * 4 + wv;
    const uint32_t ng = nsrc < nw ? nsrc : nw, G = nw / ng, g = gw / G, j = gw % G;
    if (g >= ng) return;
    const uint32_t s0 = uint32_t(uint64_t(g) * nsrc / ng), s1 = uint32_t(uint64_t(g + 1) * nsrc / ng);
    for (uint32_t s = s0; s < s1; ++s) {
        uint32_t *o = out + (unsigned long long)s * S * P;
        for (uint32_t t = j; t < ntile; t += G) {
            const uint32_t tx0 = (t % tpx) * 64, ty0 = (t / tpx) * 16;
            const uint32_t cx = tx0 + lane;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t cy = ty0 + i;
                if ((FULL ? cx < P : cx < S) && cy < S) {
                    const uint32_t v = cx ^ (cy << 12) ^ s;
                    if (NT) __builtin_nontemporal_store(v, o + cy * P + cx);
                    else o[cy * P + cx] = v;
                }
            }
        }
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    // one fresh allocation per size: is the store rate a property of the buffer's size?
    const uint32_t S = 1025, Pp = (S + 63) / 64 * 64;
    for (uint32_t nsrc : {4096u, 8192u, 12288u, 16384u}) {
        uint32_t *out;
        const unsigned long long n = (unsigned long long)nsrc * S * Pp;
        if (hipMalloc(&out, n * 4) != hipSuccess) { printf("nsrc %u: hipMalloc failed\n", nsrc); return 1; }
        const int g = 1280;
        const float ms = timeit([&] { tiles<false, true><<<g, 256>>>(out, S, Pp, nsrc); });
        printf("nsrc %5u  %.1f GB  %.3f ms  %.0f GB/s\n", nsrc, n * 4 / 1e9, ms, n * 4 / 1e6 / ms);
        (void)hipFree(out);
    }
    return 0;
}
