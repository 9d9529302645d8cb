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
    const uint32_t S = 1025, Pp = (S + 63) / 64 * 64;
    uint32_t *out;
    const unsigned long long maxn = 512ull * S * Pp;
    if (hipMalloc(&out, maxn * 4) != hipSuccess) return 1;
    for (uint32_t nsrc : {64u, 256u, 512u}) {
        for (int g : {1280, 2560}) {
            auto rep = [&](const char *name, uint32_t P, float ms) {
                const double gb = double(nsrc) * S * S * 4 / 1e9;  // useful bytes
                printf("nsrc %4u grid %5d %-26s P %5u  %.4f ms  %6.0f GB/s useful\n", nsrc, g, name, P, ms, gb / ms * 1e3);
            };
            rep("dense", S, timeit([&] { tiles<false, false><<<g, 256>>>(out, S, S, nsrc); }));
            rep("dense nt", S, timeit([&] { tiles<true, false><<<g, 256>>>(out, S, S, nsrc); }));
            rep("padded masked", Pp, timeit([&] { tiles<false, false><<<g, 256>>>(out, S, Pp, nsrc); }));
            rep("padded full", Pp, timeit([&] { tiles<false, true><<<g, 256>>>(out, S, Pp, nsrc); }));
            rep("padded full nt", Pp, timeit([&] { tiles<true, true><<<g, 256>>>(out, S, Pp, nsrc); }));
        }
    }
    return 0;
}
