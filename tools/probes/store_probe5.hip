// Store-bandwidth probe for the fill's 4 B cell words (not product code): nsrc
// sources x S rows of P cells (P = S: dense rows; P = S rounded up to 64: every
// 64-cell tile row is one aligned 256 B run), 64x16 tiles, lane = column, each
// source's tiles interleaved over its group of waves (the fill's schedule).
// FULL: tiles at the right edge store all 64 columns (the pad) instead of masking.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <bool NT, bool FULL, int TW = 64>
__global__ __launch_bounds__(256) void tiles(uint32_t *out, uint32_t S, uint32_t P, uint32_t nsrc) {
    constexpr int TH = 1024 / TW;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tpx = (S + TW - 1) / TW, tpy = (S + TH - 1) / TH, ntile = tpx * tpy;
    const uint32_t nw = gridDim.x * 4, gw = blockIdx.x * 4 + wv;
    const uint32_t ng = nsrc < nw ? nsrc : nw, G = nw / ng, g = gw / G, j = gw % G;
    if (g >= ng) return;
    const uint32_t s0 = uint32_t(uint64_t(g) * nsrc / ng), s1 = uint32_t(uint64_t(g + 1) * nsrc / ng);
    for (uint32_t s = s0; s < s1; ++s) {
        uint32_t *o = out + (unsigned long long)s * S * P;
        for (uint32_t t = j; t < ntile; t += G) {
            const uint32_t tx0 = (t % tpx) * TW, ty0 = (t / tpx) * TH;
#pragma unroll
            for (int ii = 0; ii < 16; ++ii) {
                const uint32_t cy = ty0 + ii / (TW / 64), cx = tx0 + 64 * (ii % (TW / 64)) + lane;
                const int i = ii;
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
    const uint32_t S = 1025, Pp = (S + 255) / 256 * 256, P64 = (S + 63) / 64 * 64;
    uint32_t *out;
    const unsigned long long maxn = 512ull * S * Pp;  // largest pitch
    if (hipMalloc(&out, maxn * 4) != hipSuccess) return 1;
    for (uint32_t nsrc : {512u}) {
        for (int g : {1280, 2560}) {
            auto rep = [&](const char *name, uint32_t P, float ms) {
                const double gb = double(nsrc) * S * S * 4 / 1e9;  // useful bytes
                printf("nsrc %4u grid %5d %-26s P %5u  %.4f ms  %6.0f GB/s useful\n", nsrc, g, name, P, ms, gb / ms * 1e3);
            };
            rep("64x16 full P64", P64, timeit([&] { tiles<false, true, 64><<<g, 256>>>(out, S, P64, nsrc); }));
            rep("64x16 full P256", Pp, timeit([&] { tiles<false, true, 64><<<g, 256>>>(out, S, Pp, nsrc); }));
            rep("128x8 full P256", Pp, timeit([&] { tiles<false, true, 128><<<g, 256>>>(out, S, Pp, nsrc); }));
            rep("256x4 full P256", Pp, timeit([&] { tiles<false, true, 256><<<g, 256>>>(out, S, Pp, nsrc); }));
            rep("256x4 full P256 nt", Pp, timeit([&] { tiles<true, true, 256><<<g, 256>>>(out, S, Pp, nsrc); }));
        }
    }
    return 0;
}
