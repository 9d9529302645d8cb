// Store-bandwidth probe for the fill kernel's output shape (not product code):
// 64 sources x S^2 cells x 16 B, written by waves in tiles of TW x TH cells.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// MODE 0: each wave a contiguous run of items; 1: items interleaved over waves
// (w = gw + k * nwaves); 2: each wave one source, that source's tiles interleaved
// over its waves
template <int TW, bool NT, int MODE = 0>
__global__ __launch_bounds__(256) void tiles(u32x4_t *out, uint32_t S, uint32_t nsrc) {
    constexpr int TH = 1024 / TW;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tpx = (S + TW - 1) / TW, tpy = (S + TH - 1) / TH, ntile = tpx * tpy;
    const unsigned long long total = (unsigned long long)nsrc * ntile;
    const unsigned long long nw = (unsigned long long)gridDim.x * 4, gw = blockIdx.x * 4ull + wv;
    unsigned long long w0 = gw * total / nw, w1 = (gw + 1) * total / nw, step = 1;
    if (MODE == 1) { w0 = gw; w1 = total; step = nw; }
    const unsigned long long wps = nw / nsrc;  // MODE 2: waves per source
    if (MODE == 2) { if (gw >= wps * nsrc) return; w0 = (gw % nsrc) * ntile + gw / nsrc; w1 = (gw % nsrc + 1) * ntile; step = wps; }
    for (unsigned long long w = w0; w < w1; w += step) {
        const uint32_t s = uint32_t(w / ntile), t = uint32_t(w % ntile);
        const int tx0 = int(t % tpx) * TW, ty0 = int(t / tpx) * TH;
        u32x4_t *o = out + (unsigned long long)s * S * S;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int c = i * 64 + int(lane), cx = tx0 + c % TW, cy = ty0 + c / TW;
            if (cx < int(S) && cy < int(S)) {
                u32x4_t v = {uint32_t(cx), uint32_t(cy), s, uint32_t(i)};
                if (NT) __builtin_nontemporal_store(v, o + uint32_t(cy) * S + uint32_t(cx));
                else o[uint32_t(cy) * S + uint32_t(cx)] = v;
            }
        }
    }
}

__global__ __launch_bounds__(256) void linear(u32x4_t *out, unsigned long long n) {
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
        out[i] = u32x4_t{uint32_t(i), 1u, 2u, 3u};
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
    const uint32_t S = 1025, nsrc = 64;
    const unsigned long long n = (unsigned long long)nsrc * S * S;
    u32x4_t *out;
    if (hipMalloc(&out, n * 16) != hipSuccess) return 1;
    const double gb = n * 16 / 1e9;
    for (int g : {1024, 1536, 2048}) {
        auto rep = [&](const char *name, float ms) { printf("%-22s grid %5d  %.3f ms  %.0f GB/s\n", name, g, ms, gb / ms * 1e3); };
        rep("linear", timeit([&] { linear<<<g, 256>>>(out, n); }));
        rep("tile32x32 interleave", timeit([&] { tiles<32, false, 1><<<g, 256>>>(out, S, nsrc); }));
        rep("tile64x16 interleave", timeit([&] { tiles<64, false, 1><<<g, 256>>>(out, S, nsrc); }));
        rep("tile128x8 interleave", timeit([&] { tiles<128, false, 1><<<g, 256>>>(out, S, nsrc); }));
        rep("tile256x4 interleave", timeit([&] { tiles<256, false, 1><<<g, 256>>>(out, S, nsrc); }));
        rep("tile128x8 contiguous", timeit([&] { tiles<128, false, 0><<<g, 256>>>(out, S, nsrc); }));
        rep("tile256x4 contiguous", timeit([&] { tiles<256, false, 0><<<g, 256>>>(out, S, nsrc); }));
        rep("tile1024x1 contiguous", timeit([&] { tiles<1024, false, 0><<<g, 256>>>(out, S, nsrc); }));
        rep("tile64x16 interl. nt", timeit([&] { tiles<64, true, 1><<<g, 256>>>(out, S, nsrc); }));
    }
    return 0;
}
