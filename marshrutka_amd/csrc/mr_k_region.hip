// mr_k_region.hip — the grid's region table built on the device (grid preprocessing,
// the analogue of MapGrid::parse's nearest-campfire pass, src/grid.rs:134-230,297-325).
//
// For every cell v and Scroll-of-Escape region r of a homeland (the cells whose nearest
// campfire of that homeland is region r's campfire, the Center excluded), the table
// holds {distance, rank} of the nearest region-r cell: walk distance on the 4-grid
// without the Center (walks cannot cross it, src/pathfinder.rs:30-53), ties by the
// cell's CellIndex rank (derived Ord, src/index.rs:41-46).  Layout: uint2 at
// [v * nreg + r] (the hub kernels' `near`).
//
// The walk distance is Manhattan except between two cells of one axis line on opposite
// sides of the Center (+2).  So the table is a separable L1 distance transform of the
// lexicographic pair (distance, rank), which the additive distance keeps ordered:
//   1. rows: per (row, region) the nearest region cell of the row to the left and to
//      the right (two sweeps);
//   2. columns: per (column, region) f(y) = min(g(y), f(y - 1) + 1) down and up, in
//      place (an exact two-pass L1 transform; +1 keeps the pair's order);
//   3. the axis lines: a cell of the horizontal axis reaches every cell either along
//      its own half-row (no Center crossed) or through its neighbour above or below,
//      whose entries (off the axes) are already exact:
//        T(x, H) = min(half-row(x), T(x, H - 1) + 1, T(x, H + 1) + 1),
//      and the vertical axis alike.  The Center's row is {none, none}.
// Every cell off the axes has a Manhattan path to any cell avoiding the Center, so
// passes 1-2 are exact there.  One thread per (line, region), regions fastest, so a
// wave's stores cover consecutive regions of one cell.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mr {

namespace {

constexpr uint32_t kNoneW = 0xFFFFFFFFu;
constexpr uint32_t kRegBS = 256;
constexpr int kPf = 8;  // entries loaded ahead in the column sweeps

__device__ __forceinline__ bool lex_less(uint2 a, uint2 b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }
__device__ __forceinline__ uint2 plus1(uint2 a) { return a.x == kNoneW ? a : make_uint2(a.x + 1u, a.y); }
__device__ __forceinline__ uint2 lex_min(uint2 a, uint2 b) { return lex_less(b, a) ? b : a; }

// pass 1: thread (row y, region r).  The half-row values of the Center's row (same side
// only) go to axh[x * nreg + r].
__global__ __launch_bounds__(kRegBS) void region_rows_kernel(const uint16_t *__restrict__ reg,
                                                             const uint32_t *__restrict__ rank, uint32_t S,
                                                             uint32_t nreg, uint2 *tab, uint2 *axh) {
    const uint64_t t = uint64_t(blockIdx.x) * kRegBS + threadIdx.x;
    if (t >= uint64_t(S) * nreg) return;
    const uint32_t r = uint32_t(t % nreg), y = uint32_t(t / nreg), H = S / 2;
    const bool axis = y == H;
    const uint16_t *rr = reg + uint64_t(y) * S;
    const uint32_t *rk = rank + uint64_t(y) * S;
    uint2 *out = tab + uint64_t(y) * S * nreg + r;
    const uint2 none = make_uint2(kNoneW, kNoneW);
    uint32_t L = kNoneW, rkL = kNoneW, Ls = kNoneW, rkLs = kNoneW;
    for (uint32_t x = 0; x < S; ++x) {
        if (x == H) Ls = kNoneW;  // (axis row) the Center splits it
        if (rr[x] == r) {
            L = Ls = x;
            rkL = rkLs = rk[x];
        }
        out[uint64_t(x) * nreg] = L != kNoneW ? make_uint2(x - L, rkL) : none;
        if (axis) axh[uint64_t(x) * nreg + r] = Ls != kNoneW ? make_uint2(x - Ls, rkLs) : none;
    }
    uint32_t R = kNoneW, rkR = kNoneW, Rs = kNoneW, rkRs = kNoneW;
    for (uint32_t x = S; x-- > 0;) {
        if (x == H) Rs = kNoneW;
        if (rr[x] == r) {
            R = Rs = x;
            rkR = rkRs = rk[x];
        }
        if (R != kNoneW) {
            const uint2 c = make_uint2(R - x, rkR), cur = out[uint64_t(x) * nreg];
            if (lex_less(c, cur)) out[uint64_t(x) * nreg] = c;
        }
        if (axis && Rs != kNoneW) {
            const uint2 c = make_uint2(Rs - x, rkRs), cur = axh[uint64_t(x) * nreg + r];
            if (lex_less(c, cur)) axh[uint64_t(x) * nreg + r] = c;
        }
    }
}

// pass 2: thread (column x, region r), in place.  Column H also records its half-column
// values (same side of the Center only) in axv[y * nreg + r].
__global__ __launch_bounds__(kRegBS) void region_cols_kernel(const uint16_t *__restrict__ reg,
                                                             const uint32_t *__restrict__ rank, uint32_t S,
                                                             uint32_t nreg, uint2 *tab, uint2 *axv) {
    const uint64_t t = uint64_t(blockIdx.x) * kRegBS + threadIdx.x;
    if (t >= uint64_t(S) * nreg) return;
    const uint32_t r = uint32_t(t % nreg), x = uint32_t(t / nreg), H = S / 2;
    const uint64_t pitch = uint64_t(S) * nreg;  // one row of the table
    uint2 *col = tab + uint64_t(x) * nreg + r;
    const uint2 none = make_uint2(kNoneW, kNoneW);
    uint2 f = none;
    uint2 buf[kPf];
    // down: entries read kPf rows ahead of the dependent chain
    for (uint32_t y0 = 0; y0 < S; y0 += kPf) {
        const uint32_t n = min(uint32_t(kPf), S - y0);
#pragma unroll
        for (int k = 0; k < kPf; ++k)
            if (uint32_t(k) < n) buf[k] = col[uint64_t(y0 + k) * pitch];
#pragma unroll
        for (int k = 0; k < kPf; ++k)
            if (uint32_t(k) < n) {
                f = lex_min(buf[k], plus1(f));
                col[uint64_t(y0 + k) * pitch] = f;
            }
    }
    uint2 b = none;
    for (uint32_t e = S; e > 0;) {
        const uint32_t n = min(uint32_t(kPf), e), y0 = e - n;
#pragma unroll
        for (int k = 0; k < kPf; ++k)
            if (uint32_t(k) < n) buf[k] = col[uint64_t(y0 + n - 1 - k) * pitch];
#pragma unroll
        for (int k = 0; k < kPf; ++k)
            if (uint32_t(k) < n) {
                b = lex_min(buf[k], plus1(b));
                col[uint64_t(y0 + n - 1 - k) * pitch] = b;
            }
        e = y0;
    }
    if (x != H) return;
    // the half-columns of the vertical axis (region cells of column H, same side)
    uint32_t L = kNoneW, rkL = kNoneW;
    for (uint32_t y = 0; y < S; ++y) {
        if (y == H) L = kNoneW;
        const uint64_t c = uint64_t(y) * S + x;
        if (reg[c] == r) {
            L = y;
            rkL = rank[c];
        }
        axv[uint64_t(y) * nreg + r] = L != kNoneW ? make_uint2(y - L, rkL) : none;
    }
    uint32_t R = kNoneW, rkR = kNoneW;
    for (uint32_t y = S; y-- > 0;) {
        if (y == H) R = kNoneW;
        const uint64_t c = uint64_t(y) * S + x;
        if (reg[c] == r) {
            R = y;
            rkR = rank[c];
        }
        if (R != kNoneW) {
            const uint2 cand = make_uint2(R - y, rkR), cur = axv[uint64_t(y) * nreg + r];
            if (lex_less(cand, cur)) axv[uint64_t(y) * nreg + r] = cand;
        }
    }
}

// pass 3: thread (k, r, axis); the Center's entries are {none, none}
__global__ __launch_bounds__(kRegBS) void region_axes_kernel(uint32_t S, uint32_t nreg, uint2 *tab,
                                                             const uint2 *__restrict__ axh,
                                                             const uint2 *__restrict__ axv) {
    const uint64_t t = uint64_t(blockIdx.x) * kRegBS + threadIdx.x;
    if (t >= 2ull * S * nreg) return;
    const uint32_t r = uint32_t(t % nreg), k = uint32_t((t / nreg) % S), vert = uint32_t(t / (uint64_t(S) * nreg));
    const uint32_t H = S / 2;
    const uint64_t V = uint64_t(S) * S;
    (void)V;
    if (k == H) {
        if (!vert) tab[(uint64_t(H) * S + H) * nreg + r] = make_uint2(kNoneW, kNoneW);
        return;
    }
    uint64_t v, a, b;
    uint2 own;
    if (!vert) {  // (k, H): neighbours (k, H - 1) and (k, H + 1)
        v = uint64_t(H) * S + k;
        a = v - S;
        b = v + S;
        own = axh[uint64_t(k) * nreg + r];
    } else {  // (H, k): neighbours (H - 1, k) and (H + 1, k)
        v = uint64_t(k) * S + H;
        a = v - 1;
        b = v + 1;
        own = axv[uint64_t(k) * nreg + r];
    }
    const uint2 m = lex_min(own, lex_min(plus1(tab[a * nreg + r]), plus1(tab[b * nreg + r])));
    tab[v * nreg + r] = m;
}

}  // namespace

// The region table of one homeland into tab (S * S * nreg uint2): reg = region index per
// cell (0xFFFF: none / the Center), rank = CellIndex rank per cell, axis = scratch of
// 2 * S * nreg uint2.  Enqueued on `stream`.
hipError_t region_table_build(const uint16_t *reg, const uint32_t *rank, uint32_t S, uint32_t nreg, void *tab,
                              void *axis, hipStream_t stream) {
    if (S < 3 || !(S & 1u) || nreg == 0) return hipErrorInvalidValue;
    uint2 *T = static_cast<uint2 *>(tab), *axh = static_cast<uint2 *>(axis), *axv = axh + uint64_t(S) * nreg;
    const uint64_t lines = uint64_t(S) * nreg;
    const uint32_t g1 = uint32_t((lines + kRegBS - 1) / kRegBS), g3 = uint32_t((2 * lines + kRegBS - 1) / kRegBS);
    hipLaunchKernelGGL(region_rows_kernel, dim3(g1), dim3(kRegBS), 0, stream, reg, rank, S, nreg, T, axh);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(region_cols_kernel, dim3(g1), dim3(kRegBS), 0, stream, reg, rank, S, nreg, T, axv);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(region_axes_kernel, dim3(g3), dim3(kRegBS), 0, stream, S, nreg, T, axh, axv);
    return hipGetLastError();
}

}  // namespace mr
