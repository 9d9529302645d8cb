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


// ---- the parallel build (S <= kLineMax): one workgroup per line, segmented column scans ----
//
// Round 5 ran one thread per (line, region): 4 100 threads at 1025^2, 3.25 ms of kernel time
// for a 34 MB table (latency of one dependent chain per line).  Now:
//   1. rows: one workgroup per row loads the row's regions and ranks into LDS, cuts the row
//      into runs of one region (a block-wide scan of the run heads), lists each region's runs
//      in order, and writes every (cell, region) entry from a binary search over that
//      region's runs (the nearest region cell left and right: the end of the last run that
//      starts at or before the cell, the start of the first run that ends at or after it);
//   2. columns: the L1 transform f(y) = min(g(y), f(y - 1) + 1) (down, then up) is a scan
//      with the carry c -> c + n across a segment of n rows, so each (segment, column,
//      region) thread scans its kSeg rows in registers and leaves its two aggregates, one
//      thread per (column, region) turns them into the carries entering each segment, and
//      the segment threads rescan from their carries and write min(down, up) once;
//   3. the axis lines as before (region_axes_kernel).
// The same three-pass transform as the serial kernels above (which stay for S > kLineMax),
// so tests/region_util.py models both.
constexpr uint32_t kLineMax = 8192;  // LDS: 2 + 4 + 2 + 2 + 2 B per cell of the line
constexpr uint32_t kLineBS = 256;
constexpr uint32_t kSeg = 64;        // rows per column segment (registers: kSeg uint2)
constexpr uint32_t kMaxReg = 1024;   // regions a homeland may have (LDS counters)

__device__ __forceinline__ uint2 plus_n(uint2 a, uint32_t n) { return a.x == kNoneW ? a : make_uint2(a.x + n, a.y); }

// One line of n cells (cell i at base + i * step): rows (COL = false, line = blockIdx.x)
// write their table row, and the Center's row also its same-side half-row values (axh);
// the vertical axis (COL = true, one workgroup, column H) writes its half-column values
// (axv) only.
template <bool COL>
__global__ __launch_bounds__(kLineBS) void region_line_kernel(const uint16_t *__restrict__ reg,
                                                              const uint32_t *__restrict__ rank, uint32_t S,
                                                              uint32_t nreg, uint2 *tab, uint2 *axh, uint2 *axv) {
    extern __shared__ uint32_t lds[];
    const uint32_t n = S, H = S / 2, tid = threadIdx.x;
    const uint32_t y = COL ? H : blockIdx.x;
    const uint64_t base = COL ? H : uint64_t(y) * S, step = COL ? S : 1;
    uint32_t *rk = lds;                                    // n: rank of cell i
    uint16_t *rg = reinterpret_cast<uint16_t *>(rk + n);   // n: region of cell i (0xFFFF: none)
    uint16_t *rs = rg + n;                                 // runs: start (n at most)
    uint16_t *lst = rs + n;                                // runs listed by region, in order
    uint16_t *pad = lst + n;                               // (keeps the counters 4-byte aligned)
    uint32_t *cnt = reinterpret_cast<uint32_t *>(pad + (n & 1u ? 1 : 2));  // kMaxReg + 1: region offsets
    __shared__ uint32_t part[kLineBS];
    __shared__ uint32_t nruns;
    for (uint32_t i = tid; i < n; i += kLineBS) {
        rg[i] = reg[base + i * step];
        rk[i] = rank[base + i * step];
    }
    for (uint32_t r = tid; r <= nreg; r += kLineBS) cnt[r] = 0;
    __syncthreads();
    // run heads: block-wide exclusive scan of the per-thread counts (contiguous chunks)
    const uint32_t per = (n + kLineBS - 1) / kLineBS, i0 = min(n, tid * per), i1 = min(n, i0 + per);
    uint32_t c = 0;
    for (uint32_t i = i0; i < i1; ++i) c += (i == 0 || rg[i] != rg[i - 1]) ? 1u : 0u;
    part[tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < kLineBS; d <<= 1) {
        const uint32_t v = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t k = part[tid] - c;
    for (uint32_t i = i0; i < i1; ++i)
        if (i == 0 || rg[i] != rg[i - 1]) {
            rs[k++] = uint16_t(i);
            if (rg[i] < nreg) atomicAdd(&cnt[rg[i]], 1u);
        }
    if (tid == kLineBS - 1) nruns = part[tid];
    __syncthreads();
    if (tid == 0) {  // exclusive offsets by region (cnt[nreg] = the listed runs)
        uint32_t acc = 0;
        for (uint32_t r = 0; r < nreg; ++r) {
            const uint32_t x = cnt[r];
            cnt[r] = acc;
            acc += x;
        }
        cnt[nreg] = acc;
    }
    __syncthreads();
    // each region lists its runs in line order
    const uint32_t nr = nruns;
    for (uint32_t r = tid; r < nreg; r += kLineBS) {
        uint32_t at = cnt[r];
        for (uint32_t q = 0; q < nr; ++q)
            if (rg[rs[q]] == r) lst[at++] = uint16_t(q);
    }
    __syncthreads();
    auto run_end = [&](uint32_t q) { return q + 1 < nr ? uint32_t(rs[q + 1]) - 1u : n - 1u; };
    const uint2 none = make_uint2(kNoneW, kNoneW);
    const bool half = COL || y == H;  // this line also has same-side (Center-split) values
    // entries (i, r), regions fastest
    const uint32_t di = kLineBS / nreg, dr = kLineBS % nreg;
    uint32_t i = tid / nreg, r = tid % nreg;
    for (uint64_t e = tid; e < uint64_t(n) * nreg; e += kLineBS) {
        const uint32_t lo = cnt[r], m = cnt[r + 1] - lo;
        // the last listed run of region r that starts at or before i
        uint32_t a = 0, b = m;  // answer in [a - 1, b): the count of runs starting <= i
        while (a < b) {
            const uint32_t mid = (a + b) >> 1;
            if (rs[lst[lo + mid]] <= i) a = mid + 1;
            else b = mid;
        }
        uint32_t L = kNoneW, R = kNoneW;
        if (a > 0) {
            const uint32_t q = lst[lo + a - 1], e1 = run_end(q);
            L = min(i, e1);
            if (i <= e1) R = i;
        }
        if (R == kNoneW && a < m) R = rs[lst[lo + a]];
        const uint2 cl = L != kNoneW ? make_uint2(i - L, rk[L]) : none;
        const uint2 cr = R != kNoneW ? make_uint2(R - i, rk[R]) : none;
        if (!COL) tab[(uint64_t(y) * S + i) * nreg + r] = lex_min(cl, cr);
        if (half) {  // the Center (cell H of the line, region none) splits it
            const bool ls = L != kNoneW && (L < H) == (i < H) && i != H, rsd = R != kNoneW && (R < H) == (i < H) && i != H;
            const uint2 v = lex_min(ls ? cl : none, rsd ? cr : none);
            (COL ? axv : axh)[uint64_t(i) * nreg + r] = v;
        }
        i += di;
        r += dr;
        if (r >= nreg) {
            r -= nreg;
            ++i;
        }
    }
}

// Column pass, step 1: thread (segment, column, region): the segment's down aggregate (f at
// its last row from its own rows) and up aggregate (at its first row), into agg[2 * j]
// and agg[2 * j + 1] for j = segment * S * nreg + column * nreg + region
__global__ __launch_bounds__(kLineBS) void region_seg_agg_kernel(uint32_t S, uint32_t nreg, const uint2 *__restrict__ tab,
                                                                 uint2 *agg) {
    const uint64_t cols = uint64_t(S) * nreg, t = uint64_t(blockIdx.x) * kLineBS + threadIdx.x;
    const uint32_t nseg = (S + kSeg - 1) / kSeg;
    if (t >= cols * nseg) return;
    const uint32_t seg = uint32_t(t / cols);
    const uint64_t col = t - uint64_t(seg) * cols;
    const uint32_t y0 = seg * kSeg, len = min(kSeg, S - y0);
    const uint2 none = make_uint2(kNoneW, kNoneW);
    uint2 g[kSeg];
#pragma unroll
    for (uint32_t k = 0; k < kSeg; ++k) g[k] = k < len ? tab[uint64_t(y0 + k) * cols + col] : none;
    uint2 dn = none, up = none;
#pragma unroll
    for (uint32_t k = 0; k < kSeg; ++k)
        if (k < len) dn = lex_min(g[k], plus1(dn));
#pragma unroll
    for (uint32_t k = kSeg; k-- > 0;)
        if (k < len) up = lex_min(g[k], plus1(up));
    agg[2 * t] = dn;
    agg[2 * t + 1] = up;
}

// step 2: thread (column, region): the carries entering each segment, in place (down:
// f at the row above the segment; up: f at the row below it)
__global__ __launch_bounds__(kLineBS) void region_seg_carry_kernel(uint32_t S, uint32_t nreg, uint2 *agg) {
    const uint64_t cols = uint64_t(S) * nreg, t = uint64_t(blockIdx.x) * kLineBS + threadIdx.x;
    if (t >= cols) return;
    const uint32_t nseg = (S + kSeg - 1) / kSeg;
    uint2 c = make_uint2(kNoneW, kNoneW);
    for (uint32_t s = 0; s < nseg; ++s) {
        uint2 *p = agg + 2 * (uint64_t(s) * cols + t);
        const uint2 a = p[0];
        p[0] = c;
        c = lex_min(a, plus_n(c, min(kSeg, S - s * kSeg)));
    }
    c = make_uint2(kNoneW, kNoneW);
    for (uint32_t s = nseg; s-- > 0;) {
        uint2 *p = agg + 2 * (uint64_t(s) * cols + t) + 1;
        const uint2 a = p[0];
        p[0] = c;
        c = lex_min(a, plus_n(c, min(kSeg, S - s * kSeg)));
    }
}

// step 3: thread (segment, column, region): rescan from the carries, min(down, up) out
__global__ __launch_bounds__(kLineBS) void region_seg_apply_kernel(uint32_t S, uint32_t nreg, uint2 *tab,
                                                                   const uint2 *__restrict__ agg) {
    const uint64_t cols = uint64_t(S) * nreg, t = uint64_t(blockIdx.x) * kLineBS + threadIdx.x;
    const uint32_t nseg = (S + kSeg - 1) / kSeg;
    if (t >= cols * nseg) return;
    const uint32_t seg = uint32_t(t / cols);
    const uint64_t col = t - uint64_t(seg) * cols;
    const uint32_t y0 = seg * kSeg, len = min(kSeg, S - y0);
    const uint2 none = make_uint2(kNoneW, kNoneW);
    uint2 g[kSeg];
#pragma unroll
    for (uint32_t k = 0; k < kSeg; ++k) g[k] = k < len ? tab[uint64_t(y0 + k) * cols + col] : none;
    uint2 dn = agg[2 * t];
#pragma unroll
    for (uint32_t k = 0; k < kSeg; ++k) {
        dn = lex_min(g[k], plus1(dn));
        g[k] = dn;  // (g[k] itself is no longer needed: f_down(k) <= g(k))
    }
    uint2 up = agg[2 * t + 1];
#pragma unroll
    for (uint32_t k = kSeg; k-- > 0;)
        if (k < len) {
            up = lex_min(g[k], plus1(up));  // min(f_down(k), f_up(k + 1) + 1) = the full transform
            tab[uint64_t(y0 + k) * cols + col] = up;
        }
}

}  // namespace

// The region table of one homeland into tab (S * S * nreg uint2): reg = region index per
// cell (0xFFFF: none / the Center), rank = CellIndex rank per cell, axis = scratch of
// 2 * S * nreg uint2, seg = scratch of region_table_seg_words(S, nreg) uint2 (the parallel
// build; nullptr takes the serial kernels).  Enqueued on `stream`.
uint64_t region_table_seg_words(uint32_t S, uint32_t nreg) {
    if (S > kLineMax || nreg > kMaxReg) return 0;
    return 2ull * ((S + kSeg - 1) / kSeg) * S * nreg;
}

hipError_t region_table_build(const uint16_t *reg, const uint32_t *rank, uint32_t S, uint32_t nreg, void *tab,
                              void *axis, void *seg, hipStream_t stream) {
    if (S < 3 || !(S & 1u) || nreg == 0) return hipErrorInvalidValue;
    uint2 *T = static_cast<uint2 *>(tab), *axh = static_cast<uint2 *>(axis), *axv = axh + uint64_t(S) * nreg;
    const uint64_t lines = uint64_t(S) * nreg;
    const uint32_t g1 = uint32_t((lines + kRegBS - 1) / kRegBS), g3 = uint32_t((2 * lines + kRegBS - 1) / kRegBS);
    hipError_t e;
    if (seg && region_table_seg_words(S, nreg)) {
        const size_t lds = size_t(S) * 12 + 8 + (kMaxReg + 1) * 4;
        hipLaunchKernelGGL(region_line_kernel<false>, dim3(S), dim3(kLineBS), lds, stream, reg, rank, S, nreg, T, axh, axv);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(region_line_kernel<true>, dim3(1), dim3(kLineBS), lds, stream, reg, rank, S, nreg, T, axh, axv);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        uint2 *A = static_cast<uint2 *>(seg);
        const uint64_t items = lines * ((S + kSeg - 1) / kSeg);
        const uint32_t gs = uint32_t((items + kLineBS - 1) / kLineBS), gc = uint32_t((lines + kLineBS - 1) / kLineBS);
        hipLaunchKernelGGL(region_seg_agg_kernel, dim3(gs), dim3(kLineBS), 0, stream, S, nreg, T, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(region_seg_carry_kernel, dim3(gc), dim3(kLineBS), 0, stream, S, nreg, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(region_seg_apply_kernel, dim3(gs), dim3(kLineBS), 0, stream, S, nreg, T, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(region_rows_kernel, dim3(g1), dim3(kRegBS), 0, stream, reg, rank, S, nreg, T, axh);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(region_cols_kernel, dim3(g1), dim3(kRegBS), 0, stream, reg, rank, S, nreg, T, axv);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(region_axes_kernel, dim3(g3), dim3(kRegBS), 0, stream, S, nreg, T, axh, axv);
    return hipGetLastError();
}

}  // namespace mr
