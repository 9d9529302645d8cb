// mr_k_groupq.hip — a query batch grouped by source on the device (mr_plan_create's
// host lookups and radix grouping, moved next to the data: the batch goes up raw and
// the plan's per-batch arrays are built where the kernels read them).
//
// The arrays are the host path's (mr_host.cpp build_plan / partition_sources):
//   src_v[s]    the vertex of source s, sources ascending;
//   q_begin[s]  the first grouped position of source s (q_begin[nsrc] = valid queries);
//   q_dst[k]    the destination vertex of grouped position k;
//   q_id[k]     the input query of grouped position k (each source's queries in input
//               order: the LSD radix sort is stable);
// and, for plans on hub_lane_kernel, the same with the sources of at most lane_max_q
// queries first (source order kept within both groups).  A query whose CellIndex is not
// a grid cell (the canonical forms of src/index.rs:257-312 on the map's layout; the
// reference panics, src/grid.rs:288-290) gets no position and is listed in `inv`.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../../include/marshrutka_pf.h"

namespace mr {

// the map's layout (mr_grid: the Center's vertex and the unit steps of each homeland's
// axes and border) — find()'s arithmetic path on a grid whose every cell it was checked for
struct GroupGeom {
    long long vc, ux[4], uy[4], ub[4];
    uint32_t H, V;
};

namespace {

constexpr uint32_t kGBS = 256;

__device__ __forceinline__ bool gq_find(uint2 w, const GroupGeom &g, uint32_t &v) {
    const uint32_t kind = w.x & 0xFFu, sub = (w.x >> 8) & 0xFFu, x = w.x >> 16, y = w.y & 0xFFFFu, res = w.y >> 16;
    if (res != 0) return false;
    long long r = -1;
    if (kind == MR_CELL_CENTER) {
        if (sub == 0 && x == 0 && y == 0) r = g.vc;
    } else if (kind == MR_CELL_HOMELAND) {
        if (sub < 4 && x >= 1 && y >= 1 && x <= g.H && y <= g.H) r = g.vc + x * g.ux[sub] + y * g.uy[sub];
    } else if (kind == MR_CELL_BORDER) {
        if (sub < 4 && x >= 1 && y == 0 && x <= g.H) r = g.vc + x * g.ub[sub];
    }
    if (r < 0 || r >= (long long)g.V) return false;
    v = uint32_t(r);
    return true;
}

// per query: its source vertex as the sort key (V for an invalid query: sorts last)
__global__ __launch_bounds__(kGBS) void gq_lookup_kernel(const uint4 *__restrict__ q, uint32_t n, GroupGeom g,
                                                         uint32_t *__restrict__ key, uint32_t *__restrict__ val,
                                                         uint32_t *__restrict__ dstv, uint32_t *__restrict__ inv,
                                                         uint32_t inv_cap, uint32_t *__restrict__ cnt) {
    for (uint32_t i = blockIdx.x * kGBS + threadIdx.x; i < n; i += gridDim.x * kGBS) {
        const uint4 w = q[i];
        uint32_t a = 0, b = 0;
        const bool ok = gq_find(make_uint2(w.x, w.y), g, a) && gq_find(make_uint2(w.z, w.w), g, b);
        key[i] = ok ? a : g.V;
        val[i] = i;
        dstv[i] = b;
        if (!ok) {
            const uint32_t p = atomicAdd(cnt + 4, 1u);
            if (p < inv_cap) inv[p] = i;
        }
    }
}

// head[k] = 1 where a source's run starts in the sorted keys
__global__ __launch_bounds__(kGBS) void gq_heads_kernel(const uint32_t *__restrict__ key, uint32_t n, uint32_t V,
                                                        uint32_t *__restrict__ head) {
    for (uint32_t k = blockIdx.x * kGBS + threadIdx.x; k < n; k += gridDim.x * kGBS) {
        const uint32_t s = key[k];
        head[k] = (s < V && (k == 0 || key[k - 1] != s)) ? 1u : 0u;
    }
}

// the grouped arrays; sid[k] = (inclusive count of heads) = source of position k + 1.
// cnt[0] = valid queries, cnt[1] = sources (written by the last valid position; zeroed
// by the host before)
__global__ __launch_bounds__(kGBS) void gq_write_kernel(const uint32_t *__restrict__ key,
                                                        const uint32_t *__restrict__ val,
                                                        const uint32_t *__restrict__ dstv,
                                                        const uint32_t *__restrict__ sid, uint32_t n, uint32_t V,
                                                        uint32_t *__restrict__ src_v, uint32_t *__restrict__ q_begin,
                                                        uint32_t *__restrict__ q_dst, uint32_t *__restrict__ q_id,
                                                        uint32_t *__restrict__ cnt) {
    for (uint32_t k = blockIdx.x * kGBS + threadIdx.x; k < n; k += gridDim.x * kGBS) {
        const uint32_t s = key[k];
        if (s >= V) continue;
        const uint32_t si = sid[k] - 1u, i = val[k];
        if (k == 0 || key[k - 1] != s) {
            src_v[si] = s;
            q_begin[si] = k;
        }
        q_dst[k] = dstv[i];
        q_id[k] = i;
        if (k + 1 == n || key[k + 1] >= V) {  // the last valid position
            q_begin[si + 1] = k + 1;
            cnt[0] = k + 1;
            cnt[1] = si + 1;
        }
    }
}

// per source: {small, small ? queries : 0, small ? 0 : queries, 0} (scanned next)
__global__ __launch_bounds__(kGBS) void gq_srcinfo_kernel(const uint32_t *__restrict__ q_begin,
                                                          const uint32_t *__restrict__ cnt, uint32_t n,
                                                          uint32_t lane_max_q, uint4 *__restrict__ info) {
    const uint32_t ns = cnt[1];
    for (uint32_t s = blockIdx.x * kGBS + threadIdx.x; s < n; s += gridDim.x * kGBS) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (s < ns) {
            const uint32_t c = q_begin[s + 1] - q_begin[s];
            const bool small = c <= lane_max_q;
            v = make_uint4(small ? 1u : 0u, small ? c : 0u, small ? 0u : c, 0u);
        }
        info[s] = v;
    }
}

struct Sum4 {
    __host__ __device__ uint4 operator()(const uint4 &a, const uint4 &b) const {
        return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
};

// cnt[2] = sources of at most lane_max_q queries, cnt[3] = their queries
__global__ void gq_totals_kernel(const uint4 *__restrict__ in, const uint4 *__restrict__ ex, uint32_t *__restrict__ cnt) {
    const uint32_t ns = cnt[1];
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (ns == 0) {
        cnt[2] = cnt[3] = 0;
        return;
    }
    cnt[2] = ex[ns - 1].x + in[ns - 1].x;
    cnt[3] = ex[ns - 1].y + in[ns - 1].y;
}

__global__ __launch_bounds__(kGBS) void gq_part_q_kernel(const uint32_t *__restrict__ q_dst,
                                                         const uint32_t *__restrict__ q_id,
                                                         const uint32_t *__restrict__ q_begin,
                                                         const uint32_t *__restrict__ sid,
                                                         const uint32_t *__restrict__ newoff,
                                                         const uint32_t *__restrict__ cnt, uint32_t *__restrict__ qd2,
                                                         uint32_t *__restrict__ qi2) {
    const uint32_t m = cnt[0];
    for (uint32_t k = blockIdx.x * kGBS + threadIdx.x; k < m; k += gridDim.x * kGBS) {
        const uint32_t s = sid[k] - 1u, at = newoff[s] + (k - q_begin[s]);
        qd2[at] = q_dst[k];
        qi2[at] = q_id[k];
    }
}

// the lane kernel's order (phase 2): per source its class key (its query count when at
// most lane_max_q, else lane_max_q + 1: after every small one) and its index
__global__ __launch_bounds__(kGBS) void gq_class_kernel(const uint32_t *__restrict__ q_begin, uint32_t ns,
                                                        uint32_t lane_max_q, bool desc, uint32_t *__restrict__ key,
                                                        uint32_t *__restrict__ val) {
    for (uint32_t s = blockIdx.x * kGBS + threadIdx.x; s < ns; s += gridDim.x * kGBS) {
        const uint32_t c = q_begin[s + 1] - q_begin[s];
        key[s] = c <= lane_max_q ? (desc ? lane_max_q + 1u - c : c) : lane_max_q + 1u;
        val[s] = s;
    }
}

// position j of the new order: its source's query count
__global__ __launch_bounds__(kGBS) void gq_count_sorted_kernel(const uint32_t *__restrict__ q_begin,
                                                               const uint32_t *__restrict__ order, uint32_t ns,
                                                               uint32_t *__restrict__ c) {
    for (uint32_t j = blockIdx.x * kGBS + threadIdx.x; j < ns; j += gridDim.x * kGBS) {
        const uint32_t s = order[j];
        c[j] = q_begin[s + 1] - q_begin[s];
    }
}

// the sources in the new order: index, first position, and each old source's new first
// position (for the queries)
__global__ __launch_bounds__(kGBS) void gq_reorder_src_kernel(const uint32_t *__restrict__ src_v,
                                                              const uint32_t *__restrict__ order,
                                                              const uint32_t *__restrict__ off, uint32_t ns,
                                                              const uint32_t *__restrict__ cnt, uint32_t *__restrict__ src2,
                                                              uint32_t *__restrict__ qb2, uint32_t *__restrict__ newoff) {
    for (uint32_t j = blockIdx.x * kGBS + threadIdx.x; j < ns; j += gridDim.x * kGBS) {
        const uint32_t s = order[j];
        src2[j] = src_v[s];
        qb2[j] = off[j];
        newoff[s] = off[j];
        if (j == 0) qb2[ns] = cnt[0];
    }
}

inline uint32_t grid_of(uint32_t n) { return std::max(1u, std::min(8192u, (n + kGBS - 1) / kGBS)); }
inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace

// Scratch layout of group_queries_device (n queries): key / val in and out, destinations,
// head counts, per-source info and its scan (uint4), the library's temp storage.
struct GroupScratchLayout {
    size_t key_in, key_out, val_in, val_out, dstv, sid, info, ex, temp, temp_bytes, total;
};
static GroupScratchLayout group_layout(uint32_t n, uint32_t bits) {
    GroupScratchLayout L{};
    size_t sort_b = 0, scan_b = 0, scan4_b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (uint32_t *)nullptr, int(n), 0, int(bits));
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_b, (uint32_t *)nullptr, (uint32_t *)nullptr, int(n));
    (void)hipcub::DeviceScan::ExclusiveScan(nullptr, scan4_b, (uint4 *)nullptr, (uint4 *)nullptr, Sum4(),
                                            make_uint4(0, 0, 0, 0), int(n));
    const size_t w = align256(size_t(n) * 4), w4 = align256(size_t(n) * 16);
    size_t at = 0;
    L.key_in = at, at += w;
    L.key_out = at, at += w;
    L.val_in = at, at += w;
    L.val_out = at, at += w;
    L.dstv = at, at += w;
    L.sid = at, at += w;
    L.info = at, at += w4;
    L.ex = at, at += w4;
    L.temp = at;
    L.temp_bytes = align256(std::max(sort_b, std::max(scan_b, scan4_b)));
    L.total = at + L.temp_bytes;
    return L;
}

size_t group_scratch_bytes(uint32_t n, uint32_t V) {
    const uint32_t bits = 32u - uint32_t(__builtin_clz(V));
    return group_layout(n, bits).total;
}

// Phase 1: lookups, the stable sort by source, the grouped arrays and the per-source
// counts.  q: n raw mr_query records on the device; cnt (8 words, zeroed here) ends as
// {valid queries, sources, sources of <= lane_max_q queries, their queries, invalid
// queries, -, -, -}; inv: the first inv_cap invalid query ids (any order).
hipError_t group_queries_device(const void *q, uint32_t n, const GroupGeom &geo, uint32_t lane_max_q, void *scratch,
                                uint32_t *src_v, uint32_t *q_begin, uint32_t *q_dst, uint32_t *q_id, uint32_t *cnt,
                                uint32_t *inv, uint32_t inv_cap, hipStream_t s) {
    const uint32_t bits = 32u - uint32_t(__builtin_clz(geo.V));  // V itself (the invalid key) fits
    const GroupScratchLayout L = group_layout(n, bits);
    char *b = static_cast<char *>(scratch);
    uint32_t *key_in = reinterpret_cast<uint32_t *>(b + L.key_in), *key_out = reinterpret_cast<uint32_t *>(b + L.key_out);
    uint32_t *val_in = reinterpret_cast<uint32_t *>(b + L.val_in), *val_out = reinterpret_cast<uint32_t *>(b + L.val_out);
    uint32_t *dstv = reinterpret_cast<uint32_t *>(b + L.dstv), *sid = reinterpret_cast<uint32_t *>(b + L.sid);
    uint4 *info = reinterpret_cast<uint4 *>(b + L.info), *ex = reinterpret_cast<uint4 *>(b + L.ex);
    void *temp = b + L.temp;
    size_t tb = L.temp_bytes;
    hipError_t e = hipMemsetAsync(cnt, 0, 8 * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(q_begin, 0, 4, s);  // (no valid query: q_begin[0] = 0)
    if (e != hipSuccess || n == 0) return e;
    const uint32_t gb = grid_of(n);
    hipLaunchKernelGGL(gq_lookup_kernel, dim3(gb), dim3(kGBS), 0, s, static_cast<const uint4 *>(q), n, geo, key_in,
                       val_in, dstv, inv, inv_cap, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(temp, tb, key_in, key_out, val_in, val_out, int(n), 0, int(bits), s)) !=
        hipSuccess)
        return e;
    hipLaunchKernelGGL(gq_heads_kernel, dim3(gb), dim3(kGBS), 0, s, key_out, n, geo.V, key_in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.temp_bytes;
    if ((e = hipcub::DeviceScan::InclusiveSum(temp, tb, key_in, sid, int(n), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(gq_write_kernel, dim3(gb), dim3(kGBS), 0, s, key_out, val_out, dstv, sid, n, geo.V, src_v, q_begin,
                       q_dst, q_id, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(gq_srcinfo_kernel, dim3(gb), dim3(kGBS), 0, s, q_begin, cnt, n, lane_max_q, info);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveScan(temp, tb, info, ex, Sum4(), make_uint4(0, 0, 0, 0), int(n), s)) !=
        hipSuccess)
        return e;
    hipLaunchKernelGGL(gq_totals_kernel, dim3(1), dim3(64), 0, s, info, ex, cnt);
    return hipGetLastError();
}

// Phase 2 (plans on hub_lane_kernel): the sources in the lane kernel's order into src2 /
// qb2 / qd2 / qi2 (the same sizes): by query count, 1 to lane_max_q, then the sources of
// more queries (hub_kernel's), each class in source order.  A wave of the lane kernel runs
// its destination loop as often as its busiest lane's source has queries: grouped by
// count, its 64 sources have the same.  Reads phase 1's scratch and counts; ns: the sources.
hipError_t partition_sources_device(uint32_t n, uint32_t V, uint32_t ns, uint32_t lane_max_q, bool desc, const void *scratch,
                                    const uint32_t *src_v, const uint32_t *q_begin, const uint32_t *q_dst,
                                    const uint32_t *q_id, const uint32_t *cnt, uint32_t *src2, uint32_t *qb2,
                                    uint32_t *qd2, uint32_t *qi2, hipStream_t s) {
    const uint32_t bits = 32u - uint32_t(__builtin_clz(V));
    const GroupScratchLayout L = group_layout(n, bits);
    char *b = static_cast<char *>(const_cast<void *>(scratch));
    const uint32_t *sid = reinterpret_cast<const uint32_t *>(b + L.sid);
    // phase 1's consumed words: the new first positions per source (key_in), the class
    // keys and source indices before and after the sort, the sorted counts and their scan
    uint32_t *newoff = reinterpret_cast<uint32_t *>(b + L.key_in);
    uint32_t *k_in = reinterpret_cast<uint32_t *>(b + L.key_out), *k_out = reinterpret_cast<uint32_t *>(b + L.dstv);
    uint32_t *v_in = reinterpret_cast<uint32_t *>(b + L.val_in), *v_out = reinterpret_cast<uint32_t *>(b + L.val_out);
    uint32_t *c_sorted = reinterpret_cast<uint32_t *>(b + L.info), *off = reinterpret_cast<uint32_t *>(b + L.ex);
    void *temp = b + L.temp;
    size_t tb = L.temp_bytes;
    const uint32_t gs = grid_of(ns), gb = grid_of(n);
    const uint32_t kbits = 32u - uint32_t(__builtin_clz(lane_max_q + 1u));
    {  // (phase 1's temp storage, sized for n keys of the cells' width, holds these)
        size_t need_sort = 0, need_scan = 0;
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, need_sort, k_in, k_out, v_in, v_out, int(ns), 0, int(kbits), s);
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, need_scan, c_sorted, off, int(ns), s);
        if (need_sort > tb || need_scan > tb) return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(gq_class_kernel, dim3(gs), dim3(kGBS), 0, s, q_begin, ns, lane_max_q, desc, k_in, v_in);
    hipError_t e = hipGetLastError();
    // stable: equal classes keep the source order (by cell)
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(temp, tb, k_in, k_out, v_in, v_out, int(ns), 0, int(kbits), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gq_count_sorted_kernel, dim3(gs), dim3(kGBS), 0, s, q_begin, v_out, ns, c_sorted);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(temp, tb, c_sorted, off, int(ns), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(gq_reorder_src_kernel, dim3(gs), dim3(kGBS), 0, s, src_v, v_out, off, ns, cnt, src2, qb2, newoff);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(gq_part_q_kernel, dim3(gb), dim3(kGBS), 0, s, q_dst, q_id, q_begin, sid, newoff, cnt, qd2, qi2);
    return hipGetLastError();
}

}  // namespace mr
