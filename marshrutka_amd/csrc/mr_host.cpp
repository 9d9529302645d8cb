// mr_host.cpp — host side of libmarshrutka_pf.so: grid construction and
// validation, per-query planning, the C ABI of include/marshrutka_pf.h.
//
// There is no CPU fallback: every query runs on the gfx950 device; without one
// the entry points return MR_ERR_NO_DEVICE (include/marshrutka_pf.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <chrono>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/marshrutka_pf.h"
#include "mr_engine.hpp"
#include "mr_pool.hpp"

// hipMalloc for the grid's long-lived device tables: on out-of-memory the plan block
// cache (below) is trimmed and the allocation retried once
static hipError_t dev_malloc(void **p, size_t bytes);

namespace mr {
uint32_t lds_bytes(uint32_t NS, uint32_t V, bool grid_in_lds, uint32_t algo);
hipError_t launch_solve(const KArgs *d_args, bool grid_in_lds, uint32_t algo, uint32_t NS, uint32_t V,
                        uint32_t blocks, hipStream_t stream);
int max_blocks_per_cu(bool grid_in_lds, uint32_t algo, uint32_t bytes);
uint32_t hub_lds_bytes(uint32_t NS, uint32_t nreg, uint32_t spw);
hipError_t launch_hub(const KArgs *d_args, const uint32_t perm[3], uint32_t spw, bool nonlin, uint32_t NS, uint32_t nreg,
                      uint32_t blocks, hipStream_t stream);
hipError_t launch_fill(const KArgs *d_args, const uint32_t perm[3], uint32_t gx, uint32_t gy, hipStream_t stream);
int hub_blocks_per_cu(const uint32_t perm[3], uint32_t spw, bool nonlin, uint32_t bytes);
int fill_blocks_per_cu(const uint32_t perm[3]);
hipError_t launch_hub_fill(const KArgs *hub_args, const KArgs *fill_args, const uint32_t perm[3], uint32_t spw,
                           uint32_t hub_blocks, uint32_t fill_blocks, uint32_t lds_bytes, hipStream_t stream);
int hub_fill_blocks_per_cu(const uint32_t perm[3], uint32_t spw, uint32_t lds_bytes);
uint32_t hub_wide_lds_bytes(uint32_t NS, uint32_t nreg);
uint32_t hub_wide_spl(uint32_t NS);
hipError_t launch_hub_wide(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t blocks,
                           hipStream_t stream);
int hub_wide_blocks_per_cu(const uint32_t perm[3], uint32_t NS, uint32_t bytes);
uint32_t hub_lane_entries(uint32_t NS);
hipError_t launch_hub_lane(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t n_lane,
                           bool nonlin, hipStream_t stream);
uint32_t hub_group_slots(uint32_t NS, uint32_t G);
uint32_t lane_blob_build(const SpecialStatic *sp, uint32_t NS, uint32_t nreg, uint32_t TM, uint32_t rgt,
                         uint32_t ff_num, uint32_t ff_den, const uint32_t *near_sp, std::vector<uint32_t> &blob);
uint64_t region_table_seg_words(uint32_t S, uint32_t nreg);
hipError_t region_table_build(const uint16_t *reg, const uint32_t *rank, uint32_t S, uint32_t nreg, void *tab,
                              void *axis, void *seg, hipStream_t stream);
struct GroupGeom {
    long long vc, ux[4], uy[4], ub[4];
    uint32_t H, V;
};
size_t group_scratch_bytes(uint32_t n, uint32_t V);
hipError_t group_queries_device(const void *q, uint32_t n, const GroupGeom &geo, uint32_t lane_max_q, void *scratch,
                                uint32_t *src_v, uint32_t *q_begin, uint32_t *q_dst, uint32_t *q_id, uint32_t *cnt,
                                uint32_t *inv, uint32_t inv_cap, hipStream_t s);
hipError_t partition_sources_device(uint32_t n, uint32_t V, uint32_t ns, uint32_t lane_max_q, bool desc, const void *scratch,
                                    const uint32_t *src_v, const uint32_t *q_begin, const uint32_t *q_dst,
                                    const uint32_t *q_id, const uint32_t *cnt, uint32_t *src2, uint32_t *qb2,
                                    uint32_t *qd2, uint32_t *qi2, hipStream_t s);
uint32_t hub_group_lds_bytes(uint32_t NS, uint32_t nreg, uint32_t G);
hipError_t launch_hub_group(const KArgs *d_args, const uint32_t perm[3], uint32_t NS, uint32_t nreg, uint32_t n,
                            uint32_t G, bool nonlin, hipStream_t stream);
hipError_t launch_cert_select(const KArgs *d_args, hipStream_t stream);
hipError_t launch_cert_check(const KArgs *d_args, uint32_t gx, uint32_t slots, uint32_t mark, hipStream_t stream);
hipError_t launch_cert_sweep(const KArgs *d_args, uint32_t slots, hipStream_t stream);
hipError_t launch_cert_window(const KArgs *d_args, uint32_t slots, hipStream_t stream);
hipError_t launch_cert_tile(const KArgs *d_args, uint32_t wgs, hipStream_t stream);
hipError_t launch_cert_promote(const KArgs *d_args, uint32_t slots, uint32_t *redo, hipStream_t stream);
constexpr int kCertRounds = 2;  // certificate rounds after the first (cert_promote_kernel decides each slot's)
int cert_tile_occupancy();
hipError_t launch_ovf_order(const KArgs *d_args, uint32_t nrec, OutCmd *tmp, hipStream_t stream);
hipError_t launch_wire(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, const uint32_t *nov, uint32_t ovf_cap,
                       uint32_t nrec, uint32_t nq, uint32_t mc, const uint32_t *q_id, uint32_t *rows, uint32_t *wpool,
                       uint32_t wpool_cap, hipStream_t stream);
hipError_t wire_fetch_device(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, const uint32_t *nov,
                             uint32_t ovf_cap, const uint32_t *q_id, uint32_t nrec, uint32_t nq, uint32_t mc, uint32_t *cnt,
                             uint32_t *off, void *temp, size_t *temp_bytes, uint32_t *rows, uint32_t *wpool,
                             uint32_t wpool_cap, hipStream_t stream);
hipError_t decode_records_device(const OutResult *res, const OutCmd *slots, const OutCmd *ovf, uint32_t novf,
                                 const uint32_t *q_id, uint32_t nrec, uint32_t nq, uint32_t mc,
                                 const mr_cell_index *idx_rank, uint32_t V, uint32_t rgt, uint32_t soe, uint32_t shq,
                                 uint32_t sfm, uint32_t ff, uint32_t *cnt, uint32_t *off, void *temp, size_t *temp_bytes,
                                 mr_result *out, mr_command *pool, unsigned long long pool_cap, uint32_t *err,
                                 hipStream_t stream);
}  // namespace mr



using namespace mr;

static thread_local std::string g_last_error;
// MR_TIMING=1: host phase times of plan creation and fetch on stderr (diagnostics)
static bool timing_on() {
    static const bool on = std::getenv("MR_TIMING") != nullptr;
    return on;
}
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// [0, n) in `parts` near-equal ranges: range p is [chunk_lo(n, parts, p), chunk_lo(n, parts, p + 1))
static inline uint32_t chunk_lo(uint32_t n, uint32_t parts, uint32_t p) { return uint32_t(uint64_t(n) * p / parts); }

// ------------------------------------------------------------------ CellIndex
static inline uint64_t ci_key(const mr_cell_index &c) {
    return (uint64_t(c.kind) << 48) | (uint64_t(c.sub) << 40) | (uint64_t(c.x) << 20) | uint64_t(c.y);
}
static inline mr_cell_index ci_make(uint8_t kind, uint8_t sub, uint16_t x, uint16_t y) {
    mr_cell_index c;
    c.kind = kind;
    c.sub = sub;
    c.x = x;
    c.y = y;
    c.reserved = 0;
    return c;
}
// CellIndexBuilder::build (src/index.rs:257-312)
static mr_cell_index build_homeland(int h, int x, int y) {
    if (x == 0 && y == 0) return ci_make(MR_CELL_CENTER, 0, 0, 0);
    if (x == 0) return ci_make(MR_CELL_BORDER, (h == MR_HOMELAND_YELLOW || h == MR_HOMELAND_BLUE) ? MR_BORDER_YB : MR_BORDER_RG, uint16_t(y), 0);
    if (y == 0) return ci_make(MR_CELL_BORDER, (h == MR_HOMELAND_BLUE || h == MR_HOMELAND_RED) ? MR_BORDER_BR : MR_BORDER_GY, uint16_t(x), 0);
    return ci_make(MR_CELL_HOMELAND, uint8_t(h), uint16_t(x), uint16_t(y));
}
static mr_cell_index build_border(int b, int s) {
    if (s == 0) return ci_make(MR_CELL_CENTER, 0, 0, 0);
    return ci_make(MR_CELL_BORDER, uint8_t(b), uint16_t(s), 0);
}
// CellIndexBuilder::build on a raw (homeland, x, y) / (border, shift) index
namespace mr {
mr_cell_index build_index(const mr_cell_index &c) {
    if (c.kind == MR_CELL_HOMELAND && c.sub < 4) return build_homeland(c.sub, c.x, c.y);
    if (c.kind == MR_CELL_BORDER && c.sub < 4 && c.y == 0) return build_border(c.sub, c.x);
    return c;
}
}  // namespace mr
static bool canonical(const mr_cell_index &c) {
    if (c.reserved) return false;
    if (c.kind == MR_CELL_CENTER) return c.sub == 0 && c.x == 0 && c.y == 0;
    if (c.kind == MR_CELL_HOMELAND) return c.sub < 4 && c.x >= 1 && c.y >= 1;
    if (c.kind == MR_CELL_BORDER) return c.sub < 4 && c.x >= 1 && c.y == 0;
    return false;
}
// The StandardMove/CentralMove neighbours the reference generates for a cell
// (Inflight::edges, src/pathfinder.rs:24-138), used to validate that the map's
// labels form the geometric 4-grid the kernels traverse implicitly.
static void index_neighbours(const mr_cell_index &v, int H, std::vector<uint64_t> &out) {
    static const int bn[4][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}};  // Border::neighbours
    static const int hb[4][2] = {{MR_BORDER_BR, MR_BORDER_YB}, {MR_BORDER_BR, MR_BORDER_RG},
                                 {MR_BORDER_GY, MR_BORDER_RG}, {MR_BORDER_GY, MR_BORDER_YB}};  // [h][hor, vert]
    out.clear();
    if (v.kind == MR_CELL_CENTER) {
        for (int b = 0; b < 4; ++b) out.push_back(ci_key(build_border(b, 1)));
    } else if (v.kind == MR_CELL_BORDER) {
        int b = v.sub, s = v.x;
        out.push_back(ci_key(build_border(b, s - 1)));
        if (s < H) out.push_back(ci_key(build_border(b, s + 1)));
        bool horizontal = (b == MR_BORDER_BR || b == MR_BORDER_GY);
        for (int k = 0; k < 2; ++k)
            out.push_back(ci_key(horizontal ? build_homeland(bn[b][k], s, 1) : build_homeland(bn[b][k], 1, s)));
    } else {
        int h = v.sub, x = v.x, y = v.y;
        out.push_back(ci_key(x == 1 ? build_border(hb[h][1], y) : build_homeland(h, x - 1, y)));
        out.push_back(ci_key(y == 1 ? build_border(hb[h][0], x) : build_homeland(h, x, y - 1)));
        if (x < H) out.push_back(ci_key(build_homeland(h, x + 1, y)));
        if (y < H) out.push_back(ci_key(build_homeland(h, x, y + 1)));
    }
    std::sort(out.begin(), out.end());
}

// ------------------------------------------------------------------ grid
struct mr_grid {
    uint32_t S = 0, H = 0, V = 0, vc = 0;
    std::vector<mr_cell_index> idx;
    std::vector<uint8_t> poi;
    std::unordered_map<uint64_t, uint32_t> index;
    std::vector<uint32_t> rank;
    std::vector<uint32_t> rank_inv;        // vertex of each rank
    std::vector<uint32_t> campfires;       // vertex ids, CellIndex order
    std::vector<uint32_t> nearest[4];      // nearest campfire vertex per homeland (kNone32)
    // hub solver: per homeland, the regions (campfires of the homeland, CellIndex order) and
    // (on the device, d_near) for every vertex and region the nearest cell of that region by
    // walk distance avoiding the Center, ties by CellIndex order:
    // near[2*(v*nreg+r)] = {distance, rank of the cell}
    mutable std::mutex near_mu;
    mutable std::vector<uint32_t> regions[4];
    mutable bool regions_built[4] = {false, false, false, false};
    mutable double region_ms[4] = {0, 0, 0, 0};  // device build time of each table (ms, wall)
    // wide hub solver: per homeland, each region's boundary cells (cells of the region
    // with a neighbour outside it, the Center excluded), {x | y << 16, rank}, by region
    mutable std::vector<uint32_t> rb_off[4], rb_cell[4];
    mutable bool rb_built[4] = {false, false, false, false};
    // wide hub solver without the region table: a special cell's row of {distance, rank}
    // per region, scanned from the boundary cells once per (homeland, cell)
    mutable std::unordered_map<uint32_t, std::vector<uint32_t>> near_sp_cache[4];
    // device copies of the region tables, built on first use and shared by the grid's
    // plans (the grid outlives its plans): one per (device, homeland), so a plan never
    // reads a table that lives on another device
    mutable std::map<std::pair<int, int>, uint32_t *> d_near;
    // CellIndex of each rank, built on first use by a wire fetch (idx_of_rank)
    mutable std::vector<mr_cell_index> idx_rank_h;
    // device copies shared by the grid's plans on one device (the first plan's): the rank
    // tables, and per (query homeland, HQ cell) the special / region word of every cell
    // (sinfo: it depends on the special order, fixed by those two)
    mutable int d_dev = -1;
    mutable uint32_t *d_rank = nullptr, *d_rank_inv = nullptr;
    struct SinfoDev {
        uint32_t homeland, hq_v;
        uint32_t *d;
        uint2 *cell;  // {sinfo, rank} per cell
    };
    mutable std::vector<SinfoDev> d_sinfo;
    mutable mr_cell_index *d_idx_rank = nullptr;  // device fetch: the CellIndex of every rank
    ~mr_grid() {
        if (d_idx_rank) (void)hipFree(d_idx_rank);
        for (auto &kv : d_near)
            if (kv.second) (void)hipFree(kv.second);
        for (uint32_t *p : {d_rank, d_rank_inv})
            if (p) (void)hipFree(p);
        for (const SinfoDev &e : d_sinfo) {
            (void)hipFree(e.d);
            (void)hipFree(e.cell);
        }
    }
    int32_t gx(uint32_t v) const { return int32_t(v % S) - int32_t(H); }
    int32_t gy(uint32_t v) const { return int32_t(v / S) - int32_t(H); }
    // The geometric layout (checked at creation): homeland cell (h, x, y) at vertex
    // vc + x ux[h] + y uy[h], border cell (b, s) at vc + s ub[b]; find() computes the
    // vertex and confirms it against idx[] (the hash map is the fallback).  When the
    // formula was verified for every cell at creation (`exact`), the confirmation is
    // skipped: a query batch's lookups then touch no per-cell table.
    bool fast = false, exact = false;
    bool rank_std = false;  // rank[v] = std_rank(position of v) for every cell (mr_hub_lane.hpp)
    int64_t ux[4] = {0, 0, 0, 0}, uy[4] = {0, 0, 0, 0}, ub[4] = {0, 0, 0, 0};
    bool find(const mr_cell_index &c, uint32_t &v) const {
        if (!canonical(c)) return false;
        if (fast) {
            int64_t w = -1;
            if (c.kind == MR_CELL_CENTER) w = vc;
            else if (c.kind == MR_CELL_HOMELAND && c.x <= H && c.y <= H) w = int64_t(vc) + c.x * ux[c.sub] + c.y * uy[c.sub];
            else if (c.kind == MR_CELL_BORDER && c.x <= H) w = int64_t(vc) + c.x * ub[c.sub];
            if (w >= 0 && w < int64_t(V)) {
                if (exact) {
                    v = uint32_t(w);
                    return true;
                }
                const mr_cell_index &e = idx[size_t(w)];
                if (e.kind == c.kind && e.sub == c.sub && e.x == c.x && e.y == c.y) {
                    v = uint32_t(w);
                    return true;
                }
            }
        }
        auto it = index.find(ci_key(c));
        if (it == index.end()) return false;
        v = it->second;
        return true;
    }
};

static constexpr uint32_t kNone32 = 0xFFFFFFFFu;

// CellIndex rank (position in the derived Ord, src/index.rs:41-46) of a canonical index
// on a complete map of homeland size H: Center, then Homeland{h, (x, y)} by (h, x, y),
// then Border{b, shift} by (b, shift)
static inline uint32_t closed_rank(const mr_cell_index &c, uint32_t H) {
    if (c.kind == MR_CELL_CENTER) return 0;
    if (c.kind == MR_CELL_HOMELAND) return 1u + c.sub * H * H + (c.x - 1u) * H + (c.y - 1u);
    return 1u + 4u * H * H + c.sub * H + (c.x - 1u);
}

// Grid creation's fast path (host threads, no hash map): the cells' labels are every
// canonical index of homeland size H, laid out by one unit step per homeland axis and
// border (any orientation).  It checks every cell against that layout (a bijection onto
// the V canonical indices), the index adjacency (src/pathfinder.rs:24-138) against the
// geometric 4-neighbourhood on the cells near the axes, the Center and the edges (every
// other cell repeats the neighbourhood of a homeland cell (2, 2)), and computes the
// ranks in closed form.  False (nothing decided) sends the map to the generic path,
// which also reports what is wrong with it.
static bool grid_fast_layout(mr_grid *g, const mr_cell *cells) {
    const uint32_t n = g->V, S = g->S, H = g->H;
    if (H < 3) return false;
    HostPool &pool = HostPool::get();
    const uint32_t parts = std::max(1u, std::min(pool.size(), n / 65536u));
    std::atomic<bool> bad{false};
    pool.run(parts, [&](uint32_t pt) {
        for (uint32_t i = chunk_lo(n, parts, pt); i < chunk_lo(n, parts, pt + 1); ++i) {
            const mr_cell_index c = build_index(cells[i].index);  // src/index.rs:419-431
            if (!canonical(c) || cells[i].poi > MR_POI_FORUM || cells[i].index.reserved ||
                (c.kind != MR_CELL_CENTER && (c.x > H || c.y > H)))
                bad.store(true, std::memory_order_relaxed);
            g->idx[i] = c;
            g->poi[i] = cells[i].poi;
        }
    });
    const uint32_t vc = H * S + H;
    if (bad.load() || g->idx[vc].kind != MR_CELL_CENTER) return false;
    // the unit steps, from the 5 x 5 cells round the Center
    uint32_t hv[4][3], bv[4];
    for (auto &r : hv) r[0] = r[1] = r[2] = kNone32;
    for (uint32_t &x : bv) x = kNone32;
    for (int dy = -2; dy <= 2; ++dy)
        for (int dx = -2; dx <= 2; ++dx) {
            const uint32_t v = uint32_t(int(vc) + dy * int(S) + dx);
            const mr_cell_index &c = g->idx[v];
            if (c.kind == MR_CELL_HOMELAND) {
                const int k = c.x == 1 && c.y == 1 ? 0 : (c.x == 2 && c.y == 1 ? 1 : (c.x == 1 && c.y == 2 ? 2 : -1));
                if (k >= 0) hv[c.sub][k] = v;
            } else if (c.kind == MR_CELL_BORDER && c.x == 1) {
                bv[c.sub] = v;
            }
        }
    for (int h = 0; h < 4; ++h) {
        if (hv[h][0] == kNone32 || hv[h][1] == kNone32 || hv[h][2] == kNone32 || bv[h] == kNone32) return false;
        g->ux[h] = int64_t(hv[h][1]) - int64_t(hv[h][0]);
        g->uy[h] = int64_t(hv[h][2]) - int64_t(hv[h][0]);
        g->ub[h] = int64_t(bv[h]) - int64_t(vc);
        if (int64_t(hv[h][0]) != int64_t(vc) + g->ux[h] + g->uy[h]) return false;
    }
    // every cell where its index puts it
    pool.run(parts, [&](uint32_t pt) {
        for (uint32_t v = chunk_lo(n, parts, pt); v < chunk_lo(n, parts, pt + 1); ++v) {
            const mr_cell_index &c = g->idx[v];
            int64_t w = -1;
            if (c.kind == MR_CELL_CENTER) w = vc;
            else if (c.kind == MR_CELL_HOMELAND) w = int64_t(vc) + c.x * g->ux[c.sub] + c.y * g->uy[c.sub];
            else w = int64_t(vc) + c.x * g->ub[c.sub];
            if (w != int64_t(v)) bad.store(true, std::memory_order_relaxed);
        }
    });
    if (bad.load()) return false;
    // the index adjacency on the band of cells within 2 of an axis or of the map's edge
    pool.run(parts, [&](uint32_t pt) {
        std::vector<uint64_t> a, b;
        for (uint32_t y = chunk_lo(S, parts, pt); y < chunk_lo(S, parts, pt + 1); ++y) {
            const uint32_t ay = uint32_t(std::abs(int(y) - int(H)));
            for (uint32_t x = 0; x < S; ++x) {
                const uint32_t ax = uint32_t(std::abs(int(x) - int(H)));
                if (std::min(ax, ay) > 2 && std::max(ax, ay) + 1 < H) {
                    // interior run of the row: jump to the band cell before the axis / edge
                    x = ax < H ? (x < H ? H - 3 : S - 3) : x;
                    continue;
                }
                const uint32_t v = y * S + x;
                index_neighbours(g->idx[v], int(H), a);
                b.clear();
                if (x > 0) b.push_back(ci_key(g->idx[v - 1]));
                if (x + 1 < S) b.push_back(ci_key(g->idx[v + 1]));
                if (y > 0) b.push_back(ci_key(g->idx[v - S]));
                if (y + 1 < S) b.push_back(ci_key(g->idx[v + S]));
                std::sort(b.begin(), b.end());
                if (a != b) bad.store(true, std::memory_order_relaxed);
            }
        }
    });
    if (bad.load()) return false;
    g->vc = vc;
    g->fast = g->exact = true;
    g->rank.resize(n);
    g->rank_inv.resize(n);
    std::atomic<bool> std_ok{true};
    pool.run(parts, [&](uint32_t pt) {
        bool ok = true;
        for (uint32_t v = chunk_lo(n, parts, pt); v < chunk_lo(n, parts, pt + 1); ++v) {
            const uint32_t r = closed_rank(g->idx[v], H);
            g->rank[v] = r;
            g->rank_inv[r] = v;
            ok = ok && r == std_rank(g->gx(v), g->gy(v), H);
        }
        if (!ok) std_ok.store(false, std::memory_order_relaxed);
    });
    g->rank_std = std_ok.load() && !std::getenv("MR_RANK_TABLE");  // (tests: force the table)
    for (uint32_t r = 0; r < n; ++r)
        if (g->poi[g->rank_inv[r]] == MR_POI_CAMPFIRE) g->campfires.push_back(g->rank_inv[r]);
    return true;
}

extern "C" int mr_grid_create(const mr_cell *cells, uint32_t n, mr_grid **out) {
    if (!cells || !out) return fail(MR_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    uint64_t s = 0;
    while ((s + 1) * (s + 1) <= n) ++s;
    if (s * s != n) return fail(MR_ERR_INVALID_GRID, "map grid is not square (src/grid.rs:60-63)");
    if (s < 3 || s % 2 == 0) return fail(MR_ERR_INVALID_GRID, "square size must be odd and >= 3");
    if (s > 65535) return fail(MR_ERR_LIMIT, "square size above 65535");
    auto g = new mr_grid();
    g->S = uint32_t(s);
    g->H = g->S / 2;
    g->V = n;
    g->idx.resize(n);
    g->poi.resize(n);
    // the standard layout in any orientation: the fast path; anything else, the checks
    // cell by cell with a hash map of the indices (and their error messages)
    const double tg0 = timing_on() ? now_ms() : 0.0;
    if (!grid_fast_layout(g, cells)) {
        g->fast = g->exact = false;
        g->campfires.clear();
        g->index.reserve(n * 2);
        for (uint32_t i = 0; i < n; ++i) {
            mr_cell_index c = cells[i].index;
            // MapGrid::parse builds every index canonically (src/index.rs:419-431)
            c = build_index(c);
            if (!canonical(c) || cells[i].poi > MR_POI_FORUM || cells[i].index.reserved) {
                delete g;
                return fail(MR_ERR_INVALID_GRID, "invalid cell index or poi at cell " + std::to_string(i));
            }
            if (!g->index.emplace(ci_key(c), i).second) {
                delete g;
                return fail(MR_ERR_INVALID_GRID, "duplicate cell index at cell " + std::to_string(i));
            }
            g->idx[i] = c;
            g->poi[i] = cells[i].poi;
        }
        uint32_t vc;
        if (!g->find(ci_make(MR_CELL_CENTER, 0, 0, 0), vc) || g->gx(vc) != 0 || g->gy(vc) != 0) {
            delete g;
            return fail(MR_ERR_INVALID_GRID, "Center missing or not at (0,0) (src/grid.rs:122-133)");
        }
        g->vc = vc;
        // the index adjacency must be the geometric 4-neighbourhood
        std::vector<uint64_t> a, b;
        const int S_ = int(g->S);
        for (uint32_t v = 0; v < n; ++v) {
            const mr_cell_index &c = g->idx[v];
            if ((c.kind == MR_CELL_HOMELAND && (c.x > g->H || c.y > g->H)) || (c.kind == MR_CELL_BORDER && c.x > g->H)) {
                delete g;
                return fail(MR_ERR_INVALID_GRID, "cell index outside the homeland size");
            }
            index_neighbours(c, int(g->H), a);
            b.clear();
            int x = int(v % g->S), y = int(v / g->S);
            if (x > 0) b.push_back(ci_key(g->idx[v - 1]));
            if (x + 1 < S_) b.push_back(ci_key(g->idx[v + 1]));
            if (y > 0) b.push_back(ci_key(g->idx[v - g->S]));
            if (y + 1 < S_) b.push_back(ci_key(g->idx[v + g->S]));
            std::sort(b.begin(), b.end());
            if (a != b) {
                delete g;
                return fail(MR_ERR_INVALID_GRID, "cell labels are not a consistent 4-grid at cell " + std::to_string(v));
            }
        }
        // the layout's unit steps per homeland and border (find()'s arithmetic path)
        if (g->H >= 2) {
            bool ok = true;
            for (int h = 0; h < 4 && ok; ++h) {
                uint32_t v11, v21, v12, vb;
                ok = g->find(ci_make(MR_CELL_HOMELAND, uint8_t(h), 1, 1), v11) &&
                     g->find(ci_make(MR_CELL_HOMELAND, uint8_t(h), 2, 1), v21) &&
                     g->find(ci_make(MR_CELL_HOMELAND, uint8_t(h), 1, 2), v12) && g->find(build_border(h, 1), vb);
                if (!ok) break;
                g->ux[h] = int64_t(v21) - int64_t(v11);
                g->uy[h] = int64_t(v12) - int64_t(v11);
                g->ub[h] = int64_t(vb) - int64_t(vc);
                ok = int64_t(v11) == int64_t(vc) + g->ux[h] + g->uy[h];
            }
            g->fast = ok;
            // every cell where the formula puts it: find() may then trust the formula
            bool all = ok;
            for (uint32_t v = 0; v < n && all; ++v) {
                const mr_cell_index &c = g->idx[v];
                int64_t w = -1;
                if (c.kind == MR_CELL_CENTER) w = vc;
                else if (c.kind == MR_CELL_HOMELAND) w = int64_t(vc) + c.x * g->ux[c.sub] + c.y * g->uy[c.sub];
                else if (c.kind == MR_CELL_BORDER) w = int64_t(vc) + c.x * g->ub[c.sub];
                all = w == int64_t(v);
            }
            g->exact = all;
        }
        // rank = position in the derived Ord of CellIndex (src/index.rs:41-46)
        {
            std::vector<std::pair<uint64_t, uint32_t>> keys(n);
            for (uint32_t v = 0; v < n; ++v) keys[v] = {ci_key(g->idx[v]), v};
            std::sort(keys.begin(), keys.end());
            g->rank.resize(n);
            g->rank_inv.resize(n);
            for (uint32_t r = 0; r < n; ++r) {
                g->rank[keys[r].second] = r;
                g->rank_inv[r] = keys[r].second;
            }
            for (uint32_t r = 0; r < n; ++r)
                if (g->poi[keys[r].second] == MR_POI_CAMPFIRE) g->campfires.push_back(keys[r].second);
            bool std_ok = true;
            for (uint32_t v = 0; v < n && std_ok; ++v) std_ok = g->rank[v] == std_rank(g->gx(v), g->gy(v), g->H);
            g->rank_std = std_ok && !std::getenv("MR_RANK_TABLE");  // (tests: force the table)
        }
    }
    // nearest campfire per homeland (src/grid.rs:134-230, 297-325): the argmin of
    // (Manhattan distance, |x|!=|y|, |x|+|y|, |x|, |y|) over the homeland's Homeland-indexed
    // campfires (the reference's projections give the same, tests/test_oracle_kat.py).
    // Along one row y the distance to campfire f is x - fx + |y - fy| for fx <= x and
    // fx - x + |y - fy| for fx >= x, so the best campfire at x is the better of a prefix
    // minimum of (|y - fy| - fx, key) over the campfires left of x and a suffix minimum of
    // (fx + |y - fy|, key) over those right of it: O(S + campfires) a row, rows on the
    // host threads.
    for (int h = 0; h < 4; ++h) {
        bool any = false;
        for (uint32_t v : g->campfires) any = any || (g->idx[v].kind == MR_CELL_HOMELAND && g->idx[v].sub == h);
        if (!any) {
            delete g;
            // MapGrid::parse reaches unreachable!() in this case (src/grid.rs:209)
            return fail(MR_ERR_INVALID_GRID, "a homeland has no campfire (the reference panics, src/grid.rs:209)");
        }
    }
    const double tg1 = timing_on() ? now_ms() : 0.0;
    {
        struct Cf {
            int64_t fx, fy;
            uint64_t key;
            uint32_t v;
        };
        std::vector<Cf> cfs[4];
        for (uint32_t v : g->campfires) {
            const mr_cell_index &c = g->idx[v];
            if (c.kind != MR_CELL_HOMELAND) continue;
            const int64_t fx = int64_t(v % g->S), fy = int64_t(v / g->S);
            const uint64_t ax = uint64_t(std::abs(g->gx(v))), ay = uint64_t(std::abs(g->gy(v)));
            cfs[c.sub].push_back(Cf{fx, fy, (uint64_t(ax != ay) << 62) | ((ax + ay) << 40) | (ax << 20) | ay, v});
        }
        for (int h = 0; h < 4; ++h) {
            std::sort(cfs[h].begin(), cfs[h].end(), [](const Cf &p, const Cf &q) { return p.fx < q.fx; });
            g->nearest[h].assign(n, kNone32);
        }
        const uint32_t S = g->S;
        HostPool &pool = HostPool::get();
        const uint32_t parts = std::max(1u, std::min(pool.size() * 4, S / 16u));
        pool.run(parts, [&](uint32_t pt) {
            std::vector<std::pair<int64_t, uint64_t>> suf;
            std::vector<uint32_t> sufi;
            for (uint32_t y = chunk_lo(S, parts, pt); y < chunk_lo(S, parts, pt + 1); ++y)
                for (int h = 0; h < 4; ++h) {
                    const std::vector<Cf> &cf = cfs[h];
                    const size_t k = cf.size();
                    // suffix minima of (fx + |y - fy|, key) over the campfires sorted by fx
                    suf.resize(k + 1);
                    sufi.resize(k + 1);
                    suf[k] = {INT64_MAX, ~0ull};
                    sufi[k] = kNone32;
                    for (size_t i = k; i-- > 0;) {
                        const std::pair<int64_t, uint64_t> c{cf[i].fx + std::abs(int64_t(y) - cf[i].fy), cf[i].key};
                        if (c < suf[i + 1]) {
                            suf[i] = c;
                            sufi[i] = cf[i].v;
                        } else {
                            suf[i] = suf[i + 1];
                            sufi[i] = sufi[i + 1];
                        }
                    }
                    std::pair<int64_t, uint64_t> pre{INT64_MAX, ~0ull};  // (|y - fy| - fx, key), fx <= x
                    uint32_t prei = kNone32;
                    size_t j = 0;  // first campfire with fx > x
                    uint32_t *out = &g->nearest[h][size_t(y) * S];
                    for (uint32_t x = 0; x < S; ++x) {
                        while (j < k && cf[j].fx <= int64_t(x)) {
                            const std::pair<int64_t, uint64_t> c{std::abs(int64_t(y) - cf[j].fy) - cf[j].fx, cf[j].key};
                            if (c < pre) {
                                pre = c;
                                prei = cf[j].v;
                            }
                            ++j;
                        }
                        // right of x: the campfires from the first with fx >= x (fx == x is in both)
                        size_t jj = j;
                        while (jj > 0 && cf[jj - 1].fx == int64_t(x)) --jj;
                        std::pair<int64_t, uint64_t> best{INT64_MAX, ~0ull};
                        uint32_t bi = kNone32;
                        if (prei != kNone32) {
                            best = {pre.first + int64_t(x), pre.second};
                            bi = prei;
                        }
                        if (sufi[jj] != kNone32) {
                            const std::pair<int64_t, uint64_t> c{suf[jj].first - int64_t(x), suf[jj].second};
                            if (c < best) {
                                best = c;
                                bi = sufi[jj];
                            }
                        }
                        out[x] = bi;
                    }
                }
        });
    }
    if (timing_on())
        std::fprintf(stderr, "[mr] grid_create V=%u: layout+ranks %.2f ms, nearest campfires %.2f ms (%s path)\n", n,
                     tg1 - tg0, now_ms() - tg1, g->exact ? "fast" : "generic");
    *out = g;
    return MR_OK;
}

extern "C" void mr_grid_destroy(mr_grid *g) {
    delete g;
    // the grid's plans are gone (a plan must not outlive its grid): hand the blocks they
    // cached back to the device
    mr_cache_trim();
}
extern "C" uint32_t mr_grid_square_size(const mr_grid *g) { return g ? g->S : 0; }

extern "C" void mr_params_default(mr_params *p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->scroll_of_escape_cost = 50;
    p->scroll_of_escape_hq_cost = 75;
    p->scroll_of_escape_forum_cost = 100;
    p->use_soe = 1;
    p->use_sfm = 0;
    p->use_caravans = 1;
    p->has_hq = 0;
    p->route_guru = 0;
    p->fleetfoot = 0;
    p->sort_by[0] = MR_SORT_LEGS;
    p->sort_by[1] = MR_SORT_MONEY;
    p->homeland = MR_HOMELAND_BLUE;
}

extern "C" uint32_t mr_abi_version(void) { return MR_ABI_VERSION; }
extern "C" const char *mr_last_error(void) { return g_last_error.c_str(); }

// Device properties, queried once per device (hipGetDeviceProperties costs far more
// than the rest of a small plan's creation)
static const hipDeviceProp_t *device_props(int dev) {
    static std::mutex mu;
    static std::unordered_map<int, hipDeviceProp_t> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return &it->second;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
    return &cache.emplace(dev, prop).first->second;
}

extern "C" int mr_device_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    const hipDeviceProp_t *prop = device_props(dev);
    if (!prop) return 0;
    return std::strncmp(prop->gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// The SoE regions of homeland h: its Homeland-indexed campfires in CellIndex order
// (src/grid.rs:143-146), one region per campfire.
static const std::vector<uint32_t> &region_list(const mr_grid *g, int h) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    if (!g->regions_built[h]) {
        std::vector<uint32_t> regs;
        for (uint32_t v : g->campfires) {
            const mr_cell_index &c = g->idx[v];
            if (c.kind == MR_CELL_HOMELAND && c.sub == h) regs.push_back(v);
        }
        g->regions[h] = std::move(regs);
        g->regions_built[h] = true;
    }
    return g->regions[h];
}

// The region table of homeland h on the current device, built there once per grid and
// device (mr_k_region.hip: a separable L1 transform of (distance, rank) in three passes)
// from the region of every cell (the nearest campfire, computed at grid creation) and
// the device rank table d_rank (which must live on the current device).  The grid's
// plans on that device share it; nullptr on a device error.
static const uint32_t *region_table_device(const mr_grid *g, int h, const uint32_t *d_rank) {
    const std::vector<uint32_t> &regs = region_list(g, h);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g->near_mu);
    auto it = g->d_near.find({dev, h});
    if (it != g->d_near.end()) return it->second;
    const double t0 = now_ms();
    const uint32_t V = g->V, S = g->S, nreg = uint32_t(regs.size());
    std::unordered_map<uint32_t, uint16_t> rid;
    for (uint32_t r = 0; r < nreg; ++r) rid[regs[r]] = uint16_t(r);
    std::vector<uint16_t> reg(V, 0xFFFFu);
    {
        const std::vector<uint32_t> &nearest = g->nearest[h];
        HostPool &pool = HostPool::get();
        const uint32_t parts = std::max(1u, std::min(pool.size(), V / 65536u));
        pool.run(parts, [&](uint32_t pt) {
            uint32_t last = kNone32;
            uint16_t lr = 0xFFFFu;
            for (uint32_t v = chunk_lo(V, parts, pt); v < chunk_lo(V, parts, pt + 1); ++v) {
                const uint32_t c = nearest[v];
                if (v == g->vc || c == kNone32) continue;
                if (c != last) {
                    auto it = rid.find(c);
                    lr = it == rid.end() ? 0xFFFFu : it->second;
                    last = c;
                }
                reg[v] = lr;
            }
        });
    }
    uint32_t *d = nullptr;
    uint16_t *d_reg = nullptr;
    void *d_axis = nullptr, *d_seg = nullptr;
    hipStream_t st = nullptr;
    // (MR_REGION_SERIAL=1: the serial kernels, A/B)
    static const bool serial = std::getenv("MR_REGION_SERIAL") != nullptr;
    const uint64_t segw = serial ? 0 : region_table_seg_words(S, nreg);
    bool ok = nreg > 0 && dev_malloc(reinterpret_cast<void **>(&d), size_t(V) * nreg * 8) == hipSuccess &&
              dev_malloc(reinterpret_cast<void **>(&d_reg), size_t(V) * 2) == hipSuccess &&
              dev_malloc(&d_axis, size_t(2) * S * nreg * 8) == hipSuccess &&
              (!segw || dev_malloc(&d_seg, size_t(segw) * 8) == hipSuccess) &&
              hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
              hipMemcpyAsync(d_reg, reg.data(), size_t(V) * 2, hipMemcpyHostToDevice, st) == hipSuccess &&
              region_table_build(d_reg, d_rank, S, nreg, d, d_axis, d_seg, st) == hipSuccess &&
              hipStreamSynchronize(st) == hipSuccess;
    if (st) (void)hipStreamDestroy(st);
    if (d_reg) (void)hipFree(d_reg);
    if (d_axis) (void)hipFree(d_axis);
    if (d_seg) (void)hipFree(d_seg);
    if (!ok) {
        (void)hipGetLastError();
        if (d) (void)hipFree(d);
        return nullptr;
    }
    g->d_near[{dev, h}] = d;
    g->region_ms[h] = now_ms() - t0;
    return d;
}

// Rows of the region table for the plan's specials (t = 1 .. NS) into near_sp
// ((NS + 1) x nreg x {distance, rank}), copied from the device table once per grid,
// homeland and cell (cached).
static int special_rows_from_table(const mr_grid *g, int h, const uint32_t *d_near, uint32_t nreg,
                                   const std::vector<SpecialStatic> &sp, std::vector<uint32_t> &near_sp) {
    const uint32_t NS = uint32_t(sp.size()) - 1;
    near_sp.assign(size_t(NS + 1) * nreg * 2, kNone32);
    std::lock_guard<std::mutex> lk(g->near_mu);
    auto &cache = g->near_sp_cache[h];
    for (uint32_t t = 1; t <= NS; ++t) {
        const uint32_t v = sp[t].v;
        uint32_t *row = &near_sp[size_t(t) * nreg * 2];
        auto it = cache.find(v);
        if (it == cache.end()) {
            std::vector<uint32_t> r(size_t(nreg) * 2);
            if (hipMemcpy(r.data(), d_near + size_t(v) * nreg * 2, size_t(nreg) * 8, hipMemcpyDeviceToHost) != hipSuccess)
                return MR_ERR_DEVICE;
            it = cache.emplace(v, std::move(r)).first;
        }
        std::copy(it->second.begin(), it->second.end(), row);
    }
    return MR_OK;
}

// Boundary cells of the regions (wide hub solver).  Seen from outside a region, its
// nearest cell (walk distance avoiding the Center, ties by rank) is a boundary cell:
// the last step of a shortest walk enters it from a non-Center cell outside.
static uint32_t host_walk_dist(int ax, int ay, int bx, int by) {
    uint32_t d = uint32_t(std::abs(ax - bx) + std::abs(ay - by));
    if ((ay == 0 && by == 0 && ax != 0 && bx != 0 && ((ax < 0) != (bx < 0))) ||
        (ax == 0 && bx == 0 && ay != 0 && by != 0 && ((ay < 0) != (by < 0))))
        d += 2;
    return d;
}
static void region_bounds(const mr_grid *g, int h, std::vector<uint32_t> &regs, const std::vector<uint32_t> *&off,
                          const std::vector<uint32_t> *&cell) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    regs.clear();
    for (uint32_t v : g->campfires) {
        const mr_cell_index &c = g->idx[v];
        if (c.kind == MR_CELL_HOMELAND && c.sub == h) regs.push_back(v);  // CellIndex order
    }
    off = &g->rb_off[h];
    cell = &g->rb_cell[h];
    if (g->rb_built[h]) return;
    const uint32_t V = g->V, S = g->S, nreg = uint32_t(regs.size());
    std::unordered_map<uint32_t, uint32_t> rid;
    for (uint32_t r = 0; r < nreg; ++r) rid[regs[r]] = r;
    const std::vector<uint32_t> &near = g->nearest[h];
    std::vector<uint32_t> cnt(nreg + 1, 0), which;
    std::vector<uint32_t> list;
    for (uint32_t v = 0; v < V; ++v) {
        if (v == g->vc || near[v] == kNone32) continue;
        const uint32_t x = v % S, y = v / S;
        const uint32_t nb[4] = {x > 0 ? v - 1 : kNone32, x + 1 < S ? v + 1 : kNone32, y > 0 ? v - S : kNone32,
                                y + 1 < S ? v + S : kNone32};
        bool edge = false;
        for (uint32_t w : nb)
            if (w != kNone32 && w != g->vc && near[w] != near[v]) edge = true;
        if (!edge) continue;
        auto it = rid.find(near[v]);
        if (it == rid.end()) continue;
        list.push_back(v);
        which.push_back(it->second);
        ++cnt[it->second + 1];
    }
    std::vector<uint32_t> o(nreg + 1, 0);
    for (uint32_t r = 0; r < nreg; ++r) o[r + 1] = o[r] + cnt[r + 1];
    std::vector<uint32_t> cells(size_t(o[nreg]) * 2), pos(o.begin(), o.end() - 1);
    for (size_t i = 0; i < list.size(); ++i) {
        const uint32_t v = list[i], k = pos[which[i]]++;
        cells[2 * k] = (uint32_t(uint16_t(int16_t(g->gx(v))))) | (uint32_t(uint16_t(int16_t(g->gy(v)))) << 16);
        cells[2 * k + 1] = g->rank[v];
    }
    g->rb_off[h] = std::move(o);
    g->rb_cell[h] = std::move(cells);
    g->rb_built[h] = true;
}

// ------------------------------------------------------------------ planning

namespace {

// Per-batch host arrays recycled across plans.  A fresh array of a million entries is
// mapped page by page on first touch (~1 k faults per 4 MB, the pool's threads all taking
// the address-space lock); a recycled one is mapped already, and keeps its size, so a
// resize to a batch no larger writes nothing.  Up to kSpareMax arrays and kMaxBytes per
// type are kept (mr_cache_trim releases them).
template <class T> struct SpareVecs {
    static constexpr size_t kSpareMax = 16, kMinBytes = size_t(1) << 16, kMaxBytes = size_t(256) << 20;
    std::mutex mu;
    std::vector<std::vector<T>> v;
    size_t bytes() const {
        size_t b = 0;
        for (const std::vector<T> &a : v) b += a.capacity() * sizeof(T);
        return b;
    }
    void clear() {
        std::lock_guard<std::mutex> lk(mu);
        v.clear();
        v.shrink_to_fit();
    }
    static SpareVecs &get() {
        static SpareVecs *s = new SpareVecs();
        return *s;
    }
};
// `out` = a spare of at least n entries (the smallest such, else the largest), resized to n
template <class T> static void spare_take(std::vector<T> &out, size_t n) {
    if (n * sizeof(T) >= SpareVecs<T>::kMinBytes && out.capacity() < n) {
        SpareVecs<T> &sv = SpareVecs<T>::get();
        std::lock_guard<std::mutex> lk(sv.mu);
        size_t best = sv.v.size();
        for (size_t i = 0; i < sv.v.size(); ++i) {
            const size_t c = sv.v[i].capacity();
            if (best == sv.v.size()) best = i;
            else {
                const size_t b = sv.v[best].capacity();
                if ((b < n && c > b) || (c >= n && c < b)) best = i;
            }
        }
        if (best < sv.v.size()) {
            out.swap(sv.v[best]);
            sv.v.erase(sv.v.begin() + std::ptrdiff_t(best));
        }
    }
    out.resize(n);
}
template <class T> static void spare_put(std::vector<T> &v) {
    const size_t vb = v.capacity() * sizeof(T);
    if (vb < SpareVecs<T>::kMinBytes || vb > SpareVecs<T>::kMaxBytes) return;
    SpareVecs<T> &sv = SpareVecs<T>::get();
    std::lock_guard<std::mutex> lk(sv.mu);
    // drop the smallest while full (by count or bytes), unless v is no larger
    while (!sv.v.empty() && (sv.v.size() >= SpareVecs<T>::kSpareMax || sv.bytes() + vb > SpareVecs<T>::kMaxBytes)) {
        size_t k = 0;
        for (size_t i = 1; i < sv.v.size(); ++i)
            if (sv.v[i].capacity() < sv.v[k].capacity()) k = i;
        if (sv.v[k].capacity() >= v.capacity()) return;
        sv.v.erase(sv.v.begin() + std::ptrdiff_t(k));
    }
    sv.v.emplace_back();
    sv.v.back().swap(v);
}

struct HostPlan {
    ~HostPlan() {
        for (std::vector<uint32_t> *a : {&src_v, &q_begin, &q_dst, &q_id, &q_pos}) spare_put(*a);
        spare_put(q_status);
    }
    DevParams p{};
    uint32_t homeland = 0, hq_v = 0xFFFFFFFFu;  // the key of the grid's shared sinfo (build_sinfo)
    std::vector<SpecialStatic> sp;
    std::vector<uint16_t> hubs;
    std::vector<uint32_t> src_v, q_begin, q_dst, q_id;
    std::vector<uint32_t> q_pos;    // per input query: its grouped position (output record), kNone32 if invalid
    std::vector<int32_t> q_status;  // per query: MR_OK or a host-side error
    uint32_t nq = 0;
    uint32_t fleetfoot_raw = 0;
    bool hub = false;                       // hub solver applicable (small tables)
    bool nonlin = false;                    // hub with a non-linear run time (near-tie certification)
    bool ff_magic_ok = false;               // the lane kernel's run-time magic is exact on this grid (ff_magic)
    bool near = false;                      // the grid's device region table (V x regions)
    uint32_t nreg = 0;
    bool wide = false;                      // hub_wide_kernel (NS > 63 or no V x regions table)
    std::vector<uint32_t> near_sp;          // wide: (NS+1) x nreg x {distance, rank} rows of the specials
    const std::vector<uint32_t> *rb_off = nullptr, *rb_cell = nullptr;
    // Large query batches are grouped on the device (mr_k_groupq.hip): src_v .. q_status
    // stay empty until a host caller needs them (host_arrays), the counts below hold
    bool dev_grouped = false, mirrored = false;
    uint32_t nrec = 0, nsrc = 0, n_small = 0;  // valid queries, sources, sources of <= kLaneMaxQ queries
    std::vector<uint32_t> invalid;             // device grouping: the invalid queries, ascending
};
static uint32_t nrec_of(const HostPlan &hp) { return hp.dev_grouped ? hp.nrec : uint32_t(hp.q_id.size()); }
static uint32_t nsrc_of(const HostPlan &hp) { return hp.dev_grouped ? hp.nsrc : uint32_t(hp.src_v.size()); }

// (c1, c2) -> (c1, c2', c3): CostComparator::eval_next (src/cost.rs:387-405)
static void comparator_order(uint8_t s1, uint8_t s2, uint8_t out[3]) {
    uint8_t c2 = s2;
    if (s1 == s2) c2 = (s1 == MR_SORT_LEGS) ? MR_SORT_TIME : MR_SORT_LEGS;
    uint8_t c3 = uint8_t(3 - s1 - c2);  // the remaining one of {0,1,2}
    out[0] = s1;
    out[1] = c2;
    out[2] = c3;
}
static uint32_t metric_index(uint8_t c) { return c == MR_SORT_LEGS ? 0u : (c == MR_SORT_MONEY ? 1u : 2u); }

// RouteGuru (src/skill.rs:43-52) on CARAVAN_TIME = 240 s: ceil(240 * r), raw out of range
static uint32_t caravan_unit_time(uint32_t route_guru) {
    static const uint32_t rgn[6] = {1, 19, 7, 73, 31, 51}, rgd[6] = {1, 24, 10, 120, 60, 120};
    const uint32_t rg = route_guru <= 5 ? route_guru : 0;
    return uint32_t((240ull * rgn[rg] + rgd[rg] - 1) / rgd[rg]);
}

// Per calling thread: the grouping scratch of build_plan (about 20 B per query of the
// thread's largest batch), registered so that mr_cache_trim can release every thread's.
struct GroupScratch;
static std::mutex g_scratch_mu;
static std::vector<GroupScratch *> g_scratch;
struct GroupScratch {
    std::mutex mu;  // held by build_plan while it uses the vectors, and by the trim
    std::vector<uint64_t> kv, tmp;  // source << 32 | query index
    std::vector<uint32_t> hist, dst;
    GroupScratch() {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        g_scratch.push_back(this);
    }
    ~GroupScratch() {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        g_scratch.erase(std::find(g_scratch.begin(), g_scratch.end(), this));
    }
    void release() {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<uint64_t>().swap(kv);
        std::vector<uint64_t>().swap(tmp);
        std::vector<uint32_t>().swap(hist);
        std::vector<uint32_t>().swap(dst);
    }
};
static void trim_group_scratch() {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (GroupScratch *g : g_scratch) g->release();
}

// ---- query batches grouped on the device (mr_k_groupq.hip) -------------------------
// Batches of at least kDevGroupMin queries on a grid whose cells are all where the
// layout's formula puts them (mr_grid::exact) go up raw: the lookups, the stable sort by
// source and the lane kernel's partition run on the device, and the host learns counts
// only.  MR_DEV_GROUP=0: never, =1: any batch on such a grid.
constexpr uint32_t kDevGroupMin = 32768;
static bool dev_group_ok(const mr_grid *g, uint32_t n) {
    if (!g->exact || n == 0 || n >= (1u << 30)) return false;
    const char *e = std::getenv("MR_DEV_GROUP");
    if (e && !std::strcmp(e, "0")) return false;
    if (e && !std::strcmp(e, "1")) return true;
    return n >= kDevGroupMin;
}

// The lane kernel's Fleetfoot run time ceil(c k / den) as umulhi(c k + den - 1, magic) >>
// shift (LaneHub::rtime): the least shift whose magic ceil(2^(32 + shift) / den) fits 32
// bits and gives the exact quotient for every k <= kmax (checked here, k by k: every walk
// on the grid is shorter than 2 S + 8 legs, and the path scan's period check reads up to
// 2 den + 1 past one: kmax = 2 S + 256).  False: no such pair (the plan then stays off
// the lane kernel).
static bool ff_magic(uint32_t c, uint32_t den, uint32_t kmax, uint32_t &magic, uint32_t &shift) {
    magic = 1;
    shift = 0;
    if (den <= 1) return true;  // linear: rtime does not use it
    if (uint64_t(c) * kmax + den - 1 > 0xFFFFFFFFull) return false;
    for (uint32_t s = 0; s < 32; ++s) {
        const uint64_t m = ((uint64_t(1) << (32 + s)) + den - 1) / den;
        if (m > 0xFFFFFFFFull) break;
        bool ok = true;
        for (uint64_t k = 0; k <= kmax && ok; ++k) {
            const uint64_t x = uint64_t(c) * k + den - 1;
            ok = ((x * m) >> (32 + s)) == x / den;
        }
        if (ok) {
            magic = uint32_t(m);
            shift = s;
            return true;
        }
    }
    return false;
}

static int build_plan(const mr_grid *g, const mr_params *prm, const mr_query *qs, uint32_t n, uint32_t max_cmds,
                      HostPlan &hp, bool allow_dev_group = false) {
    const double tbs = timing_on() ? now_ms() : 0.0;
    if (!g || !prm) return fail(MR_ERR_INVALID_ARG, "null grid or params");
    if (prm->sort_by[0] > 2 || prm->sort_by[1] > 2 || prm->homeland > 3)
        return fail(MR_ERR_INVALID_ARG, "invalid sort_by or homeland");
    DevParams &p = hp.p;
    p.S = g->S;
    p.H = g->H;
    p.V = g->V;
    p.vc = g->vc;
    uint8_t ord[3];
    comparator_order(prm->sort_by[0], prm->sort_by[1], ord);
    for (int i = 0; i < 3; ++i) p.perm[i] = metric_index(ord[i]);
    if (ord[0] == MR_SORT_LEGS) p.bucket_mode = kBucketLegs;
    else if (ord[0] == MR_SORT_TIME) p.bucket_mode = kBucketTime;
    else p.bucket_mode = (ord[1] == MR_SORT_LEGS) ? kBucketMoneyLegs : kBucketMoneyTime;
    // Fleetfoot (src/skill.rs:65-71): out-of-range levels leave the time raw
    static const uint32_t ffn[4] = {1, 50, 100, 25}, ffd[4] = {1, 53, 109, 28};
    uint32_t ff = prm->fleetfoot <= 3 ? prm->fleetfoot : 0;
    p.ff = prm->fleetfoot;
    hp.fleetfoot_raw = prm->fleetfoot;
    p.ff_num = ffn[ff];
    p.ff_den = ffd[ff];
    p.W = uint32_t((180ull * p.ff_num) / p.ff_den);  // floor(r*180): min StandardMove increment
    p.ff_c = 180u * p.ff_num;
    hp.ff_magic_ok = ff_magic(p.ff_c, p.ff_den, 2u * g->S + 256u, p.ff_magic, p.ff_shift);
    p.rgt = caravan_unit_time(prm->route_guru);
    p.soe_cost = prm->scroll_of_escape_cost;
    p.shq_cost = prm->scroll_of_escape_hq_cost;
    p.sfm_cost = prm->scroll_of_escape_forum_cost;
    p.use_soe = prm->use_soe ? 1 : 0;
    p.use_sfm = prm->use_sfm ? 1 : 0;
    p.use_caravans = prm->use_caravans ? 1 : 0;
    p.max_cmds = max_cmds;
    // specials: 1 Center, 2..5 border-1 cells, campfires, HQ
    std::unordered_map<uint32_t, uint32_t> tixm;  // vertex -> table entry of the specials
    tixm.reserve(2 * g->campfires.size() + 16);
    auto tix = [&](uint32_t v) {
        auto it = tixm.find(v);
        return it == tixm.end() ? kNone10 : it->second;
    };
    std::vector<uint32_t> order;
    order.push_back(0);  // entry 0 = source (dynamic)
    auto add = [&](uint32_t v) {
        auto it = tixm.find(v);
        if (it != tixm.end()) return it->second;
        const uint32_t t = uint32_t(order.size());
        tixm.emplace(v, t);
        order.push_back(v);
        return t;
    };
    add(g->vc);
    for (int b = 0; b < 4; ++b) {
        uint32_t v;
        g->find(build_border(b, 1), v);
        add(v);
    }
    // the query homeland's campfires (the SoE regions) first: hub_lane_kernel keeps its
    // region candidates to entries 6 .. 6 + kLaneRegs - 1 (the table order decides
    // nothing else: equal labels are ordered by their command lists)
    for (uint32_t v : g->campfires)
        if (g->idx[v].kind == MR_CELL_HOMELAND && g->idx[v].sub == prm->homeland) add(v);
    for (uint32_t v : g->campfires) add(v);
    uint32_t hq_v = kNone32;
    if (prm->has_hq) {
        if (!g->find(prm->hq_position, hq_v)) return fail(MR_ERR_INVALID_INDEX, "hq_position is not a grid cell");
        add(hq_v);
    }
    const uint32_t NS = uint32_t(order.size()) - 1;
    if (NS > kMaxSpecials) return fail(MR_ERR_LIMIT, "too many campfires (special table limit)");
    p.NS = NS;
    p.hq_t = prm->has_hq ? tix(hq_v) : 0;
    hp.hq_v = hq_v;
    hp.homeland = prm->homeland;
    const std::vector<uint32_t> &near = g->nearest[prm->homeland];
    hp.sp.assign(NS + 1, SpecialStatic{});
    hp.hubs.clear();
    for (uint32_t t = 1; t <= NS; ++t) {
        uint32_t v = order[t];
        SpecialStatic &s = hp.sp[t];
        s.v = v;
        s.rk = g->rank[v];
        s.x = g->gx(v);
        s.y = g->gy(v);
        bool is_cf = g->poi[v] == MR_POI_CAMPFIRE;
        s.flags = (t == 1 ? kSpCenter : 0u) | ((t >= 2 && t <= 5) ? kSpBorder1 : 0u) | ((t == 1 || is_cf) ? kSpHub : 0u);
        s.region = near[v] == kNone32 ? kNone10 : tix(near[v]);
        const mr_cell_index &c = g->idx[v];
        bool coef2 = c.kind == MR_CELL_CENTER || (c.kind == MR_CELL_HOMELAND && c.sub == prm->homeland);
        s.coef5 = coef2 ? 0u : 1u;
        if (s.flags & kSpHub) hp.hubs.push_back(uint16_t(t));
    }
    p.n_hubs = uint32_t(hp.hubs.size());
    for (uint32_t t = 1; t <= NS; ++t) hp.sp[t].rid = kNone10;
    // hub solver: the closed form is exact when the StandardMove run time is linear
    // (Fleetfoot level 0 or out of range) — DESIGN.md §3a; the one non-isotone case is
    // detected per source and re-solved by the SSSP kernel.  With Fleetfoot 1..3 every
    // closed-form label is also certified against near-ties of the time gap (§3a''), the
    // narrow kernel only.  MR_ALGO=sssp|generic disables the hub, MR_HUB_NONLIN=0 its
    // non-linear use.  Up to 63 specials and a V x regions table of <= 16 GB: one
    // special per lane (hub_kernel); otherwise up to 511 specials (hub_wide_kernel,
    // forced by MR_HUB_WIDE=1 for the tests).
    bool linear = p.ff_num == p.ff_den, nonlin_ok = !linear;
    if (const char *e = std::getenv("MR_HUB_NONLIN"))
        if (!std::strcmp(e, "0")) nonlin_ok = false;
    if (const char *e = std::getenv("MR_ALGO"))
        if (!std::strcmp(e, "sssp") || !std::strcmp(e, "generic")) linear = nonlin_ok = false;
    size_t nregs = 0;
    for (uint32_t v : g->campfires)
        if (g->idx[v].kind == MR_CELL_HOMELAND && g->idx[v].sub == prm->homeland) ++nregs;
    const char *fw = std::getenv("MR_HUB_WIDE");
    const bool force_wide = fw && (!std::strcmp(fw, "1") || !std::strcmp(fw, "scan"));
    // the V x regions table (grid preprocessing, shared by the grid's plans) up to
    // 16 GB of HBM (c5: 8.6 GB); beyond it the wide kernel scans boundary cells
    const bool table_ok = nregs <= 256 && size_t(g->V) * nregs * 8 <= (size_t(16) << 30) &&
                          !(fw && !std::strcmp(fw, "scan"));
    const bool narrow_ok = NS <= 63 && nregs <= 63 && table_ok;
    hp.hub = hp.wide = hp.nonlin = false;
    if ((linear || nonlin_ok) && narrow_ok && !force_wide) {
        hp.nonlin = !linear;
        const std::vector<uint32_t> &regs = region_list(g, prm->homeland);
        hp.hub = true;
        hp.nreg = uint32_t(regs.size());
        hp.near = true;  // the device table (built at plan creation) and the specials' rows
        for (uint32_t r = 0; r < hp.nreg; ++r) hp.sp[tix(regs[r])].rid = r;
    } else if (linear && hub_wide_spl(NS) != 0 && nregs <= 256) {
        std::vector<uint32_t> regs;
        region_bounds(g, prm->homeland, regs, hp.rb_off, hp.rb_cell);
        hp.near = table_ok;  // the source's row read from the device table instead of scanned
        hp.hub = hp.wide = true;
        hp.nreg = uint32_t(regs.size());
        for (uint32_t r = 0; r < hp.nreg; ++r) hp.sp[tix(regs[r])].rid = r;
        // the specials' rows (row 0, the source, is computed per source on the device);
        // with the table they are its rows, copied at plan creation
        const uint32_t nr = hp.nreg;
        hp.near_sp.assign(size_t(NS + 1) * nr * 2, kNone32);
        const std::vector<uint32_t> &nearh = g->nearest[prm->homeland];
        const std::vector<uint32_t> &off = *hp.rb_off, &cell = *hp.rb_cell;
        // With the grid's region table the rows are its rows (the same (distance, rank)
        // minimum: seen from outside a region its nearest cell is a boundary cell); without
        // it each row scans the boundary cells once per grid and special cell (cached: the
        // scan is O(boundary cells) per special, 28 ms a plan at c5 when done per plan).
        for (uint32_t t = 1; t <= NS; ++t) {
            const uint32_t v = order[t];
            if (v == g->vc || hp.near) continue;
            uint32_t *row = &hp.near_sp[size_t(t) * nr * 2];
            {
                std::lock_guard<std::mutex> lk(g->near_mu);
                auto it = g->near_sp_cache[prm->homeland].find(v);
                if (it != g->near_sp_cache[prm->homeland].end()) {
                    std::copy(it->second.begin(), it->second.end(), row);
                    continue;
                }
            }
            const int vx = g->gx(v), vy = g->gy(v);
            for (uint32_t r = 0; r < nr; ++r) {
                uint32_t bd = kNone32, br = kNone32;
                if (nearh[v] == regs[r]) {
                    bd = 0;
                    br = g->rank[v];
                } else {
                    for (uint32_t i = off[r]; i < off[r + 1]; ++i) {
                        const int ux = int16_t(cell[2 * i] & 0xFFFFu), uy = int16_t(cell[2 * i] >> 16);
                        const uint32_t d = host_walk_dist(vx, vy, ux, uy), rk = cell[2 * i + 1];
                        if (d < bd || (d == bd && rk < br)) {
                            bd = d;
                            br = rk;
                        }
                    }
                }
                row[2 * r] = bd;
                row[2 * r + 1] = br;
            }
            std::lock_guard<std::mutex> lk(g->near_mu);
            g->near_sp_cache[prm->homeland][v].assign(row, row + 2 * nr);
        }
    }
    // Queries grouped by source vertex, sources ascending, each source's queries in
    // input order: a stable sort of the queries by source, 13-bit LSD radix passes over
    // the batch (two while V < 2^26).  The counting sort it replaces touched two
    // V-sized arrays at random (5.5 ms at 125k queries on 1025^2).  Large batches run
    // every phase over host threads (HostPool): per part a histogram, the parts' offsets
    // by (digit, part) keep the sort stable, then each part scatters its own keys.
    const uint32_t V = g->V;
    hp.nq = n;
    if (allow_dev_group && dev_group_ok(g, n)) {  // grouped by plan_create on the device
        hp.dev_grouped = true;
        return MR_OK;
    }
    const double tb0 = timing_on() ? now_ms() : 0.0;
    HostPool &pool = HostPool::get();
    // at least 8k queries a part (a part's work must outweigh waking a thread; 125k
    // queries on 3 parts took 1.2 ms)
    const uint32_t parts = std::max(1u, std::min(pool.size(), n / 8192u));
    constexpr uint32_t kBits = 13, kB = 1u << kBits;
    // An invalid query gets the source key 2^32 - 1: its low bits are all ones, so with
    // enough passes to cover every vertex id (two while V < 2^26) it sorts after every
    // valid query, and the grouping stops at the first one.
    const uint32_t passes = V < (1u << (2 * kBits)) ? 2u : 3u;
    // scratch reused across plans of this thread (no fresh pages per batch); the pool's
    // workers reach it through these references (a thread_local named inside a lambda
    // would be the worker's own); mr_cache_trim releases it
    static thread_local GroupScratch scr;
    std::lock_guard<std::mutex> scr_lk(scr.mu);
    std::vector<uint64_t> &kv = scr.kv, &tmp = scr.tmp;
    std::vector<uint32_t> &hist = scr.hist, &qs_dst = scr.dst;
    kv.resize(n);
    tmp.resize(n);
    qs_dst.resize(n);
    hist.resize(size_t(parts) * kB);
    spare_take(hp.q_status, n);
    spare_take(hp.q_pos, n);
    std::vector<uint32_t> bad(parts + 1, 0);
    // lookups, fused with the first pass's histogram
    pool.run(parts, [&](uint32_t pt) {
        uint32_t *h = &hist[size_t(pt) * kB];
        std::fill(h, h + kB, 0u);
        uint32_t c = 0;
        for (uint32_t i = chunk_lo(n, parts, pt), e = chunk_lo(n, parts, pt + 1); i < e; ++i) {
            uint32_t a, b;
            uint64_t key;
            if (!g->find(qs[i].from, a) || !g->find(qs[i].to, b)) {
                hp.q_status[i] = MR_ERR_INVALID_INDEX;
                hp.q_pos[i] = kNone32;
                key = (uint64_t(kNone32) << 32) | i;
                ++c;
            } else {
                hp.q_status[i] = MR_OK;
                qs_dst[i] = b;
                key = (uint64_t(a) << 32) | i;
            }
            kv[i] = key;
            ++h[uint32_t(key >> 32) & (kB - 1)];
        }
        bad[pt + 1] = c;
    });
    uint32_t nbad = 0;
    for (uint32_t pt = 0; pt < parts; ++pt) nbad += bad[pt + 1];
    const uint32_t m = n - nbad;
    const double tb1 = timing_on() ? now_ms() : 0.0;
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const uint32_t sh = 32 + kBits * pass;
        if (pass > 0)
            pool.run(parts, [&](uint32_t pt) {
                uint32_t *h = &hist[size_t(pt) * kB];
                std::fill(h, h + kB, 0u);
                for (uint32_t k = chunk_lo(n, parts, pt), e = chunk_lo(n, parts, pt + 1); k < e; ++k)
                    ++h[uint32_t(kv[k] >> sh) & (kB - 1)];
            });
        // offsets by (digit, part): the digits' totals, their prefix, then per digit the
        // parts in order (ranges of digits per thread: each part's row is read in order)
        if (parts == 1) {
            uint32_t acc = 0;
            for (uint32_t j = 0; j < kB; ++j) {
                const uint32_t c = hist[j];
                hist[j] = acc;
                acc += c;
            }
        } else {
            std::vector<uint32_t> base(kB + 1, 0);
            pool.run(parts, [&](uint32_t pt) {
                for (uint32_t j = chunk_lo(kB, parts, pt), e = chunk_lo(kB, parts, pt + 1); j < e; ++j) {
                    uint32_t c = 0;
                    for (uint32_t q = 0; q < parts; ++q) c += hist[size_t(q) * kB + j];
                    base[j + 1] = c;
                }
            });
            for (uint32_t j = 0; j < kB; ++j) base[j + 1] += base[j];
            pool.run(parts, [&](uint32_t pt) {
                for (uint32_t j = chunk_lo(kB, parts, pt), e = chunk_lo(kB, parts, pt + 1); j < e; ++j) {
                    uint32_t acc = base[j];
                    for (uint32_t q = 0; q < parts; ++q) {
                        const uint32_t c = hist[size_t(q) * kB + j];
                        hist[size_t(q) * kB + j] = acc;
                        acc += c;
                    }
                }
            });
        }
        pool.run(parts, [&](uint32_t pt) {
            uint32_t *h = &hist[size_t(pt) * kB];
            for (uint32_t k = chunk_lo(n, parts, pt), e = chunk_lo(n, parts, pt + 1); k < e; ++k)
                tmp[h[uint32_t(kv[k] >> sh) & (kB - 1)]++] = kv[k];
        });
        kv.swap(tmp);
    }
    const double tb2 = timing_on() ? now_ms() : 0.0;
    // sources: a new one starts where the sorted source changes; per part the count of
    // starts, then each part writes its sources and its records' destinations / ids
    std::vector<uint32_t> starts(parts + 1, 0);
    pool.run(parts, [&](uint32_t pt) {
        uint32_t c = 0;
        for (uint32_t k = chunk_lo(m, parts, pt), e = chunk_lo(m, parts, pt + 1); k < e; ++k)
            c += (k == 0 || (kv[k] >> 32) != (kv[k - 1] >> 32)) ? 1u : 0u;
        starts[pt + 1] = c;
    });
    for (uint32_t pt = 0; pt < parts; ++pt) starts[pt + 1] += starts[pt];
    spare_take(hp.src_v, starts[parts]);
    spare_take(hp.q_begin, starts[parts] + 1);
    spare_take(hp.q_dst, m);
    spare_take(hp.q_id, m);
    pool.run(parts, [&](uint32_t pt) {
        uint32_t si = starts[pt];
        for (uint32_t k = chunk_lo(m, parts, pt), e = chunk_lo(m, parts, pt + 1); k < e; ++k) {
            const uint32_t a = uint32_t(kv[k] >> 32), i = uint32_t(kv[k]);
            if (k == 0 || a != uint32_t(kv[k - 1] >> 32)) {
                hp.src_v[si] = a;
                hp.q_begin[si] = k;
                ++si;
            }
            hp.q_dst[k] = qs_dst[i];
            hp.q_id[k] = i;
            hp.q_pos[i] = k;  // the device writes query i's record at grouped position k
        }
    });
    hp.q_begin[starts[parts]] = m;
    if (timing_on())
        std::fprintf(stderr, "MR_TIMING build_plan n=%u parts=%u: specials %.2f ms, lookups %.2f, radix %.2f, grouping %.2f\n", n,
                     parts, tb0 - tbs, tb1 - tb0, tb2 - tb1, now_ms() - tb2);
    return MR_OK;
}

// The special / region word of every cell for the plan's special table (sp[t].v) and
// query homeland: sinfo[v] = table entry of v (kNone10) | entry of v's region campfire << 10.
static std::vector<uint32_t> build_sinfo(const mr_grid *g, const HostPlan &hp) {
    const uint32_t V = g->V;
    std::vector<uint32_t> tix(V, kNone10), out(V);
    for (uint32_t t = 1; t < hp.sp.size(); ++t) tix[hp.sp[t].v] = t;
    const std::vector<uint32_t> &near = g->nearest[hp.homeland];
    for (uint32_t v = 0; v < V; ++v) {
        const uint32_t r = near[v] == kNone32 ? kNone10 : tix[near[v]];
        out[v] = (tix[v] & kNone10) | (r << 10);
    }
    return out;
}

// The grid's shared device tables for a plan on device `dev`: rank, rank_inv and the
// sinfo of (homeland, HQ), uploaded once; false when the grid's tables live on another
// device (the plan then uploads its own).
// {sinfo, rank} per cell (hub_lane_kernel reads both words of a cell in one line)
static std::vector<uint2> build_cell(const mr_grid *g, const std::vector<uint32_t> &sinfo) {
    std::vector<uint2> out(sinfo.size());
    for (size_t v = 0; v < sinfo.size(); ++v) out[v] = make_uint2(sinfo[v], g->rank[v]);
    return out;
}

// The grid's device rank tables (rank, rank_inv), uploaded on the first device that asks
// (the caller holds near_mu); false on an upload error.
static bool grid_rank_upload(const mr_grid *g, int dev) {
    auto up = [](uint32_t *&d, const std::vector<uint32_t> &h) {
        if (dev_malloc(reinterpret_cast<void **>(&d), std::max<size_t>(h.size(), 1) * 4) != hipSuccess) return false;
        if (!h.empty() && hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            d = nullptr;
            return false;
        }
        return true;
    };
    if (!up(g->d_rank, g->rank)) return false;
    if (!up(g->d_rank_inv, g->rank_inv)) {
        (void)hipFree(g->d_rank);
        g->d_rank = nullptr;
        return false;
    }
    g->d_dev = dev;
    return true;
}
// The device rank table on `dev`: the grid's shared copy, nullptr when it lives on another
// device (or cannot be uploaded)
static const uint32_t *grid_rank_device(const mr_grid *g, int dev) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    if (g->d_dev == -1 && !grid_rank_upload(g, dev)) return nullptr;
    return g->d_dev == dev ? g->d_rank : nullptr;
}

static bool grid_tables(const mr_grid *g, int dev, const HostPlan &hp, uint32_t *&rank, uint32_t *&rank_inv,
                        uint32_t *&sinfo, uint2 *&cell) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    if (g->d_dev != -1 && g->d_dev != dev) return false;
    auto up = [](uint32_t *&d, const std::vector<uint32_t> &h) {
        if (dev_malloc(reinterpret_cast<void **>(&d), std::max<size_t>(h.size(), 1) * 4) != hipSuccess) return false;
        if (!h.empty() && hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            d = nullptr;
            return false;
        }
        return true;
    };
    if (g->d_dev == -1 && !grid_rank_upload(g, dev)) return false;
    uint32_t *ds = nullptr;
    uint2 *dc = nullptr;
    for (const mr_grid::SinfoDev &e : g->d_sinfo)
        if (e.homeland == hp.homeland && e.hq_v == hp.hq_v) {
            ds = e.d;
            dc = e.cell;
        }
    if (!ds) {
        if (g->d_sinfo.size() >= 8) return false;
        const std::vector<uint32_t> si = build_sinfo(g, hp);
        if (!up(ds, si)) return false;
        const std::vector<uint2> ce = build_cell(g, si);
        if (dev_malloc(reinterpret_cast<void **>(&dc), std::max<size_t>(ce.size(), 1) * sizeof(uint2)) != hipSuccess) {
            (void)hipFree(ds);
            return false;
        }
        if (!ce.empty() && hipMemcpy(dc, ce.data(), ce.size() * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(ds);
            (void)hipFree(dc);
            return false;
        }
        g->d_sinfo.push_back(mr_grid::SinfoDev{hp.homeland, hp.hq_v, ds, dc});
    }
    rank = g->d_rank;
    rank_inv = g->d_rank_inv;
    sinfo = ds;
    cell = dc;
    return true;
}

// Plan buffers come from a cache of freed device blocks (size classes per device: powers
// of two up to 64 MiB, 64 MiB steps above): a plan for each fresh batch then costs no
// hipMalloc / hipFree (tens of microseconds each, milliseconds for large blocks).  A
// block returns to the cache when its plan is destroyed, after mr_plan_destroy has
// waited for the plan's work; the cache keeps up to 16 GiB and is emptied before a
// hipMalloc that would otherwise fail.
struct BlockCache {
    std::mutex mu;
    std::unordered_map<void *, std::pair<int, size_t>> live;  // block -> (device, class bytes)
    std::unordered_map<uint64_t, std::vector<void *>> free;   // (device, class) -> blocks
    size_t cached = 0;
};
static BlockCache &block_cache() {
    static BlockCache *c = new BlockCache();  // never destroyed: plans may outlive static destructors
    return *c;
}
static size_t size_class(size_t b) {
    constexpr size_t kBig = size_t(64) << 20;
    if (b > kBig) return (b + kBig - 1) / kBig * kBig;
    size_t c = 256;
    while (c < b) c <<= 1;
    return c;
}
static uint64_t cache_key(int dev, size_t cls) { return (uint64_t(cls) << 8) | uint64_t(dev & 0xFF); }
static void trim_cache(int dev) {  // hipFree every cached block of `dev` (caller holds the lock)
    BlockCache &c = block_cache();
    for (auto it = c.free.begin(); it != c.free.end(); ++it) {
        if (int(it->first & 0xFF) != (dev & 0xFF)) continue;
        for (void *q : it->second) {
            (void)hipFree(q);
            c.cached -= size_t(it->first >> 8);
        }
        it->second.clear();
    }
}
static hipError_t pmalloc(void **p, size_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    const size_t cls = size_class(std::max<size_t>(bytes, 1));
    BlockCache &c = block_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.free.find(cache_key(dev, cls));
    if (it != c.free.end() && !it->second.empty()) {
        *p = it->second.back();
        it->second.pop_back();
        c.cached -= cls;
        c.live[*p] = {dev, cls};
        return hipSuccess;
    }
    hipError_t e = hipMalloc(p, cls);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        trim_cache(dev);
        e = hipMalloc(p, cls);
    }
    if (e == hipSuccess) c.live[*p] = {dev, cls};
    return e;
}
static void pfree(void *p) {
    if (!p) return;
    BlockCache &c = block_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) {
        (void)hipFree(p);
        return;
    }
    const int dev = it->second.first;
    const size_t cls = it->second.second;
    c.live.erase(it);
    if (c.cached + cls > (size_t(16) << 30)) {
        (void)hipFree(p);
        return;
    }
    c.free[cache_key(dev, cls)].push_back(p);
    c.cached += cls;
}
static void trim_cache_all() {
    BlockCache &c = block_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto &kv : c.free) {
        for (void *q : kv.second) {
            (void)hipFree(q);
            c.cached -= size_t(kv.first >> 8);
        }
        kv.second.clear();
    }
}

// Plan streams come from a per-device pool as well: a destroyed plan (which waited for
// its work) returns its streams, and the next plan takes them without hipStreamCreate.
struct StreamPool {
    std::mutex mu;
    std::vector<std::pair<int, hipStream_t>> free;
};
static StreamPool &stream_pool() {
    static StreamPool *p = new StreamPool();
    return *p;
}
static hipError_t pstream_create(hipStream_t *s) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        StreamPool &p = stream_pool();
        std::lock_guard<std::mutex> lk(p.mu);
        for (size_t i = p.free.size(); i-- > 0;)
            if (p.free[i].first == dev) {
                *s = p.free[i].second;
                p.free.erase(p.free.begin() + long(i));
                return hipSuccess;
            }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
static void pstream_release(hipStream_t s) {
    if (!s) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    StreamPool &p = stream_pool();
    std::lock_guard<std::mutex> lk(p.mu);
    if (p.free.size() >= 64) {
        (void)hipStreamDestroy(s);
        return;
    }
    p.free.emplace_back(dev, s);
}

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return fail(MR_ERR_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

template <class T>
static int upload(T *&dptr, const std::vector<T> &h) {
    dptr = nullptr;
    size_t bytes = std::max<size_t>(h.size(), 1) * sizeof(T);
    HIPCHK(pmalloc(reinterpret_cast<void **>(&dptr), bytes));
    if (!h.empty()) HIPCHK(hipMemcpy(dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return MR_OK;
}

}  // namespace

// Pinned host staging for the per-batch copies (the query block up, a fetch's results
// and commands down): a pageable hipMemcpy runs at a fraction of the DMA rate.  One
// grow-only buffer per direction; a copy holds its mutex while it uses the buffer.
struct PinnedStage {
    std::mutex mu;
    void *p = nullptr;
    size_t bytes = 0;
    void *get(size_t want) {  // caller holds mu; nullptr if pinned memory is not available
        if (bytes >= want) return p;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        const size_t cls = (want + (size_t(8) << 20) - 1) / (size_t(8) << 20) * (size_t(8) << 20);
        if (hipHostMalloc(&p, cls, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return nullptr;
        }
        bytes = cls;
        return p;
    }
};
static PinnedStage &stage_up() {
    static PinnedStage *s = new PinnedStage();
    return *s;
}
static PinnedStage &stage_down() {
    static PinnedStage *s = new PinnedStage();
    return *s;
}
// true when [p, p + bytes) is page-locked host memory HIP can DMA into directly
// Caller ranges page-locked through mr_host_register: start -> bytes.  A fetch takes the
// direct DMA only into a destination range one of them covers whole (a range registered
// shorter than the fetch writes goes through the pinned stage).
static std::mutex g_reg_mu;
static std::map<uintptr_t, size_t> g_reg;
static bool host_pinned(const void *p, size_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(a);
    if (it == g_reg.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second;
}
// Device -> host copies of `n` segments into caller memory on `s`: straight DMA when the
// destination is pinned, else through the pinned stage in 16 MB chunks, two in flight:
// the DMA of chunk c + 1 runs while host threads copy chunk c out of the stage.
struct D2HSeg {
    void *dst;
    const void *src;
    size_t bytes;
};
static hipError_t copy_d2h(const D2HSeg *seg, int n, hipStream_t s) {
    hipError_t e = hipSuccess;
    bool direct = true;
    for (int i = 0; i < n; ++i)
        if (seg[i].bytes && !host_pinned(seg[i].dst, seg[i].bytes)) direct = false;
    if (direct) {
        for (int i = 0; i < n && e == hipSuccess; ++i)
            if (seg[i].bytes) e = hipMemcpyAsync(seg[i].dst, seg[i].src, seg[i].bytes, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    }
    constexpr size_t kChunk = size_t(4) << 20;  // (16 MB: 1M fetch 5.3 ms, one chunk's DMA and copy-out not overlapped)
    PinnedStage &st = stage_down();
    std::lock_guard<std::mutex> lk(st.mu);
    char *buf = static_cast<char *>(st.get(2 * kChunk));
    if (!buf) {  // no pinned memory: pageable copies
        for (int i = 0; i < n && e == hipSuccess; ++i)
            if (seg[i].bytes) e = hipMemcpyAsync(seg[i].dst, seg[i].src, seg[i].bytes, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    }
    struct Chunk {
        char *dst;
        const char *src;
        size_t bytes;
    };
    std::vector<Chunk> ch;
    for (int i = 0; i < n; ++i)
        for (size_t o = 0; o < seg[i].bytes; o += kChunk)
            ch.push_back({static_cast<char *>(seg[i].dst) + o, static_cast<const char *>(seg[i].src) + o,
                          std::min(kChunk, seg[i].bytes - o)});
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (hipEvent_t &x : ev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x, hipEventDisableTiming);
    auto issue = [&](size_t c) {
        if (e == hipSuccess) e = hipMemcpyAsync(buf + (c % 2) * kChunk, ch[c].src, ch[c].bytes, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(ev[c % 2], s);
    };
    for (size_t c = 0; c < ch.size() && c < 2; ++c) issue(c);
    HostPool &pool = HostPool::get();
    for (size_t c = 0; c < ch.size() && e == hipSuccess; ++c) {
        e = hipEventSynchronize(ev[c % 2]);
        if (e != hipSuccess) break;
        const char *from = buf + (c % 2) * kChunk;
        const uint32_t parts = ch[c].bytes >= (size_t(1) << 20) ? pool.size() : 1u;
        pool.run(parts, [&](uint32_t pt) {
            const size_t a = ch[c].bytes * pt / parts, b = ch[c].bytes * (pt + 1) / parts;
            std::memcpy(ch[c].dst + a, from + a, b - a);
        });
        if (c + 2 < ch.size()) issue(c + 2);
    }
    (void)hipStreamSynchronize(s);  // nothing may still write the stage once it is unlocked
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    return e;
}

static hipError_t dev_malloc(void **p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        trim_cache_all();
        e = hipMalloc(p, bytes);
    }
    return e;
}

extern "C" int mr_grid_region_table(mr_grid *g, uint32_t homeland, uint32_t *out, uint64_t cap_words, uint32_t *nreg,
                                    double *build_ms) {
    if (!g || homeland > 3) return fail(MR_ERR_INVALID_ARG, "mr_grid_region_table: null grid or homeland > 3");
    if (!mr_device_available()) return fail(MR_ERR_NO_DEVICE, "no gfx950 device visible (no CPU fallback)");
    const std::vector<uint32_t> &regs = region_list(g, int(homeland));
    const uint64_t words = uint64_t(g->V) * regs.size() * 2;
    if (nreg) *nreg = uint32_t(regs.size());
    if (out && cap_words < words) return fail(MR_ERR_CAPACITY, "mr_grid_region_table: output shorter than V x nreg x 2");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(MR_ERR_DEVICE, "hipGetDevice");
    const uint32_t *rank = grid_rank_device(g, dev);
    uint32_t *own = nullptr;
    if (!rank) {  // the grid's tables live on another device: this one gets its own rank copy
        if (dev_malloc(reinterpret_cast<void **>(&own), size_t(g->V) * 4) != hipSuccess ||
            hipMemcpy(own, g->rank.data(), size_t(g->V) * 4, hipMemcpyHostToDevice) != hipSuccess) {
            if (own) (void)hipFree(own);
            return fail(MR_ERR_DEVICE, "rank table upload");
        }
        rank = own;
    }
    const uint32_t *d = region_table_device(g, int(homeland), rank);
    if (own) (void)hipFree(own);
    if (!d) return fail(MR_ERR_DEVICE, "region table build");
    if (build_ms) *build_ms = g->region_ms[homeland];
    if (out && words && hipMemcpy(out, d, words * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "region table copy");
    return MR_OK;
}

extern "C" void mr_cache_trim(void) {
    trim_cache_all();
    SpareVecs<uint32_t>::get().clear();
    SpareVecs<int32_t>::get().clear();
    trim_group_scratch();
}

extern "C" int mr_host_register(void *p, uint64_t bytes) {
    if (!p || !bytes) return fail(MR_ERR_INVALID_ARG, "mr_host_register: null or empty range");
    if (!mr_device_available()) return fail(MR_ERR_NO_DEVICE, "no gfx950 device visible");
    const hipError_t e = hipHostRegister(p, size_t(bytes), hipHostRegisterDefault);
    if (e != hipSuccess) return fail(MR_ERR_DEVICE, std::string("hipHostRegister: ") + hipGetErrorString(e));
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[reinterpret_cast<uintptr_t>(p)] = size_t(bytes);
    return MR_OK;
}

extern "C" int mr_host_unregister(void *p) {
    if (!p) return fail(MR_ERR_INVALID_ARG, "mr_host_unregister: null pointer");
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.erase(reinterpret_cast<uintptr_t>(p));
    }
    const hipError_t e = hipHostUnregister(p);
    if (e != hipSuccess) return fail(MR_ERR_DEVICE, std::string("hipHostUnregister: ") + hipGetErrorString(e));
    return MR_OK;
}

struct mr_plan {
    const mr_grid *grid = nullptr;
    HostPlan hp;
    KArgs ka{};
    bool grid_in_lds = false;
    uint32_t blocks = 0;
    uint32_t *d_sinfo = nullptr, *d_rank = nullptr, *d_rank_inv = nullptr, *d_src = nullptr, *d_qb = nullptr,
             *d_qd = nullptr, *d_qi = nullptr;
    KArgs *d_args = nullptr;
    KArgs *d_args_fb = nullptr;           // SSSP launch over the hub solver's fallback list
    KArgs *d_args_hub_last = nullptr;     // hub launch that ends the pass (fallback known to be empty)
    KArgs *d_args_lane = nullptr;         // hub_lane_kernel launch (sources [0, n_lane))
    KArgs *d_args_lane_last = nullptr;    // the same, ending the pass
    uint32_t n_lane = 0;                  // sources on the lane kernel; the rest on hub_kernel
    uint32_t lane_g = 0;                  // > 0: the n_lane sources run G lanes each (hub_group_kernel)
    KArgs *d_args_fill = nullptr;         // all-destinations mode: the fill launch (ends the pass)
    bool all_mode = false;
    CellWord *d_rec = nullptr;            // all-destinations outputs (KArgs::out_rec ...)
    Rec *d_tab = nullptr;
    uint32_t *d_lex = nullptr, *d_sstate = nullptr;
    std::vector<uint32_t> src_of_input;   // caller's source i -> plan source index
    bool fb_none = false;                 // a completed pass of this plan had no fallback sources
    uint32_t runs = 0;
    double fill_ms = 0.0;                 // all-destinations: average fill launch of the last window
    uint32_t *d_near = nullptr, *d_fb = nullptr;
    uint32_t *d_near_sp = nullptr, *d_rb_off = nullptr, *d_rb_cell = nullptr;  // wide hub tables
    uint32_t *d_lane_blob = nullptr;  // lane / group kernels: the plan's LDS block (lane_blob_build)
    uint32_t *d_relist = nullptr;     // lane kernel (Fleetfoot): uncertain sources for hub_kernel (KArgs::relist)
    OutCmd *d_ovf = nullptr;              // command-overflow pool (labels longer than max_cmds)
    // outputs bound with an overflow buffer (a collective gathers them raw): each pass
    // ends with ovf_order_kernel, which puts the pool in record order (d_ovf_tmp: its staging)
    OutCmd *d_ovf_tmp = nullptr;
    bool ovf_order = false;
    uint32_t hub_blocks = 0, fb_blocks = 0, spw = 1, cus = 256, fill_per_cu = 8;
    unsigned long long *d_dbg = nullptr;  // diagnostic builds: per-workgroup phase cycles
    uint32_t algo = kAlgoGeneric;
    SpecialStatic *d_sp = nullptr;
    uint16_t *d_hubs = nullptr;
    OutResult *d_res = nullptr;
    OutCmd *d_cmd = nullptr;
    uint32_t *d_ws = nullptr, *d_counter = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t last_stream = nullptr;    // the stream the latest pass ran on
    hipEvent_t ev_last = nullptr;         // the end event of the latest pass (on the caller's stream)
    bool ev_last_orphan = false;          // ev_last was folded out of `timed` and is owned here
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timed;  // pending event pairs
    // whole: the pass is the fill launch (the pass pair times it)
    struct FillTimed {
        hipEvent_t first, second;
        bool whole;
    };
    std::vector<FillTimed> timed_fill;  // all-destinations: fill launches
    // timings of event pairs already folded (a caller that never asks for kernel_ms
    // must not pile up events: mr_plan_run folds the oldest beyond kMaxTimed)
    double acc_ms = 0.0, acc_fill_ms = 0.0;
    uint32_t acc_n = 0, acc_fill_n = 0;
    int device = 0;
    // All-destinations plans run the specials' solves of the next passes (hub kernels,
    // in order on the plan's hub stream) beside the fill of pass k (on the caller's
    // stream).  The per-pass buffers and kernel arguments come in slots taken round
    // robin; the d_* fields above always name the slot of the latest pass (use_slot).
    // One hub stream for every slot: more streams than the process's hardware queues
    // (GPU_MAX_HW_QUEUES, 4) alias, and a hub queued behind a fill serialises the two.
    struct Slot {
        Rec *tab = nullptr;
        uint32_t *lex = nullptr, *sstate = nullptr, *fb = nullptr, *counter = nullptr;
        KArgs *args = nullptr, *args_fb = nullptr, *args_fill = nullptr;
        hipEvent_t ev_hub = nullptr, ev_fill = nullptr;
        bool used = false;    // a pass has run in this slot
        bool solved = false;  // fused: a launch has solved the specials of this slot's next pass
    };
    std::vector<Slot> slots;  // slot 0 holds the plan's first buffers; empty: no overlap
    hipStream_t hub_stream = nullptr;
    bool overlap = false;
    // overlap in one launch per pass (hub_fill_kernel): the specials of pass k + 1 are
    // solved by the first workgroups of pass k's fill launch (MR_FILL_FUSED=0: the two
    // streams instead)
    bool fused = false;
    uint32_t hub_lds = 0, fused_per_cu = 0;
    uint32_t slot = 0;     // slot index of the d_* fields
    bool own_tables = true;  // d_sinfo / d_rank / d_rank_inv / d_cell: false = the grid's shared copies
    uint2 *d_cell = nullptr;
    uint32_t *d_qblock = nullptr;  // the per-batch arrays (d_src, d_qb, d_qd, d_qi point into it)
    void *d_gscratch = nullptr;    // device grouping: phase 1's scratch, until the partition (plan_create)
    uint32_t *d_gcnt = nullptr;    // device grouping: its counts
    // certified fallback (query hub plans): per slot a label table,
    // boundary ranks, source, cell words, check state and sweep list; the fill's
    // argument block over the slots
    uint32_t cert_cap = 0, cert_fill_gx = 1, cert_check_gx = 1, cert_tile_wgs = 0;
    Rec *d_cert_tab = nullptr;
    uint32_t *d_cert_win = nullptr;               // per slot the repair window (cert_window_kernel)
    uint32_t *d_cert_redo = nullptr;              // per slot: redone in the second round (cert_promote_kernel)
    KArgs *d_args_r2 = nullptr, *d_args_cert_r2 = nullptr;  // the second round's argument blocks
    unsigned long long *d_cert_pub = nullptr;     // the tile sweep's publish areas
    uint32_t *d_cert_lex = nullptr, *d_cert_src = nullptr, *d_cert_st = nullptr, *d_cert_aux = nullptr,
             *d_fb_cert = nullptr, *d_cert_ones = nullptr;
    CellWord *d_cert_rec = nullptr;
    KArgs *d_args_cert = nullptr;
    Rec *d_cert_stage_tab = nullptr;
    uint32_t *d_cert_stage_lex = nullptr, *d_cert_stage_src = nullptr;
    ~mr_plan() {
        if (!slots.empty()) {  // the d_* fields may name another slot: free each slot's once
            Slot &k = slots[0];
            d_tab = k.tab;
            d_lex = k.lex;
            d_sstate = k.sstate;
            d_fb = k.fb;
            d_counter = k.counter;
            d_args = k.args;
            d_args_fb = k.args_fb;
            d_args_fill = k.args_fill;
            k.tab = nullptr;
            k.lex = k.sstate = k.fb = k.counter = nullptr;
            k.args = k.args_fb = k.args_fill = nullptr;
        }
        for (Slot &k : slots) {
            for (void *p : {(void *)k.tab, (void *)k.lex, (void *)k.sstate, (void *)k.fb, (void *)k.counter,
                            (void *)k.args, (void *)k.args_fb, (void *)k.args_fill})
                if (p) (void)pfree(p);
            for (hipEvent_t e : {k.ev_hub, k.ev_fill})
                if (e) (void)hipEventDestroy(e);
        }
        pstream_release(hub_stream);
        d_src = d_qb = d_qd = d_qi = nullptr;  // inside d_qblock
        pfree(d_qblock);
        pfree(d_gscratch);
        pfree(d_gcnt);
        if (!own_tables) {  // the grid's
            d_sinfo = d_rank = d_rank_inv = nullptr;
            d_cell = nullptr;
        }
        if (d_cell) (void)pfree(d_cell);
        for (void *p : {(void *)d_cert_tab, (void *)d_cert_lex, (void *)d_cert_src, (void *)d_cert_st,
                        (void *)d_cert_aux, (void *)d_fb_cert, (void *)d_cert_ones, (void *)d_cert_rec,
                        (void *)d_args_cert, (void *)d_cert_stage_tab, (void *)d_cert_stage_lex,
                        (void *)d_cert_stage_src, (void *)d_cert_win, (void *)d_cert_pub, (void *)d_cert_redo,
                        (void *)d_args_r2, (void *)d_args_cert_r2})
            if (p) (void)pfree(p);
        for (void *p : {(void *)d_sinfo, (void *)d_rank, (void *)d_rank_inv, (void *)d_src, (void *)d_qb, (void *)d_qd,
                        (void *)d_qi, (void *)d_sp, (void *)d_hubs, (void *)d_res, (void *)d_cmd, (void *)d_ws,
                        (void *)d_counter, (void *)d_args, (void *)d_dbg, (void *)d_args_fb, (void *)d_near,
                        (void *)d_fb, (void *)d_args_hub_last, (void *)d_args_fill, (void *)d_rec,
                        (void *)d_args_lane, (void *)d_args_lane_last, (void *)d_relist,
                        (void *)d_tab,
                        (void *)d_lex, (void *)d_sstate, (void *)d_near_sp, (void *)d_rb_off, (void *)d_rb_cell, (void *)d_ovf,
                        (void *)d_lane_blob, (void *)d_ovf_tmp})
            if (p) (void)pfree(p);
        if (ev_last && ev_last_orphan) (void)hipEventDestroy(ev_last);
        for (auto &e : timed) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        for (auto &f : timed_fill)  // its end event is the pass's, destroyed above
            if (f.first) (void)hipEventDestroy(f.first);
        pstream_release(stream);
    }
};

// all-destinations overlap: make slot i's buffers and argument blocks current
static void use_slot(mr_plan *pl, uint32_t i) {
    const mr_plan::Slot &k = pl->slots[i];
    pl->d_tab = k.tab;
    pl->d_lex = k.lex;
    pl->d_sstate = k.sstate;
    pl->d_fb = k.fb;
    pl->d_counter = k.counter;
    pl->d_args = k.args;
    pl->d_args_fb = k.args_fb;
    pl->d_args_fill = k.args_fill;
    pl->ka.out_tab = k.tab;
    pl->ka.out_lex = k.lex;
    pl->ka.src_state = k.sstate;
    pl->ka.fb_list = k.fb;
    pl->ka.counter = k.counter;
    pl->slot = i;
}

// Kernel-argument blocks of a plan: the main launch, and for hub plans the fallback
// launch and the hub launch that ends a pass on its own (last_launch marks the
// kernel whose last workgroup resets the per-pass counters).
static int upload_args(mr_plan *pl) {
    // every block queued on the plan's stream, then one synchronisation (a blocking copy
    // each cost ~10 us: up to six per plan); the host copies live in `held` until then.
    // Callers hold a drained plan, so nothing of the stream's is in flight.
    KArgs held[8];
    uint32_t nh = 0;
    bool ok = true;
    auto put = [&](KArgs *d, const KArgs &k) {
        held[nh] = k;
        ok = ok && hipMemcpyAsync(d, &held[nh], sizeof(KArgs), hipMemcpyHostToDevice, pl->stream) == hipSuccess;
        ++nh;
        return ok;
    };
    struct Drain {
        mr_plan *pl;
        ~Drain() { (void)hipStreamSynchronize(pl->stream); }
    } drain{pl};
    KArgs k = pl->ka;
    const bool hub = pl->hp.hub;
    // tests: MR_DBG_INJECT_SLOT=<slot> makes the fill of that slot's passes raise a
    // device error flag (checks that errors of either overlap slot are reported)
    if (const char *e = std::getenv("MR_DBG_INJECT_SLOT"))
        if (pl->all_mode && uint32_t(std::atoi(e)) == pl->slot) k.dbg_flags |= kDbgInjectFlag;
    // the pass ends with: the SSSP kernel (no hub), the fill kernel (all-destinations
    // hub plans), else the fallback launch or a lone hub launch
    k.last_launch = hub ? 0u : 1u;
    if (!put(pl->d_args, k)) return MR_ERR_DEVICE;
    if (hub) {
        KArgs f = k;
        f.fb_mode = 1;
        f.last_launch = pl->all_mode ? 0u : 1u;
        if (!put(pl->d_args_fb, f)) return MR_ERR_DEVICE;
        KArgs l = k;
        l.last_launch = 1;
        if (!put(pl->all_mode ? pl->d_args_fill : pl->d_args_hub_last, l)) return MR_ERR_DEVICE;
        if (pl->d_args_cert) {  // the fill over the certificate slots the hub kernel exported
            KArgs c = k;
            c.nsrc = pl->cert_cap;
            c.nsrc_dev = pl->d_counter + kCtrCert;
            c.src_v = pl->d_cert_src;
            c.src_state = pl->d_cert_ones;
            c.out_tab = pl->d_cert_tab;
            c.out_lex = pl->d_cert_lex;
            c.out_rec = pl->d_cert_rec;
            if (!put(pl->d_args_cert, c)) return MR_ERR_DEVICE;
            if (pl->d_args_r2) {  // the second round: only the slots cert_promote_kernel marked
                KArgs r = k;
                r.cert_redo = pl->d_cert_redo;
                c.src_state = pl->d_cert_redo;
                if (!put(pl->d_args_r2, r) || !put(pl->d_args_cert_r2, c)) return MR_ERR_DEVICE;
            }
        }
        // (the lane kernel as the pass's only launch has no hub launch after it to relist into)
        KArgs ll = l;
        ll.relist = nullptr;
        if (pl->d_args_lane && (!put(pl->d_args_lane, k) || !put(pl->d_args_lane_last, ll))) return MR_ERR_DEVICE;
    }
    return ok && hipStreamSynchronize(pl->stream) == hipSuccess ? MR_OK : MR_ERR_DEVICE;
}

// The lane kernel adds metrics without overflow checks and keeps distances in 16
// bits (S <= 4097): it only takes plans whose longest possible label (2 NS + 4 commands: each
// table entry once with at most two tail commands, plus the final walk) stays below
// 2^32 in every metric at the per-command maxima.
static bool lane_bounds_ok(const DevParams &p) {
    const uint64_t ncmd = 2ull * p.NS + 4, dmax = 2ull * p.S + 2;
    const uint64_t money = std::max<uint64_t>(std::max<uint64_t>(p.soe_cost, p.shq_cost),
                                              std::max<uint64_t>(p.sfm_cost, 5 * dmax));
    const uint64_t time = std::max<uint64_t>(uint64_t(p.rgt) * dmax, 180 * dmax);
    const uint64_t lim = 0xFFFFFFFEull;  // c1 = 2^32 - 1 marks an absent label in the lane kernel
    return p.S <= 4097 && ncmd * dmax <= lim && ncmd * money <= lim && ncmd * time <= lim;
}
// hub_lane_kernel's fixed table layout: no caravan hub among the border-1 entries 2..5
// and every region campfire (and so every SoE target) in entries 6 .. 6 + kLaneRegs - 1
static bool lane_layout_ok(const HostPlan &hp) {
    for (uint32_t t = 2; t <= 5 && t <= hp.p.NS; ++t)
        if (hp.sp[t].flags & kSpHub) return false;
    for (uint32_t t = 1; t <= hp.p.NS; ++t)
        if (hp.sp[t].rid != kNone10 && (t < 6 || t >= 6 + kLaneRegs)) return false;
    for (uint32_t t = 1; t <= hp.p.NS; ++t) {  // SoE targets: the specials' region campfires
        const uint32_t r = hp.sp[t].region;
        if (r != kNone10 && (r < 6 || r >= 6 + kLaneRegs || hp.sp[r].rid == kNone10)) return false;
    }
    return true;
}

// sources that would run on the lane kernel (at most kLaneMaxQ queries)
static uint32_t lane_sources(const HostPlan &hp) {
    if (hp.dev_grouped) return hp.n_small;
    uint32_t c = 0;
    for (size_t i = 0; i + 1 < hp.q_begin.size(); ++i) c += hp.q_begin[i + 1] - hp.q_begin[i] <= kLaneMaxQ;
    return c;
}
// the lane kernel from 160 sources a CU (40 960 on MI355X): below, a plan's lane-kernel
// waves run one round at a wave per SIMD or less, latency-bound, and the group kernel is
// faster (1025^2 map: 20k sources 66 us against 97, 40k even, 60k 149 against 105);
// MR_HUB_LANE_MIN overrides
static uint32_t lane_min_sources() {
    if (const char *e = std::getenv("MR_HUB_LANE_MIN")) return uint32_t(std::strtoul(e, nullptr, 10));
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return uint32_t(cus) * 160u;
}

// The lane kernel's count order: the busiest sources first (MR_LANE_ORDER=asc: the
// least busy first), so the last waves of a launch are the shortest ones
static bool lane_order_desc() {
    const char *e = std::getenv("MR_LANE_ORDER");
    return !(e && !std::strcmp(e, "asc"));
}

// Hub plans on the lane kernel: the sources with at most kLaneMaxQ queries first (one
// source per lane, hub_lane_kernel), by query count (a wave runs its destination loop as
// often as its busiest lane's source has queries: c4's uniform batch, 1.55 queries a
// source, ran it ~4 times a wave in source order), then the others (hub_kernel, a lane
// per query); each class in source order, each source's records contiguous (the device
// partition, mr_k_groupq.hip, gives the same order).  Returns the count of the first group.
static uint32_t partition_sources(HostPlan &hp) {
    const uint32_t ns = uint32_t(hp.src_v.size());
    std::vector<uint32_t> order(ns), start(kLaneMaxQ + 3, 0);
    const bool desc = lane_order_desc();
    auto cls = [&](uint32_t i) {
        const uint32_t c = hp.q_begin[i + 1] - hp.q_begin[i];
        return c <= kLaneMaxQ ? (desc ? kLaneMaxQ + 1u - c : c) : kLaneMaxQ + 1u;
    };
    for (uint32_t i = 0; i < ns; ++i) ++start[cls(i) + 1];
    for (uint32_t c = 1; c < start.size(); ++c) start[c] += start[c - 1];
    const uint32_t n_lane = start[kLaneMaxQ + 1];
    for (uint32_t i = 0; i < ns; ++i) order[start[cls(i)]++] = i;
    std::vector<uint32_t> src, qb, qd, qi;
    spare_take(src, ns);
    spare_take(qb, ns + 1);
    spare_take(qd, hp.q_dst.size());
    spare_take(qi, hp.q_id.size());
    uint32_t off = 0;
    for (uint32_t j = 0; j < ns; ++j) {
        const uint32_t i = order[j];
        src[j] = hp.src_v[i];
        qb[j] = off;
        for (uint32_t k = hp.q_begin[i]; k < hp.q_begin[i + 1]; ++k, ++off) {
            qd[off] = hp.q_dst[k];
            qi[off] = hp.q_id[k];
            hp.q_pos[hp.q_id[k]] = off;
        }
    }
    qb[ns] = off;
    hp.src_v.swap(src);
    hp.q_begin.swap(qb);
    hp.q_dst.swap(qd);
    hp.q_id.swap(qi);
    for (std::vector<uint32_t> *a : {&src, &qb, &qd, &qi}) spare_put(*a);
    return n_lane;
}

// ---- query batches grouped on the device (mr_k_groupq.hip; dev_group_ok above) -----
// The per-batch block's layout for n queries (src_v, q_begin, q_dst, q_id: each bounded
// by n words, 64-word aligned)
static void qblock_layout(size_t n, size_t at[5]) {
    const size_t w = (n + 1 + 63) / 64 * 64;
    for (int j = 0; j <= 4; ++j) at[j] = size_t(j) * w;
}

// Phase 1 on the plan's stream: the raw queries up (straight from caller memory that
// mr_host_register page-locked, else through the pinned stage in 4 MB chunks, host
// threads copying chunk c + 1 while chunk c's DMA runs), the device grouping into a new
// query block, then the counts (and any invalid queries' ids) back.
static int group_on_device(mr_plan *pl, const mr_query *qs, uint32_t n) {
    HostPlan &hp = pl->hp;
    const mr_grid *g = pl->grid;
    GroupGeom geo{};
    geo.vc = g->vc;
    for (int h = 0; h < 4; ++h) {
        geo.ux[h] = g->ux[h];
        geo.uy[h] = g->uy[h];
        geo.ub[h] = g->ub[h];
    }
    geo.H = g->H;
    geo.V = g->V;
    size_t at[5];
    qblock_layout(n, at);
    void *d_q = nullptr;
    const size_t qbytes = size_t(n) * sizeof(mr_query);
    if (pmalloc(reinterpret_cast<void **>(&pl->d_qblock), at[4] * 4) != hipSuccess ||
        pmalloc(&d_q, qbytes) != hipSuccess || pmalloc(&pl->d_gscratch, group_scratch_bytes(n, g->V)) != hipSuccess ||
        pmalloc(reinterpret_cast<void **>(&pl->d_gcnt), 8 * 4 + 4096 * 4) != hipSuccess) {
        pfree(d_q);
        return fail(MR_ERR_DEVICE, "hipMalloc device grouping");
    }
    pl->d_src = pl->d_qblock + at[0];
    pl->d_qb = pl->d_qblock + at[1];
    pl->d_qd = pl->d_qblock + at[2];
    pl->d_qi = pl->d_qblock + at[3];
    hipError_t e = hipSuccess;
    if (host_pinned(qs, qbytes)) {
        e = hipMemcpyAsync(d_q, qs, qbytes, hipMemcpyHostToDevice, pl->stream);
    } else {
        PinnedStage &su = stage_up();
        std::lock_guard<std::mutex> lk(su.mu);
        constexpr size_t kUp = size_t(4) << 20;
        char *stage = static_cast<char *>(su.get(std::min(qbytes, 2 * kUp)));
        if (!stage) {
            e = hipMemcpyAsync(d_q, qs, qbytes, hipMemcpyHostToDevice, pl->stream);
        } else {
            // two stage halves in turn: a half is refilled only after its previous DMA
            hipEvent_t done[2] = {nullptr, nullptr};
            for (hipEvent_t &ev : done)
                if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            HostPool &hpool = HostPool::get();
            const char *src = reinterpret_cast<const char *>(qs);
            uint32_t c = 0;
            for (size_t lo = 0; lo < qbytes && e == hipSuccess; lo += kUp, ++c) {
                const size_t len = std::min(kUp, qbytes - lo);
                char *half = stage + (c & 1u) * kUp;
                if (c >= 2 && (e = hipEventSynchronize(done[c & 1u])) != hipSuccess) break;
                const uint32_t parts = len >= (size_t(1) << 20) ? hpool.size() : 1u;
                hpool.run(parts, [&](uint32_t pt) {
                    const size_t a = len * pt / parts, b = len * (pt + 1) / parts;
                    std::memcpy(half + a, src + lo + a, b - a);
                });
                e = hipMemcpyAsync(static_cast<char *>(d_q) + lo, half, len, hipMemcpyHostToDevice, pl->stream);
                if (e == hipSuccess) e = hipEventRecord(done[c & 1u], pl->stream);
            }
            const hipError_t es = hipStreamSynchronize(pl->stream);  // (the stage is in use until here)
            if (e == hipSuccess) e = es;
            for (hipEvent_t ev : done)
                if (ev) (void)hipEventDestroy(ev);
        }
    }
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (e == hipSuccess)
        e = group_queries_device(d_q, n, geo, kLaneMaxQ, pl->d_gscratch, pl->d_src, pl->d_qb, pl->d_qd, pl->d_qi,
                                 pl->d_gcnt, pl->d_gcnt + 8, 4096, pl->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(cnt, pl->d_gcnt, sizeof(cnt), hipMemcpyDeviceToHost, pl->stream);
    const hipError_t es = hipStreamSynchronize(pl->stream);
    if (e == hipSuccess) e = es;
    pfree(d_q);  // (after the sync: the cache hands blocks out without one)
    if (e != hipSuccess) return fail(MR_ERR_DEVICE, std::string("device grouping: ") + hipGetErrorString(e));
    hp.nrec = cnt[0];
    hp.nsrc = cnt[1];
    hp.n_small = cnt[2];
    const uint32_t ninv = cnt[4];
    if (ninv != n - cnt[0]) return fail(MR_ERR_DEVICE, "device grouping: inconsistent counts");
    hp.invalid.clear();
    if (ninv) {
        if (ninv <= 4096) {
            hp.invalid.resize(ninv);
            if (hipMemcpy(hp.invalid.data(), pl->d_gcnt + 8, size_t(ninv) * 4, hipMemcpyDeviceToHost) != hipSuccess)
                return fail(MR_ERR_DEVICE, "device grouping: invalid list");
        } else {  // many invalid queries: every query not among the grouped ids
            std::vector<uint32_t> ids(cnt[0]);
            if (cnt[0] && hipMemcpy(ids.data(), pl->d_qi, size_t(cnt[0]) * 4, hipMemcpyDeviceToHost) != hipSuccess)
                return fail(MR_ERR_DEVICE, "device grouping: query ids");
            std::vector<uint8_t> seen(n, 0);
            for (uint32_t i : ids) seen[i] = 1;
            for (uint32_t i = 0; i < n; ++i)
                if (!seen[i]) hp.invalid.push_back(i);
        }
        std::sort(hp.invalid.begin(), hp.invalid.end());
    }
    return MR_OK;
}

// Phase 2 (plans on hub_lane_kernel): the small sources first, into a new block
static uint32_t partition_on_device(mr_plan *pl) {
    HostPlan &hp = pl->hp;
    if (hp.nsrc == 0) return 0;
    size_t at[5];
    qblock_layout(hp.nq, at);
    uint32_t *blk = nullptr;
    if (pmalloc(reinterpret_cast<void **>(&blk), at[4] * 4) != hipSuccess) return kNone32;
    hipError_t e = partition_sources_device(hp.nq, pl->grid->V, hp.nsrc, kLaneMaxQ, lane_order_desc(), pl->d_gscratch, pl->d_src, pl->d_qb,
                                            pl->d_qd, pl->d_qi, pl->d_gcnt, blk + at[0], blk + at[1], blk + at[2],
                                            blk + at[3], pl->stream);
    const hipError_t es = hipStreamSynchronize(pl->stream);
    if (e == hipSuccess) e = es;
    if (e != hipSuccess) {
        pfree(blk);
        return kNone32;
    }
    pfree(pl->d_qblock);
    pl->d_qblock = blk;
    pl->d_src = blk + at[0];
    pl->d_qb = blk + at[1];
    pl->d_qd = blk + at[2];
    pl->d_qi = blk + at[3];
    return hp.n_small;
}

// The host copies of a device-grouped plan's arrays (record order, the fallback
// sources' cells, the host decoder), fetched on first use
static int host_arrays(const mr_plan *cpl) {
    mr_plan *pl = const_cast<mr_plan *>(cpl);
    HostPlan &hp = pl->hp;
    if (!hp.dev_grouped || hp.mirrored) return MR_OK;
    hp.src_v.assign(hp.nsrc, 0u);
    hp.q_begin.assign(size_t(hp.nsrc) + 1, 0u);
    hp.q_dst.assign(hp.nrec, 0u);
    hp.q_id.assign(hp.nrec, 0u);
    const std::pair<std::vector<uint32_t> *, const uint32_t *> arr[4] = {
        {&hp.src_v, pl->d_src}, {&hp.q_begin, pl->d_qb}, {&hp.q_dst, pl->d_qd}, {&hp.q_id, pl->d_qi}};
    for (const auto &a : arr)
        if (!a.first->empty() &&
            hipMemcpy(a.first->data(), a.second, a.first->size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(MR_ERR_DEVICE, "copy grouped arrays");
    hp.q_pos.assign(hp.nq, kNone32);
    hp.q_status.assign(hp.nq, MR_OK);
    for (uint32_t k = 0; k < hp.nrec; ++k) hp.q_pos[hp.q_id[k]] = k;
    for (uint32_t i : hp.invalid) hp.q_status[i] = MR_ERR_INVALID_INDEX;
    hp.mirrored = true;
    return MR_OK;
}

static int plan_create(const mr_grid *g, const mr_params *prm, const mr_query *qs, uint32_t n, uint32_t max_cmds,
                       mr_plan **out, bool all_mode = false) {
    if (!out || (n && !qs)) return fail(MR_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    if (!mr_device_available()) return fail(MR_ERR_NO_DEVICE, "no gfx950 device visible (no CPU fallback)");
    const double tm0 = timing_on() ? now_ms() : 0.0;
    double tm_build = 0, tm_upload = 0, tm_alloc = 0;
    auto pl = new mr_plan();
    pl->grid = g;
    int st = build_plan(g, prm, qs, n, max_cmds, pl->hp, !all_mode);
    if (st == MR_OK && pl->hp.dev_grouped) {  // the batch grouped on the device (counts back)
        if (hipGetDevice(&pl->device) != hipSuccess) st = fail(MR_ERR_DEVICE, "hipGetDevice");
        else if (pstream_create(&pl->stream) != hipSuccess) st = fail(MR_ERR_DEVICE, "stream");
        else st = group_on_device(pl, qs, n);
    }
    if (timing_on()) tm_build = now_ms();
    if (st != MR_OK) {
        delete pl;
        return st;
    }
    HostPlan &hp = pl->hp;
    // all destinations: hub_kernel + fill only, linear run times (the fill's keys)
    if (all_mode && (hp.wide || hp.nonlin)) hp.hub = hp.wide = hp.nonlin = false;
    // query plans with a linear run time and a table that fits a lane's registers: the
    // sources with few queries run one per lane, when there are enough of them to give
    // half of the SIMDs a wave (lane_min_sources); a lane-kernel wave runs a whole
    // Dijkstra, so fewer waves than SIMDs leave it latency-bound and hub_kernel (a wave
    // per source) is faster.  MR_HUB_LANE=0: never, =1: whenever applicable.
    const char *hl = std::getenv("MR_HUB_LANE");
    const bool lane_off = hl && !std::strcmp(hl, "0"), lane_force = hl && !std::strcmp(hl, "1");
    // Plans the lane kernel does not take (too few sources to fill the GPU, or a table
    // layout it does not hold) run one source per group of G lanes when the table fits 32
    // entries: a source's Dijkstra is then ~G times shorter in wave instructions, which
    // is what a small plan's pass time is (hub_group_kernel).  MR_HUB_GROUP=0: never,
    // =8 / =16 / =32: the group size; MR_HUB_GROUP_FORCE=1: even where the lane
    // kernel applies.  The certificate's table export is hub_kernel's, so
    // MR_HUB_FALLBACK_ALL keeps hub_kernel.
    const char *hg = std::getenv("MR_HUB_GROUP");
    const uint32_t hgv = hg ? uint32_t(std::strtoul(hg, nullptr, 10)) : 8u;
    const bool group_off = hg && hgv == 0, group_force = std::getenv("MR_HUB_GROUP_FORCE") != nullptr;
    // default size by sources (tools/gpu_r04zi.sh): 32 lanes up to 1 024 (a lone
    // source: 23 us against 31 with 16), 16 up to 4 096 (c2, 3 821 sources: 37 us against
    // 44 with 8), else 8 (1025^2 map, 5k / 20k sources: 34 / 66 us against 53 / 129 with
    // 16: more groups per wave, fewer waves)
    const size_t nsrc_g = nsrc_of(hp);
    const uint32_t group_g = hg ? (hgv == 16 ? 16u : (hgv == 32 ? 32u : 8u))
                                : (nsrc_g <= 1024 ? 32u : (nsrc_g <= 4096 ? 16u : 8u));
    const bool lane_ok = hp.hub && !hp.wide && !all_mode && hp.near && lane_bounds_ok(hp.p);
    // Fleetfoot 1..3 on the lane kernel (its NL instantiation: the walk certification of
    // hub_kernel's §3a'').  A source it cannot certify (Time first: 1 in 118k at 1025^2)
    // is relisted for a hub_kernel launch right after it, whose fallback reaches the
    // certificate (§3d) instead of the SSSP kernel.  MR_LANE_NONLIN=0: never; =1: the group
    // kernel for Time-first orders too.
    const char *lnl = std::getenv("MR_LANE_NONLIN");
    const bool lane_nl = hp.nonlin && hp.ff_magic_ok && !(lnl && !std::strcmp(lnl, "0"));
    if (lane_ok && (!hp.nonlin || lane_nl) && !group_force && !lane_off && hub_lane_entries(hp.p.NS) != 0 &&
        lane_layout_ok(hp) && (lane_force || lane_sources(hp) >= lane_min_sources()))
        pl->n_lane = hp.dev_grouped ? partition_on_device(pl) : partition_sources(hp);
    // (the group kernel takes Fleetfoot plans that do not lead with Time: on Time-first
    // ones, c2-sized, hub_kernel's pass was 0.4-0.5 ms shorter, tools/r05/gpu_rates.sh)
    else if (lane_ok && (!hp.nonlin || (lane_nl && (hp.p.perm[0] != 2u || (lnl && !std::strcmp(lnl, "1"))))) &&
             !group_off && !lane_force && hub_group_slots(hp.p.NS, group_g) != 0 &&
             !std::getenv("MR_HUB_FALLBACK_ALL")) {
        pl->n_lane = nsrc_of(hp);
        pl->lane_g = group_g;
    }
    if (pl->d_gscratch) {  // phase 1's scratch is done with (the partition synchronised)
        pfree(pl->d_gscratch);
        pl->d_gscratch = nullptr;
    }
    auto bail = [&](int code) {
        delete pl;
        return code;
    };
    if (pl->n_lane == kNone32) return bail(fail(MR_ERR_DEVICE, "device partition of the sources"));
    if (hipGetDevice(&pl->device) != hipSuccess) return bail(fail(MR_ERR_DEVICE, "hipGetDevice"));
    if (grid_tables(g, pl->device, hp, pl->d_rank, pl->d_rank_inv, pl->d_sinfo, pl->d_cell)) {
        pl->own_tables = false;
    } else {
        const std::vector<uint32_t> si = build_sinfo(g, hp);
        if ((st = upload(pl->d_sinfo, si)) || (st = upload(pl->d_cell, build_cell(g, si))) ||
            (st = upload(pl->d_rank, g->rank)) || (st = upload(pl->d_rank_inv, g->rank_inv)))
            return bail(st);
    }
    if ((st = upload(pl->d_sp, hp.sp)) || (st = upload(pl->d_hubs, hp.hubs)))
        return bail(st);
    if (!hp.dev_grouped) {  // the per-batch arrays in one device block and one copy (sources, offsets, destinations, query ids)
        const size_t a0 = 0, a1 = a0 + (hp.src_v.size() + 63) / 64 * 64, a2 = a1 + (hp.q_begin.size() + 63) / 64 * 64,
                     a3 = a2 + (hp.q_dst.size() + 63) / 64 * 64, a4 = a3 + (hp.q_id.size() + 63) / 64 * 64;
        // packed in the pinned upload stage (host threads for large batches), one DMA
        const size_t words = std::max<size_t>(a4, 1);
        if (pmalloc(reinterpret_cast<void **>(&pl->d_qblock), words * 4) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "hipMalloc query block"));
        {
            PinnedStage &su = stage_up();
            std::lock_guard<std::mutex> lk(su.mu);
            uint32_t *pack = static_cast<uint32_t *>(su.get(words * 4));
            std::vector<uint32_t> pv;
            if (!pack) {
                pv.assign(words, 0u);
                pack = pv.data();
            }
            const std::vector<uint32_t> *arr[4] = {&hp.src_v, &hp.q_begin, &hp.q_dst, &hp.q_id};
            const size_t at[4] = {a0, a1, a2, a3};
            // words [a, b) of the block: the pieces of the four arrays that fall in them
            auto pack_range = [&](size_t a, size_t b) {
                for (int j = 0; j < 4; ++j) {
                    const size_t s = std::max(a, at[j]), e = std::min(b, at[j] + arr[j]->size());
                    if (s < e) std::memcpy(pack + s, arr[j]->data() + (s - at[j]), (e - s) * 4);
                }
            };
            HostPool &hpool = HostPool::get();
            if (words < (size_t(1) << 18)) {
                pack_range(0, words);
                if (hipMemcpy(pl->d_qblock, pack, words * 4, hipMemcpyHostToDevice) != hipSuccess)
                    return bail(fail(MR_ERR_DEVICE, "upload query block"));
            } else {
                // 4 MB chunks: the DMA of chunk c runs while host threads pack chunk c + 1
                // (packed and copied in one go: 0.85 ms at 1M queries)
                constexpr size_t kUp = size_t(1) << 20;
                const uint32_t parts = hpool.size();
                hipError_t e = hipSuccess;
                for (size_t lo = 0; lo < words && e == hipSuccess; lo += kUp) {
                    const size_t hi = std::min(words, lo + kUp);
                    hpool.run(parts, [&](uint32_t pt) {
                        pack_range(lo + (hi - lo) * pt / parts, lo + (hi - lo) * (pt + 1) / parts);
                    });
                    e = hipMemcpyAsync(pl->d_qblock + lo, pack + lo, (hi - lo) * 4, hipMemcpyHostToDevice, nullptr);
                }
                // (the stage is not unlocked, nor the block used, before the copies are done)
                const hipError_t es = hipStreamSynchronize(nullptr);
                if (e != hipSuccess || es != hipSuccess) return bail(fail(MR_ERR_DEVICE, "upload query block"));
            }
        }
        pl->d_src = pl->d_qblock + a0;
        pl->d_qb = pl->d_qblock + a1;
        pl->d_qd = pl->d_qblock + a2;
        pl->d_qi = pl->d_qblock + a3;
    }
    if (timing_on()) tm_upload = now_ms();
    size_t nres = std::max<uint32_t>(n, 1);
    if (pmalloc(reinterpret_cast<void **>(&pl->d_res), nres * sizeof(OutResult)) != hipSuccess ||
        pmalloc(reinterpret_cast<void **>(&pl->d_cmd), nres * size_t(max_cmds) * sizeof(OutCmd)) != hipSuccess ||
        pmalloc(reinterpret_cast<void **>(&pl->d_ovf), std::max<size_t>(4096, size_t(n) * 8) * sizeof(OutCmd)) !=
            hipSuccess ||
        pmalloc(reinterpret_cast<void **>(&pl->d_counter), kCtrWords * 4) != hipSuccess ||
        hipMemset(pl->d_counter, 0, kCtrWords * 4) != hipSuccess)
        return bail(fail(MR_ERR_DEVICE, "hipMalloc outputs"));
    // algorithm: level-synchronous when the comparator leads with Legs (MR_ALGO=generic forces the
    // bucketed solver, used by the tests to cover both); grid state in LDS when it fits 3
    // workgroups per CU, else per-workgroup HBM slots (MR_GRID_STATE=hbm|lds overrides)
    const uint32_t NS = hp.p.NS, V = hp.p.V;
    const uint32_t nsrc = nsrc_of(hp);
    pl->algo = hp.p.bucket_mode == kBucketLegs ? kAlgoLegs : kAlgoGeneric;
    if (const char *e = std::getenv("MR_ALGO"))
        if (!std::strcmp(e, "generic")) pl->algo = kAlgoGeneric;
    const uint32_t lds_full = lds_bytes(NS, V, true, pl->algo);
    pl->grid_in_lds = V <= 65535 && lds_full <= 53 * 1024;
    if (const char *e = std::getenv("MR_GRID_STATE")) {
        if (!std::strcmp(e, "hbm")) pl->grid_in_lds = false;
        else if (!std::strcmp(e, "lds") && V <= 65535 && lds_full <= 160 * 1024) pl->grid_in_lds = true;
    }
    uint32_t bytes = lds_bytes(NS, V, pl->grid_in_lds, pl->algo);
    if (bytes > 160 * 1024) return bail(fail(MR_ERR_LIMIT, "special table exceeds LDS"));
    const hipDeviceProp_t *propp = device_props(pl->device);
    if (!propp) return bail(fail(MR_ERR_DEVICE, "props"));
    const hipDeviceProp_t &prop = *propp;
    pl->cus = uint32_t(prop.multiProcessorCount);
    int per_cu = std::max(1, max_blocks_per_cu(pl->grid_in_lds, pl->algo, bytes));
    uint64_t resident = uint64_t(per_cu) * uint64_t(prop.multiProcessorCount);
    uint64_t blocks = std::min<uint64_t>(std::max<uint32_t>(nsrc, 1), resident);
    if (hp.hub) blocks = std::min<uint64_t>(blocks, 2ull * prop.multiProcessorCount);  // fallback launches only
    if (!pl->grid_in_lds) {
        const uint64_t slot_bytes = 5ull * V * 4ull;
        // HBM budget for solve slots; hub plans only solve the (few) fallback sources
        // (a hub plan's slots serve the few sources its closed form cannot certify: 2 GB
        // is ~95 slots at 1025^2 and ~6 at 4097^2, each looping over the sources)
        const uint64_t budget = (hp.hub ? 2ull : 64ull) << 30;
        blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, budget / slot_bytes));
        if (pmalloc(reinterpret_cast<void **>(&pl->d_ws), blocks * slot_bytes) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "hipMalloc workspace"));
    }
    pl->blocks = uint32_t(blocks);
    if (timing_on()) tm_alloc = now_ms();
    if (!pl->stream && pstream_create(&pl->stream) != hipSuccess)
        return bail(fail(MR_ERR_DEVICE, "stream"));
    KArgs &ka = pl->ka;
    ka.p = hp.p;
    ka.sinfo = pl->d_sinfo;
    ka.rank = pl->d_rank;
    ka.rank_inv = pl->d_rank_inv;
    ka.cell = pl->d_cell;
    ka.sp = pl->d_sp;
    ka.hubs = pl->d_hubs;
    ka.src_v = pl->d_src;
    ka.q_begin = pl->d_qb;
    ka.q_dst = pl->d_qd;
    ka.q_id = pl->d_qi;
    ka.out_res = pl->d_res;
    ka.out_cmd = pl->d_cmd;
    ka.ws = pl->d_ws;
    ka.counter = pl->d_counter;
    ka.ovf = pl->d_ovf;
    ka.ovf_cap = uint32_t(std::min<size_t>(std::max<size_t>(4096, size_t(n) * 8), 0xFFFFFFFFu));
    ka.nsrc = nsrc;
    ka.early_exit_max = 64;
    ka.grid_in_lds = pl->grid_in_lds ? 1u : 0u;
    ka.algo = pl->algo;
    ka.dbg = nullptr;
    ka.near = nullptr;
    ka.nreg = 0;
    ka.fb_list = nullptr;
    ka.fb_mode = 0;
    ka.fb_all = std::getenv("MR_HUB_FALLBACK_ALL") ? 1u : 0u;  // tests cover the fallback path
    ka.n_lane = pl->n_lane;
    ka.rank_std = g->rank_std ? 1u : 0u;
    ka.src_off = pl->n_lane;
    if (const char *e = std::getenv("MR_DBG_FLAGS")) ka.dbg_flags = uint32_t(std::atoi(e));
    pl->all_mode = all_mode;
    if (all_mode) {  // per source: a record per cell, the label table, the boundary ranks
        const size_t T = size_t(NS) + 1;
        // rows padded to whole 128 B lines (rec_pitch; MR_REC_ALIGN=64 pads to whole
        // 64-cell tile rows): the fill never stores part of a line
        uint32_t align = 32;
        if (const char *e = std::getenv("MR_REC_ALIGN"))
            if (std::atoi(e) == 64) align = 64;
        const uint32_t pitch = (hp.p.S + align - 1) / align * align;
        ka.rec_pitch = pitch;
        if (pmalloc(reinterpret_cast<void **>(&pl->d_rec),
                      std::max<size_t>(nsrc, 1) * hp.p.S * pitch * sizeof(CellWord)) != hipSuccess ||
            pmalloc(reinterpret_cast<void **>(&pl->d_tab), std::max<size_t>(nsrc, 1) * T * sizeof(Rec)) != hipSuccess ||
            pmalloc(reinterpret_cast<void **>(&pl->d_lex), std::max<size_t>(nsrc, 1) * T * 4) != hipSuccess ||
            pmalloc(reinterpret_cast<void **>(&pl->d_sstate), std::max<size_t>(nsrc, 1) * 4) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "hipMalloc all-destinations outputs"));
        ka.all_mode = 1;
        ka.out_rec = pl->d_rec;
        ka.out_tab = pl->d_tab;
        ka.out_lex = pl->d_lex;
        ka.src_state = pl->d_sstate;
        ka.early_exit_max = 0;  // every cell must settle
        pl->src_of_input.assign(n, kNone32);
        for (uint32_t si = 0; si < nsrc; ++si)
            for (uint32_t k = hp.q_begin[si]; k < hp.q_begin[si + 1]; ++k) pl->src_of_input[hp.q_id[k]] = si;
    }
    if (hp.hub) {
        if (pmalloc(reinterpret_cast<void **>(&pl->d_fb), std::max<size_t>(nsrc, 1) * 4) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "hub tables"));
        if (hp.near) {
            ka.near = region_table_device(g, prm->homeland, pl->d_rank);
            if (!ka.near) return bail(fail(MR_ERR_DEVICE, "region table build"));
            if ((st = special_rows_from_table(g, prm->homeland, ka.near, hp.nreg, hp.sp, hp.near_sp)) != MR_OK)
                return bail(fail(st, "region table rows"));
        }
        if (hp.wide) {
            std::vector<uint32_t> off(hp.rb_off->begin(), hp.rb_off->end());
            if (off.empty()) off.push_back(0);
            if (upload(pl->d_near_sp, hp.near_sp) != MR_OK || upload(pl->d_rb_off, off) != MR_OK ||
                upload(pl->d_rb_cell, *hp.rb_cell) != MR_OK)
                return bail(fail(MR_ERR_DEVICE, "wide hub tables"));
            ka.near_sp = pl->d_near_sp;
            ka.rb_off = pl->d_rb_off;
            ka.rb_cell = pl->d_rb_cell;
        }
        ka.nreg = hp.nreg;
        ka.fb_list = pl->d_fb;
        // two sources per wave when the specials fit 32 lanes (MR_HUB_SPW=1 forces one);
        // the wide kernel runs one source per wave
        pl->spw = !hp.wide && NS + 1 <= 32 ? 2u : 1u;
        if (const char *e = std::getenv("MR_HUB_SPW"))
            if (std::atoi(e) == 1) pl->spw = 1;
        const uint32_t hb = hp.wide ? hub_wide_lds_bytes(NS, hp.nreg) : hub_lds_bytes(NS, hp.nreg, pl->spw);
        if (hb > 160 * 1024) return bail(fail(MR_ERR_LIMIT, "hub tables exceed LDS"));
        const int hper = std::max(1, hp.wide ? hub_wide_blocks_per_cu(hp.p.perm, NS, hb)
                                             : hub_blocks_per_cu(hp.p.perm, pl->spw, hp.nonlin, hb));
        // (a lane kernel with Fleetfoot relists its uncertain sources for hub_kernel: room
        // for a few hundred of them in one round)
        const bool relist = pl->n_lane && hp.nonlin;
        const uint64_t per_block = 4ull * pl->spw, hub_src = std::max<uint64_t>(nsrc - pl->n_lane, relist ? 512u : 0u);
        pl->hub_blocks = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((hub_src + per_block - 1) / per_block,
                                                                           uint64_t(hper) * prop.multiProcessorCount)));
        if (const char *e = std::getenv("MR_HUB_BLOCKS")) pl->hub_blocks = uint32_t(std::max(1, std::atoi(e)));
        pl->fb_blocks = pl->blocks;
        pl->fill_per_cu = uint32_t(std::max(1, fill_blocks_per_cu(hp.p.perm)));
        if (pmalloc(reinterpret_cast<void **>(&pl->d_args_fb), sizeof(KArgs)) != hipSuccess ||
            pmalloc(reinterpret_cast<void **>(&pl->d_args_hub_last), sizeof(KArgs)) != hipSuccess ||
            pmalloc(reinterpret_cast<void **>(&pl->d_args_fill), sizeof(KArgs)) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "kernel args"));
        // Certified fallback for query plans on hub_kernel (MR_CERT=0: off; MR_CERT_SLOTS:
        // slots per pass, default by grid size): a flagged source's table goes to a slot, the fill
        // writes its closed form over every cell, the check and one repair sweep decide
        // whether its labels need the SSSP kernel at all.
        const char *ce = std::getenv("MR_CERT");
        if (!all_mode && !hp.wide && !(ce && !std::strcmp(ce, "0"))) {
            // slots: as many as 512 MB of cell words and sweep lists hold, 8 to 64 (1025^2:
            // 60; 4097^2: 8).  A Time-first Fleetfoot 1 batch of 125k on c4's map hands
            // over ~40 sources, and every one without a slot costs a whole SSSP solve.
            const size_t T = size_t(NS) + 1;
            const uint32_t pitch = (hp.p.S + 31) / 32 * 32;
            const size_t slot_bytes = size_t(V) * 4 + size_t(hp.p.S) * pitch * 4 + T * (sizeof(Rec) + 4);
            uint32_t cap = uint32_t(std::min<size_t>(64, std::max<size_t>(8, (size_t(512) << 20) / slot_bytes)));
            if (const char *e = std::getenv("MR_CERT_SLOTS")) cap = uint32_t(std::min(64, std::max(1, std::atoi(e))));
            std::vector<uint32_t> ones(cap, 1u);
            // staging for every fallback entry up to kCertStageMax (mr_engine.hpp): a
            // pass with more hands nothing to the certificate
            const uint32_t stage = uint32_t(std::min<size_t>(kCertStageMax, std::max<size_t>(nsrc, 1)));
            if (pmalloc(reinterpret_cast<void **>(&pl->d_cert_stage_tab), stage * T * sizeof(Rec)) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_stage_lex), stage * T * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_stage_src), stage * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_tab), cap * T * sizeof(Rec)) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_lex), cap * T * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_src), cap * 4) != hipSuccess ||

                pmalloc(reinterpret_cast<void **>(&pl->d_cert_aux), size_t(cap) * V * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_cert_rec), size_t(cap) * hp.p.S * pitch * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_fb_cert), std::max<size_t>(nsrc, 1) * 4) != hipSuccess ||
                pmalloc(reinterpret_cast<void **>(&pl->d_args_cert), sizeof(KArgs)) != hipSuccess ||
                upload(pl->d_cert_ones, ones) != MR_OK)
                return bail(fail(MR_ERR_DEVICE, "certificate slots"));
            pl->cert_cap = cap;
            ka.cert_cap = cap;
            ka.cert_stage_cap = stage;
            ka.cert_stage_tab = pl->d_cert_stage_tab;
            ka.cert_stage_lex = pl->d_cert_stage_lex;
            ka.cert_stage_src = pl->d_cert_stage_src;
            ka.cert_tab = pl->d_cert_tab;
            ka.cert_lex = pl->d_cert_lex;
            ka.cert_src = pl->d_cert_src;
            ka.cert_st = pl->d_cert_st;
            ka.cert_aux = pl->d_cert_aux;
            ka.cert_rec = pl->d_cert_rec;
            ka.fb_cert = pl->d_fb_cert;
            ka.rec_pitch = pitch;
            const uint64_t tiles = uint64_t((hp.p.S + kFillTW - 1) / kFillTW) * ((hp.p.S + kFillTH - 1) / kFillTH);
            // (a workgroup's four waves a tile each, for every slot: the fill spreads the slots
            // over groups of waves, and workgroups past the slots in use exit.  One slot's
            // worth of workgroups left a small grid's 8 slots to 3 workgroups, one after the
            // other: 0.34 ms of Fleetfoot fill at 65^2)
            pl->cert_fill_gx = uint32_t(std::max<uint64_t>(
                1, std::min<uint64_t>((tiles + 3) / 4 * cap, uint64_t(pl->fill_per_cu) * prop.multiProcessorCount)));
            pl->cert_check_gx = uint32_t(std::max<uint64_t>(
                1, std::min<uint64_t>((uint64_t(V) + 4 * 256 - 1) / (4 * 256), 4ull * prop.multiProcessorCount)));
            // the check's state: one partial per slot and check workgroup, reduced by its readers
            if (pmalloc(reinterpret_cast<void **>(&pl->d_cert_st), size_t(cap) * pl->cert_check_gx * kCertSt * 4) !=
                hipSuccess)
                return bail(fail(MR_ERR_DEVICE, "certificate slots"));
            ka.cert_st = pl->d_cert_st;
            ka.cert_parts = pl->cert_check_gx;
            // the repair: per slot its window; the tile sweep's persistent grid (one
            // workgroup a CU, each with two publish areas).  MR_CERT_TILE=0: the round-5
            // sweep for every slot (A/B)
            static const bool no_tile = [] {
                const char *e = std::getenv("MR_CERT_TILE");
                return e && std::atoi(e) == 0;
            }();
            const int occ = no_tile ? 0 : cert_tile_occupancy();
            pl->cert_tile_wgs = occ > 0 ? uint32_t(occ) * uint32_t(prop.multiProcessorCount) : 0u;
            // (+ one word: cert_window_kernel's completion count, zero between launches)
            if (pmalloc(reinterpret_cast<void **>(&pl->d_cert_win), (size_t(cap) * kWinWords + 1) * 4) != hipSuccess ||
                hipMemset(pl->d_cert_win, 0, (size_t(cap) * kWinWords + 1) * 4) != hipSuccess ||
                (pl->cert_tile_wgs && pmalloc(reinterpret_cast<void **>(&pl->d_cert_pub),
                                              size_t(pl->cert_tile_wgs) * 2 * kTileT * kTileT * 8) != hipSuccess))
                return bail(fail(MR_ERR_DEVICE, "certificate slots"));
            ka.cert_win = pl->d_cert_win;
            ka.cert_pub = pl->d_cert_pub;
            ka.cert_pub_wgs = pl->cert_tile_wgs;
            // the second round after promotions (MR_CERT_PROMOTE=0: none)
            static const bool no_promote = [] {
                const char *e = std::getenv("MR_CERT_PROMOTE");
                return e && std::atoi(e) == 0;
            }();
            if (!no_promote && (pmalloc(reinterpret_cast<void **>(&pl->d_cert_redo), size_t(cap) * 4) != hipSuccess ||
                                pmalloc(reinterpret_cast<void **>(&pl->d_args_r2), sizeof(KArgs)) != hipSuccess ||
                                pmalloc(reinterpret_cast<void **>(&pl->d_args_cert_r2), sizeof(KArgs)) != hipSuccess))
                return bail(fail(MR_ERR_DEVICE, "certificate slots"));
        }
        if (pl->n_lane && (pmalloc(reinterpret_cast<void **>(&pl->d_args_lane), sizeof(KArgs)) != hipSuccess ||
                           pmalloc(reinterpret_cast<void **>(&pl->d_args_lane_last), sizeof(KArgs)) != hipSuccess))
            return bail(fail(MR_ERR_DEVICE, "kernel args"));
        if (relist) {
            if (pmalloc(reinterpret_cast<void **>(&pl->d_relist), size_t(pl->n_lane) * 4) != hipSuccess)
                return bail(fail(MR_ERR_DEVICE, "relist"));
            ka.relist = pl->d_relist;
        }
        if (pl->n_lane) {  // the lane / group kernels' LDS block, built once per plan
            const uint32_t TM = pl->lane_g ? pl->lane_g * hub_group_slots(NS, pl->lane_g) : hub_lane_entries(NS);
            std::vector<uint32_t> blob;
            lane_blob_build(hp.sp.data(), NS, hp.nreg, TM, hp.p.rgt, hp.p.ff_num, hp.p.ff_den, hp.near_sp.data(), blob);
            if (upload(pl->d_lane_blob, blob) != MR_OK) return bail(fail(MR_ERR_DEVICE, "lane tables"));
            ka.lane_blob = reinterpret_cast<const uint4 *>(pl->d_lane_blob);
        }
    }
#ifdef MR_HUBDUMP
    if (const char *e = std::getenv("MR_DEBUG_SRC"))
        if (pmalloc(reinterpret_cast<void **>(&pl->d_dbg), 64 * 16 * 4) == hipSuccess) {
            (void)hipMemset(pl->d_dbg, 0, 64 * 16 * 4);
            ka.dbg = pl->d_dbg;
            ka.dbg_blocks = uint32_t(std::atoi(e));
        }
#endif
#ifdef MR_STAMPS
    if (pmalloc(reinterpret_cast<void **>(&pl->d_dbg), (size_t(pl->blocks) * 10 + 16) * 8) == hipSuccess) {
        (void)hipMemset(pl->d_dbg, 0, (size_t(pl->blocks) * 10 + 16) * 8);
        ka.dbg = pl->d_dbg;
        ka.dbg_blocks = pl->blocks;
    }
#endif
    if (pmalloc(reinterpret_cast<void **>(&pl->d_args), sizeof(KArgs)) != hipSuccess || upload_args(pl) != MR_OK)
        return bail(fail(MR_ERR_DEVICE, "kernel args"));
    // all destinations with the hub: slots of per-pass buffers, so that the specials'
    // solves of the next passes overlap this pass's fill (MR_FILL_OVERLAP=0: off;
    // MR_FILL_SLOTS: the slot count, 2..8, default 2 — at c3 the specials' solve of a
    // pass is shorter than a fill, and 3 or 4 slots measured the same pass time)
    const char *ov = std::getenv("MR_FILL_OVERLAP");
    if (all_mode && hp.hub && !(ov && !std::strcmp(ov, "0"))) {
        uint32_t nslots = 2;
        if (const char *e = std::getenv("MR_FILL_SLOTS")) nslots = uint32_t(std::min(8, std::max(2, std::atoi(e))));
        const size_t T = size_t(NS) + 1, ns = std::max<size_t>(nsrc, 1);
        pl->slots.resize(nslots);
        mr_plan::Slot &k0 = pl->slots[0];
        k0.tab = pl->d_tab;
        k0.lex = pl->d_lex;
        k0.sstate = pl->d_sstate;
        k0.fb = pl->d_fb;
        k0.counter = pl->d_counter;
        k0.args = pl->d_args;
        k0.args_fb = pl->d_args_fb;
        k0.args_fill = pl->d_args_fill;
        for (uint32_t i = 0; i < nslots; ++i) {
            mr_plan::Slot &k = pl->slots[i];
            if (i > 0 &&
                (pmalloc(reinterpret_cast<void **>(&k.tab), ns * T * sizeof(Rec)) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.lex), ns * T * 4) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.sstate), ns * 4) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.fb), ns * 4) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.counter), kCtrWords * 4) != hipSuccess ||
                 hipMemset(k.counter, 0, kCtrWords * 4) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.args), sizeof(KArgs)) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.args_fb), sizeof(KArgs)) != hipSuccess ||
                 pmalloc(reinterpret_cast<void **>(&k.args_fill), sizeof(KArgs)) != hipSuccess))
                return bail(fail(MR_ERR_DEVICE, "all-destinations slots"));
            if (hipEventCreateWithFlags(&k.ev_hub, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&k.ev_fill, hipEventDisableTiming) != hipSuccess)
                return bail(fail(MR_ERR_DEVICE, "overlap streams"));
            if (i > 0) {
                use_slot(pl, i);
                const int ua = upload_args(pl);
                use_slot(pl, 0);
                if (ua != MR_OK) return bail(fail(MR_ERR_DEVICE, "kernel args"));
            }
        }
        if (pstream_create(&pl->hub_stream) != hipSuccess)
            return bail(fail(MR_ERR_DEVICE, "hub stream"));
        pl->overlap = true;
        const char *fz = std::getenv("MR_FILL_FUSED");
        if (!hp.wide && !hp.nonlin && !(fz && !std::strcmp(fz, "0"))) {
            pl->hub_lds = hub_lds_bytes(NS, hp.nreg, pl->spw);
            pl->fused_per_cu = uint32_t(std::max(0, hub_fill_blocks_per_cu(hp.p.perm, pl->spw, pl->hub_lds)));
            pl->fused = pl->fused_per_cu > 0;
        }
    }
    if (timing_on())
        std::fprintf(stderr, "MR_TIMING plan_create n=%u: build %.2f ms, upload %.2f, outputs+workspace %.2f, rest %.2f\n", n,
                     tm_build - tm0, tm_upload - tm_build, tm_alloc - tm_upload, now_ms() - tm_alloc);
    *out = pl;
    return MR_OK;
}

extern "C" int mr_plan_create(const mr_grid *g, const mr_params *prm, const mr_query *qs, uint32_t n, mr_plan **out) {
    return plan_create(g, prm, qs, n, 16, out);
}

extern "C" int mr_plan_create_ex(const mr_grid *g, const mr_params *prm, const mr_query *qs, uint32_t n,
                                 uint32_t max_cmds, mr_plan **out) {
    if (max_cmds == 0 || max_cmds > 4096) return fail(MR_ERR_INVALID_ARG, "max_cmds must be 1..4096");
    return plan_create(g, prm, qs, n, max_cmds, out);
}



static hipError_t launch_hub_plan(const mr_plan *pl, const KArgs *d_args, hipStream_t s) {
    if (pl->hp.wide) return launch_hub_wide(d_args, pl->ka.p.perm, pl->ka.p.NS, pl->ka.nreg, pl->hub_blocks, s);
    return launch_hub(d_args, pl->ka.p.perm, pl->spw, pl->hp.nonlin, pl->ka.p.NS, pl->ka.nreg, pl->hub_blocks, s);
}

static void fold_timed(mr_plan *pl, size_t keep);
static constexpr size_t kMaxTimed = 1024;  // pending timing event pairs per plan

extern "C" int mr_plan_run(mr_plan *pl, void *stream) {
    if (!pl) return fail(MR_ERR_INVALID_ARG, "null plan");
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : pl->stream;
    if (pl->ka.nsrc == 0) return MR_OK;
    if (pl->timed.size() >= kMaxTimed) fold_timed(pl, kMaxTimed / 4);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipEventCreate(&e0) != hipSuccess) return fail(MR_ERR_DEVICE, "event");
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return fail(MR_ERR_DEVICE, "event");
    }
    // Passes of one plan run in submission order whatever streams they are given:
    // a pass reads what the previous one left (the fused look-ahead tables, the
    // counters it resets, a slot the previous fill read), so a pass on another stream
    // first waits for the previous pass's end.  plan_sync then only needs the last.
    if (pl->ev_last && pl->last_stream != s && hipStreamWaitEvent(s, pl->ev_last, 0) != hipSuccess) {
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        return fail(MR_ERR_DEVICE, "wait for the previous pass");
    }
    const uint32_t prev_slot = pl->slot;
    if (pl->hp.hub && pl->all_mode && pl->fused) {  // one launch per pass, see below
        const uint32_t cur = pl->runs >= 1 ? (pl->slot + 1) % uint32_t(pl->slots.size()) : 0u;
        use_slot(pl, cur);
    } else if (pl->hp.hub && pl->all_mode && pl->overlap) {
        // overlap plans: this pass takes the next slot once the fill that last read it
        // has released it; nothing is launched or recorded before that wait is in place
        const uint32_t prev = pl->slot, next = pl->runs >= 1 ? (pl->slot + 1) % uint32_t(pl->slots.size()) : 0u;
        use_slot(pl, next);
        if (pl->slots[next].used && hipStreamWaitEvent(pl->hub_stream, pl->slots[next].ev_fill, 0) != hipSuccess) {
            use_slot(pl, prev);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            return fail(MR_ERR_DEVICE, "wait");
        }
        pl->slots[next].used = true;
    }
    (void)hipEventRecord(e0, s);
    hipError_t e;
    ++pl->runs;
    if (pl->hp.hub && pl->all_mode && pl->fused) {
        // Fused: this pass's specials were solved into its slot by the previous pass's
        // launch (the first pass solves its own first).  The SSSP kernel takes the
        // sources that solve flagged, then one launch fills this pass's cells while its
        // first workgroups solve the next pass's specials into the next slot (which the
        // previous launch's fill has finished reading: stream order).  Each pass thus runs
        // one specials' solve and one fill; the last pass's look-ahead solve is extra work.
        const uint32_t nslots = uint32_t(pl->slots.size()), cur = pl->slot, nxt = (cur + 1) % nslots;
        const uint64_t items = uint64_t(pl->ka.nsrc) * ((pl->ka.p.S + kFillTW - 1) / kFillTW) *
                               ((pl->ka.p.S + kFillTH - 1) / kFillTH);
        const uint64_t resident = uint64_t(pl->fused_per_cu) * pl->cus;
        // the look-ahead solve takes at most a quarter of the resident workgroups: with
        // as many hub workgroups as fit (8 k+ sources a pass at 1025^2) the fill was left
        // with one workgroup (12 288 sources: 4.3 s a pass; 17 ms with 256 fill workgroups)
        const uint32_t hub_fused = uint32_t(std::min<uint64_t>(pl->hub_blocks, std::max<uint64_t>(1, resident / 4)));
        const uint32_t fb_blocks = uint32_t(std::max<uint64_t>(
            1, std::min<uint64_t>((items + 3) / 4, resident > hub_fused ? resident - hub_fused : 1)));
        e = hipSuccess;
        // the first pass (or one after a failed launch) solves its own specials first
        const bool solve_own = !pl->slots[cur].solved;
        if (solve_own) e = launch_hub_plan(pl, pl->slots[cur].args, s);
        if (e == hipSuccess) pl->slots[cur].solved = true;
        if (e == hipSuccess && !pl->fb_none)
            e = launch_solve(pl->d_args_fb, pl->grid_in_lds, pl->algo, pl->ka.p.NS, pl->ka.p.V, pl->fb_blocks, s);
        // with no SSSP launch the pass is the fused launch: its time is the pass's (an
        // event of its own costs command-processor time, see ev_last below)
        hipEvent_t f0 = nullptr;
        const bool own = solve_own || !pl->fb_none;
        if (e == hipSuccess && own && hipEventCreate(&f0) == hipSuccess) (void)hipEventRecord(f0, s);
        if (e == hipSuccess)
            e = launch_hub_fill(pl->slots[nxt].args, pl->slots[cur].args_fill, pl->ka.p.perm, pl->spw, hub_fused,
                                fb_blocks, pl->hub_lds, s);
        if (e == hipSuccess) {
            pl->slots[cur].used = true;  // a fill ran in it: its counters hold a finished pass
            pl->slots[nxt].solved = true;
        } else {
            // nothing of this pass is trusted: the next run re-takes this slot, and the
            // slot the failed launch may have half-written is solved again
            pl->slots[nxt].solved = false;
            --pl->runs;
            use_slot(pl, prev_slot);
            if (pl->runs == 0) pl->slots[cur].solved = false;
        }
        pl->timed_fill.push_back({f0, nullptr, !own});
    } else if (pl->hp.hub && pl->all_mode) {
        // hub solve + table export, the SSSP kernel for flagged sources, then the fill:
        // (source, tile) items, one per wave, over a resident-sized grid
        const uint64_t items = uint64_t(pl->ka.nsrc) * ((pl->ka.p.S + kFillTW - 1) / kFillTW) *
                               ((pl->ka.p.S + kFillTH - 1) / kFillTH);
        uint32_t gx = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((items + 3) / 4, uint64_t(pl->fill_per_cu) * pl->cus)));
        if (const char *e = std::getenv("MR_FILL_GX")) gx = uint32_t(std::max(1, std::atoi(e)));
        const uint32_t gy = 1;
        // overlap: this pass took its slot above, and its hub kernel runs on the slot's
        // stream behind the wait for the fill that last read the slot.  The hub writes
        // only the slot's tables; everything that writes the records (the SSSP kernel for
        // flagged sources, the fill) stays on the caller's stream, in stream order.
        hipStream_t hs = pl->overlap ? pl->hub_stream : s;
        e = launch_hub_plan(pl, pl->d_args, hs);
        if (e == hipSuccess && pl->overlap) {
            if (hipEventRecord(pl->slots[pl->slot].ev_hub, hs) != hipSuccess ||
                hipStreamWaitEvent(s, pl->slots[pl->slot].ev_hub, 0) != hipSuccess)
                e = hipErrorUnknown;
        }
        if (e == hipSuccess && !pl->fb_none)
            e = launch_solve(pl->d_args_fb, pl->grid_in_lds, pl->algo, pl->ka.p.NS, pl->ka.p.V, pl->fb_blocks, s);
        hipEvent_t f0 = nullptr;
        if (e == hipSuccess && hipEventCreate(&f0) == hipSuccess) (void)hipEventRecord(f0, s);
        if (e == hipSuccess) e = launch_fill(pl->d_args_fill, pl->ka.p.perm, gx, gy, s);
        // the slot's tables are free again once this fill has read them
        if (e == hipSuccess && pl->overlap && hipEventRecord(pl->slots[pl->slot].ev_fill, s) != hipSuccess)
            e = hipErrorUnknown;
        pl->timed_fill.push_back({f0, nullptr, false});  // one per pass (f0 may be null), as in `timed`
    } else if (pl->hp.hub) {
        // closed-form hub solve: the lane kernel for the sources with few queries, the
        // hub kernel for the others, then the SSSP kernel for the sources they flagged
        // (usually none; those workgroups exit at once).  Once a pass of this plan (same
        // inputs, deterministic result) had no fallback source, the hub launches end the
        // pass on their own.
        // (a Fleetfoot lane plan relaunches hub_kernel for the sources its lane kernel
        // relisted, until a pass had none)
        const bool big = pl->ka.nsrc > pl->n_lane || (pl->d_relist && !pl->fb_none);
        e = hipSuccess;
        if (pl->n_lane) {
            const KArgs *la = pl->fb_none && !big ? pl->d_args_lane_last : pl->d_args_lane;
            e = pl->lane_g ? launch_hub_group(la, pl->ka.p.perm, pl->ka.p.NS, pl->ka.nreg, pl->n_lane, pl->lane_g, pl->hp.nonlin, s)
                           : launch_hub_lane(la, pl->ka.p.perm, pl->ka.p.NS, pl->ka.nreg, pl->n_lane, pl->hp.nonlin, s);
        }
        if (e == hipSuccess && big) e = launch_hub_plan(pl, pl->fb_none ? pl->d_args_hub_last : pl->d_args, s);
        // certified fallback: the slots given to the staged sources in source order,
        // their closed forms, the check, one repair sweep, the check again (each exits at
        // once without slots); the SSSP launch then
        // emits every certified source from its slot and solves the rest
        if (e == hipSuccess && !pl->fb_none && pl->cert_cap) {
            e = launch_cert_select(pl->d_args, s);
            if (e == hipSuccess) e = launch_fill(pl->d_args_cert, pl->ka.p.perm, pl->cert_fill_gx, 1, s);
            // (MR_CERT_NOSWEEP=1: diagnostics, the first check's state stays for MR_CERT_DEBUG)
            static const bool nosweep = std::getenv("MR_CERT_NOSWEEP") != nullptr;
            // the first check marks its failing cells: the sweep's seeds
            if (e == hipSuccess) e = launch_cert_check(pl->d_args, pl->cert_check_gx, pl->cert_cap, nosweep ? 0u : 1u, s);
            if (!nosweep) {
                // the repair: each slot's window, the tile sweep (Legs / Time first), the
                // round-5 sweep for the others
                if (e == hipSuccess) e = launch_cert_window(pl->d_args, pl->cert_cap, s);
                if (e == hipSuccess && pl->cert_tile_wgs) e = launch_cert_tile(pl->d_args, pl->cert_tile_wgs, s);
                if (e == hipSuccess) e = launch_cert_sweep(pl->d_args, pl->cert_cap, s);
                if (e == hipSuccess) e = launch_cert_check(pl->d_args, pl->cert_check_gx, pl->cert_cap, 0u, s);
                // further rounds for the slots whose last check still failed: the closed form
                // again after a promotion, else the sweep again from the repaired words
                for (int round = 0; round < kCertRounds && e == hipSuccess && pl->d_args_r2; ++round) {
                    e = launch_cert_promote(pl->d_args, pl->cert_cap, pl->d_cert_redo, s);
                    if (e == hipSuccess) e = launch_fill(pl->d_args_cert_r2, pl->ka.p.perm, pl->cert_fill_gx, 1, s);
                    if (e == hipSuccess) e = launch_cert_check(pl->d_args_r2, pl->cert_check_gx, pl->cert_cap, 1u, s);
                    if (e == hipSuccess) e = launch_cert_window(pl->d_args_r2, pl->cert_cap, s);
                    if (e == hipSuccess && pl->cert_tile_wgs) e = launch_cert_tile(pl->d_args_r2, pl->cert_tile_wgs, s);
                    if (e == hipSuccess) e = launch_cert_sweep(pl->d_args_r2, pl->cert_cap, s);
                    if (e == hipSuccess) e = launch_cert_check(pl->d_args_r2, pl->cert_check_gx, pl->cert_cap, 0u, s);
                }
            }
        }
        if (e == hipSuccess && !pl->fb_none)
            e = launch_solve(pl->d_args_fb, pl->grid_in_lds, pl->algo, pl->ka.p.NS, pl->ka.p.V, pl->fb_blocks, s);
    } else {
        e = launch_solve(pl->d_args, pl->grid_in_lds, pl->algo, pl->ka.p.NS, pl->ka.p.V, pl->blocks, s);
    }
    // raw outputs for a collective: the overflow pool in record order (byte-deterministic)
    if (e == hipSuccess && pl->ovf_order && !pl->all_mode) e = launch_ovf_order(pl->d_args, nrec_of(pl->hp), pl->d_ovf_tmp, s);
    (void)hipEventRecord(e1, s);
    // the pass's end event doubles as the plan's last event (plan_sync): a record of
    // its own cost ~6 us of command-processor time per pass
    if (pl->ev_last_orphan) (void)hipEventDestroy(pl->ev_last);
    pl->ev_last = e1;
    pl->ev_last_orphan = false;
    pl->last_stream = s;
    pl->timed.push_back({e0, e1});
    if (!pl->timed_fill.empty() && !pl->timed_fill.back().second) pl->timed_fill.back().second = e1;
    if (e != hipSuccess) return fail(MR_ERR_DEVICE, std::string("launch: ") + hipGetErrorString(e));
    return MR_OK;
}

// Waits for this plan's passes only (the caller's stream up to the last pass, the
// plan's own and hub streams), never for the whole device.
static bool plan_sync(mr_plan *pl) {
    bool ok = true;
    if (pl->runs && pl->ev_last) ok = hipEventSynchronize(pl->ev_last) == hipSuccess;
    if (pl->stream) ok = hipStreamSynchronize(pl->stream) == hipSuccess && ok;
    if (pl->hub_stream) ok = hipStreamSynchronize(pl->hub_stream) == hipSuccess && ok;
    return ok;
}

// counters after the plan's passes have drained; notes a pass without fallback sources
static int read_counters(mr_plan *pl, uint32_t ctr[kCtrWords]) {
    if (!plan_sync(pl) || hipMemcpy(ctr, pl->d_counter, kCtrWords * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "copy counter");
    if (pl->hp.hub && pl->runs && !pl->ka.fb_all && ctr[kCtrLastFb] == 0 && ctr[kCtrLastRelist] == 0) pl->fb_none = true;
    return MR_OK;
}

// Folds the pending event pairs into the plan's running totals, all but the newest
// `keep` of them (waits for those passes; the fill pairs share their end event
// with the pass pairs, which destroy it).
static void fold_timed(mr_plan *pl, size_t keep) {
    const size_t nf = pl->timed_fill.size() > keep ? pl->timed_fill.size() - keep : 0;
    for (size_t i = 0; i < nf; ++i) {
        auto &f = pl->timed_fill[i];
        float ms = 0.f;
        // all-destinations plans push one pair to each list per pass: the lists align
        const hipEvent_t f0 = f.whole && pl->timed.size() == pl->timed_fill.size() ? pl->timed[i].first : f.first;
        if (f0 && f.second && hipEventSynchronize(f.second) == hipSuccess &&
            hipEventElapsedTime(&ms, f0, f.second) == hipSuccess) {
            pl->acc_fill_ms += ms;
            ++pl->acc_fill_n;
        }
        if (f.first) (void)hipEventDestroy(f.first);
    }
    pl->timed_fill.erase(pl->timed_fill.begin(), pl->timed_fill.begin() + ptrdiff_t(nf));
    const size_t n = pl->timed.size() > keep ? pl->timed.size() - keep : 0;
    for (size_t i = 0; i < n; ++i) {
        auto &e = pl->timed[i];
        float ms = 0.f;
        if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
            pl->acc_ms += ms;
            ++pl->acc_n;
        }
        (void)hipEventDestroy(e.first);
        if (e.second == pl->ev_last) pl->ev_last_orphan = true;  // plan_sync still waits on it
        else (void)hipEventDestroy(e.second);
    }
    pl->timed.erase(pl->timed.begin(), pl->timed.begin() + ptrdiff_t(n));
}

extern "C" double mr_plan_kernel_ms(mr_plan *pl, uint32_t *n_launches) {
    if (!pl) return 0.0;
    // all-destinations passes: the fill launches' own time (their end event is the pass's)
    fold_timed(pl, 0);
    pl->fill_ms = pl->acc_fill_n ? pl->acc_fill_ms / pl->acc_fill_n : 0.0;
    const double tot = pl->acc_ms;
    const uint32_t k = pl->acc_n;
    pl->acc_ms = pl->acc_fill_ms = 0.0;
    pl->acc_n = pl->acc_fill_n = 0;
    uint32_t ctr[kCtrWords];
    (void)read_counters(pl, ctr);
    if (n_launches) *n_launches = k;
    return k ? tot / k : 0.0;
}

extern "C" int mr_plan_bind_outputs_ex(mr_plan *pl, void *d_results, void *d_commands, void *d_overflow,
                                       uint32_t overflow_cap) {
    if (!pl || !d_results || !d_commands || (overflow_cap && !d_overflow))
        return fail(MR_ERR_INVALID_ARG, "null argument");
    // all-destinations plans write per-cell records, not query records (and keep two
    // slots of argument blocks)
    if (pl->all_mode) return fail(MR_ERR_INVALID_ARG, "bind_outputs: not a query plan");
    if (!plan_sync(pl)) return fail(MR_ERR_DEVICE, "sync");
    pl->ka.out_res = reinterpret_cast<OutResult *>(d_results);
    pl->ka.out_cmd = reinterpret_cast<OutCmd *>(d_commands);
    if (d_overflow && overflow_cap) {  // overflow_cap 0 keeps the plan's own pool
        // the pool in record order after every pass (ovf_order_kernel): its staging buffer
        pfree(pl->d_ovf_tmp);
        pl->d_ovf_tmp = nullptr;
        pl->ovf_order = false;
        if (pmalloc(reinterpret_cast<void **>(&pl->d_ovf_tmp), size_t(overflow_cap) * sizeof(OutCmd)) != hipSuccess)
            return fail(MR_ERR_DEVICE, "bind_outputs: overflow staging");
        pl->ka.ovf = reinterpret_cast<OutCmd *>(d_overflow);
        pl->ka.ovf_cap = overflow_cap;
        pl->ovf_order = true;
    }
    if (upload_args(pl) != MR_OK) return fail(MR_ERR_DEVICE, "kernel args");
    return MR_OK;
}

extern "C" int mr_plan_bind_outputs(mr_plan *pl, void *d_results, void *d_commands) {
    return mr_plan_bind_outputs_ex(pl, d_results, d_commands, nullptr, 0);
}

extern "C" uint32_t mr_plan_num_sources(const mr_plan *pl) { return pl ? pl->ka.nsrc : 0; }

extern "C" int mr_plan_record_queries(const mr_plan *pl, uint32_t *query_of_record, uint32_t n) {
    if (!pl || (n && !query_of_record)) return fail(MR_ERR_INVALID_ARG, "null argument");
    if (int st = host_arrays(pl)) return st;
    const std::vector<uint32_t> &ids = pl->hp.q_id;
    for (uint32_t k = 0; k < n; ++k) query_of_record[k] = k < ids.size() ? ids[k] : kNone32;
    return MR_OK;
}

extern "C" double mr_plan_fill_ms(const mr_plan *pl) { return pl ? pl->fill_ms : 0.0; }

// The last pass's fallback entries (source indices, kFbCertified on those the certificate
// answered), sorted by source
static int handed_over(mr_plan *pl, std::vector<uint32_t> &fb) {
    fb.clear();
    if (!plan_sync(pl)) return fail(MR_ERR_DEVICE, "sync");
    uint32_t ctr[kCtrWords];
    if (int st = read_counters(pl, ctr)) return st;
    const uint32_t nf = pl->hp.hub && pl->d_fb ? std::min(ctr[kCtrLastFb], pl->ka.nsrc) : 0u;
    fb.resize(nf);
    if (nf && hipMemcpy(fb.data(), pl->d_fb, size_t(nf) * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "copy fallback list");
    std::sort(fb.begin(), fb.end(), [](uint32_t a, uint32_t b) { return (a & ~kFbCertified) < (b & ~kFbCertified); });
    if (!fb.empty())
        if (int st = host_arrays(pl)) return st;
    return MR_OK;
}

extern "C" int mr_plan_fallback_sources(mr_plan *pl, mr_cell_index *out, uint32_t cap, uint32_t *n) {
    if (!pl || !n || (cap && !out)) return fail(MR_ERR_INVALID_ARG, "null argument");
    *n = 0;
    std::vector<uint32_t> fb;
    if (int st = handed_over(pl, fb)) return st;
    // entries the certificate answered carry kFbCertified: no search was run for them
    fb.erase(std::remove_if(fb.begin(), fb.end(), [](uint32_t s) { return (s & kFbCertified) != 0; }), fb.end());
    for (uint32_t k = 0; k < fb.size() && k < cap; ++k) out[k] = pl->grid->idx[pl->hp.src_v[fb[k]]];
    *n = uint32_t(fb.size());
    return MR_OK;
}

extern "C" int mr_plan_handed_over_sources(mr_plan *pl, mr_cell_index *out, uint8_t *certified, uint32_t cap,
                                           uint32_t *n) {
    if (!pl || !n) return fail(MR_ERR_INVALID_ARG, "null argument");
    *n = 0;
    std::vector<uint32_t> fb;
    if (int st = handed_over(pl, fb)) return st;
    for (uint32_t k = 0; k < fb.size() && k < cap; ++k) {
        if (out) out[k] = pl->grid->idx[pl->hp.src_v[fb[k] & ~kFbCertified]];
        if (certified) certified[k] = (fb[k] & kFbCertified) ? 1u : 0u;
    }
    *n = uint32_t(fb.size());
    return MR_OK;
}

extern "C" int mr_plan_get_stats(mr_plan *pl, mr_plan_stats *out) {
    if (!pl || !out) return fail(MR_ERR_INVALID_ARG, "null argument");
    std::memset(out, 0, sizeof(*out));
    uint32_t ctr[kCtrWords];
    if (int st = read_counters(pl, ctr)) return st;
    if (std::getenv("MR_CERT_DEBUG") && pl->cert_cap) {  // diagnostics: each slot's last check
        const size_t parts = pl->cert_check_gx, n = size_t(pl->cert_cap) * parts * kCertSt;
        std::vector<uint32_t> cs(n), src(pl->cert_cap);
        if (hipMemcpy(cs.data(), pl->d_cert_st, n * 4, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(src.data(), pl->d_cert_src, src.size() * 4, hipMemcpyDeviceToHost) == hipSuccess)
            for (uint32_t k = 0; k < pl->cert_cap; ++k) {
                uint32_t key = kNone32, fails = 0, x0 = kNone32, x1 = 0, y0 = kNone32, y1 = 0;
                for (size_t j = 0; j < parts; ++j) {
                    const uint32_t *q = &cs[(k * parts + j) * kCertSt];
                    if (!q[kCertFails]) continue;
                    key = std::min(key, q[kCertKey]);
                    fails += q[kCertFails];
                    x0 = std::min(x0, q[kCertX0]);
                    x1 = std::max(x1, q[kCertX1]);
                    y0 = std::min(y0, q[kCertY0]);
                    y1 = std::max(y1, q[kCertY1]);
                }
                const uint32_t v = src[k] < pl->grid->V ? src[k] : 0;
                uint32_t wn[16] = {0};
                if (pl->d_cert_win) (void)hipMemcpy(wn, pl->d_cert_win + size_t(k) * kWinWords, sizeof(wn), hipMemcpyDeviceToHost);
                std::fprintf(stderr,
                             "MR_CERT_DEBUG slot %u src (%d,%d): fails %u key %u box x %d..%d y %d..%d | repair mode %u "
                             "tiles %ux%u steps %u fail %u promoted %08x%08x | tile 0: steps %.1f us, %u exchanges %.1f us\n",
                             k, pl->grid->gx(v), pl->grid->gy(v), fails, key, int(x0) - int(pl->grid->H),
                             int(x1) - int(pl->grid->H), int(y0) - int(pl->grid->H), int(y1) - int(pl->grid->H), wn[kWinMode],
                             wn[kWinNtx], wn[kWinNty], wn[kWinSteps], wn[kWinFail], wn[kWinProm1], wn[kWinProm0],
                             wn[kWinTStep] * 0.01, wn[kWinNXchg],
                             wn[kWinTXchg] * 0.01);
                {
                    uint32_t wy[29] = {0};
                    if (hipMemcpy(wy, pl->d_cert_win + size_t(k) * kWinWords + kWinWhy, sizeof(wy), hipMemcpyDeviceToHost) == hipSuccess)
                        for (uint32_t f = 0; f < std::min(wy[0], 7u); ++f)
                            std::fprintf(stderr, "MR_CERT_DEBUG   failing cell (%d,%d)%s tests %#x own %u best %u\n",
                                         int(wy[1 + 4 * f] & 0xFFFFu) - int(pl->grid->H), int(wy[1 + 4 * f] >> 16) - int(pl->grid->H),
                                         (wy[2 + 4 * f] >> 31) ? " special" : "", wy[2 + 4 * f] & 0x7FFFFFFFu, wy[3 + 4 * f], wy[4 + 4 * f]);
                }
                if (wn[kWinMode] == kWinTile) {  // the tiles' step / exchange times and settles
                    const uint32_t nt = std::min(wn[kWinNtx] * wn[kWinNty], kTileMaxTiles);
                    std::vector<uint32_t> ts(size_t(nt) * 4);
                    if (hipMemcpy(ts.data(), pl->d_cert_win + size_t(k) * kWinWords + kWinStat, ts.size() * 4,
                                  hipMemcpyDeviceToHost) == hipSuccess)
                        for (uint32_t t = 0; t < nt; ++t)
                            std::fprintf(stderr, "MR_CERT_DEBUG   tile %u: steps %u in %.1f us, exchanges %.1f us (publish %.1f, wait %.1f)\n", t,
                                         ts[4 * t + 3], ts[4 * t] * 0.01, ts[4 * t + 1] * 0.01, (ts[4 * t + 2] >> 16) * 0.01,
                                         (ts[4 * t + 2] & 0xFFFFu) * 0.01);
                }
            }
    }
    out->solver = pl->hp.hub ? (pl->hp.wide ? MR_SOLVER_HUB_WIDE : MR_SOLVER_HUB)
                             : (pl->algo == kAlgoLegs ? MR_SOLVER_LEVELS : MR_SOLVER_BUCKETED);
    out->grid_state_in_lds = pl->grid_in_lds ? 1u : 0u;
    out->num_sources = pl->ka.nsrc;
    out->fallback_sources = pl->hp.hub ? ctr[kCtrLastFb] : 0u;
    out->num_specials = pl->ka.p.NS;
    out->num_regions = pl->hp.nreg;
    out->hub_workgroups = pl->hub_blocks;
    out->sssp_workgroups = pl->blocks;
    out->specials_per_lane = !pl->hp.hub ? 0u : (pl->hp.wide ? hub_wide_spl(pl->ka.p.NS) : 1u);
    out->region_boundary_cells = pl->hp.wide && pl->hp.rb_off && !pl->hp.rb_off->empty() ? pl->hp.rb_off->back() : 0u;
    out->lane_sources = pl->lane_g ? 0u : pl->n_lane;
    out->lanes_per_source = !pl->n_lane ? 0u : (pl->lane_g ? pl->lane_g : 1u);
    out->certified_sources = ctr[kCtrLastCert];
    out->fill_launch = !(pl->hp.hub && pl->all_mode) ? MR_FILL_NONE
                       : pl->fused                   ? MR_FILL_FUSED
                       : pl->overlap                 ? MR_FILL_STREAMS
                                                     : MR_FILL_SERIAL;
    return MR_OK;
}

// Makes `stream` (or, with NULL, the calling thread) wait until every pass enqueued
// on the plan so far has finished: how a consumer on another stream reads the device
// outputs without a host sync (passes are chained, so the last pass's end suffices).
extern "C" int mr_plan_wait(mr_plan *pl, void *stream) {
    if (!pl) return fail(MR_ERR_INVALID_ARG, "null plan");
    if (!stream) return plan_sync(pl) ? MR_OK : fail(MR_ERR_DEVICE, "sync");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // (a pass's hub-stream work is waited for by its own records' stream before the
    // pass's end event, so that event covers it)
    if (pl->ev_last && hipStreamWaitEvent(s, pl->ev_last, 0) != hipSuccess) return fail(MR_ERR_DEVICE, "wait");
    return MR_OK;
}

extern "C" int mr_plan_device_outputs(mr_plan *pl, void **d_results, uint64_t *rb, void **d_commands, uint64_t *cb) {
    if (!pl) return fail(MR_ERR_INVALID_ARG, "null plan");
    // the pointers are handed out once the plan's passes so far have finished, so a
    // raw read right after this call sees whole records (mr_plan_wait orders a stream
    // instead of the host)
    if (!plan_sync(pl)) return fail(MR_ERR_DEVICE, "sync");
    if (d_results) *d_results = pl->ka.out_res;
    if (rb) *rb = uint64_t(pl->hp.nq) * sizeof(OutResult);
    if (d_commands) *d_commands = pl->ka.out_cmd;
    if (cb) *cb = uint64_t(pl->hp.nq) * pl->hp.p.max_cmds * sizeof(OutCmd);
    return MR_OK;
}

// What a compact command's payload scales by (mr_engine.hpp Cmd): the caravan
// seconds per distance unit, the scroll prices and the raw Fleetfoot level.
struct CmdScale {
    uint32_t rgt, soe, shq, sfm, ff;
};
static CmdScale cmd_scale(const HostPlan &hp) {
    return CmdScale{hp.p.rgt, hp.p.soe_cost, hp.p.shq_cost, hp.p.sfm_cost, hp.fleetfoot_raw};
}
static CmdScale cmd_scale(const mr_params &prm) {
    return CmdScale{caravan_unit_time(prm.route_guru), prm.scroll_of_escape_cost, prm.scroll_of_escape_hq_cost,
                    prm.scroll_of_escape_forum_cost, prm.fleetfoot};
}

// expand one compact command (mr_engine.hpp) into the ABI's mr_command; false if it
// names no cell of the grid
static bool expand_cmd(const mr_grid *g, const CmdScale &cs, const OutCmd &c, mr_command &o) {
    std::memset(&o, 0, sizeof(o));
    uint32_t kind = c.kp >> 29, pay = c.kp & 0x1FFFFFFFu;
    o.kind = uint8_t(kind);
    switch (kind) {
        case kCentral: o.time_s = int64_t(10) * pay; break;
        case kStandard:
            o.legs = pay;
            o.time_s = int64_t(180) * pay;
            o.fleetfoot = cs.ff;
            break;
        case kCaravan: {
            uint32_t d = pay >> 1;
            o.time_s = int64_t(cs.rgt) * d;
            o.money = d * ((pay & 1u) ? 5u : 2u);
            break;
        }
        case kSoE: o.money = cs.soe; break;
        case kSHQ: o.money = cs.shq; break;
        case kSFm: o.money = cs.sfm; break;
        default: break;
    }
    if (kind > kSFm || c.from >= g->V || c.to >= g->V) return false;
    o.from = g->idx[g->rank_inv[c.from]];  // device commands name cells by rank
    o.to = g->idx[g->rank_inv[c.to]];
    return true;
}

// Decodes compact record `o` (its max_cmds slots at `slots`, the overflow pool
// `ovf` of novf commands) into r, its commands into pool[off..] when they fit
// (else *ret = MR_ERR_CAPACITY).  Returns MR_OK, or MR_ERR_DEVICE for a record
// that is not well formed (an overflow tag outside the pool, a bad cell rank).
static int decode_record(const mr_grid *g, const CmdScale &cs, const OutResult &o, const OutCmd *slots, uint32_t mc,
                         const OutCmd *ovf, uint64_t novf, mr_result &r, mr_command *pool, uint64_t pool_cap,
                         uint64_t &off, int &ret) {
    std::memset(&r, 0, sizeof(r));
    int status = int(o.ncmd_status >> 16) - 16;
    r.legs = o.legs;
    r.money = o.money;
    r.time_s = int64_t(o.time);
    r.n_commands = o.ncmd_status & 0xFFFFu;
    r.status = status;
    r.command_offset = uint32_t(off);
    if (status == MR_NOT_FOUND) {
        r.n_commands = 0;
        return MR_OK;
    }
    // a long label: its commands are in the overflow pool at {offset, count}
    const OutCmd *src = slots;
    if (status == int(kStatusOverflow)) {
        const OutCmd &tag = slots[0];
        if (!mc || tag.kp != kOvfTag || tag.to != r.n_commands || uint64_t(tag.from) + tag.to > novf)
            return fail(MR_ERR_DEVICE, "overflow pool record");
        src = &ovf[tag.from];
        status = MR_OK;
        r.status = MR_OK;
    } else if (status == MR_OK && r.n_commands > mc) {
        return fail(MR_ERR_DEVICE, "record longer than its command slots");
    }
    if (status != MR_OK) {
        if (ret == MR_OK) ret = status;
        return MR_OK;
    }
    if (off + r.n_commands <= pool_cap && pool) {
        for (uint32_t j = 0; j < r.n_commands; ++j)
            if (!expand_cmd(g, cs, src[j], pool[off + j])) return fail(MR_ERR_DEVICE, "command names no cell");
    } else {
        ret = MR_ERR_CAPACITY;
    }
    off += r.n_commands;
    return MR_OK;
}

static int check_device_errors(mr_plan *pl, uint32_t &flags, uint32_t *ctr_out = nullptr) {
    uint32_t ctr[kCtrWords];
    if (int st = read_counters(pl, ctr)) return st;
    if (ctr_out) std::memcpy(ctr_out, ctr, sizeof(ctr));  // (read before the flags are collected)
    flags = ctr[kCtrFlags];
    if (flags) (void)hipMemset(pl->d_counter + kCtrFlags, 0, 4);  // collected
    // overlap plans: the other slots' counter blocks belong to earlier passes; their
    // flags and written counts are checked (and collected) as well
    for (uint32_t i = 0; i < pl->slots.size(); ++i) {
        const mr_plan::Slot &k = pl->slots[i];
        if (i == pl->slot || !k.counter) continue;
        uint32_t oc[kCtrWords];
        if (hipMemcpy(oc, k.counter, kCtrWords * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(MR_ERR_DEVICE, "copy counter");
        if (oc[kCtrFlags]) (void)hipMemset(k.counter + kCtrFlags, 0, 4);
        flags |= oc[kCtrFlags];  // a fused plan's look-ahead solve may have flagged a slot not yet filled
        if (flags == 0 && k.used && oc[kCtrLastWritten] != nrec_of(pl->hp))
            return fail(MR_ERR_DEVICE, "internal: " + std::to_string(oc[kCtrLastWritten]) + " of " +
                                           std::to_string(nrec_of(pl->hp)) + " records written (an earlier pass)");
    }
#ifdef MR_HUBDUMP
    if (pl->d_dbg) {
        std::vector<uint32_t> d(64 * 16);
        (void)hipMemcpy(d.data(), pl->d_dbg, d.size() * 4, hipMemcpyDeviceToHost);
        for (uint32_t t = 0; t <= pl->ka.p.NS; ++t) {
            const uint32_t *r = &d[t * 16];
            const uint32_t v = t ? pl->hp.sp[t].v : pl->ka.dbg_blocks;
            const mr_cell_index &c = pl->grid->idx[v];
            Rec rec;
            std::memcpy(&rec, r, sizeof(Rec));
            const uint32_t ut = rec.u < pl->grid->V ? rec.u : 0;
            const mr_cell_index &cu = pl->grid->idx[pl->grid->rank_inv[ut]];
            std::fprintf(stderr, "T%2u (%u,%u,%u,%u) R.m=(%u,%u,%u) len=%u ntail=%u state=%u par=%u k%u p%u u=(%u,%u,%u,%u)",
                         t, c.kind, c.sub, c.x, c.y, r[0], r[1], r[2], rec.len(), rec.ntail(), rec.state(), rec.parent(),
                         rec.kp0 >> 29, rec.kp0 & 0x1FFFFFFF, cu.kind, cu.sub, cu.x, cu.y);
            std::fprintf(stderr, " st=%u my=(%u,%u,%u) %08x\n", r[11], r[12], r[13], r[14], r[15]);
        }
    }
#endif
    if (std::getenv("MR_DEBUG")) {
        std::fprintf(stderr, "MR_DEBUG hub=%d sources=%u fallback=%u flags=%u hub_blocks=%u\n", int(pl->hp.hub),
                     pl->ka.nsrc, ctr[kCtrLastFb], ctr[kCtrFlags], pl->hub_blocks);
        if (pl->d_fb && ctr[kCtrLastFb] <= pl->ka.nsrc && host_arrays(pl) == MR_OK) {
            std::vector<uint32_t> fb(ctr[kCtrLastFb]);
            (void)hipMemcpy(fb.data(), pl->d_fb, fb.size() * 4, hipMemcpyDeviceToHost);
            std::fprintf(stderr, "MR_DEBUG fallback sources (vertex):");
            for (uint32_t s : fb) std::fprintf(stderr, " %u%s", pl->hp.src_v[s & ~kFbCertified], (s & kFbCertified) ? "c" : "");
            std::fprintf(stderr, "\n");
        }
    }
    if (flags && std::getenv("MR_DEBUG_FLAGS_OK")) {  // diagnostics: report, then read the records anyway
        std::fprintf(stderr, "MR_DEBUG_FLAGS_OK: device flags %u ignored\n", flags);
        flags = 0;
    }
    if (flags & (kErrKOverflow | kErrMetricOverflow))
        return fail(MR_ERR_LIMIT, "a label exceeds the engine's 32-bit metric or run-length limits");
    if (flags) return fail(MR_ERR_DEVICE, "internal invariant violated on device (flags " + std::to_string(flags) + ")");
    if (pl->runs && ctr[kCtrLastWritten] != nrec_of(pl->hp))
        return fail(MR_ERR_DEVICE, "internal: " + std::to_string(ctr[kCtrLastWritten]) + " of " +
                                       std::to_string(nrec_of(pl->hp)) + " result records written");
    return MR_OK;
}

// Copies the compact outputs and expands them.  Queries whose label needs more
// than max_cmds commands come back with status MR_ERR_CAPACITY in *over.
static int plan_collect(mr_plan *pl, std::vector<OutResult> &res, std::vector<OutCmd> &cmd,
                        std::vector<OutCmd> &ovf) {
    uint32_t flags = 0, ctr[kCtrWords];
    const int st = check_device_errors(pl, flags, ctr);  // (syncs the plan)
    if (st != MR_OK) return st;
    const uint32_t nov = std::min(ctr[kCtrLastOvf], pl->ka.ovf_cap);
    ovf.resize(nov);
    if (nov && hipMemcpy(ovf.data(), pl->ka.ovf, size_t(nov) * sizeof(OutCmd), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "copy overflow pool");
    const uint32_t n = pl->hp.nq, mc = pl->hp.p.max_cmds;
    res.resize(n);
    cmd.resize(size_t(n) * mc);
    if (n) {
        if (hipMemcpy(res.data(), pl->ka.out_res, n * sizeof(OutResult), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(cmd.data(), pl->ka.out_cmd, size_t(n) * mc * sizeof(OutCmd), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(MR_ERR_DEVICE, "copy outputs");
    }
    return MR_OK;
}

// the commands record k adds to the output pool (decode_record's `off` step)
static uint32_t record_cmds(const OutResult &o) {
    const int status = int(o.ncmd_status >> 16) - 16;
    return (status == MR_OK || status == int(kStatusOverflow)) ? (o.ncmd_status & 0xFFFFu) : 0u;
}

// the grid's CellIndex-by-rank table on the plan's device (uploaded once)
static const mr_cell_index *grid_idx_rank(const mr_grid *g, int dev) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    if (g->d_dev != dev) return nullptr;
    if (!g->d_idx_rank) {
        std::vector<mr_cell_index> t(g->V);
        for (uint32_t r = 0; r < g->V; ++r) t[r] = g->idx[g->rank_inv[r]];
        mr_cell_index *d = nullptr;
        if (dev_malloc(reinterpret_cast<void **>(&d), std::max<size_t>(t.size(), 1) * sizeof(mr_cell_index)) != hipSuccess)
            return nullptr;
        if (!t.empty() && hipMemcpy(d, t.data(), t.size() * sizeof(mr_cell_index), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return nullptr;
        }
        g->d_idx_rank = d;
    }
    return g->d_idx_rank;
}

// mr_plan_fetch with the records expanded on the device (mr_k_decode.hip) into the ABI
// layout, then one copy of the results and one of the commands; the host only marks the
// queries that had no record (invalid indices) and finds the status to return.  Returns
// false (nothing written) when the device path does not apply (the host decoder runs).
static bool plan_fetch_device(mr_plan *pl, mr_result *results, mr_command *pool, uint64_t pool_cap, int &ret) {
    const HostPlan &hp = pl->hp;
    const uint32_t nq = hp.nq, nrec = nrec_of(hp), mc = hp.p.max_cmds;
    if (const char *e = std::getenv("MR_HOST_DECODE"))
        if (!std::strcmp(e, "1")) return false;
    if (!pool || !nq || pl->all_mode) return false;
    const mr_cell_index *idx_rank = grid_idx_rank(pl->grid, pl->device);
    if (!idx_rank) return false;
    const double tm0 = timing_on() ? now_ms() : 0.0;
    uint32_t flags = 0, ctr[kCtrWords];
    if ((ret = check_device_errors(pl, flags, ctr)) != MR_OK) return true;  // (syncs the plan)
    const uint32_t nov = std::min(ctr[kCtrLastOvf], pl->ka.ovf_cap);
    const uint64_t bound = uint64_t(nrec) * mc + nov, pcap = std::min<uint64_t>(pool_cap, std::max<uint64_t>(bound, 1));
    const CmdScale cs = cmd_scale(hp);
    size_t temp_bytes = 0;
    (void)decode_records_device(nullptr, nullptr, nullptr, 0, nullptr, 0, nq, mc, nullptr, 0, 0, 0, 0, 0, 0, nullptr,
                                nullptr, nullptr, &temp_bytes, nullptr, nullptr, 0, nullptr, pl->stream);
    void *scratch = nullptr, *d_out = nullptr, *d_pool = nullptr;
    const size_t cnt_b = (size_t(nq) * 4 + 255) / 256 * 256, tail = 256;
    if (pmalloc(&scratch, 2 * cnt_b + temp_bytes + tail) != hipSuccess ||
        pmalloc(&d_out, size_t(nq) * sizeof(mr_result)) != hipSuccess ||
        pmalloc(&d_pool, size_t(pcap) * sizeof(mr_command)) != hipSuccess) {
        pfree(scratch);
        pfree(d_out);
        return false;  // the host decoder needs no device memory
    }
    uint32_t *cnt = static_cast<uint32_t *>(scratch), *off = reinterpret_cast<uint32_t *>(static_cast<char *>(scratch) + cnt_b);
    uint32_t *err = reinterpret_cast<uint32_t *>(static_cast<char *>(scratch) + 2 * cnt_b);
    void *temp = static_cast<char *>(scratch) + 2 * cnt_b + tail;
    hipError_t e = decode_records_device(pl->ka.out_res, pl->ka.out_cmd, pl->ka.ovf, nov, pl->d_qi, nrec, nq, mc, idx_rank,
                                         pl->grid->V, cs.rgt, cs.soe, cs.shq, cs.sfm, cs.ff, cnt, off, temp, &temp_bytes,
                                         static_cast<mr_result *>(d_out), static_cast<mr_command *>(d_pool), pcap, err,
                                         pl->stream);
    uint32_t tailw[3] = {0, 0, 0};  // err, off and count of the last query: the commands written
    if (e == hipSuccess) e = hipMemcpyAsync(&tailw[0], err, 4, hipMemcpyDeviceToHost, pl->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&tailw[1], off + (nq - 1), 4, hipMemcpyDeviceToHost, pl->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&tailw[2], cnt + (nq - 1), 4, hipMemcpyDeviceToHost, pl->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(pl->stream);
    // every command fits the caller's pool (offsets are the prefix of the counts): results
    // and commands in one pipelined copy, else the results first, to find the cut
    const uint64_t total = uint64_t(tailw[1]) + tailw[2];
    const bool fits = !(tailw[0] & 1u) && total <= pool_cap && total <= pcap;
    if (e == hipSuccess) {
        const D2HSeg sg[2] = {{results, d_out, size_t(nq) * sizeof(mr_result)},
                              {pool, d_pool, fits ? size_t(total) * sizeof(mr_command) : 0}};
        e = copy_d2h(sg, 2, pl->stream);
    }
    // queries without a record (an invalid index), and the status to return: the first
    // error in query order, or MR_ERR_CAPACITY once a label's commands do not fit the
    // caller's pool (written up to the first such label), as the host decoder does; per
    // part of the queries on the host pool, combined in order
    uint64_t end = total;
    ret = MR_OK;
    if (e == hipSuccess && !(tailw[0] & 1u)) {
        HostPool &hpool = HostPool::get();
        const uint32_t parts = nq >= 65536u ? hpool.size() : 1u;
        std::vector<uint64_t> p_end(parts, total);
        std::vector<int32_t> p_ret(parts, MR_OK);
        hpool.run(parts, [&](uint32_t pt) {
            uint64_t en = total;
            int32_t rt = MR_OK;
            const uint32_t i0 = chunk_lo(nq, parts, pt);
            // (device-grouped plans: the invalid queries from their sorted list)
            auto inv = std::lower_bound(hp.invalid.begin(), hp.invalid.end(), i0);
            for (uint32_t i = i0, ie = chunk_lo(nq, parts, pt + 1); i < ie; ++i) {
                mr_result &r = results[i];
                int32_t qs = MR_OK;
                if (hp.dev_grouped) {
                    if (inv != hp.invalid.end() && *inv == i) {
                        qs = MR_ERR_INVALID_INDEX;
                        ++inv;
                    }
                } else {
                    qs = hp.q_status[i];
                }
                if (qs != MR_OK) {
                    std::memset(&r, 0, sizeof(r));
                    r.status = qs;
                }
                if (r.status == MR_OK && uint64_t(r.command_offset) + r.n_commands > pool_cap) {
                    en = std::min<uint64_t>(en, r.command_offset);
                    rt = MR_ERR_CAPACITY;  // (the host decoder's rule: a short pool wins over other errors)
                } else if (rt == MR_OK && r.status != MR_OK) {
                    rt = r.status;
                }
            }
            p_end[pt] = en;
            p_ret[pt] = rt;
        });
        for (uint32_t pt = 0; pt < parts; ++pt) {
            end = std::min(end, p_end[pt]);
            if (p_ret[pt] == MR_ERR_CAPACITY) ret = MR_ERR_CAPACITY;
            else if (ret == MR_OK) ret = p_ret[pt];
        }
    }
    const uint64_t ncopy = std::min<uint64_t>(end, pcap);
    if (e == hipSuccess && !fits && ncopy && !(tailw[0] & 1u)) {
        const D2HSeg sg{pool, d_pool, size_t(ncopy) * sizeof(mr_command)};
        e = copy_d2h(&sg, 1, pl->stream);
    }
    // the blocks go back to the cache, which hands them out with no implicit sync: on
    // every path (a failed enqueue included) the work queued on them must be done first
    (void)hipStreamSynchronize(pl->stream);
    pfree(scratch);
    pfree(d_out);
    pfree(d_pool);
    const double tm1 = timing_on() ? now_ms() : 0.0;
    if (e != hipSuccess) return (ret = fail(MR_ERR_DEVICE, std::string("device fetch: ") + hipGetErrorString(e))), true;
    if (tailw[0] & 1u) return (ret = fail(MR_ERR_DEVICE, "malformed record (overflow tag or cell rank)")), true;
    if (timing_on())
        std::fprintf(stderr, "MR_TIMING fetch n=%u (device decode): kernels + copies %.2f ms, host %.2f ms\n", nq,
                     tm1 - tm0, now_ms() - tm1);
    return true;
}

static bool plan_fetch_wire(mr_plan *pl, mr_result *results, mr_command *pool, uint64_t pool_cap, int &ret);

extern "C" int mr_plan_fetch(mr_plan *pl, mr_result *results, mr_command *pool, uint64_t pool_cap) {
    if (!pl || (pl->hp.nq && !results)) return fail(MR_ERR_INVALID_ARG, "null argument");
    {
        int ret = MR_OK;
        if (plan_fetch_wire(pl, results, pool, pool_cap, ret)) return ret;
        if (plan_fetch_device(pl, results, pool, pool_cap, ret)) return ret;
    }
    const double tm0 = timing_on() ? now_ms() : 0.0;
    if (int sh = host_arrays(pl)) return sh;
    std::vector<OutResult> res;
    std::vector<OutCmd> cmd, ovf;
    int st = plan_collect(pl, res, cmd, ovf);
    if (st != MR_OK) return st;
    const double tm1 = timing_on() ? now_ms() : 0.0;
    const HostPlan &hp = pl->hp;
    const CmdScale cs = cmd_scale(hp);
    const uint32_t mc = hp.p.max_cmds;
    uint64_t off = 0;
    int ret = MR_OK;
    // Large batches decode on host threads: each query's pool offset is the prefix sum
    // of the commands before it, so chunks write disjoint pool ranges; the first error
    // status in query order is the one returned, as in the serial loop below.
    const uint32_t nthr = std::min<uint32_t>(16, std::max(1u, std::thread::hardware_concurrency() / 2));
    if (hp.nq >= 65536 && nthr > 1 && pool) {
        std::vector<uint64_t> first(hp.nq + 1, 0);
        for (uint32_t i = 0; i < hp.nq; ++i)
            first[i + 1] = first[i] + (hp.q_status[i] == MR_OK ? record_cmds(res[hp.q_pos[i]]) : 0u);
        if (first[hp.nq] <= pool_cap) {
            std::vector<int> rets(nthr, MR_OK), errs(nthr, MR_OK);
            std::vector<std::string> msgs(nthr);
            std::vector<std::thread> th;
            const uint32_t chunk = (hp.nq + nthr - 1) / nthr;
            for (uint32_t t = 0; t < nthr; ++t)
                th.emplace_back([&, t]() {
                    const uint32_t a = t * chunk, b = std::min(hp.nq, a + chunk);
                    uint64_t o = first[std::min(a, hp.nq)];
                    for (uint32_t i = a; i < b; ++i) {
                        mr_result &r = results[i];
                        if (hp.q_status[i] != MR_OK) {
                            std::memset(&r, 0, sizeof(r));
                            r.status = hp.q_status[i];
                            if (rets[t] == MR_OK) rets[t] = hp.q_status[i];
                            continue;
                        }
                        const uint32_t k = hp.q_pos[i];
                        if (int e = decode_record(pl->grid, cs, res[k], mc ? &cmd[size_t(k) * mc] : nullptr, mc, ovf.data(),
                                                  ovf.size(), r, pool, pool_cap, o, rets[t])) {
                            errs[t] = e;
                            msgs[t] = g_last_error;  // (thread-local)
                            return;
                        }
                    }
                });
            for (auto &x : th) x.join();
            for (uint32_t t = 0; t < nthr; ++t)
                if (errs[t] != MR_OK) return fail(errs[t], msgs[t]);
            for (uint32_t t = 0; t < nthr && ret == MR_OK; ++t) ret = rets[t];
            if (timing_on())
                std::fprintf(stderr, "MR_TIMING fetch n=%u: collect %.2f ms, decode %.2f ms (%u threads)\n", hp.nq, tm1 - tm0,
                             now_ms() - tm1, nthr);
            return ret;
        }
    }
    for (uint32_t i = 0; i < hp.nq; ++i) {
        mr_result &r = results[i];
        if (hp.q_status[i] != MR_OK) {
            std::memset(&r, 0, sizeof(r));
            r.status = hp.q_status[i];
            if (ret == MR_OK) ret = hp.q_status[i];
            continue;
        }
        const uint32_t k = hp.q_pos[i];  // records are in grouped (by source) order
        if ((st = decode_record(pl->grid, cs, res[k], mc ? &cmd[size_t(k) * mc] : nullptr, mc, ovf.data(), ovf.size(), r,
                                pool, pool_cap, off, ret)))
            return st;
    }
    return ret;
}

extern "C" int mr_decode_records(const mr_grid *g, const mr_params *prm, const void *results, const void *commands,
                                 uint32_t n, uint32_t max_cmds, const void *overflow, uint64_t overflow_n,
                                 mr_result *out, mr_command *pool, uint64_t pool_cap) {
    if (!g || !prm || (n && (!results || !out || (max_cmds && !commands))) || (overflow_n && !overflow))
        return fail(MR_ERR_INVALID_ARG, "null argument");
    const CmdScale cs = cmd_scale(*prm);
    const OutResult *res = static_cast<const OutResult *>(results);
    const OutCmd *cmd = static_cast<const OutCmd *>(commands), *ovf = static_cast<const OutCmd *>(overflow);
    uint64_t off = 0;
    int ret = MR_OK;
    for (uint32_t k = 0; k < n; ++k)
        if (int st = decode_record(g, cs, res[k], cmd ? cmd + size_t(k) * max_cmds : nullptr, max_cmds, ovf, overflow_n,
                                   out[k], pool, pool_cap, off, ret))
            return st;
    return ret;
}

extern "C" uint32_t mr_wire_row_bytes(uint32_t max_cmds) { return 4u + 8u * max_cmds; }

extern "C" int mr_plan_wire_records(mr_plan *pl, void *d_rows, void *d_pool, uint32_t pool_cap, void *stream) {
    if (!pl || (pl->hp.nq && !d_rows) || (pool_cap && !d_pool)) return fail(MR_ERR_INVALID_ARG, "null argument");
    if (pl->all_mode) return fail(MR_ERR_INVALID_ARG, "wire_records: not a query plan");
    if (pl->grid->V > kWireRankMask + 1u) return fail(MR_ERR_INVALID_ARG, "wire_records: grid too large for wire records");
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : pl->stream;
    // ordered after the plan's last pass, whichever stream that ran on
    if (pl->ev_last && pl->last_stream != s && hipStreamWaitEvent(s, pl->ev_last, 0) != hipSuccess)
        return fail(MR_ERR_DEVICE, "wait for the last pass");
    const uint32_t nq = pl->hp.nq, nrec = pl->runs ? nrec_of(pl->hp) : 0u;
    if (launch_wire(pl->ka.out_res, pl->ka.out_cmd, pl->ka.ovf, pl->d_counter + kCtrLastOvf, pl->ka.ovf_cap, nrec, nq,
                    pl->hp.p.max_cmds, nullptr, static_cast<uint32_t *>(d_rows), static_cast<uint32_t *>(d_pool), pool_cap,
                    s) !=
        hipSuccess)
        return fail(MR_ERR_DEVICE, "wire kernel");
    // on a stream of its own (overlapping the next plan's pass), the encoding reads the
    // plan's outputs after the pass: the plan's next pass waits for it as for a pass
    if (pl->ev_last && pl->last_stream != s) {
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, s) != hipSuccess) {
            if (ev) (void)hipEventDestroy(ev);
            (void)hipStreamSynchronize(s);  // (ordered the slow way)
            return MR_OK;
        }
        if (pl->ev_last_orphan) (void)hipEventDestroy(pl->ev_last);
        pl->ev_last = ev;
        pl->ev_last_orphan = true;
        pl->last_stream = s;
    }
    return MR_OK;
}

// Metrics of a label from its commands (the reference's TotalCost sums, src/cost.rs:299-313;
// a StandardMove run's time is its Fleetfoot ceil, src/skill.rs:21-30).
static void wire_metrics(const CmdScale &cs, const uint32_t *cmd, uint32_t n, mr_result &r) {
    static const uint32_t ffn[4] = {1, 50, 100, 25}, ffd[4] = {1, 53, 109, 28};
    const uint32_t ff = cs.ff <= 3 ? cs.ff : 0;
    uint64_t legs = 0, money = 0, t = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t kind = cmd[2 * j] >> 29, pay = cmd[2 * j] & 0x1FFFFFFFu;
        switch (kind) {
            case kCentral: t += uint64_t(10) * pay; break;
            case kStandard:
                legs += pay;
                t += (uint64_t(180) * pay * ffn[ff] + ffd[ff] - 1) / ffd[ff];
                break;
            case kCaravan:
                t += uint64_t(cs.rgt) * (pay >> 1);
                money += uint64_t(pay >> 1) * ((pay & 1u) ? 5u : 2u);
                break;
            case kSoE: money += cs.soe; break;
            case kSHQ: money += cs.shq; break;
            case kSFm: money += cs.sfm; break;
            default: break;
        }
    }
    r.legs = uint32_t(legs);
    r.money = uint32_t(money);
    r.time_s = int64_t(t);
}

// Decodes wire row `row` (max_cmds mc, the pool wp of pool_n commands) into r, its commands
// into cmds[off..] when they fit cmd_cap (else *ret = MR_ERR_CAPACITY).  MR_OK, or
// MR_ERR_DEVICE for a row that is not well formed.
static int decode_wire_row(const mr_grid *g, const CmdScale &cs, const uint32_t *row, uint32_t mc, const uint32_t *wp,
                           uint64_t pool_n, mr_result &r, mr_command *cmds, uint64_t cmd_cap, uint64_t &off, int &ret) {
    std::memset(&r, 0, sizeof(r));
    r.command_offset = uint32_t(off);
    const uint32_t code = row[0] >> kWireRankBits;
    uint32_t from = row[0] & kWireRankMask, nc = 0;
    const uint32_t *src = row + 1;
    if (code >= kWireStatus) {
        r.status = int32_t(code) - int32_t(kWireStatus) - 32;
        if (r.status != MR_NOT_FOUND && ret == MR_OK) ret = r.status;
        return MR_OK;
    }
    if (code == kWireOvf) {
        if (!mc || uint64_t(row[1]) + row[2] > pool_n) return fail(MR_ERR_DEVICE, "wire pool record");
        src = wp + 2ull * row[1];
        nc = row[2];
    } else {
        if (code > mc) return fail(MR_ERR_DEVICE, "wire record longer than its command slots");
        nc = code;
    }
    r.status = MR_OK;
    r.n_commands = nc;
    wire_metrics(cs, src, nc, r);
    if (cmds && off + nc <= cmd_cap) {
        for (uint32_t j = 0; j < nc; ++j) {
            const OutCmd c{src[2 * j], from, src[2 * j + 1], 0u};
            if (!expand_cmd(g, cs, c, cmds[off + j])) return fail(MR_ERR_DEVICE, "command names no cell");
            from = c.to;
        }
    } else {
        ret = MR_ERR_CAPACITY;
    }
    off += nc;
    return MR_OK;
}

extern "C" int mr_decode_wire(const mr_grid *g, const mr_params *prm, const void *rows, uint32_t n, uint32_t max_cmds,
                              const void *pool, uint64_t pool_n, mr_result *out, mr_command *cmds, uint64_t cmd_cap) {
    if (!g || !prm || (n && (!rows || !out)) || (pool_n && !pool)) return fail(MR_ERR_INVALID_ARG, "null argument");
    const CmdScale cs = cmd_scale(*prm);
    const uint32_t rw = 1u + 2u * max_cmds;
    const uint32_t *w = static_cast<const uint32_t *>(rows), *wp = static_cast<const uint32_t *>(pool);
    uint64_t off = 0;
    int ret = MR_OK;
    for (uint32_t k = 0; k < n; ++k)
        if (int st = decode_wire_row(g, cs, w + size_t(k) * rw, max_cmds, wp, pool_n, out[k], cmds, cmd_cap, off, ret))
            return st;
    return ret;
}

// the grid's CellIndex-by-rank table on the host (one lookup a command instead of two)
static const mr_cell_index *idx_of_rank(const mr_grid *g) {
    std::lock_guard<std::mutex> lk(g->near_mu);
    if (g->idx_rank_h.size() != g->V) {
        std::vector<mr_cell_index> t(g->V);
        for (uint32_t r = 0; r < g->V; ++r) t[r] = g->idx[g->rank_inv[r]];
        g->idx_rank_h.swap(t);
    }
    return g->idx_rank_h.data();
}

static inline uint64_t cell_bits(const mr_cell_index &c) {
    uint64_t b;
    std::memcpy(&b, &c, 8);
    return b;
}
static inline void nt_store(void *dst, const uint64_t *q, int n) {
    uint64_t *d = static_cast<uint64_t *>(dst);
    for (int i = 0; i < n; ++i) __builtin_nontemporal_store(q[i], d + i);
}

// decode_wire_row for the fetch: the same outputs, written with streaming stores (the
// caller's arrays are written once and not read back here: no read-for-ownership of
// their lines), cells from the rank table, a command's `from` as the previous `to`.
// Returns MR_OK or MR_ERR_DEVICE (a row that is not well formed; *bad names it).
static int fetch_wire_row(const uint32_t *row, uint32_t mc, const uint32_t *wp, uint64_t pool_n, const mr_cell_index *cell,
                          uint32_t V, const CmdScale &cs, const uint32_t ffn, const uint32_t ffd, mr_result &r,
                          mr_command *cmds, uint64_t cmd_cap, uint64_t &off, int &ret, const char *&bad) {
    const uint32_t code = row[0] >> kWireRankBits;
    uint32_t from = row[0] & kWireRankMask, nc = 0;
    const uint32_t *src = row + 1;
    uint64_t q[5];
    if (code >= kWireStatus) {
        const int32_t st = int32_t(code) - int32_t(kWireStatus) - 32;
        if (st != MR_NOT_FOUND && ret == MR_OK) ret = st;
        q[0] = q[1] = 0;
        q[2] = uint64_t(uint32_t(off)) << 32;
        q[3] = uint64_t(uint32_t(st));
        nt_store(&r, q, 4);
        return MR_OK;
    }
    if (code == kWireOvf) {
        if (!mc || uint64_t(row[1]) + row[2] > pool_n) return (bad = "wire pool record"), MR_ERR_DEVICE;
        src = wp + 2ull * row[1];
        nc = row[2];
    } else {
        if (code > mc) return (bad = "wire record longer than its command slots"), MR_ERR_DEVICE;
        nc = code;
    }
    const bool put = cmds && off + nc <= cmd_cap;
    if (!put) ret = MR_ERR_CAPACITY;
    uint64_t legs = 0, money = 0, t = 0;
    if (nc && from >= V) return (bad = "command names no cell"), MR_ERR_DEVICE;
    uint64_t fbits = nc ? cell_bits(cell[from]) : 0;
    for (uint32_t j = 0; j < nc; ++j) {
        const uint32_t kp = src[2 * j], to = src[2 * j + 1], kind = kp >> 29, pay = kp & 0x1FFFFFFFu;
        if (kind > kSFm || to >= V) return (bad = "command names no cell"), MR_ERR_DEVICE;
        uint32_t cl = 0, cm = 0, cf = 0;
        uint64_t ct = 0;
        switch (kind) {
            case kCentral: ct = uint64_t(10) * pay; break;
            case kStandard:
                cl = pay;
                ct = uint64_t(180) * pay;
                cf = cs.ff;
                t += (ct * ffn + ffd - 1) / ffd;
                ct = uint64_t(180) * pay;
                break;
            case kCaravan:
                ct = uint64_t(cs.rgt) * (pay >> 1);
                cm = (pay >> 1) * ((pay & 1u) ? 5u : 2u);
                break;
            case kSoE: cm = cs.soe; break;
            case kSHQ: cm = cs.shq; break;
            case kSFm: cm = cs.sfm; break;
            default: break;
        }
        legs += cl;
        money += cm;
        if (kind != kStandard) t += ct;
        const uint64_t tbits = cell_bits(cell[to]);
        if (put) {
            q[0] = uint64_t(kind) | uint64_t(cl) << 32;
            q[1] = uint64_t(cm) | uint64_t(cf) << 32;
            q[2] = ct;
            q[3] = fbits;
            q[4] = tbits;
            nt_store(&cmds[off + j], q, 5);
        }
        fbits = tbits;
    }
    q[0] = uint64_t(uint32_t(legs)) | uint64_t(uint32_t(money)) << 32;
    q[1] = t;
    q[2] = uint64_t(nc) | uint64_t(uint32_t(off)) << 32;
    q[3] = uint64_t(uint32_t(MR_OK));
    nt_store(&r, q, 4);
    off += nc;
    return MR_OK;
}

// mr_plan_fetch through wire rows: the pass re-encoded on the device in query order
// (wire_kernel, 4 + 8 max_cmds bytes a query instead of the 32 B result and 32 B per
// command the device decoder writes), copied in chunks into the pinned stage, and decoded
// on the host pool while the next chunk is in flight; a chunk's command offsets continue
// the previous chunk's.  Same outputs and status rules as plan_fetch_device.  Returns
// false (nothing written) when it does not apply.
static bool plan_fetch_wire(mr_plan *pl, mr_result *results, mr_command *pool, uint64_t pool_cap, int &ret) {
    const HostPlan &hp = pl->hp;
    const uint32_t nq = hp.nq, nrec = nrec_of(hp), mc = hp.p.max_cmds, rw = 2u + 2u * mc;  // (+ the offset word)
    // Opt-in (MR_FETCH_WIRE=1).  In a quiet process it fetches 1M labels in 1.7-1.9 ms
    // against 3.5-5 ms for the device decoder; in bench.py's process (torch loaded, the CPU
    // baseline's threads just run) its host writes took 5.8-6.1 ms, so the device decoder
    // (plan_fetch_device: no host threads, direct DMA into page-locked arrays) stays the
    // default
    const char *fw = std::getenv("MR_FETCH_WIRE");
    if (!(fw && !std::strcmp(fw, "1")) || !pool || !nq || pl->all_mode || pl->grid->V > kWireRankMask + 1u || !pl->d_qi)
        return false;
    if (const char *e = std::getenv("MR_HOST_DECODE"))
        if (!std::strcmp(e, "1")) return false;
    const double tm0 = timing_on() ? now_ms() : 0.0;
    uint32_t flags = 0, ctr[kCtrWords];
    if ((ret = check_device_errors(pl, flags, ctr)) != MR_OK) return true;  // (syncs the plan)
    const uint32_t nov = std::min(ctr[kCtrLastOvf], pl->ka.ovf_cap);
    const size_t rows_b = size_t(nq) * rw * 4, pool_b = size_t(nov) * 8, cnt_b = (size_t(nq) * 4 + 255) / 256 * 256;
    size_t temp_b = 0;
    (void)wire_fetch_device(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, nq, mc, nullptr, nullptr, nullptr, &temp_b,
                            nullptr, nullptr, 0, pl->stream);
    const size_t rows_at = 2 * cnt_b + (temp_b + 255) / 256 * 256;
    void *d_wire = nullptr;
    if (pmalloc(&d_wire, rows_at + rows_b + pool_b + 8) != hipSuccess) return false;
    char *dw = static_cast<char *>(d_wire);
    uint32_t *d_cnt = reinterpret_cast<uint32_t *>(dw), *d_off = reinterpret_cast<uint32_t *>(dw + cnt_b);
    uint32_t *d_rows = reinterpret_cast<uint32_t *>(dw + rows_at), *d_pool = d_rows + size_t(nq) * rw;
    PinnedStage &stg = stage_down();
    std::lock_guard<std::mutex> lk(stg.mu);
    char *h = static_cast<char *>(stg.get(rows_b + pool_b + 8));
    if (!h) {
        pfree(d_wire);
        return false;
    }
    const uint32_t *h_rows = reinterpret_cast<const uint32_t *>(h), *h_pool = h_rows + size_t(nq) * rw;
    // chunks of rows copied one after the other, the pool first (the rows of any chunk may
    // point into it); each host part decodes its share of a chunk once that has landed
    // (one chunk: the caller waits for the copies, then the pool decodes; the pool's threads
    // waiting on per-chunk events spun through the process's CPU share on busy hosts)
    const uint32_t nch = 1u;
    std::vector<hipEvent_t> ev(nch, nullptr);
    hipError_t e = wire_fetch_device(pl->ka.out_res, pl->ka.out_cmd, pl->ka.ovf, pl->d_counter + kCtrLastOvf, pl->ka.ovf_cap,
                                     pl->d_qi, nrec, nq, mc, d_cnt, d_off, dw + 2 * cnt_b, &temp_b, d_rows, d_pool, nov,
                                     pl->stream);
    if (e == hipSuccess && pool_b) e = hipMemcpyAsync(h + rows_b, d_pool, pool_b, hipMemcpyDeviceToHost, pl->stream);
    for (uint32_t c = 0; c < nch && e == hipSuccess; ++c) {
        const size_t lo = size_t(chunk_lo(nq, nch, c)) * rw * 4, hi = size_t(chunk_lo(nq, nch, c + 1)) * rw * 4;
        e = hipMemcpyAsync(h + lo, reinterpret_cast<char *>(d_rows) + lo, hi - lo, hipMemcpyDeviceToHost, pl->stream);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[c], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ev[c], pl->stream);
    }
    const double tm1 = timing_on() ? now_ms() : 0.0;
    HostPool &hpool = HostPool::get();
    const CmdScale cs = cmd_scale(hp);
    static const uint32_t ffn_t[4] = {1, 50, 100, 25}, ffd_t[4] = {1, 53, 109, 28};
    const uint32_t ffn = ffn_t[cs.ff <= 3 ? cs.ff : 0], ffd = ffd_t[cs.ff <= 3 ? cs.ff : 0];
    const mr_cell_index *cell = idx_of_rank(pl->grid);
    const uint32_t V = pl->grid->V;
    const uint32_t parts = nq >= 65536u ? hpool.size() : 1u;
    if (e == hipSuccess) e = hipEventSynchronize(ev[nch - 1]);
    // per (chunk, part): the first error status in its queries, or MR_ERR_CAPACITY
    std::vector<int32_t> p_ret(size_t(nch) * parts, MR_OK), p_err(parts, MR_OK);
    std::vector<const char *> p_msg(parts, nullptr);
    std::vector<hipError_t> p_e(parts, hipSuccess);
    if (e == hipSuccess)
        hpool.run(parts, [&](uint32_t pt) {
            for (uint32_t c = 0; c < nch; ++c) {
                if (hipError_t x = hipEventSynchronize(ev[c])) {
                    p_e[pt] = x;
                    break;
                }
                const uint32_t q0 = chunk_lo(nq, nch, c), nc = chunk_lo(nq, nch, c + 1) - q0;
                const uint32_t i0 = q0 + chunk_lo(nc, parts, pt), i1 = q0 + chunk_lo(nc, parts, pt + 1);
                // (device-grouped plans: the invalid queries from their sorted list)
                auto inv = std::lower_bound(hp.invalid.begin(), hp.invalid.end(), i0);
                int32_t rt = MR_OK;
                for (uint32_t i = i0; i < i1; ++i) {
                    mr_result &r = results[i];
                    int32_t qs = MR_OK;
                    if (hp.dev_grouped) {
                        if (inv != hp.invalid.end() && *inv == i) {
                            qs = MR_ERR_INVALID_INDEX;
                            ++inv;
                        }
                    } else {
                        qs = hp.q_status[i];
                    }
                    if (qs != MR_OK) {
                        const uint64_t z[4] = {0, 0, 0, uint64_t(uint32_t(qs))};
                        nt_store(&r, z, 4);
                        if (rt == MR_OK) rt = qs;
                        continue;
                    }
                    const uint32_t *row = h_rows + size_t(i) * rw;
                    uint64_t o = row[rw - 1];
                    int rr = MR_OK;
                    const char *bad = nullptr;
                    if (int st = fetch_wire_row(row, mc, h_pool, nov, cell, V, cs, ffn, ffd, r, pool, pool_cap, o, rr, bad)) {
                        p_err[pt] = st;
                        p_msg[pt] = bad;
                        __builtin_ia32_sfence();
                        return;
                    }
                    if (rr == MR_ERR_CAPACITY) rt = MR_ERR_CAPACITY;  // (a short pool wins over other errors)
                    else if (rt == MR_OK && rr != MR_OK) rt = rr;
                }
                p_ret[size_t(c) * parts + pt] = rt;
            }
            __builtin_ia32_sfence();  // (the streaming stores drain before the pool's completion count)
        });
    ret = MR_OK;
    int32_t err = MR_OK;
    const char *msg = nullptr;
    for (uint32_t pt = 0; pt < parts; ++pt) {
        if (e == hipSuccess && p_e[pt] != hipSuccess) e = p_e[pt];
        if (err == MR_OK && p_err[pt] != MR_OK) {
            err = p_err[pt];
            msg = p_msg[pt];
        }
    }
    for (int32_t x : p_ret) {  // (chunk-major, part-minor: query order)
        if (x == MR_ERR_CAPACITY) ret = MR_ERR_CAPACITY;
        else if (ret == MR_OK) ret = x;
    }
    // the device block goes back to the cache, which hands it out with no implicit sync
    (void)hipStreamSynchronize(pl->stream);
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    pfree(d_wire);
    if (e != hipSuccess) return (ret = fail(MR_ERR_DEVICE, std::string("wire fetch: ") + hipGetErrorString(e))), true;
    if (err != MR_OK) return (ret = fail(err, msg ? msg : "wire row")), true;
    if (timing_on())
        std::fprintf(stderr, "MR_TIMING fetch n=%u (wire, %u chunks, %u parts): enqueue %.2f ms, copies + host decode %.2f ms\n",
                     nq, nch, parts, tm1 - tm0, now_ms() - tm1);
    return true;
}

extern "C" void mr_plan_destroy(mr_plan *pl) {
#ifdef MR_STAMPS
    if (pl && pl->d_dbg) {  // diagnostic summary: phase cycles summed over workgroups (last launch)
        std::vector<unsigned long long> d(size_t(pl->blocks) * 10 + 16);
        if (hipMemcpy(d.data(), pl->d_dbg, d.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            unsigned long long acc[9] = {0};
            for (uint32_t b = 0; b < pl->blocks; ++b)
                for (int i = 0; i < 9; ++i) acc[i] += d[size_t(b) * 10 + i];
            std::fprintf(stderr,
                         "MR_STAMPS blocks=%u sources=%llu cycles: init=%llu fire=%llu specials=%llu next=%llu "
                         "bar1=%llu claim=%llu bar2=%llu frontier_vertices=%llu\n",
                         pl->blocks, acc[8], acc[0], acc[1], acc[2], acc[3], acc[4], acc[5], acc[6], acc[7]);
            const unsigned long long *h = &d[size_t(pl->blocks) * 10];
            if (pl->hp.hub)
                std::fprintf(stderr,
                             "MR_STAMPS hub (sum over waves): sources=%llu iterations=%llu boundaries=%llu cycles: "
                             "init=%llu select=%llu edges=%llu boundary=%llu emit=%llu dequeue=%llu\n",
                             h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]);
            if (h[9])
                std::fprintf(stderr,
                             "MR_STAMPS lane/group (per wave, %llu waves, last pass): setup=%.0f own_edges=%.0f scan_min=%.0f "
                             "settle=%.0f relax=%.0f cmds_cert=%.0f destinations=%.0f\n",
                             h[9], double(h[10]) / h[9], double(h[11]) / h[9], double(h[12]) / h[9], double(h[13]) / h[9],
                             double(h[14]) / h[9], double(h[7]) / h[9], double(h[15]) / h[9]);
        }
    }
#endif
    // passes may still be in flight on the caller's stream and the plan's hub stream
    if (pl) (void)plan_sync(pl);
    delete pl;
}

extern "C" int mr_find_path_batch(const mr_grid *g, const mr_params *prm, const mr_query *qs, uint32_t n,
                                  mr_result *results, mr_command *pool, uint64_t pool_cap) {
    if (!g || !prm || (n && (!qs || !results))) return fail(MR_ERR_INVALID_ARG, "null argument");
    uint32_t max_cmds = 16;
    for (int attempt = 0; attempt < 4; ++attempt) {
        mr_plan *pl = nullptr;
        int st = plan_create(g, prm, qs, n, max_cmds, &pl);
        if (st != MR_OK) return st;
        st = mr_plan_run(pl, nullptr);
        if (st != MR_OK) {
            mr_plan_destroy(pl);
            return st;
        }
        st = mr_plan_fetch(pl, results, pool, pool_cap);
        mr_plan_destroy(pl);
        // a label longer than the device command slots: re-run with more slots
        uint32_t need = 0;
        for (uint32_t i = 0; i < n; ++i)
            if (results[i].status == MR_ERR_CAPACITY) need = std::max(need, results[i].n_commands);
        if (need == 0) return st;
        max_cmds = std::max(need, max_cmds * 4);
    }
    return fail(MR_ERR_LIMIT, "label length");
}

extern "C" int mr_find_path(const mr_grid *g, const mr_params *prm, mr_cell_index from, mr_cell_index to,
                            mr_result *out, mr_command *cmds, uint32_t cap) {
    if (!out) return fail(MR_ERR_INVALID_ARG, "null result");
    mr_query q;
    q.from = from;
    q.to = to;
    std::vector<mr_command> pool(std::max<uint32_t>(cap, 64));
    int st = mr_find_path_batch(g, prm, &q, 1, out, pool.data(), pool.size());
    if (st < 0 && st != MR_ERR_CAPACITY) return st;
    if (out->status != MR_OK) return out->status;
    out->command_offset = 0;
    if (out->n_commands > cap) {
        out->status = MR_ERR_CAPACITY;
        return MR_ERR_CAPACITY;
    }
    if (cmds) std::memcpy(cmds, pool.data(), out->n_commands * sizeof(mr_command));
    return MR_OK;
}

// ------------------------------------------------------------ all destinations
extern "C" int mr_sssp_plan_create(const mr_grid *g, const mr_params *prm, const mr_cell_index *sources, uint32_t n,
                                   mr_plan **out) {
    if (!g || !prm || !out || (n && !sources)) return fail(MR_ERR_INVALID_ARG, "null argument");
    std::vector<mr_query> qs(n);
    for (uint32_t i = 0; i < n; ++i) qs[i].from = qs[i].to = sources[i];
    const int st = plan_create(g, prm, qs.data(), n, 16, out, true);
    if (st == MR_OK) {
        for (uint32_t i = 0; i < n; ++i)
            if ((*out)->hp.q_status[i] != MR_OK) {
                mr_plan_destroy(*out);
                *out = nullptr;
                return fail(MR_ERR_INVALID_INDEX, "source " + std::to_string(i) + " is not a grid cell");
            }
    }
    return st;
}

static int sssp_source(mr_plan *pl, uint32_t i, uint32_t &si) {
    if (!pl || !pl->all_mode) return fail(MR_ERR_INVALID_ARG, "not an all-destinations plan");
    if (i >= pl->src_of_input.size() || pl->src_of_input[i] == kNone32) return fail(MR_ERR_INVALID_ARG, "source index");
    si = pl->src_of_input[i];
    uint32_t flags = 0;
    return check_device_errors(pl, flags);
}

// The source's label table (NS + 1 entries) as the last pass exported it.
static int sssp_table(mr_plan *pl, uint32_t si, std::vector<Rec> &tab) {
    const uint32_t T = pl->ka.p.NS + 1;
    tab.resize(T);
    if (hipMemcpy(tab.data(), pl->d_tab + size_t(si) * T, T * sizeof(Rec), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "copy label table");
    return MR_OK;
}

// A cell word (CellWord, mr_engine.hpp) over its source's table: the label's metrics
// (the table label's plus the final walk's) and `via`.  False if it names no entry.
static bool expand_word(const HostPlan &hp, const std::vector<Rec> &tab, CellWord w, mr_label_record &o) {
    const uint32_t T = uint32_t(tab.size());
    if (w == kViaSource) {
        o = mr_label_record{0, 0, 0, kViaSource};
        return true;
    }
    if (w & kViaSpecial) {
        const uint32_t t = w & kNone10;
        if (t >= T || (w & ~(kViaSpecial | kNone10))) return false;
        o = mr_label_record{tab[t].m[0], tab[t].m[1], tab[t].m[2], w};
        return true;
    }
    const uint32_t b = w >> kStBShift, k = w & kStKMask;
    if (b >= T) return false;
    // AggregatedCost::time of the walk's run (src/cost.rs:122-124): Fleetfoot's ceil
    const uint64_t t = (uint64_t(180) * k * hp.p.ff_num + hp.p.ff_den - 1) / hp.p.ff_den;
    o = mr_label_record{tab[b].m[0] + k, tab[b].m[1], uint32_t(tab[b].m[2] + t), b};
    return true;
}

// A source's cell words in row-major order (S x S, the device rows' padding dropped):
// one contiguous copy of its padded rows, compacted on the host.  (A pitched
// hipMemcpy2D into pageable memory here twice ended in an illegal memory access on the
// GPU box, intermittently, with every kernel of the plan long finished.)
static int copy_source_words(mr_plan *pl, uint32_t si, std::vector<CellWord> &words) {
    const uint32_t S = pl->ka.p.S, pitch = pl->ka.rec_pitch;
    std::vector<CellWord> rows(size_t(S) * pitch);
    if (hipError_t e = hipMemcpy(rows.data(), pl->d_rec + size_t(si) * S * pitch, rows.size() * sizeof(CellWord),
                                 hipMemcpyDeviceToHost))
        return fail(MR_ERR_DEVICE, std::string("copy records: ") + hipGetErrorString(e));
    words.resize(size_t(S) * S);
    for (uint32_t y = 0; y < S; ++y)
        std::memcpy(&words[size_t(y) * S], &rows[size_t(y) * pitch], S * sizeof(CellWord));
    return MR_OK;
}

extern "C" int mr_sssp_records(mr_plan *pl, uint32_t i, mr_label_record *out) {
    uint32_t si = 0;
    if (int st = sssp_source(pl, i, si)) return st;
    if (!out) return fail(MR_ERR_INVALID_ARG, "null output");
    const uint32_t V = pl->ka.p.V;
    std::vector<CellWord> words(V);
    std::vector<Rec> tab;
    if (int st = copy_source_words(pl, si, words)) return st;
    if (int st = sssp_table(pl, si, tab)) return st;
    for (uint32_t v = 0; v < V; ++v)
        if (!expand_word(pl->hp, tab, words[v], out[v])) return fail(MR_ERR_DEVICE, "cell word names no table entry");
    return MR_OK;
}

extern "C" int mr_sssp_device_records(mr_plan *pl, void **d_records, uint64_t *bytes) {
    if (!pl || !pl->all_mode) return fail(MR_ERR_INVALID_ARG, "not an all-destinations plan");
    if (!plan_sync(pl)) return fail(MR_ERR_DEVICE, "sync");  // whole records behind the pointer
    if (d_records) *d_records = pl->d_rec;
    if (bytes) *bytes = uint64_t(pl->ka.nsrc) * pl->ka.p.S * pl->ka.rec_pitch * sizeof(CellWord);
    return MR_OK;
}

extern "C" int mr_sssp_record_pitch(mr_plan *pl, uint32_t *cells_per_row) {
    if (!pl || !pl->all_mode) return fail(MR_ERR_INVALID_ARG, "not an all-destinations plan");
    if (!cells_per_row) return fail(MR_ERR_INVALID_ARG, "null output");
    *cells_per_row = pl->ka.rec_pitch;
    return MR_OK;
}

extern "C" int mr_sssp_device_tables(mr_plan *pl, void **d_tables, uint64_t *bytes) {
    if (!pl || !pl->all_mode) return fail(MR_ERR_INVALID_ARG, "not an all-destinations plan");
    if (!plan_sync(pl)) return fail(MR_ERR_DEVICE, "sync");  // the latest pass's slot, finished
    if (d_tables) *d_tables = pl->d_tab;
    if (bytes) *bytes = uint64_t(pl->ka.nsrc) * (pl->ka.p.NS + 1) * sizeof(Rec);
    return MR_OK;
}

// The full label of destination dst from source i: the record's boundary chain in
// the source's label table, plus the final walk (its length is the boundary's
// grid distance to dst).
// The label of cell w from plan source si, given its cell word and the source's
// table: metrics into rec, compact commands into seq.  MR_OK or MR_ERR_DEVICE for a
// word that names no entry or whose walk is not the boundary's distance.
static int sssp_expand(const mr_plan *pl, uint32_t si, const std::vector<Rec> &tab, uint32_t w, CellWord word,
                       mr_label_record &rec, std::vector<OutCmd> &seq) {
    const mr_grid *g = pl->grid;
    const uint32_t T = pl->ka.p.NS + 1;
    seq.clear();
    if (!expand_word(pl->hp, tab, word, rec)) return fail(MR_ERR_DEVICE, "cell word names no table entry");
    const uint32_t src = pl->hp.src_v[si];
    // rank of table entry e's cell (entry 0: the source)
    auto rk = [&](uint32_t e) { return g->rank[e == 0 ? src : pl->hp.sp[e].v]; };
    auto chain = [&](uint32_t t) {  // commands of table label t (parent 0 ends the chain)
        uint32_t path[kMaxSpecials + 2];
        uint32_t np = 0;
        for (uint32_t e = t, guard = 0; e != 0 && guard <= T && np < kMaxSpecials + 2; e = tab[e].parent(), ++guard)
            path[np++] = e;
        for (uint32_t j = np; j-- > 0;) {
            const Rec &r = tab[path[j]];  // tails as Rec (mr_engine.hpp) derives them
            seq.push_back(OutCmd{r.kp0, r.from0, r.u, 0});
            if (r.ntail() == 2) seq.push_back(OutCmd{kSoE << 29, r.u, rk(path[j]), 0});
        }
    };
    if (rec.via == kViaSource) {
        seq.push_back(OutCmd{kNoMove << 29, g->rank[src], g->rank[src], 0});
    } else if (rec.via & kViaSpecial) {
        const uint32_t t = rec.via & kNone10;
        if (t >= T) return fail(MR_ERR_DEVICE, "record names no table entry");
        chain(t);
    } else {
        const uint32_t b = rec.via;
        if (b >= T) return fail(MR_ERR_DEVICE, "record names no boundary");
        const uint32_t vb = b == 0 ? src : pl->hp.sp[b].v;
        chain(b);
        int32_t ax = g->gx(vb), ay = g->gy(vb), bx = g->gx(w), by = g->gy(w);
        uint32_t k = uint32_t(std::abs(ax - bx) + std::abs(ay - by));
        if ((ay == 0 && by == 0 && ax != 0 && bx != 0 && ((ax < 0) != (bx < 0))) ||
            (ax == 0 && bx == 0 && ay != 0 && by != 0 && ((ay < 0) != (by < 0))))
            k += 2;  // the walk goes round the Center
        if (k != (word & kStKMask)) return fail(MR_ERR_DEVICE, "cell word's walk is not the boundary's distance");
        seq.push_back(OutCmd{(kStandard << 29) | k, g->rank[vb], g->rank[w], 0});
    }
    return MR_OK;
}

extern "C" int mr_sssp_label(mr_plan *pl, uint32_t i, mr_cell_index dst, mr_result *res, mr_command *cmds, uint32_t cap) {
    uint32_t si = 0;
    if (int st = sssp_source(pl, i, si)) return st;
    if (!res) return fail(MR_ERR_INVALID_ARG, "null result");
    const mr_grid *g = pl->grid;
    uint32_t w;
    if (!g->find(dst, w)) return fail(MR_ERR_INVALID_INDEX, "destination is not a grid cell");
    CellWord word;
    std::vector<Rec> tab;
    const size_t at = (size_t(si) * g->S + w / g->S) * pl->ka.rec_pitch + w % g->S;  // padded rows
    if (hipMemcpy(&word, pl->d_rec + at, sizeof(word), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MR_ERR_DEVICE, "copy label");
    if (int st = sssp_table(pl, si, tab)) return st;
    mr_label_record rec;
    std::vector<OutCmd> seq;
    if (int st = sssp_expand(pl, si, tab, w, word, rec, seq)) return st;
    std::memset(res, 0, sizeof(*res));
    res->legs = rec.legs;
    res->money = rec.money;
    res->time_s = int64_t(rec.time_s);
    res->n_commands = uint32_t(seq.size());
    if (seq.size() > cap || (!cmds && !seq.empty())) {
        res->status = MR_ERR_CAPACITY;
        return MR_ERR_CAPACITY;
    }
    const CmdScale cs = cmd_scale(pl->hp);
    for (size_t j = 0; j < seq.size(); ++j)
        if (!expand_cmd(g, cs, seq[j], cmds[j])) return fail(MR_ERR_DEVICE, "command names no cell");
    return MR_OK;
}

extern "C" int mr_sssp_labels(mr_plan *pl, uint32_t i, mr_result *results, mr_command *pool, uint64_t pool_cap) {
    uint32_t si = 0;
    if (int st = sssp_source(pl, i, si)) return st;
    if (!results) return fail(MR_ERR_INVALID_ARG, "null results");
    const mr_grid *g = pl->grid;
    const uint32_t V = pl->ka.p.V;
    std::vector<CellWord> words(V);
    std::vector<Rec> tab;
    if (int st = copy_source_words(pl, si, words)) return st;
    if (int st = sssp_table(pl, si, tab)) return st;
    const CmdScale cs = cmd_scale(pl->hp);
    std::vector<OutCmd> seq;
    uint64_t off = 0;
    int ret = MR_OK;
    for (uint32_t w = 0; w < V; ++w) {
        mr_label_record rec;
        if (int st = sssp_expand(pl, si, tab, w, words[w], rec, seq)) return st;
        mr_result &r = results[w];
        std::memset(&r, 0, sizeof(r));
        r.legs = rec.legs;
        r.money = rec.money;
        r.time_s = int64_t(rec.time_s);
        r.n_commands = uint32_t(seq.size());
        r.command_offset = uint32_t(std::min<uint64_t>(off, 0xFFFFFFFFu));
        r.status = MR_OK;
        if (pool && off + seq.size() <= pool_cap && off + seq.size() <= 0xFFFFFFFFull) {
            for (size_t j = 0; j < seq.size(); ++j)
                if (!expand_cmd(g, cs, seq[j], pool[off + j])) return fail(MR_ERR_DEVICE, "command names no cell");
        } else {
            ret = MR_ERR_CAPACITY;
        }
        off += seq.size();
    }
    return ret;
}
