// mr_device.hpp — gfx950 device code of the pathfinder hot path (included by the
// mr_k_*.hip translation units, one per kernel family, so they compile in parallel).
//
// Replaces the body of FindPath::eval (src/pathfinder.rs:199-248): the binary
// heap frontier (src/binary_heap.rs) becomes bucketed parallel settling, the
// per-pop edge generator (Inflight::edges, src/pathfinder.rs:24-180) becomes
// implicit grid neighbours + a small table of teleport edges, and the ~240 B
// cloned labels (src/cost.rs:187-315) become one 32-bit word per grid vertex.
// See mr_engine.hpp for the layout and DESIGN.md §3 for the exactness argument.
//
// One 256-thread workgroup solves one source at a time (sources are dequeued
// from a global counter; no grid-wide barrier, no co-residency assumption).
// Two solvers share the special-table machinery (Core):
//
//  * LegsSolver   (comparator leads with Legs — the app's default): level-
//    synchronous.  At legs level L every candidate label of a plain vertex is
//    walk(b, L - legs(b)), so candidates order by the boundary b alone: wave 0
//    ranks the boundaries once per level (prio[]), and a plain vertex's label
//    is FINAL the moment it is claimed.  Two barriers per level:
//      [specials] wave 0: Scroll-of-Escape region argmins fire, an exact
//                 Dijkstra settles the specials of level L, boundaries are
//                 ranked for level L+1;
//      [claim]    every frontier vertex of level L claims the unsettled
//                 neighbours it owns (lowest-direction frontier neighbour owns;
//                 a parity bit tells level-L vertices apart), picking the
//                 best-prio boundary among their level-L neighbours.
//  * GenericSolver (Time- or Money-first): buckets of the leading metric
//    (the bucket rises by 1 or 2 per StandardMove): settle -> specials ->
//    pull -> next, with full label comparisons in the pull.
//
// Grid state lives in LDS when it fits (G=false) and in a per-workgroup HBM
// slot otherwise (G=true; cross-thread words then go through sc1 loads/stores).
#pragma once
#include <hip/hip_runtime.h>

#include "mr_engine.hpp"

#include <map>
#include <mutex>
#include <tuple>

namespace mr {

constexpr int kBS = 256;

// hipOccupancyMaxActiveBlocksPerMultiprocessor, once per (kernel, block size, LDS bytes)
// and device: plan creation asks for several, and the query is not free
inline int occupancy_cached(const void *fn, int bs, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<const void *, int, size_t, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(fn, bs, lds, dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, bs, lds);
    cache.emplace(key, n);
    return n;
}
constexpr uint32_t kOwn = 0xFFFFu;
constexpr uint32_t kNone32 = 0xFFFFFFFFu;
constexpr unsigned long long kInf64 = ~0ull;
constexpr uint32_t kStPar = kStDirty;  // LegsSolver: parity of the settle level (settled words only)

struct Shared {
    unsigned long long B;   // generic: current bucket
    unsigned long long smin;
    uint32_t cnt[3];        // list counts
    uint32_t lb;            // generic: list rotation base / legs: current frontier buffer
    uint32_t nd;            // generic: dirty count
    uint32_t sidx;
    uint32_t sslot;         // fallback launch: the source's certificate slot (kNone32: none)
    uint32_t sentry;        // fallback launch: the source's fallback entry
    uint32_t done;
    uint32_t L;             // legs: current level
    uint32_t nbnd;          // legs: number of boundaries
    uint32_t jump;          // legs: 1 if the frontier is empty and L jumps
    uint32_t ndst;          // destinations of the current source
    uint32_t ranked;        // legs: nbnd when prio[] was last computed (linear run time)
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Exact floor(x / d) for 0 < d < 2^31 and |x| < 2^50 without an integer division (a
// 64-bit divide expands to ~150 VALU instructions on gfx950; the non-linear hub's
// certification divides per path cell): the correctly rounded double quotient is
// within one of the result, and one remainder step corrects it.
__device__ __forceinline__ long long floor_div(long long x, long long d) {
    long long q = (long long)floor(double(x) / double(d));
    const long long r = x - q * d;
    q += r >= d ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

// Diagnostic phase stamps (build with -DMR_STAMPS; never in the product build):
// thread 0 of each workgroup accumulates shader cycles per phase.
#ifdef MR_STAMPS
struct Stamps {
    unsigned long long last, acc[8];
    __device__ void start() {
        last = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 8; ++i) acc[i] = 0;
    }
    __device__ void mark(int slot) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[slot] += t - last;
        last = t;
    }
};
#define MR_STAMP(st, slot) \
    do {                   \
        if (threadIdx.x == 0) (st).mark(slot); \
    } while (0)
#else
struct Stamps {
    __device__ void start() {}
    __device__ void mark(int) {}
};
#define MR_STAMP(st, slot) \
    do {                   \
    } while (0)
#endif

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- wave-wide minimum on the DPP network (all 64 lanes active) ----------------------
// row_shr 1/2/4/8 leave each row's minimum in its lane 15, row_bcast 15/31 carry it
// to lane 63; rows outside the mask keep the identity, so min() leaves them intact.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_min(uint32_t x) {
    const uint32_t y = uint32_t(__builtin_amdgcn_update_dpp(-1, int(x), CTRL, ROWS, 0xF, false));
    return y < x ? y : x;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = dpp_min<0x111, 0xF>(x);  // row_shr:1
    x = dpp_min<0x112, 0xF>(x);  // row_shr:2
    x = dpp_min<0x114, 0xF>(x);  // row_shr:4
    x = dpp_min<0x118, 0xF>(x);  // row_shr:8
    x = dpp_min<0x142, 0xA>(x);  // row_bcast:15
    x = dpp_min<0x143, 0xC>(x);  // row_bcast:31
    return uint32_t(__builtin_amdgcn_readlane(int(x), 63));
}
// keep in c only the lanes whose key is the minimum over the lanes in c
__device__ __forceinline__ void narrow(bool &c, uint32_t key) {
    const uint32_t m = wave_min_u32(c ? key : 0xFFFFFFFFu);
    c = c && key == m;
}
// value of x in (uniform) lane l, without LDS
__device__ __forceinline__ uint32_t bcast(uint32_t x, uint32_t l) {
    return uint32_t(__builtin_amdgcn_readlane(int(x), int(l)));
}

// A label viewed for comparison: metrics, length, prefix pointer (table
// index, 0 = empty prefix) and the last <= 2 commands.  Scalar fields only, so
// nothing is runtime-indexed (no scratch).
struct View {
    uint32_t m0, m1, m2;  // legs, money, time
    uint32_t len, parent, ntail;
    Cmd t0, t1;
};
__device__ __forceinline__ Cmd bcast(const Cmd &c, uint32_t l) { return Cmd{bcast(c.kp, l), bcast(c.from, l), bcast(c.to, l)}; }
__device__ __forceinline__ View bcast(const View &x, uint32_t l) {
    View y;
    y.m0 = bcast(x.m0, l);
    y.m1 = bcast(x.m1, l);
    y.m2 = bcast(x.m2, l);
    y.len = bcast(x.len, l);
    y.parent = bcast(x.parent, l);
    y.ntail = bcast(x.ntail, l);
    y.t0 = bcast(x.t0, l);
    y.t1 = bcast(x.t1, l);
    return y;
}
// selected with masks rather than ?: so the optimiser cannot turn it into a
// load through a selected pointer (which would force the View into scratch)
__device__ __forceinline__ Cmd tail_at(const View &x, int i) {
    const uint32_t m = 0u - uint32_t(i == 0);
    return Cmd{(x.t0.kp & m) | (x.t1.kp & ~m), (x.t0.from & m) | (x.t1.from & ~m), (x.t0.to & m) | (x.t1.to & ~m)};
}
// A tentative label held in registers by the hub solvers: a View without the fields
// every such label derives.  The label builders (start, walk, SoE from a region,
// ext_view, SHQ/SFm) all give t0.from = the rank of the parent entry's cell (the
// source's for parent 0), t0.to = u (the special's own rank unless ntail = 2), and
// t1 = {SoE, u, own rank} when ntail = 2; so 6 words hold it where a View takes 12,
// and an improvement selects 6 fields.
struct RLab {
    uint32_t m0, m1, m2;
    uint32_t lpn;  // len | parent << 16 | (ntail - 1) << 31
    uint32_t kp0, u;
};
__device__ __forceinline__ RLab compact(const View &c) {
    return RLab{c.m0, c.m1, c.m2, c.len | (c.parent << 16) | ((c.ntail - 1u) << 31), c.t0.kp, c.t0.to};
}
__device__ __forceinline__ uint32_t rl_len(const RLab &x) { return x.lpn & 0xFFFFu; }
__device__ __forceinline__ void sel_rlab(bool take, RLab &d, const RLab &c) {
    d.m0 = take ? c.m0 : d.m0;
    d.m1 = take ? c.m1 : d.m1;
    d.m2 = take ? c.m2 : d.m2;
    d.lpn = take ? c.lpn : d.lpn;
    d.kp0 = take ? c.kp0 : d.kp0;
    d.u = take ? c.u : d.u;
}

template <bool G>
struct Core {
    const KArgs *__restrict__ a;
    Shared *sh;
    Rec *R;
    uint32_t *state;
    // Register copies of the launch constants: wave_sync's fences make the compiler
    // re-load anything read through `a` after every sync.
    DevParams P;
    const uint32_t *rank;     // a->rank
    const uint32_t *sinfo;    // a->sinfo
    uint32_t *counter;        // a->counter
    const SpecialStatic *sp;  // LDS copy of a->sp (loaded once per workgroup)
    const uint16_t *hubs;     // LDS copy of a->hubs
    uint32_t *dst;            // LDS: destinations of the current source (<= early_exit_max)
    uint32_t src, src_rk;

    // ---- memory helpers -----------------------------------------------------
    __device__ __forceinline__ uint32_t ld_state(uint32_t v) const {
        if constexpr (G) return __hip_atomic_load(state + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return state[v];
    }
    __device__ __forceinline__ void st_state(uint32_t v, uint32_t x) const {
        if constexpr (G) __hip_atomic_store(state + v, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else state[v] = x;
    }
    __device__ __forceinline__ uint32_t or_state(uint32_t v, uint32_t x) const {
        if constexpr (G) return __hip_atomic_fetch_or(state + v, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return atomicOr(state + v, x);
    }
    template <class IdxT>
    __device__ __forceinline__ uint32_t ld_idx(const IdxT *l, uint32_t i) const {
        if constexpr (G) return __hip_atomic_load(l + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return l[i];
    }
    template <class IdxT>
    __device__ __forceinline__ void st_idx(IdxT *l, uint32_t i, uint32_t v) const {
        if constexpr (G) __hip_atomic_store(l + i, IdxT(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else l[i] = IdxT(v);
    }
    __device__ __forceinline__ void flag(uint32_t e) const { atomicOr(counter + kCtrFlags, e); }
    // metric overflow is sticky per lane and reported once, at the end of the launch
    // (flush_err): a branch and an atomic per addition would cost issue slots
    mutable uint32_t err = 0;
    __device__ __forceinline__ void flush_err() const {
        if (err) flag(err);
    }
    __device__ __forceinline__ uint32_t special_of(uint32_t v) const { return sinfo[v] & kNone10; }
    __device__ __forceinline__ uint32_t region_of(uint32_t v) const { return (sinfo[v] >> 10) & kNone10; }
    __device__ __forceinline__ uint32_t vert_of(uint32_t t) const { return t == 0 ? src : sp[t].v; }
    // commands name cells by CellIndex rank, so comparing them needs no memory access
    __device__ __forceinline__ uint32_t rk_of(uint32_t t) const { return t == 0 ? src_rk : sp[t].rk; }
    // the View of register label x of the special whose cell has rank `own` (RLab)
    __device__ __forceinline__ View expand(const RLab &x, uint32_t own) const {
        View v;
        v.m0 = x.m0;
        v.m1 = x.m1;
        v.m2 = x.m2;
        v.len = x.lpn & 0xFFFFu;
        v.parent = (x.lpn >> 16) & kNone10;
        v.ntail = (x.lpn >> 31) + 1u;
        v.t0 = Cmd{x.kp0, rk_of(v.parent), x.u};
        v.t1 = v.ntail == 2 ? Cmd{kSoE << 29, x.u, own} : Cmd{0, 0, 0};
        return v;
    }

    // ---- arithmetic (u32 like the reference; overflow is reported, not wrapped)
    __device__ __forceinline__ uint32_t add32(uint32_t x, uint32_t y) const {
        uint32_t r = x + y;
        err |= r < x ? kErrMetricOverflow : 0u;
        return r;
    }
    // AggregatedCost::time of a StandardMove run of k legs: Fleetfoot ceil of
    // 180k seconds (src/cost.rs:122-124, src/skill.rs:21-30)
    __device__ __forceinline__ uint32_t run_time(uint32_t k) const {
        const DevParams &p = P;
        unsigned long long t = 180ull * k;
        if (p.ff_num != p.ff_den) t = (unsigned long long)floor_div((long long)(t * p.ff_num + p.ff_den - 1), p.ff_den);
        err |= t > 0xFFFFFFFFull ? kErrMetricOverflow : 0u;
        return uint32_t(t);
    }
    __device__ __forceinline__ unsigned long long key_of(uint32_t m0, uint32_t m1, uint32_t m2) const {
        const DevParams &p = P;
        switch (p.bucket_mode) {
            case kBucketLegs: return m0;
            case kBucketTime: return m2 / p.W;
            case kBucketMoneyLegs: return (unsigned long long)m1 << 32 | m0;
            default: return (unsigned long long)m1 << 32 | (m2 / p.W);
        }
    }
    __device__ __forceinline__ unsigned long long key_rec(uint32_t t) const { return key_of(R[t].m[0], R[t].m[1], R[t].m[2]); }

    // ---- views ------------------------------------------------------------------
    __device__ __forceinline__ void view_rec(uint32_t t, View &x) const {
        const Rec &r = R[t];
        x.m0 = r.m[0];
        x.m1 = r.m[1];
        x.m2 = r.m[2];
        x.len = r.len();
        x.parent = r.parent();
        x.ntail = r.ntail();
        x.t0 = Cmd{r.kp0, r.from0, r.u};
        x.t1 = x.ntail == 2 ? Cmd{kSoE << 29, r.u, rk_of(t)} : Cmd{0, 0, 0};
    }
    // the start label TotalCost::new(src) (src/cost.rs:196-205)
    __device__ __forceinline__ void view_start(View &x) const {
        x.m0 = x.m1 = x.m2 = 0;
        x.len = 1;
        x.parent = 0;
        x.ntail = 1;
        x.t0 = Cmd{kNoMove << 29, src_rk, src_rk};
        x.t1 = Cmd{0, 0, 0};
    }
    // walk label of v (rank vr): full(b) ++ [StandardMove{k} vert(b) -> v]
    __device__ __forceinline__ void view_walk(uint32_t b, uint32_t k, uint32_t vr, View &x) const {
        if (b == 0 && k == 0) {
            view_start(x);
            return;
        }
        const Rec &rb = R[b];
        x.m0 = add32(rb.m[0], k);
        x.m1 = rb.m[1];
        x.m2 = add32(rb.m[2], run_time(k));
        x.len = (b == 0 ? 0u : rb.len()) + 1u;
        x.parent = b;
        x.ntail = 1;
        x.t0 = Cmd{(kStandard << 29) | k, rk_of(b), vr};
        x.t1 = Cmd{0, 0, 0};
    }

    // the same, from b's label lb held in registers
    __device__ __forceinline__ void view_walk_lab(const View &lb, uint32_t b, uint32_t k, uint32_t vr, View &x) const {
        if (b == 0 && k == 0) {
            view_start(x);
            return;
        }
        x.m0 = add32(lb.m0, k);
        x.m1 = lb.m1;
        x.m2 = add32(lb.m2, run_time(k));
        x.len = (b == 0 ? 0u : lb.len) + 1u;
        x.parent = b;
        x.ntail = 1;
        x.t0 = Cmd{(kStandard << 29) | k, rk_of(b), vr};
        x.t1 = Cmd{0, 0, 0};
    }
    __device__ __forceinline__ void write_rec(uint32_t t, const View &c, uint32_t state) const {
        Rec &r = R[t];
        r.m[0] = c.m0;
        r.m[1] = c.m1;
        r.m[2] = c.m2;
        r.meta = Rec::pack(c.len, c.parent, c.ntail, state);
        r.kp0 = c.t0.kp;
        r.from0 = c.t0.from;
        r.u = c.t0.to;
    }

    // ---- comparator: CostComparator::and_then (src/cost.rs:411-426) ------------
    __device__ __forceinline__ int cmp_cmd(const Cmd &x, const Cmd &y) const {
        if (x.kp != y.kp) return x.kp < y.kp ? -1 : 1;
        if (x.from != y.from) return x.from < y.from ? -1 : 1;  // ranks: CellIndex order
        if (x.to != y.to) return x.to < y.to ? -1 : 1;
        return 0;
    }
    // command i of table entry t, by value (no pointer into LDS escapes)
    __device__ __forceinline__ Cmd rec_tail(uint32_t t, int i) const {
        const Rec &r = R[t];
        return i == 0 ? Cmd{r.kp0, r.from0, r.u} : Cmd{kSoE << 29, r.u, rk_of(t)};
    }
    // lexicographic compare of two command lists of equal length, walking from
    // the last command towards the first; xid/yid name the table entries the
    // views were read from (kOwn for built views) so a shared prefix stops the walk.
    __device__ __forceinline__ int cmp_list(const View &x, uint32_t xid, const View &y, uint32_t yid) const {
        uint32_t xe = xid, ye = yid;
        int xt = int(x.ntail) - 1, yt = int(y.ntail) - 1;
        int res = 0;
        for (uint32_t guard = 0; guard < 8192u; ++guard) {
            if (xe != kOwn && xe == ye && xt == yt) return res;
            const Cmd cx = (xe == kOwn) ? tail_at(x, xt) : rec_tail(xe, xt);
            const Cmd cy = (ye == kOwn) ? tail_at(y, yt) : rec_tail(ye, yt);
            int r = cmp_cmd(cx, cy);
            if (r) res = r;
            if (xt > 0) --xt;
            else {
                uint32_t pp = (xe == kOwn) ? x.parent : R[xe].parent();
                if (pp == 0) return res;
                xe = pp;
                xt = int(R[pp].ntail()) - 1;
            }
            if (yt > 0) --yt;
            else {
                uint32_t pp = (ye == kOwn) ? y.parent : R[ye].parent();
                if (pp == 0) return res;
                ye = pp;
                yt = int(R[pp].ntail()) - 1;
            }
        }
        flag(kErrChain);
        return res;
    }
    __device__ __forceinline__ int cmp_metrics(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t y0, uint32_t y1,
                                               uint32_t y2) const {
        const DevParams &p = P;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t pi = p.perm[i];
            const uint32_t u = pi == 0 ? x0 : (pi == 1 ? x1 : x2);
            const uint32_t w = pi == 0 ? y0 : (pi == 1 ? y1 : y2);
            if (u != w) return u < w ? -1 : 1;
        }
        return 0;
    }
    __device__ __forceinline__ int cmp_view(const View &x, uint32_t xid, const View &y, uint32_t yid) const {
        int r = cmp_metrics(x.m0, x.m1, x.m2, y.m0, y.m1, y.m2);
        if (r) return r;
        if (x.len != y.len) return x.len < y.len ? -1 : 1;
        return cmp_list(x, xid, y, yid);
    }
    __device__ __forceinline__ int cmp_entries(uint32_t s, uint32_t t) const {
        const Rec &rs = R[s], &rt = R[t];
        int r = cmp_metrics(rs.m[0], rs.m[1], rs.m[2], rt.m[0], rt.m[1], rt.m[2]);
        if (r) return r;
        if (rs.len() != rt.len()) return rs.len() < rt.len() ? -1 : 1;
        View x, y;
        view_rec(s, x);
        view_rec(t, y);
        return cmp_list(x, s, y, t);
    }

    // ---- special table updates --------------------------------------------------
    __device__ __forceinline__ void try_improve(uint32_t t, const View &c) const {
        const Rec &r = R[t];
        if (r.state() == 2) return;
        if (r.state() == 1) {
            int cm = cmp_metrics(c.m0, c.m1, c.m2, r.m[0], r.m[1], r.m[2]);
            if (cm > 0) return;
            if (cm == 0) {
                if (c.len > r.len()) return;
                if (c.len == r.len()) {
                    View cur;
                    view_rec(t, cur);
                    if (cmp_list(c, kOwn, cur, t) >= 0) return;
                }
            }
        }
        write_rec(t, c, 1);
    }
    // extend the settled label r of special s (rank rs) by a non-Standard edge
    // to the cell of rank rt (TotalCost += edge, src/cost.rs:208-315)
    __device__ __forceinline__ void ext_view(const View &r, uint32_t s, uint32_t rs, uint32_t kind, uint32_t payload,
                                             uint32_t dm_money, uint32_t dm_time, uint32_t rt, View &c) const {
        const Cmd last = r.ntail == 2 ? r.t1 : r.t0;
        const uint32_t lk = last.kp >> 29;
        c.t1 = Cmd{0, 0, 0};
        if (lk == kNoMove) {  // the start label: NoMove is replaced, its from kept
            c.m0 = 0;
            c.m1 = dm_money;
            c.m2 = dm_time;
            c.len = 1;
            c.parent = 0;
            c.ntail = 1;
            c.t0 = Cmd{(kind << 29) | payload, last.from, rt};
        } else if (kind == kCentral && lk == kCentral) {  // CentralMoves merge (ntail is 1)
            c.m0 = r.m0;
            c.m1 = r.m1;
            c.m2 = add32(r.m2, dm_time);
            c.len = r.len;
            c.parent = r.parent;
            c.ntail = 1;
            c.t0 = Cmd{last.kp + 1u, last.from, rt};
        } else {
            c.m0 = r.m0;
            c.m1 = add32(r.m1, dm_money);
            c.m2 = add32(r.m2, dm_time);
            c.len = r.len + 1u;
            c.parent = s;
            c.ntail = 1;
            c.t0 = Cmd{(kind << 29) | payload, rs, rt};
        }
    }
    __device__ __forceinline__ void ext_special(uint32_t s, uint32_t kind, uint32_t payload, uint32_t dm_money,
                                                uint32_t dm_time, uint32_t t, View &c) const {
        View r;
        view_rec(s, r);
        ext_view(r, s, sp[s].rk, kind, payload, dm_money, dm_time, sp[t].rk, c);
    }
    // the SoE candidate for campfire t from plain vertex u (rank ur) with walk label (b,k)
    __device__ __forceinline__ void soe_from_plain(uint32_t b, uint32_t k, uint32_t ur, uint32_t t, View &c) const {
        const DevParams &p = P;
        const uint32_t vt = sp[t].rk;
        if (b == 0 && k == 0) {  // u is the source: [SoE src->c]
            c.m0 = 0;
            c.m1 = p.soe_cost;
            c.m2 = 0;
            c.len = 1;
            c.parent = 0;
            c.ntail = 1;
            c.t0 = Cmd{kSoE << 29, src_rk, vt};
            c.t1 = Cmd{0, 0, 0};
        } else {  // full(b) ++ [Std{k} b->u, SoE u->c]
            view_walk(b, k, ur, c);
            c.m1 = add32(c.m1, p.soe_cost);
            c.len += 1;
            c.ntail = 2;
            c.t1 = Cmd{kSoE << 29, ur, vt};
        }
    }

    // ---- grid helpers -------------------------------------------------------------
    // geometric neighbour d (0:-x 1:+x 2:-y 3:+y) of v, or kNone32
    __device__ __forceinline__ uint32_t nbr(uint32_t v, int d) const {
        const DevParams &p = P;
        const uint32_t x = v % p.S;
        switch (d) {
            case 0: return x == 0 ? kNone32 : v - 1;
            case 1: return x + 1 == p.S ? kNone32 : v + 1;
            case 2: return v < p.S ? kNone32 : v - p.S;
            default: return v + p.S >= p.V ? kNone32 : v + p.S;
        }
    }

    // ---- specials: settle + relax (one wave, uniform s) ----------------------------
    // Seeds the grid word of s, then relaxes CentralMove (src/pathfinder.rs:30-53),
    // caravan (:140-160, 251-273) and Scroll-of-Escape (:162-170) edges.
    // Returns whether s is a boundary (its label does not end in a StandardMove).
    __device__ __forceinline__ bool settle_special(uint32_t s, uint32_t par_bits) const {
        const DevParams &p = P;
        const uint32_t lane = lane_id();
        const uint32_t vs = sp[s].v;
        Rec &r = R[s];
        const uint32_t last_kp = r.ntail() == 2 ? (kSoE << 29) : r.kp0;
        const uint32_t lk = last_kp >> 29;
        uint32_t seed;
        bool boundary;
        if (lk == kNoMove) {  // the source itself
            seed = 0;
            boundary = false;
        } else if (lk == kStandard) {  // continues the walk of its parent boundary
            seed = (r.parent() << kStBShift) | (last_kp & kStKMask);
            boundary = false;
        } else {  // a boundary: walks restart here
            seed = s << kStBShift;
            boundary = true;
        }
        wave_sync();
        if (lane == 0) {
            r.set_state(2);
            st_state(vs, kStSettled | par_bits | seed);
        }
        wave_sync();
        const uint32_t fl = sp[s].flags;
        if (fl & kSpCenter) {
            if (lane < 4) {
                View c;
                ext_special(s, kCentral, 1, 0, 10, 2 + lane, c);
                try_improve(2 + lane, c);
            }
        } else if (fl & kSpBorder1) {
            if (lane == 0) {
                View c;
                ext_special(s, kCentral, 1, 0, 10, 1, c);
                try_improve(1, c);
            }
        }
        wave_sync();
        if (p.use_caravans && (fl & kSpHub)) {
            const SpecialStatic ss = sp[s];
            for (uint32_t h = lane; h < p.n_hubs; h += 64) {
                const uint32_t t = hubs[h];
                if (t == s || R[t].state() == 2) continue;
                const SpecialStatic st = sp[t];
                const uint32_t d = uint32_t(abs(ss.x - st.x) + abs(ss.y - st.y));
                const uint32_t coef = st.coef5 ? 5u : 2u;
                View c;
                ext_special(s, kCaravan, (d << 1) | st.coef5, coef * d, p.rgt * d, t, c);
                try_improve(t, c);
            }
        }
        wave_sync();
        if (p.use_soe && lane == 0) {
            const uint32_t t = sp[s].region;
            if (t != kNone10 && t != s) {
                View c;
                ext_special(s, kSoE, 0, p.soe_cost, 0, t, c);
                try_improve(t, c);
            }
        }
        wave_sync();
        return boundary;
    }

    // wave argmin (full comparator) over tentative specials whose key == K
    __device__ __forceinline__ uint32_t argmin_special(unsigned long long K) const {
        const DevParams &p = P;
        const uint32_t lane = lane_id();
        uint32_t mine = kNone32;
        for (uint32_t t = 1 + lane; t <= p.NS; t += 64) {
            if (R[t].state() != 1) continue;
            const unsigned long long k = key_rec(t);
            if (k < K) flag(kErrBucket);
            if (k > K) continue;
            if (mine == kNone32 || cmp_entries(t, mine) < 0) mine = t;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t other = __shfl_xor(mine, off, 64);
            if (other != kNone32 && (mine == kNone32 || cmp_entries(other, mine) < 0)) mine = other;
        }
        return mine;
    }
    // ---- register-resident exact Dijkstra over the specials of bucket K -------------
    // (wave 0, NS <= 63): lane t holds the tentative label of special t; the LDS
    // table R[] stays an exact mirror (every improvement is written back) because
    // other phases and the list comparator read it.  Per iteration select_lane picks
    // the settle candidate, then every lane relaxes the edges from the settled
    // special into itself — no shared-write races.
    __device__ __forceinline__ static uint32_t metric(const View &x, uint32_t i) {
        return i == 0 ? x.m0 : (i == 1 ? x.m1 : x.m2);
    }
    __device__ __forceinline__ static uint32_t metric(const RLab &x, uint32_t i) {
        return i == 0 ? x.m0 : (i == 1 ? x.m1 : x.m2);
    }
    // among the lanes with c set, the one holding the smallest table label (lane t holds
    // entry t, mirrored in `my`): metrics in comparator order, then length on the DPP
    // network; only exact ties of both reach the command-list compare.  kNone32 if none.
    __device__ __forceinline__ uint32_t select_lane(bool c, const View &my) const {
        if (__ballot(c) == 0) return kNone32;
        const DevParams &p = P;
        narrow(c, metric(my, p.perm[0]));
        narrow(c, metric(my, p.perm[1]));
        narrow(c, metric(my, p.perm[2]));
        narrow(c, my.len);
        const unsigned long long bal = __ballot(c);
        if (__popcll(bal) == 1) return uint32_t(__ffsll((long long)bal) - 1);
        uint32_t m = c ? lane_id() : kNone32;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t o = __shfl_xor(m, off, 64);
            if (o != kNone32 && (m == kNone32 || cmp_entries(o, m) < 0)) m = o;
        }
        return m;
    }
    __device__ __forceinline__ void improve_own(uint32_t t, uint32_t &st, View &my, const View &c) const {
        if (st == 2) return;
        if (st == 1) {
            int cm = cmp_metrics(c.m0, c.m1, c.m2, my.m0, my.m1, my.m2);
            if (cm > 0) return;
            if (cm == 0) {
                if (c.len > my.len) return;
                if (c.len == my.len && cmp_list(c, kOwn, my, t) >= 0) return;
            }
        }
        my = c;
        st = 1;
        write_rec(t, c, 1);
    }
    template <class OnSettle>
    __device__ __forceinline__ void specials_reg(unsigned long long K, uint32_t par_bits, OnSettle on_settle) const {
        const DevParams &p = P;
        const uint32_t t = lane_id();
        const bool mine = t >= 1 && t <= p.NS;
        View my;
        uint32_t st = 0;
        SpecialStatic ss{};
        if (mine) {
            st = R[t].state();
            view_rec(t, my);
            ss = sp[t];
        } else {
            my.m0 = my.m1 = my.m2 = 0;
        }
        for (uint32_t it = 0; it <= p.NS; ++it) {
            const bool tent = mine && st == 1;
            const unsigned long long key = tent ? key_of(my.m0, my.m1, my.m2) : kInf64;
            if (tent && key < K) flag(kErrBucket);
            const bool cand = tent && key == K;
            const uint32_t s = select_lane(cand, my);
            if (s == kNone32) break;
            // settle s
            View ls;
            view_rec(s, ls);
            const Cmd last = ls.ntail == 2 ? ls.t1 : ls.t0;
            const uint32_t lk = last.kp >> 29;
            uint32_t seed;
            bool boundary;
            if (lk == kNoMove) {  // the source itself
                seed = 0;
                boundary = false;
            } else if (lk == kStandard) {  // continues the walk of its parent boundary
                seed = (ls.parent << kStBShift) | (last.kp & kStKMask);
                boundary = false;
            } else {  // a boundary: walks restart here
                seed = s << kStBShift;
                boundary = true;
            }
            const SpecialStatic sS = sp[s];
            if (t == s) st = 2;
            wave_sync();
            if (t == 0) {
                R[s].set_state(2);
                st_state(sS.v, kStSettled | par_bits | seed);
            }
            on_settle(s, sS.v, boundary);
            // relax the CentralMove / caravan / SoE edges s -> t into lane t
            if (mine && st != 2) {
                View c;
                if (((sS.flags & kSpCenter) && (ss.flags & kSpBorder1)) ||
                    ((sS.flags & kSpBorder1) && (ss.flags & kSpCenter))) {
                    ext_view(ls, s, sS.rk, kCentral, 1, 0, 10, ss.rk, c);
                    improve_own(t, st, my, c);
                }
                if (p.use_caravans && (sS.flags & kSpHub) && (ss.flags & kSpHub)) {
                    const uint32_t d = uint32_t(abs(sS.x - ss.x) + abs(sS.y - ss.y));
                    const uint32_t coef = ss.coef5 ? 5u : 2u;
                    ext_view(ls, s, sS.rk, kCaravan, (d << 1) | ss.coef5, coef * d, p.rgt * d, ss.rk, c);
                    improve_own(t, st, my, c);
                }
                if (p.use_soe && sS.region == t) {
                    ext_view(ls, s, sS.rk, kSoE, 0, p.soe_cost, 0, ss.rk, c);
                    improve_own(t, st, my, c);
                }
            }
            wave_sync();
        }
    }
    __device__ __forceinline__ unsigned long long min_special_key() const {
        const DevParams &p = P;
        unsigned long long smin = kInf64;
        for (uint32_t t = 1 + lane_id(); t <= p.NS; t += 64)
            if (R[t].state() == 1) {
                const unsigned long long k = key_rec(t);
                if (k < smin) smin = k;
            }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(smin, off, 64);
            if (o < smin) smin = o;
        }
        return smin;
    }

    // ---- per-source init / output ----------------------------------------------------
    // Untouched grid words carry the vertex's static info in their k field
    // (special index | region << 10), so a claim needs no extra global load.
    __device__ __forceinline__ void init_source(uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t tid = threadIdx.x;
        src = a->src_v[s_idx];
        src_rk = rank[src];
        if constexpr (G) {
            const uint4 *i4 = reinterpret_cast<const uint4 *>(a->sinfo);
            uint4 *s4 = reinterpret_cast<uint4 *>(state);
            for (uint32_t i = tid; i < p.V / 4; i += kBS) {
                uint4 x = i4[i];
                x.x |= kStUntouched;
                x.y |= kStUntouched;
                x.z |= kStUntouched;
                x.w |= kStUntouched;
                s4[i] = x;
            }
            for (uint32_t v = (p.V & ~3u) + tid; v < p.V; v += kBS) state[v] = kStUntouched | a->sinfo[v];
        } else {
            for (uint32_t v = tid; v < p.V; v += kBS) state[v] = kStUntouched | a->sinfo[v];
        }
        for (uint32_t t = tid; t <= p.NS; t += kBS) R[t].set_state(0);
        const uint32_t q0 = a->q_begin[s_idx], q1 = a->q_begin[s_idx + 1];
        if (tid == 0) sh->ndst = q1 - q0;
        if (q1 - q0 <= a->early_exit_max)
            for (uint32_t i = tid; i < q1 - q0; i += kBS) dst[i] = a->q_dst[q0 + i];
    }
    // SHQ / SFm: only the source's own edges can be minimal (any prefix only adds
    // metrics and length), src/pathfinder.rs:172-178
    __device__ __forceinline__ void seed_scrolls() const {
        const DevParams &p = P;
        if (p.hq_t) {
            View c;
            view_start(c);
            c.m1 = p.shq_cost;
            c.t0 = Cmd{kSHQ << 29, src_rk, sp[p.hq_t].rk};
            try_improve(p.hq_t, c);
        }
        if (p.use_sfm) {
            View c;
            view_start(c);
            c.m1 = p.sfm_cost;
            c.t0 = Cmd{kSFm << 29, src_rk, sp[1].rk};  // entry 1 = the Center
            try_improve(1, c);
        }
    }
    // materialise label x as a result record and command slots
    // the output record of the query at grouped position qi (queries grouped by source,
    // so a source's records are contiguous: whole lines, not scattered 16 B stores; the
    // host maps positions back to query ids)
    __device__ __forceinline__ void emit(const View &x, uint32_t qi) const {
        const DevParams &p = P;
        OutResult &o = a->out_res[qi];
        OutCmd *oc = a->out_cmd + (unsigned long long)qi * p.max_cmds;
        uint32_t status = 16;
        if (x.len > p.max_cmds) {  // the overflow pool, else MR_ERR_CAPACITY (the host re-runs with more slots)
            const uint32_t off = atomicAdd(a->counter + kCtrOvf, x.len);
            if (p.max_cmds == 0 || off + x.len > a->ovf_cap || off + x.len < off) {
                o = OutResult{x.m0, x.m1, x.m2, (uint32_t(16 - 4) << 16) | (x.len & 0xFFFFu)};
                return;
            }
            oc[0] = OutCmd{kOvfTag, off, x.len, 0};
            oc = a->ovf + off;
            status = 16 + kStatusOverflow;
        }
        int pos = int(x.len) - 1;
        if (x.ntail == 2 && pos >= 0) {
            oc[pos] = OutCmd{x.t1.kp, x.t1.from, x.t1.to, 0};
            --pos;
        }
        if (pos >= 0) {
            oc[pos] = OutCmd{x.t0.kp, x.t0.from, x.t0.to, 0};
            --pos;
        }
        uint32_t pp = x.parent;
        while (pp != 0 && pos >= 0) {
            const Rec &r = R[pp];
            for (int j = int(r.ntail()) - 1; j >= 0 && pos >= 0; --j, --pos) {
                const Cmd cj = rec_tail(pp, j);
                oc[pos] = OutCmd{cj.kp, cj.from, cj.to, 0};
            }
            pp = r.parent();
        }
        if (pos != -1 || pp != 0) flag(kErrChain);
        o = OutResult{x.m0, x.m1, x.m2, (status << 16) | (x.len & 0xFFFFu)};
    }
    __device__ __forceinline__ void write_output(uint32_t w, uint32_t qi) const {
        const uint32_t sw = ld_state(w);
        if (!(sw & kStSettled)) {
            a->out_res[qi] = OutResult{0, 0, 0, uint32_t(16 + 1) << 16};  // MR_NOT_FOUND
            return;
        }
        View x;
        const uint32_t t = special_of(w);
        if (t != kNone10) view_rec(t, x);
        else view_walk((sw >> kStBShift) & kNone10, sw & kStKMask, rank[w], x);
        emit(x, qi);
    }
    __device__ __forceinline__ void write_outputs(uint32_t s_idx) const {
        if (a->all_mode) {
            write_all(s_idx);
            return;
        }
        const uint32_t q0 = a->q_begin[s_idx], q1 = a->q_begin[s_idx + 1];
        for (uint32_t i = q0 + threadIdx.x; i < q1; i += kBS) write_output(a->q_dst[i], i);
    }
    // all-destinations mode: the label table and a cell word for every cell (CellWord:
    // the settled state word's walk (b, k) as it stands)
    __device__ __forceinline__ void write_all(uint32_t s_idx) const {
        const DevParams &p = P;
        const unsigned long long tb = (unsigned long long)s_idx * (p.NS + 1);
        for (uint32_t t = threadIdx.x; t <= p.NS; t += kBS) {
            a->out_tab[tb + t] = R[t];
            a->out_lex[tb + t] = kNone32;
        }
        const uint32_t pitch = a->rec_pitch;
        CellWord *out = a->out_rec + (unsigned long long)s_idx * p.S * pitch;
        for (uint32_t v = threadIdx.x; v < p.V; v += kBS) {
            CellWord r = kViaSource;
            const uint32_t sw = ld_state(v);
            const uint32_t t = special_of(v);
            if (v == src) {
            } else if (t != kNone10) {
                r = kViaSpecial | t;
            } else if (sw & kStSettled) {
                r = sw & ((kNone10 << kStBShift) | kStKMask);
            } else {
                flag(kErrBucket);  // every cell of the connected grid settles
            }
            const uint32_t y = v / p.S;
            out[y * pitch + (v - y * p.S)] = r;
        }
        if (threadIdx.x == 0) a->src_state[s_idx] = 2;
    }
    // Certified fallback: the label of vertex d from certificate
    // slot words w (the cell words of a fill, repaired by the sweep) and the slot's table in R
    __device__ __forceinline__ void cert_view(const CellWord *w, uint32_t d, View &x) const {
        const DevParams &p = P;
        const uint32_t y = d / p.S, cw = w[(unsigned long long)y * a->rec_pitch + (d - y * p.S)];
        if (cw == kViaSource) view_start(x);
        else if (cw & kViaSpecial) view_rec(cw & kNone10, x);
        else view_walk((cw >> kStBShift) & kNone10, cw & kStKMask, rank[d], x);
    }
    // Source s_idx's records from certificate slot k when the leading metric of each of
    // its labels lies below the slot's failure key (those labels are the reference's:
    // the fixed-point argument of section 3d); false, with nothing written, otherwise
    __device__ __forceinline__ bool cert_emit(uint32_t s_idx, uint32_t k) {
        const DevParams &p = P;
        const uint32_t T = p.NS + 1;
        for (uint32_t t = threadIdx.x; t < T; t += kBS) R[t] = a->cert_tab[(unsigned long long)k * T + t];
        src = a->src_v[s_idx];
        src_rk = rank[src];
        // the slot's key: the least over the check's workgroups
        uint32_t key = 0xFFFFFFFFu;
        for (uint32_t j = threadIdx.x; j < a->cert_parts; j += kBS)
            key = min(key, a->cert_st[((unsigned long long)k * a->cert_parts + j) * kCertSt + kCertKey]);
        key = wave_min_u32(key);
        if (threadIdx.x == 0) sh->done = 0xFFFFFFFFu;
        __syncthreads();
        if (lane_id() == 0) atomicMin(&sh->done, key);
        const CellWord *w = a->cert_rec + (unsigned long long)k * p.S * a->rec_pitch;
        __syncthreads();
        key = sh->done;
        const uint32_t q0 = a->q_begin[s_idx], q1 = a->q_begin[s_idx + 1];
        int ok = 1;
        for (uint32_t i = q0 + threadIdx.x; i < q1; i += kBS) {
            View x;
            cert_view(w, a->q_dst[i], x);
            const uint32_t c1 = p.perm[0] == 0 ? x.m0 : (p.perm[0] == 1 ? x.m1 : x.m2);
            ok &= c1 < key ? 1 : 0;
        }
        if (!__syncthreads_and(ok)) return false;
        for (uint32_t i = q0 + threadIdx.x; i < q1; i += kBS) {
            View x;
            cert_view(w, a->q_dst[i], x);
            emit(x, i);
        }
        __syncthreads();
        return true;
    }
    // 1 if every destination of this source (when <= early_exit_max) is settled
    __device__ __forceinline__ uint32_t dsts_done() const {
        const uint32_t lane = lane_id();
        const uint32_t nd = sh->ndst;
        if (nd > a->early_exit_max) return 0;
        bool ok = true;
        if (lane < nd) ok = (ld_state(dst[lane]) & kStSettled) != 0;
        return __all(ok) ? 1u : 0u;
    }
    __device__ __forceinline__ void seed_root() const {
        View st;
        view_start(st);
        write_rec(0, st, 2);  // entry 0: the source, root of every command chain
    }
};

// ===================================================================================
// Legs-first level-synchronous solver
// ===================================================================================
template <bool G, class IdxT>
struct LegsSolver : Core<G> {
    using Core<G>::a;
    using Core<G>::sh;
    using Core<G>::R;
    using Core<G>::state;
    using Core<G>::src;
    using Core<G>::P;
    using Core<G>::rank;
    using Core<G>::sinfo;
    using Core<G>::counter;
    IdxT *F0, *F1;                 // frontier ping-pong lists
    uint32_t *prio;                // per boundary rank for the next level
    uint32_t *bnd;                 // boundary list (table indices), bnd[0] = 0 (the source)
    unsigned long long *best64;    // per region: (prio << 32 | rank) of the level's best vertex
    uint32_t *fired;

    Stamps *stamps;                // diagnostic builds only

    __device__ __forceinline__ IdxT *frontier(uint32_t i) const { return i ? F1 : F0; }

    // walk(b1, L - legs(b1)) vs walk(b2, L - legs(b2)) at one vertex: legs tie at L
    __device__ __forceinline__ int cmp_boundaries(uint32_t b1, uint32_t b2, uint32_t L) const {
        const Rec &r1 = R[b1], &r2 = R[b2];
        const uint32_t k1 = L - r1.m[0], k2 = L - r2.m[0];
        const uint32_t t1 = this->add32(r1.m[2], this->run_time(k1)), t2 = this->add32(r2.m[2], this->run_time(k2));
        int c = this->cmp_metrics(L, r1.m[1], t1, L, r2.m[1], t2);
        if (c) return c;
        const uint32_t l1 = (b1 == 0 ? 0u : r1.len()), l2 = (b2 == 0 ? 0u : r2.len());
        if (l1 != l2) return l1 < l2 ? -1 : 1;
        if (b1 == b2) return 0;
        View x, y;  // equal prefix lengths >= 1: both are table entries; compare full(b1), full(b2)
        this->view_rec(b1, x);
        this->view_rec(b2, y);
        return this->cmp_list(x, b1, y, b2);
    }
    // wave 0: rank the boundaries for level L (prio[b] = number of better boundaries)
    __device__ __forceinline__ void rank_boundaries(uint32_t L) const {
        const uint32_t nb = sh->nbnd;
        for (uint32_t i = lane_id(); i < nb; i += 64) {
            const uint32_t b = bnd[i];
            uint32_t r = 0;
            for (uint32_t j = 0; j < nb; ++j)
                if (j != i && cmp_boundaries(bnd[j], b, L) < 0) ++r;
            prio[b] = r;
        }
        wave_sync();
    }
    // wave 0: SoE candidates from the level-L region argmins
    __device__ __forceinline__ void fire_regions() const {
        const DevParams &p = P;
        for (uint32_t t = 1 + lane_id(); t <= p.NS; t += 64) {
            const unsigned long long key = best64[t];
            if (key == kInf64) continue;
            best64[t] = kInf64;
            fired[t] = 1;
            if (R[t].state() == 2) continue;
            const uint32_t u = a->rank_inv[uint32_t(key)];
            const uint32_t su = this->ld_state(u);
            View c;
            this->soe_from_plain((su >> kStBShift) & kNone10, su & kStKMask, uint32_t(key), t, c);
            this->try_improve(t, c);
        }
        wave_sync();
    }
    // claim the unsettled StandardMove neighbours of frontier vertex v (level L)
    __device__ __forceinline__ void claim_from(uint32_t v, uint32_t L, IdxT *Fn, uint32_t cn) const {
        const DevParams &p = P;
        if (v == p.vc) return;  // the Center's out-edges are CentralMoves
        const uint32_t parL = (L & 1u) ? kStPar : 0u;
        const uint32_t parN = parL ^ kStPar;
        const uint32_t sv = this->ld_state(v);
        const uint32_t bv = (sv >> kStBShift) & kNone10, kv = sv & kStKMask;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t w = this->nbr(v, d);
            if (w == kNone32 || w == p.vc) continue;
            const uint32_t sw = this->ld_state(w);
            if (sw & kStSettled) continue;
            const int dw = d ^ 1;  // direction of v as seen from w
            // ownership: the frontier neighbour of w with the lowest direction claims w;
            // best candidate: lowest prio among w's level-L neighbours
            bool owner = true;
            uint32_t bb = bv, bk = kv + 1u, bp = prio[bv];
#pragma unroll
            for (int d2 = 0; d2 < 4; ++d2) {
                if (d2 == dw) continue;
                const uint32_t u = this->nbr(w, d2);
                if (u == kNone32 || u == p.vc) continue;
                const uint32_t su = this->ld_state(u);
                if (!(su & kStSettled) || (su & kStPar) != parL) continue;
                if (d2 < dw) owner = false;
                const uint32_t b = (su >> kStBShift) & kNone10;
                const uint32_t pr = prio[b];
                if (pr < bp) {
                    bp = pr;
                    bb = b;
                    bk = (su & kStKMask) + 1u;
                }
            }
            if (!owner) continue;
            if (bk > kStKMask) {
                this->flag(kErrKOverflow);
                continue;
            }
            const uint32_t t = sw & kNone10;  // static info of the untouched word
            if (t != kNone10) {  // a special: offer the walk label to the table
                View c;
                this->view_walk(bb, bk, this->sp[t].rk, c);
                this->try_improve(t, c);
                continue;
            }
            this->st_state(w, kStSettled | parN | (bb << kStBShift) | bk);
            const uint32_t i = atomicAdd(&sh->cnt[cn], 1u);
            this->st_idx(Fn, i, w);
            if (p.use_soe) {
                const uint32_t r = (sw >> 10) & kNone10;
                if (r != kNone10 && !fired[r]) atomicMin(best64 + r, ((unsigned long long)bp << 32) | rank[w]);
            }
        }
    }

    __device__ __forceinline__ void solve(uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t tid = threadIdx.x;
        this->init_source(s_idx);
        for (uint32_t t = tid; t <= p.NS; t += kBS) {
            best64[t] = kInf64;
            fired[t] = 0;
        }
        if (tid == 0) {
            sh->cnt[0] = sh->cnt[1] = 0;
            sh->lb = 0;
            sh->L = 0;
            sh->done = 0;
            sh->jump = 0;
            sh->nbnd = 1;
            sh->ranked = 1;
            bnd[0] = 0;
            prio[0] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            this->seed_root();
            View st;
            this->view_start(st);
            const uint32_t ts = this->special_of(src);
            if (ts != kNone10) {
                this->try_improve(ts, st);
            } else {
                this->st_state(src, kStSettled);  // level 0 (parity 0), walk (0,0) = the start label
                sh->cnt[0] = 1;
                this->st_idx(F0, 0, src);
                const uint32_t r = this->region_of(src);
                if (p.use_soe && r != kNone10) {  // [SoE src -> nearest campfire]
                    View c;
                    this->soe_from_plain(0, 0, this->src_rk, r, c);
                    this->try_improve(r, c);
                    fired[r] = 1;
                }
            }
            this->seed_scrolls();
        }
        __syncthreads();
        MR_STAMP(*stamps, 0);  // init
        for (uint32_t guard = 0;; ++guard) {
            // ---- specials of level L (wave 0) ----
            if (tid < 64) {
                const uint32_t L = sh->L;
                const uint32_t cur = sh->lb;
                if (p.use_soe) fire_regions();
                MR_STAMP(*stamps, 1);  // fire regions
                const uint32_t par = (L & 1u) ? kStPar : 0u;
                auto on_settle = [&](uint32_t s, uint32_t vs, bool boundary) {
                    if (lane_id() == 0) {
                        const uint32_t i = sh->cnt[cur]++;
                        this->st_idx(frontier(cur), i, vs);
                        if (boundary) bnd[sh->nbnd++] = s;
                    }
                    wave_sync();
                };
                if (p.NS <= 63) {
                    this->specials_reg(L, par, on_settle);
                } else {
                    for (uint32_t it = 0; it <= p.NS; ++it) {
                        const uint32_t s = this->argmin_special(L);
                        if (s == kNone32) break;
                        const bool boundary = this->settle_special(s, par);
                        on_settle(s, this->sp[s].v, boundary);
                    }
                }
                MR_STAMP(*stamps, 2);  // specials Dijkstra
                const uint32_t done = this->dsts_done();
                const uint32_t n = sh->cnt[cur];
                if (n == 0) {  // empty frontier: jump to the next special level
                    const unsigned long long smin = this->min_special_key();
                    if (lane_id() == 0) {
                        sh->jump = 1;
                        sh->done = (smin == kInf64 || done) ? 1u : 0u;
                        if (smin != kInf64) sh->L = uint32_t(smin);
                    }
                } else {
                    // with a linear run time (Fleetfoot 0 / out of range) the order of
                    // boundaries does not depend on the level: re-rank only when one is added
                    if (p.ff_num != p.ff_den || sh->ranked != sh->nbnd) {
                        rank_boundaries(L + 1);
                        if (lane_id() == 0) sh->ranked = sh->nbnd;
                    }
                    if (lane_id() == 0) {
                        sh->jump = 0;
                        sh->done = done;
                        sh->cnt[cur ^ 1u] = 0;
                    }
                }
                MR_STAMP(*stamps, 3);  // next level / ranking
            }
            __syncthreads();
            MR_STAMP(*stamps, 4);  // barrier after specials
            if (sh->done) break;
            if (guard > p.V + p.NS + 64u) {
                this->flag(kErrBucket);
                break;
            }
            if (sh->jump) continue;
            // ---- claim level L+1 from the level-L frontier (all threads) ----
            {
                const uint32_t L = sh->L, cur = sh->lb, n = sh->cnt[cur];
                const IdxT *Fc = frontier(cur);
                IdxT *Fn = frontier(cur ^ 1u);
                for (uint32_t i = tid; i < n; i += kBS) claim_from(this->ld_idx(Fc, i), L, Fn, cur ^ 1u);
#ifdef MR_STAMPS
                if (tid == 0) stamps->acc[7] += n;  // frontier vertices processed
#endif
            }
            MR_STAMP(*stamps, 5);  // own claims
            __syncthreads();
            if (tid == 0) {
                sh->lb ^= 1u;
                sh->L += 1;
            }
            __syncthreads();
            MR_STAMP(*stamps, 6);  // claim barriers
        }
        this->write_outputs(s_idx);
        __syncthreads();
    }
};

// ===================================================================================
// Generic bucketed solver (Time- or Money-first comparators)
// ===================================================================================
template <bool G, class IdxT>
struct GenericSolver : Core<G> {
    using Core<G>::a;
    using Core<G>::sh;
    using Core<G>::R;
    using Core<G>::state;
    using Core<G>::src;
    using Core<G>::P;
    using Core<G>::rank;
    using Core<G>::sinfo;
    using Core<G>::counter;
    IdxT *L0b, *dirty;  // the three bucket lists are L0b + i * lstride
    uint32_t lstride;
    uint32_t *best;
    uint32_t *fired;

    __device__ __forceinline__ IdxT *lbuf(uint32_t i) const { return L0b + i * lstride; }

    __device__ __forceinline__ void mark_dirty(uint32_t v, uint32_t n) const {
        const DevParams &p = P;
        if (n == kNone32 || v == p.vc || n == p.vc) return;
        const uint32_t old = this->or_state(n, kStDirty);
        if (old & (kStSettled | kStDirty)) return;
        const uint32_t i = atomicAdd(&sh->nd, 1u);
        this->st_idx(dirty, i, n);
    }
    __device__ __forceinline__ void region_offer(uint32_t r, uint32_t v) const {
        uint32_t cur = best[r];
        for (;;) {
            if (cur != kNone32) {
                const uint32_t su = this->ld_state(cur), sv = this->ld_state(v);
                View xu, xv;
                this->view_walk((su >> kStBShift) & kNone10, su & kStKMask, rank[cur], xu);
                this->view_walk((sv >> kStBShift) & kNone10, sv & kStKMask, rank[v], xv);
                if (this->cmp_view(xu, kOwn, xv, kOwn) <= 0) return;
            }
            const uint32_t prev = atomicCAS(best + r, cur, v);
            if (prev == cur) return;
            cur = prev;
        }
    }
    __device__ __forceinline__ void settle_plain(uint32_t v) const {
        const DevParams &p = P;
        this->or_state(v, kStSettled);
        if (p.use_soe) {
            const uint32_t r = this->region_of(v);
            if (r != kNone10 && !fired[r]) region_offer(r, v);
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) mark_dirty(v, this->nbr(v, d));
    }
    __device__ __forceinline__ void fire_regions() const {
        const DevParams &p = P;
        for (uint32_t t = 1 + lane_id(); t <= p.NS; t += 64) {
            const uint32_t u = best[t];
            if (u == kNone32) continue;
            best[t] = kNone32;
            fired[t] = 1;
            if (R[t].state() == 2) continue;
            const uint32_t su = this->ld_state(u);
            View c;
            this->soe_from_plain((su >> kStBShift) & kNone10, su & kStKMask, rank[u], t, c);
            this->try_improve(t, c);
        }
        wave_sync();
    }
    __device__ __forceinline__ void pull(uint32_t w) const {
        const DevParams &p = P;
        // a vertex marked dirty may have been settled later in the same bucket
        if (this->ld_state(w) & kStSettled) return;
        const uint32_t t = this->special_of(w);
        uint32_t bb = kNone10, bk = 0;
        if (w != p.vc) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const uint32_t n = this->nbr(w, d);
                if (n == kNone32 || n == p.vc) continue;
                const uint32_t sn = this->ld_state(n);
                if (!(sn & kStSettled)) continue;
                const uint32_t b = (sn >> kStBShift) & kNone10, k = (sn & kStKMask) + 1u;
                if (k > kStKMask) {
                    this->flag(kErrKOverflow);
                    continue;
                }
                if (bb == kNone10) {
                    bb = b;
                    bk = k;
                } else if (b == bb) {
                    if (k < bk) bk = k;  // same boundary: fewer legs is smaller in every order
                } else {
                    View xc, xb;  // same endpoint: its rank cannot decide, any value serves
                    this->view_walk(b, k, 0, xc);
                    this->view_walk(bb, bk, 0, xb);
                    if (this->cmp_view(xc, kOwn, xb, kOwn) < 0) {
                        bb = b;
                        bk = k;
                    }
                }
            }
        }
        if (t != kNone10) {
            this->st_state(w, this->ld_state(w) & ~kStDirty);
            if (bb != kNone10) {
                View c;
                this->view_walk(bb, bk, this->sp[t].rk, c);
                this->try_improve(t, c);
            }
            return;
        }
        const uint32_t old = this->ld_state(w);
        if (bb == kNone10) {  // cannot happen: a dirty vertex has a settled StandardMove neighbour
            this->st_state(w, old & ~kStDirty);
            this->flag(kErrBucket);
            return;
        }
        this->st_state(w, (bb << kStBShift) | bk);
        if (((old >> kStBShift) & kNone10) == kNone10) {  // first touch: list it (its bucket is final)
            View c;
            this->view_walk(bb, bk, 0, c);  // metrics only
            const unsigned long long X = this->key_of(c.m0, c.m1, c.m2), B = sh->B;
            uint32_t j;
            if (X == B + 1) j = 1;
            else if (X == B + 2) j = 2;
            else {
                this->flag(kErrBucket);
                return;
            }
            const uint32_t buf = (sh->lb + j) % 3u;
            const uint32_t i = atomicAdd(&sh->cnt[buf], 1u);
            this->st_idx(lbuf(buf), i, w);
        }
    }
    __device__ __forceinline__ void next_bucket(uint32_t s_idx) const {
        const unsigned long long smin = this->min_special_key();
        const uint32_t all_done = this->dsts_done();
        if (lane_id() == 0) {
            const unsigned long long B = sh->B;
            const uint32_t lb = sh->lb;
            const uint32_t n1 = sh->cnt[(lb + 1) % 3u], n2 = sh->cnt[(lb + 2) % 3u];
            unsigned long long nb = n1 ? B + 1 : (n2 ? B + 2 : kInf64);
            if (smin < nb) nb = smin;
            sh->cnt[lb] = 0;
            if (nb == B + 1) sh->lb = (lb + 1) % 3u;
            else if (nb == B + 2) sh->lb = (lb + 2) % 3u;
            sh->nd = 0;
            sh->B = nb;
            sh->done = (nb == kInf64 || all_done) ? 1u : 0u;
        }
    }
    __device__ __forceinline__ void solve(uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t tid = threadIdx.x;
        this->init_source(s_idx);
        for (uint32_t t = tid; t <= p.NS; t += kBS) {
            best[t] = kNone32;
            fired[t] = 0;
        }
        if (tid == 0) {
            sh->cnt[0] = sh->cnt[1] = sh->cnt[2] = 0;
            sh->lb = 0;
            sh->nd = 0;
            sh->B = 0;
            sh->done = 0;
        }
        __syncthreads();
        if (tid == 0) {
            this->seed_root();
            View st;
            this->view_start(st);
            const uint32_t ts = this->special_of(src);
            if (ts != kNone10) {
                this->try_improve(ts, st);
            } else {
                this->st_state(src, 0u);  // walk label (0,0) = the start label
                sh->cnt[0] = 1;
                this->st_idx(L0b, 0, src);
            }
            this->seed_scrolls();
        }
        __syncthreads();
        for (uint32_t guard = 0;; ++guard) {
            {
                const uint32_t lb = sh->lb, n0 = sh->cnt[lb];
                const IdxT *L0 = lbuf(lb);
                for (uint32_t i = tid; i < n0; i += kBS) settle_plain(this->ld_idx(L0, i));
            }
            __syncthreads();
            if (tid < 64) {
                if (p.use_soe) fire_regions();
                const unsigned long long B = sh->B;
                auto on_settle = [&](uint32_t, uint32_t vs, bool) {
                    if (lane_id() < 4) mark_dirty(vs, this->nbr(vs, int(lane_id())));
                    wave_sync();
                };
                if (p.NS <= 63) {
                    this->specials_reg(B, 0u, on_settle);
                } else {
                    for (uint32_t it = 0; it <= p.NS; ++it) {
                        const uint32_t s = this->argmin_special(B);
                        if (s == kNone32) break;
                        this->settle_special(s, 0u);
                        on_settle(s, this->sp[s].v, false);
                    }
                }
            }
            __syncthreads();
            {
                const uint32_t nd = sh->nd;
                for (uint32_t i = tid; i < nd; i += kBS) pull(this->ld_idx(dirty, i));
            }
            __syncthreads();
            if (tid < 64) next_bucket(s_idx);
            __syncthreads();
            if (sh->done) break;
            if (guard > p.V + p.NS + 64u) {
                this->flag(kErrBucket);
                break;
            }
        }
        this->write_outputs(s_idx);
        __syncthreads();
    }
};

// End of a workgroup (thread 0, after a barrier): add its written records; in the
// pass's last kernel the last workgroup to finish publishes the pass's counts and
// zeroes the per-pass counters for the next pass.
__device__ __forceinline__ void finish_launch(const KArgs *__restrict__ a, uint32_t written,
                                              uint32_t nblocks = 0xFFFFFFFFu) {
    uint32_t *c = a->counter;
    if (!a->last_launch) {
        if (written) atomicAdd(c + kCtrWritten, written);
        return;
    }
    // No fence before the count: the counters this workgroup added to were updated by
    // atomics whose returned values it waited for, and the records need no ordering
    // (the host reads them after the kernel).  An agent-scope release here writes the
    // XCD's L2 back: one per workgroup made the fill 1.7x slower.
    // One atomic per workgroup: {done, written} share a 64-bit word (a grid's workgroups
    // end together, and same-address atomics serialise at ~11 ns each)
    static_assert(kCtrDone % 2 == 0 && kCtrWritten == kCtrDone + 1, "counter pair");
    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long *>(c + kCtrDone),
                                             ((unsigned long long)written << 32) | 1ull);
    // the grid's last workgroup (nblocks: the workgroups that count, when a launch fuses
    // two kernels' work)
    const uint32_t nb = nblocks != 0xFFFFFFFFu ? nblocks : gridDim.x * gridDim.y * gridDim.z;
    if (uint32_t(old) == nb - 1) {
        __threadfence();
        const uint32_t fb = atomicAdd(c + kCtrFbCount, 0u), wr = uint32_t(old >> 32) + written,
                       ov = atomicAdd(c + kCtrOvf, 0u);
        c[kCtrLastFb] = fb;
        c[kCtrLastWritten] = wr;
        c[kCtrLastOvf] = ov;
        c[kCtrLastCert] = atomicAdd(c + kCtrCertDone, 0u);
        c[kCtrLastRelist] = atomicAdd(c + kCtrRelist, 0u);
        c[kCtrRelist] = 0;
        c[kCtrCertDone] = 0;
        c[kCtrOvf] = 0;
        c[kCtrDequeue] = 0;
        c[kCtrFbCount] = 0;
        c[kCtrFbDequeue] = 0;
        c[kCtrCert] = 0;
        c[kCtrWritten] = 0;
        c[kCtrDone] = 0;
        __threadfence();
    }
}

// A source handed to the SSSP launch: fallback entry i, with its certificate slot
// (kNone32: none, the SSSP kernel solves it)
// (kNone32: none, the SSSP kernel solves it; kFbStaged: its table is staged for
// cert_select_kernel).  Returns i.
__device__ __forceinline__ uint32_t push_fallback(const KArgs *__restrict__ a, uint32_t *counter, uint32_t s_idx,
                                                  uint32_t slot) {
    const uint32_t i = atomicAdd(counter + kCtrFbCount, 1u);
    a->fb_list[i] = s_idx;
    if (a->fb_cert) a->fb_cert[i] = slot;
    return i;
}

// ===================================================================================
// Hub solver (linear StandardMove run time: Fleetfoot level 0 or out of range)
// ===================================================================================
// With a linear run time, extending two walk labels by the same StandardMove
// preserves their order (metrics shift equally, lengths and prefixes are
// unchanged), so every plain vertex's label is min over boundaries b of
// walk(b, d_b(v)), d_b = grid distance avoiding the Center (Manhattan, +2 when
// the straight line crosses it).  One wave per source runs an exact Dijkstra
// over the specials (lane t owns special t) whose edges are those walks, the
// CentralMove/caravan/SoE edges, and SoE edges from each region's nearest cell
// (precomputed table).  The only step that is not order-preserving — extending
// a boundary special whose label ties a walk candidate on all three metrics
// (the tie is then decided by length/commands, which a StandardMove can flip) —
// is detected and such sources are re-solved by the SSSP kernel.  DESIGN.md §3b.
__host__ __device__ __forceinline__ uint32_t walk_dist(int ax, int ay, int bx, int by) {
    uint32_t d = uint32_t(abs(ax - bx) + abs(ay - by));
    if ((ay == 0 && by == 0 && ax != 0 && bx != 0 && ((ax < 0) != (bx < 0))) ||
        (ax == 0 && bx == 0 && ay != 0 && by != 0 && ((ay < 0) != (by < 0))))
        d += 2;  // both on one axis, on opposite sides of the Center: detour
    return d;
}

// Lanes are split into SPW segments of LPS = 64 / SPW lanes; segment h solves its
// own source with lane t (within the segment) owning special t.  Per-source values
// (source, settled special, boundary count) are segment-uniform per-lane values.
template <uint32_t LPS>
__device__ __forceinline__ uint32_t seg_min_u32(uint32_t x) {
    x = dpp_min<0x111, 0xF>(x);  // row_shr:1
    x = dpp_min<0x112, 0xF>(x);  // row_shr:2
    x = dpp_min<0x114, 0xF>(x);  // row_shr:4
    x = dpp_min<0x118, 0xF>(x);  // row_shr:8
    x = dpp_min<0x142, 0xA>(x);  // row_bcast:15: lanes 31 and 63 hold the two 32-lane minima
    if constexpr (LPS == 64) {
        x = dpp_min<0x143, 0xC>(x);  // row_bcast:31
        return bcast(x, 63);
    } else {
        const uint32_t lo = bcast(x, 31), hi = bcast(x, 63);
        return lane_id() >= 32 ? hi : lo;
    }
}
template <uint32_t LPS>
__device__ __forceinline__ void narrow_seg(bool &c, uint32_t key) {
    const uint32_t m = seg_min_u32<LPS>(c ? key : 0xFFFFFFFFu);
    c = c && key == m;
}
// this lane's segment of a wave ballot
template <uint32_t LPS>
__device__ __forceinline__ unsigned long long seg_bits(unsigned long long bal) {
    if constexpr (LPS == 64) return bal;
    else return lane_id() >= 32 ? (bal >> 32) : (bal & 0xFFFFFFFFull);
}
template <uint32_t LPS>
__device__ __forceinline__ uint32_t seg_max_u32(uint32_t x) {
    return ~seg_min_u32<LPS>(~x);
}
// every segment of wave ballot `bal` has at most one lane set (SALU: the ballot is uniform)
template <uint32_t LPS>
__device__ __forceinline__ bool seg_single(unsigned long long bal) {
    if constexpr (LPS == 64) return __popcll(bal) <= 1;
    else return __popc(uint32_t(bal)) <= 1 && __popc(uint32_t(bal >> 32)) <= 1;
}
// Keeps in c, per segment, the lanes holding the smallest (k1, k2, k3, len) and returns
// the final ballot; stops once every segment has at most one lane left.  The first
// round narrows on k1 and k2 packed into one word (k1 saturated to W1 bits, k2 to
// 32 - W1): packing is monotone, so the survivors are exactly the lanes of the least
// (k1, k2) unless the least packed word holds a saturated field, in which case k1 and
// k2 get rounds of their own.
template <uint32_t LPS, uint32_t W1>
__device__ __forceinline__ unsigned long long seg_narrow(bool &c, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t len) {
    constexpr uint32_t M1 = (1u << W1) - 1u, M2 = (W1 == 0u) ? 0xFFFFFFFFu : (0xFFFFFFFFu >> W1);
    unsigned long long bal = __ballot(c);
    if (seg_single<LPS>(bal)) return bal;
    const uint32_t pk = (min(k1, M1) << (32u - W1)) | min(k2, M2);
    const uint32_t m = seg_min_u32<LPS>(c ? pk : 0xFFFFFFFFu);
    c = c && pk == m;
    bal = __ballot(c);
    if (seg_single<LPS>(bal)) return bal;
    if (__any(c && ((m >> (32u - W1)) == M1 || (m & M2) == M2))) {  // a saturated field: exact rounds
        narrow_seg<LPS>(c, k1);
        narrow_seg<LPS>(c, k2);
        bal = __ballot(c);
        if (seg_single<LPS>(bal)) return bal;
    }
    narrow_seg<LPS>(c, k3);
    bal = __ballot(c);
    if (seg_single<LPS>(bal)) return bal;
    narrow_seg<LPS>(c, len);
    return __ballot(c);
}

template <uint32_t SPW>
struct HubSolver : Core<false> {
    static constexpr uint32_t LPS = 64 / SPW;
    uint32_t *bnd;          // LDS: this segment's boundary list (table indices; bnd[0] = 0, the source)
    uint32_t *lexs;         // LDS: all-destinations mode, rank of each table entry among the boundaries
    const uint32_t *nearS;  // LDS: region rows {distance, rank} of every special (row t at t*2*nreg)
    uint32_t *srow;         // LDS: this segment's region row of its source
    uint32_t *blk;          // LDS: this segment's blocking specials (see avail)
    uint32_t nreg;
    uint32_t written = 0;   // result records this lane emitted for (segment lane 0)
#ifdef MR_STAMPS
    mutable unsigned long long hs_last = 0, hs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    __device__ void hmark(int slot) const {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        hs[slot] += t - hs_last;
        hs_last = t;
    }
#define MR_HSTAMP(slot) hmark(slot)
#define MR_HCOUNT(slot, n) (hs[slot] += (n))
#else
#define MR_HSTAMP(slot) \
    do {                \
    } while (0)
#define MR_HCOUNT(slot, n) \
    do {                   \
    } while (0)
#endif
    __device__ __forceinline__ static uint32_t seg_lane() { return lane_id() % LPS; }

    // tentative labels live only in registers (lane t = special t); the LDS table
    // receives a label when it settles (command chains and list compares read it).
    // The update is a per-field select under an explicit mask, never a divergent
    // block assignment.
    // (own: the rank of the lane's special, for the rare command-list compare)
    __device__ __forceinline__ void improve_reg(bool active, uint32_t &st, RLab &my, const View &c, uint32_t own) const {
        bool take = active && st != 2;
        if (take && st == 1) {
            const int cm = cmp_metrics(c.m0, c.m1, c.m2, my.m0, my.m1, my.m2);
            if (cm != 0) take = cm < 0;
            else if (c.len != rl_len(my)) take = c.len < rl_len(my);
            else take = cmp_list(c, kOwn, expand(my, own), kOwn) < 0;
        }
        sel_rlab(take, my, compact(c));
        st = take ? 1u : st;
    }
    // Per segment, the settle candidate: the smallest tentative label, resolved
    // metric by metric on the DPP network (exit once every segment has at most one
    // lane left).  Exact ties of metrics and length publish the tied labels to the
    // table and compare command lists.  Returns the segment lane, or kNone32.
    __device__ __forceinline__ uint32_t select_reg(bool c, const RLab &my, uint32_t own) const {
        const DevParams &p = P;
        const uint32_t mm3[3] = {my.m0, my.m1, my.m2};
        // (the packed first round: a time-first key takes 20 bits, legs or money 16)
        unsigned long long bal;
        if (p.perm[0] == 2u)
            bal = seg_narrow<LPS, 20u>(c, mm3[p.perm[0]], mm3[p.perm[1]], mm3[p.perm[2]], rl_len(my));
        else
            bal = seg_narrow<LPS, 16u>(c, mm3[p.perm[0]], mm3[p.perm[1]], mm3[p.perm[2]], rl_len(my));
        const unsigned long long m = seg_bits<LPS>(bal);
#ifndef MR_HUB_SETTLE_TIES
        // Exact ties of metrics and length between specials need no list compare: either
        // may settle first (every candidate out of a settled special is strictly greater
        // than its label in (metrics, length)), so the lowest lane
        (void)own;
        return m ? uint32_t(__ffsll((long long)m) - 1) : kNone32;
#endif
        uint32_t win = __popcll(m) == 1 ? uint32_t(__ffsll((long long)m) - 1) : kNone32;
        if (!seg_single<LPS>(bal)) {
            const bool tied = __popcll(m) > 1;
            const uint32_t t = seg_lane();
            if (tied && c) write_rec(t, expand(my, own), 1);
            wave_sync();
            uint32_t mm = (tied && c) ? t : kNone32;
#pragma unroll
            for (int off = LPS / 2; off >= 1; off >>= 1) {
                const uint32_t o = __shfl_xor(mm, off, 64);
                if (o != kNone32 && (mm == kNone32 || cmp_entries(o, mm) < 0)) mm = o;
            }
            if (tied) win = mm;
        }
        return win;
    }
    __device__ __forceinline__ void note_walk(bool on, const View &c, uint32_t &bwh, uint32_t &b0, uint32_t &b1,
                                              uint32_t &b2) const {
        const bool take = on && (!bwh || cmp_metrics(c.m0, c.m1, c.m2, b0, b1, b2) < 0);
        bwh = take ? 1u : bwh;
        b0 = take ? c.m0 : b0;
        b1 = take ? c.m1 : b1;
        b2 = take ? c.m2 : b2;
    }
    // walks and SoE-region edges from boundary b (label lb, at bx, by) into lane t's special
    __device__ __forceinline__ void relax_boundary(bool live, const View &lb, uint32_t b, int bx, int by, uint32_t t,
                                                   uint32_t &st, RLab &my, const SpecialStatic &ss, uint32_t &bwh,
                                                   uint32_t &b0, uint32_t &b1, uint32_t &b2) const {
        const DevParams &p = P;
        live = live && st != 2;
        relax_walk(live, lb, b, bx, by, t, st, my, ss, bwh, b0, b1, b2);
        if (p.use_soe) {  // [Std{d} b->u, SoE u->c] from the region cell u nearest to b
            uint32_t d = kNone32, u = 0;
            if (live && ss.rid != kNone10) {
                const uint32_t *e = (b == 0 ? srow : nearS + 2u * b * nreg) + 2u * ss.rid;
                d = e[0];
                u = e[1];
            }
            relax_soe(live, lb, b, t, st, my, ss, d, u);
        }
    }
    // the walk from boundary b into lane t's special: not into the Center (entry 1)
    // nor b's own cell
    __device__ __forceinline__ void relax_walk(bool live, const View &lb, uint32_t b, int bx, int by, uint32_t t,
                                               uint32_t &st, RLab &my, const SpecialStatic &ss, uint32_t &bwh,
                                               uint32_t &b0, uint32_t &b1, uint32_t &b2) const {
        const bool on = live && st != 2 && t != 1 && t != b && !(b == 0 && ss.v == src);
        View c;
        view_walk_lab(lb, b, walk_dist(bx, by, ss.x, ss.y), ss.rk, c);
        note_walk(on, c, bwh, b0, b1, b2);
        improve_reg(on, st, my, c, ss.rk);
    }
    // the SoE-region edge from boundary b into lane t's special, with b's region row
    // entry {d, u} for t's region already read
    __device__ __forceinline__ void relax_soe(bool live, const View &lb, uint32_t b, uint32_t t, uint32_t &st, RLab &my,
                                              const SpecialStatic &ss, uint32_t d, uint32_t u) const {
        const DevParams &p = P;
        (void)t;
        {
            const bool on = live && st != 2 && d != kNone32 && (d != 0 || b == 0);  // d == 0, b special: its own SoE edge
            View c;
            view_walk_lab(lb, b, on ? d : 0u, u, c);
            if (d == 0) {  // b is the source, standing on the region: [SoE src->c]
                c.ntail = 1;
                c.t0 = Cmd{kSoE << 29, src_rk, ss.rk};
                c.m1 = p.soe_cost;
            } else {
                c.m1 = add32(c.m1, p.soe_cost);
                c.len += 1;
                c.ntail = 2;
                c.t1 = Cmd{kSoE << 29, u, ss.rk};
            }
            improve_reg(on, st, my, c, ss.rk);
        }
    }

    // A boundary special s whose label tied a walk candidate on all three metrics and
    // won on length/commands is a blocker: past s that walk's extension can win (the
    // run merges, so its length stops growing), yet Dijkstra never offers it through
    // s.  walk(b, d_b(v)) is therefore only certain when some shortest walk from b to
    // v avoids the blockers.  A strict metric loss needs no care: the winner at s
    // stays ahead along every extension, so such a b is never the closed-form minimum
    // there.  Returns false when it cannot rule the blockers out: several of them in
    // the b-v rectangle, the Center in it too, a Center detour near one, or a
    // one-cell-wide rectangle through one.  (One blocker inside a rectangle at least
    // two cells wide leaves a monotone walk around it.)
    __device__ __forceinline__ bool avail(uint32_t nbk, uint32_t b, int bx, int by, int vx, int vy) const {
        if (nbk == 0) return true;
        const int x0 = min(bx, vx), x1 = max(bx, vx), y0 = min(by, vy), y1 = max(by, vy);
        const bool detour = walk_dist(bx, by, vx, vy) != uint32_t(x1 - x0 + y1 - y0);
        uint32_t inside = 0;
        for (uint32_t i = 0; i < nbk; ++i) {
            const uint32_t k = blk[i];
            if (k == b) continue;
            const int kx = sp[k].x, ky = sp[k].y;
            if (kx >= x0 && kx <= x1 && ky >= y0 && ky <= y1) inside += 1;
            else if (detour && kx >= x0 - 1 && kx <= x1 + 1 && ky >= y0 - 1 && ky <= y1 + 1) inside += 2;
        }
        if (inside == 0) return true;
        if (inside > 1 || detour) return false;
        if (x0 <= 0 && 0 <= x1 && y0 <= 0 && 0 <= y1) return false;  // the Center in the rectangle too
        return x0 != x1 && y0 != y1;
    }
    // the settled label x of special (tx, ty): its walk, or the walk to the cell its
    // Scroll of Escape is read from, must be certain (labels of other kinds extend
    // settled labels and are exact)
    __device__ __forceinline__ bool label_avail(const View &x, uint32_t nbk, int tx, int ty, int sx, int sy) const {
        if (nbk == 0) return true;
        const uint32_t k0 = x.t0.kp >> 29;
        if (k0 != kStandard) return true;
        int bx, by;
        bpos(x.parent, sx, sy, bx, by);
        if (x.ntail == 1) return avail(nbk, x.parent, bx, by, tx, ty);
        const uint32_t u = a->rank_inv[x.t0.to];
        return avail(nbk, x.parent, bx, by, int(u % P.S) - int(P.H), int(u / P.S) - int(P.H));
    }

    // ---- non-linear run times (Fleetfoot 1..3; DESIGN.md section 3a'') ------------
    // With f(k) = ceil(180 k num / den) a StandardMove extension shifts the time gap of
    // two walks (k' = k + m legs) by delta = f(k'+1) - f(k') - (f(k+1) - f(k)) in
    // {-1, 0, 1}, 0 whenever m = 0; the other metrics, lengths and command lists keep
    // their order.  So a walk q that beats walk(b, .) at a cell u can lose to it one
    // step further only when every metric before Time in the comparator ties at u, the
    // time gap there is -1 or 0 and delta = +1.  If no boundary can do that on a
    // shortest b-path to v, walk(b, .) wins along the whole path, and the closed-form
    // label of v is the reference's (the last cell where b lost would need such a q).
    __device__ __forceinline__ bool ff_linear() const { return P.ff_num == P.ff_den; }
    // the gap f(k + m) - f(k) takes one of {lo, hi} for every k (cm = 180 m num / den)
    __device__ __forceinline__ bool gap_hits(long long d0, long long m) const {
        const long long a = 180ll * (long long)P.ff_num * (m < 0 ? -m : m), den = (long long)P.ff_den;
        long long lo = floor_div(a, den), hi = floor_div(a + den - 1, den);
        if (m < 0) {
            const long long t = lo;
            lo = -hi;
            hi = -t;
        }
        return d0 + lo == -1 || d0 + lo == 0 || d0 + hi == -1 || d0 + hi == 0;
    }
    // Can boundary q (at qx, qy) beat walk(b, .) non-isotonically somewhere on a shortest
    // b-path to (vx, vy)?  Every cell of those paths lies in the b-v rectangle, where
    // m = d_q(u) - d_b(u) runs within [L1(q, v) - L1(b, v), L1(q, b) + 2].
    __device__ __forceinline__ bool near_tie(uint32_t q, int qx, int qy, uint32_t b, int bx, int by, int vx,
                                             int vy) const {
        const DevParams &p = P;
        const int mlo = abs(qx - vx) + abs(qy - vy) - abs(bx - vx) - abs(by - vy);
        const int mhi = abs(qx - bx) + abs(qy - by) + 2;
        const long long d0 = (long long)R[q].m[2] - (long long)R[b].m[2];
        const bool legs_before = p.perm[0] == 0 || (p.perm[1] == 0 && p.perm[0] != 2);
        const bool money_before = p.perm[0] == 1 || (p.perm[1] == 1 && p.perm[0] != 2);
        if (money_before && R[q].m[1] != R[b].m[1]) return false;
        if (legs_before) {  // the legs tie where m = L_b - L_q
            const long long m = (long long)R[b].m[0] - (long long)R[q].m[0];
            return m != 0 && m >= mlo && m <= mhi && gap_hits(d0, m);
        }
        // d0 + 180 m num / den within (-2, 1): m next to -d0 den / (180 num)
        const long long c = 180ll * (long long)p.ff_num, num = (-2 - d0) * (long long)p.ff_den;
        const long long m0 = floor_div(num, c);
        for (long long m = m0 - 1; m <= m0 + 2; ++m)
            if (m != 0 && m >= mlo && m <= mhi && gap_hits(d0, m)) return true;
        return false;
    }
    // Along one L-shaped shortest path from b to v (x first, or y first), is there a
    // cell u (v excluded) where walk(q, .) beats walk(b, .) and the next leg w of the
    // path flips their order?  That needs the metrics before Time to tie at u, q's
    // distance to grow on that leg, a time gap of -1 or 0 at u that does not shrink
    // (delta >= 0), q ahead at u and b ahead at w on (gap, tail) — the tail being the
    // metric after Time, then the length (a walk from q's own cell appends a command:
    // the flip of a blocker), then the command lists: two walks of equal length that
    // both append a command compare as q's and b's own lists do (`lists`, the same at
    // every cell: their last commands end at different cells, so the lists differ);
    // other list ties count as undecided.  A path through the Center is not a walk: true.
    __device__ __forceinline__ bool path_tie(uint32_t q, int qx, int qy, uint32_t b, int bx, int by, int vx, int vy,
                                             bool x_first, int lists) const {
        const DevParams &p = P;
        const bool legs_before = p.perm[0] == 0 || (p.perm[1] == 0 && p.perm[0] != 2);
        const bool money_before = p.perm[0] == 1 || (p.perm[1] == 1 && p.perm[0] != 2);
        // the metric after Time, if any (legs 0, money 1; 3 = none)
        const uint32_t after = p.perm[0] == 2 ? p.perm[1] : (p.perm[1] == 2 ? p.perm[2] : 3u);
        if (money_before && R[q].m[1] != R[b].m[1]) return false;
        const int sx = vx > bx ? 1 : -1, sy = vy > by ? 1 : -1;
        const int K = abs(vx - bx) + abs(vy - by), kx = abs(vx - bx), ky = K - kx;
        const long long tb = R[b].m[2], tq = R[q].m[2], lb = R[b].m[0], lq = R[q].m[0];
        const long long mb = R[b].m[1], mq = R[q].m[1];
        // the walks' lengths (the source's walk replaces its NoMove: length 1)
        const long long nq0 = q == 0 ? 1 : R[q].len(), nq1 = q == 0 ? 1 : R[q].len() + 1;
        const long long nb0 = b == 0 ? 1 : R[b].len(), nb1 = b == 0 ? 1 : R[b].len() + 1;
        auto cell = [&](int k, int &ux, int &uy) {
            if (x_first) {
                ux = k < kx ? bx + sx * k : vx;
                uy = k < kx ? by : by + sy * (k - kx);
            } else {
                uy = k < ky ? by + sy * k : vy;
                ux = k < ky ? bx : bx + sx * (k - ky);
            }
        };
        // Skips: on a run of steps where q moves away from the path (its distance grows by
        // one a step, no axis crossed) every quantity below is constant or periodic in k
        // with period den (run_time(k + den) = run_time(k) + 180 num), so a run of at least
        // den steps is decided by one period of the time gaps and skipped whole (a shorter
        // one after den checked steps); a stretch approaching q cannot flip and is skipped
        // too (tests/test_path_tie_skip.py restates this loop and checks it against the
        // cell-by-cell scan).
        // the order after Time at a cell (dd, kk: q's and b's legs there): -1 q ahead, +1 b
        // ahead, 0 undecided (the command lists)
        auto tail = [&](long long dd, long long kk) -> int {
            if (after == 0) {
                if (lq + dd != lb + kk) return lq + dd < lb + kk ? -1 : 1;
            } else if (after == 1) {
                if (mq != mb) return mq < mb ? -1 : 1;
            }
            const long long nq = dd > 0 ? nq1 : nq0, nbb = kk > 0 ? nb1 : nb0;
            if (nq != nbb) return nq < nbb ? -1 : 1;
            return (dd > 0 && kk > 0) ? lists : 0;
        };
        const int den = int(p.ff_den);
        int ux, uy, run = 0;
        cell(0, ux, uy);
        uint32_t dq = walk_dist(qx, qy, ux, uy);
        for (int k = 0; k < K;) {
            if (ux == 0 && uy == 0) return true;
            {  // Approach skip: moving towards q's column (row), q's distance drops by one a step
                // until the walk reaches it (or the step before the axis being crossed: the
                // Center detour's term stays constant), and only a step on which it grows can flip
                const bool ax = x_first ? k < kx : k >= ky;
                const int seg = ax ? (x_first ? kx : K) : (x_first ? K : ky);
                const int c0 = ax ? ux : uy, qc = ax ? qx : qy, sd = ax ? sx : sy;
                if (sd * (c0 - qc) < 0) {
                    int j = min(seg, k + abs(c0 - qc));
                    if (c0 * sd < 0) j = min(j, k + abs(c0) - 1);
                    if (j > k + 1) {
                        k = j;
                        run = 0;
                        cell(k, ux, uy);
                        dq = walk_dist(qx, qy, ux, uy);
                        continue;
                    }
                }
            }
            int wx, wy;
            cell(k + 1, wx, wy);
            const uint32_t dqn = walk_dist(qx, qy, wx, wy);
            const bool tie_before = !legs_before || lq + dq == lb + k;
            if (tie_before && dqn > dq) {  // (q getting nearer stays ahead)
                const long long fq = run_time(dq), fb = run_time(uint32_t(k));
                const long long delta = ((long long)run_time(dqn) - fq) - ((long long)run_time(uint32_t(k) + 1) - fb);
                const long long gap = tq + fq - tb - fb;
                if ((gap == -1 || gap == 0) && delta >= 0) {
                    const bool q_beats_u = gap == -1 || tail(dq, k) != 1;
                    const long long gw = gap + delta;
                    const bool b_beats_w = gw > 0 || (gw == 0 && tail(dqn, k + 1) != -1);
                    if (q_beats_u && b_beats_w) return true;
                }
            }
            const bool along_x = x_first ? k < kx : k >= ky;
            const bool plain = k >= 1 && (along_x ? (ux != 0 && wx != 0 && sx * (ux - qx) >= 0)
                                                  : (uy != 0 && wy != 0 && sy * (uy - qy) >= 0));
            // the next step that is not plain: the segment's end, or the step before the one
            // whose cell lies on the axis being crossed
            int j = along_x ? (x_first ? kx : K) : (x_first ? K : ky);
            {
                const int c0 = along_x ? ux : uy, sd = along_x ? sx : sy;
                if (c0 * sd < 0) j = min(j, k + abs(c0) - 1);
            }
            // A plain run of at least den steps from here (q off the walk, so the tail is the
            // run's): its steps see every residue of k mod den, and the time gaps at a step
            // and the next are d0 + F(r), d0 + F(r + 1), F(r) = f(r + m) - f(r) with m = dq - k
            // constant on the run.  One period of F decides whether some step of the run
            // flips; the run is then skipped whole.
            if (plain && tie_before && dq > 0 && j - k >= den) {
                const int m = int(dq) - k, T = tail(dq, k);
                const long long d0 = tq - tb;
                const int base = den * ((max(0, -m) + den - 1) / den);  // (r + m >= 0)
                for (int i = 0; i < den; ++i) {
                    const int r = base + i;
                    const long long g = d0 + (long long)run_time(uint32_t(r + m)) - (long long)run_time(uint32_t(r));
                    const long long gw = d0 + (long long)run_time(uint32_t(r + 1 + m)) - (long long)run_time(uint32_t(r + 1));
                    if ((g == -1 || g == 0) && gw >= g && (g == -1 || T != 1) && (gw > 0 || (gw == 0 && T != -1)))
                        return true;
                }
                k = j;
                run = 0;
                cell(k, ux, uy);
                dq = walk_dist(qx, qy, ux, uy);
                continue;
            }
            run = plain ? run + 1 : 0;
            // (Legs before Time: the legs gap is constant on a plain run too, so a run that
            // starts untied stays untied and is skipped at once)
            if (run >= den || (plain && !tie_before)) {
                if (j > k + 1) {
                    k = j;
                    run = 0;
                    cell(k, ux, uy);
                    dq = walk_dist(qx, qy, ux, uy);
                    continue;
                }
            }
            ++k;
            ux = wx;
            uy = wy;
            dq = dqn;
        }
        return false;
    }
    // Which of the two L-paths from b to v does boundary q leave clean?  Bit 0: the
    // x-first path, bit 1: the y-first one (3 for q = b, the Center, kNone32 or a q
    // that fails near_tie; 0 when the b-v walks detour round the Center).  The label
    // is certain when one path is clean for every boundary: the argument above needs
    // ONE path on which no boundary flips.
    __device__ __forceinline__ uint32_t walk_clear(uint32_t q, uint32_t b, int vx, int vy, int sx, int sy) const {
        int bx, by;
        bpos(b, sx, sy, bx, by);
        if ((by == 0 && vy == 0 && bx != 0 && vx != 0 && (bx < 0) != (vx < 0)) ||
            (bx == 0 && vx == 0 && by != 0 && vy != 0 && (by < 0) != (vy < 0)))
            return 0u;  // shortest walks detour round the Center
        if (q == kNone32 || q == b || vert_of(q) == P.vc) return 3u;
        int qx, qy;
        bpos(q, sx, sy, qx, qy);
        if (!near_tie(q, qx, qy, b, bx, by, vx, vy)) return 3u;
        int lists = 0;  // the order of q's and b's command lists when their walks' lengths tie
        if (q != 0 && b != 0 && R[q].len() == R[b].len()) {
            View xq, xb;
            view_rec(q, xq);
            view_rec(b, xb);
            lists = cmp_list(xq, q, xb, b);
        }
        return (path_tie(q, qx, qy, b, bx, by, vx, vy, true, lists) ? 0u : 1u) |
               (path_tie(q, qx, qy, b, bx, by, vx, vy, false, lists) ? 0u : 2u);
    }
    // Is the closed-form walk(b, d_b(v)) certain to be the reference's label of v?
    // Linear run times: always (the blocker check, avail, covers ties).  Otherwise
    // one L-path must be clean for every boundary.
    __device__ __forceinline__ bool walk_certain(uint32_t b, int vx, int vy, uint32_t nb, int sx, int sy) const {
        if (ff_linear()) return true;
        uint32_t paths = 3u;
        for (uint32_t j = 0; j < nb && paths; ++j) paths &= walk_clear(bnd[j], b, vx, vy, sx, sy);
        return paths != 0;
    }
    // the same for a settled special's label x at (tx, ty): its walk, or the walk to the
    // cell its Scroll of Escape is read from
    __device__ __forceinline__ bool label_certain(const View &x, uint32_t nb, int tx, int ty, int sx, int sy) const {
        if (ff_linear() || (x.t0.kp >> 29) != kStandard) return true;
        if (x.ntail == 1) return walk_certain(x.parent, tx, ty, nb, sx, sy);
        const uint32_t u = a->rank_inv[x.t0.to];
        return walk_certain(x.parent, int(u % P.S) - int(P.H), int(u / P.S) - int(P.H), nb, sx, sy);
    }

    __device__ __forceinline__ void bpos(uint32_t b, int sx, int sy, int &bx, int &by) const {
        bx = b == 0 ? sx : sp[b].x;
        by = b == 0 ? sy : sp[b].y;
    }
    // the walk label of plain w from boundary b
    __device__ __forceinline__ void walk_to(uint32_t b, int sx, int sy, int wx, int wy, uint32_t wr, View &x) const {
        int bx, by;
        bpos(b, sx, sy, bx, by);
        view_walk(b, walk_dist(bx, by, wx, wy), wr, x);
    }
    // label of destination w (not the source, not a special) by a serial scan of the boundaries
    __device__ __forceinline__ uint32_t plain_label_serial(uint32_t w, uint32_t nb, int sx, int sy, View &x) const {
        const DevParams &p = P;
        const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
        const uint32_t wr = rank[w];
        bool have = false;
        uint32_t win = 0;
        for (uint32_t j = 0; j < nb; ++j) {
            const uint32_t b = bnd[j];
            if (vert_of(b) == p.vc) continue;
            View c;
            walk_to(b, sx, sy, wx, wy, wr, c);
            if (!have || cmp_view(c, kOwn, x, kOwn) < 0) {
                x = c;
                win = b;
                have = true;
            }
        }
        return win;
    }
    // is the closed-form label of plain w (walk from boundary b) certain?
    __device__ __forceinline__ bool dest_avail(uint32_t nbk, uint32_t b, uint32_t w, int sx, int sy) const {
        if (nbk == 0) return true;
        int bx, by;
        bpos(b, sx, sy, bx, by);
        return avail(nbk, b, bx, by, int(w % P.S) - int(P.H), int(w / P.S) - int(P.H));
    }

    // Destinations.  A segment with few (<= kEmitWaveMax) picks each one's winning
    // boundary in turn, lane j evaluating boundary j's walk and the winner found on the
    // DPP network (exact metric + length ties: full compare); lane i loads destination
    // i's cell data up front and writes its record at the end, so the queries' loads and
    // records overlap instead of queueing one query at a time.  A segment with many
    // gives each lane a query.
    static constexpr uint32_t kEmitWaveMax = 32;
    __device__ __forceinline__ bool emit_all(uint32_t qa, uint32_t qb, uint32_t nb, uint32_t nbk, int sx, int sy,
                                             const View &st0) const {
        static_assert(kEmitWaveMax <= LPS, "one lane per destination");
        bool unc = false;
        const DevParams &p = P;
        const uint32_t t = seg_lane();
        const uint32_t nq = qb - qa;
        const bool few = nq <= kEmitWaveMax;
        const uint32_t trip = seg_max_u32<64>(few ? nq : 0u);  // wave-uniform trip count
        const uint32_t bj = t < nb ? bnd[t] : 0u;
        const bool usable = t < nb && vert_of(bj) != p.vc;
        int bx, by;
        bpos(bj, sx, sy, bx, by);
        // lane t: destination t's cell, its special entry and rank
        const bool mine_q = few && t < nq;
        const uint32_t wq = mine_q ? a->q_dst[qa + t] : src;
        const uint32_t twq = sinfo[wq] & kNone10, wrq = rank[wq];
        const uint32_t seg0 = lane_id() - t;
        uint32_t wbq = 0;  // lane t: destination t's winning boundary (plain destinations)
        for (uint32_t i = 0; i < trip; ++i) {
            const bool qon = few && i < nq;
            const uint32_t from = seg0 + (qon ? i : 0u);
            const uint32_t w = qon ? uint32_t(__shfl(int(wq), int(from), 64)) : src;
            const uint32_t tw = uint32_t(__shfl(int(twq), int(from), 64));
            const uint32_t wr = uint32_t(__shfl(int(wrq), int(from), 64));
            const bool plain = qon && w != src && tw == kNone10;
            const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
            View c;
            view_walk(bj, walk_dist(bx, by, wx, wy), wr, c);
            bool cand = usable && plain;
            // metric by metric, until every segment has at most one candidate left
            unsigned long long bal;
            if (p.perm[0] == 2u)
                bal = seg_narrow<LPS, 20u>(cand, metric(c, p.perm[0]), metric(c, p.perm[1]), metric(c, p.perm[2]), c.len);
            else
                bal = seg_narrow<LPS, 16u>(cand, metric(c, p.perm[0]), metric(c, p.perm[1]), metric(c, p.perm[2]), c.len);
            const unsigned long long m = seg_bits<LPS>(bal);
            uint32_t win = __popcll(m) >= 1 ? uint32_t(__ffsll((long long)m) - 1) : 0u;
            if (!seg_single<LPS>(bal)) {  // equal metrics and length: compare the command lists
                const bool tied = __popcll(m) > 1;
                uint32_t mm = (tied && cand) ? t : kNone32;
#pragma unroll
                for (int off = LPS / 2; off >= 1; off >>= 1) {
                    const uint32_t o = __shfl_xor(mm, off, 64);
                    if (o == kNone32) continue;
                    if (mm == kNone32) {
                        mm = o;
                        continue;
                    }
                    View co, cm;
                    walk_to(bnd[o], sx, sy, wx, wy, wr, co);
                    walk_to(bnd[mm], sx, sy, wx, wy, wr, cm);
                    if (cmp_view(co, kOwn, cm, kOwn) < 0) mm = o;
                }
                if (tied) win = mm;
            }
            wbq = (qon && t == i) ? win : wbq;
            // non-linear run times: lane j clears boundary j; one path clean for all
            if (!ff_linear() && !(a->dbg_flags & 8u)) {
                const uint32_t pc = (qon && plain) ? walk_clear(t < nb ? bnd[t] : kNone32, bnd[win], wx, wy, sx, sy) : 3u;
                const bool x_bad = seg_bits<LPS>(__ballot(!(pc & 1u))) != 0;
                const bool y_bad = seg_bits<LPS>(__ballot(!(pc & 2u))) != 0;
                if (x_bad && y_bad && t == 0) unc = true;
            }
        }
        if (mine_q) {  // lane t writes destination t's record
            View x;
            const bool plain = wq != src && twq == kNone10;
            const int wx = int(wq % p.S) - int(p.H), wy = int(wq / p.S) - int(p.H);
            if (plain) walk_to(bnd[wbq], sx, sy, wx, wy, wrq, x);
            else if (wq == src) x = st0;
            else view_rec(twq, x);
            emit(x, qa + t);
            if (plain && !dest_avail(nbk, bnd[wbq], wq, sx, sy)) unc = true;
        }
        for (uint32_t i = qa + t; !few && i < qb; i += LPS) {
            const uint32_t w = a->q_dst[i];
            View x;
            const uint32_t tw = sinfo[w] & kNone10;
            if (w == src) {
                x = st0;
            } else if (tw != kNone10) {
                view_rec(tw, x);
            } else {
                const uint32_t b = plain_label_serial(w, nb, sx, sy, x);
                if (!dest_avail(nbk, b, w, sx, sy)) unc = true;
                if (!(a->dbg_flags & 8u) && !walk_certain(b, int(w % p.S) - int(p.H), int(w / p.S) - int(p.H), nb, sx, sy))
                    unc = true;
            }
            emit(x, i);
        }
        wave_sync();
        return unc;
    }

    // All-destinations mode: publish the label table and rank the boundaries by
    // (length, command list) — the order in which their walks tie-break at any cell
    // (equal metrics and lengths leave the lists to decide, and two walks' lists
    // first differ inside the boundaries' own labels).  The source (b = 0) ranks first.
    __device__ __forceinline__ void export_table(bool ok, bool have, bool fallback, uint32_t s_idx, uint32_t nb) const {
        const DevParams &p = P;
        const uint32_t t = seg_lane();
        if (t <= p.NS) lexs[t] = kNone32;
        wave_sync();
        if (ok && t < nb) {
            const uint32_t bj = bnd[t];
            uint32_t r = 0;
            for (uint32_t i = 0; i < nb; ++i) {
                const uint32_t bi = bnd[i];
                if (bi == bj) continue;
                bool less;
                if (bi == 0 || bj == 0) {
                    less = bi == 0;
                } else if (R[bi].len() != R[bj].len()) {
                    less = R[bi].len() < R[bj].len();
                } else {
                    View xi, xj;
                    view_rec(bi, xi);
                    view_rec(bj, xj);
                    less = cmp_list(xi, bi, xj, bj) < 0;
                }
                r += less ? 1u : 0u;
            }
            lexs[bj] = r;
        }
        wave_sync();
        const unsigned long long tb = (unsigned long long)s_idx * (p.NS + 1);
        if (ok && t <= p.NS) {
            a->out_tab[tb + t] = R[t];
            a->out_lex[tb + t] = lexs[t];
        }
        if (have && t == 0) a->src_state[s_idx] = fallback ? 2u : 1u;
        wave_sync();
    }

    // Certified fallback: the same ranks and table into staging entry `slot` (the
    // source's fallback entry), with the source's vertex
    __device__ __forceinline__ void export_cert(bool go, uint32_t slot, uint32_t nb) const {
        const DevParams &p = P;
        const uint32_t t = seg_lane();
        if (t <= p.NS) lexs[t] = kNone32;
        wave_sync();
        if (go && t < nb) {
            const uint32_t bj = bnd[t];
            uint32_t r = 0;
            for (uint32_t i = 0; i < nb; ++i) {
                const uint32_t bi = bnd[i];
                if (bi == bj) continue;
                bool less;
                if (bi == 0 || bj == 0) {
                    less = bi == 0;
                } else if (R[bi].len() != R[bj].len()) {
                    less = R[bi].len() < R[bj].len();
                } else {
                    View xi, xj;
                    view_rec(bi, xi);
                    view_rec(bj, xj);
                    less = cmp_list(xi, bi, xj, bj) < 0;
                }
                r += less ? 1u : 0u;
            }
            lexs[bj] = r;
        }
        wave_sync();
        if (go && t <= p.NS) {
            const unsigned long long tb = (unsigned long long)slot * (p.NS + 1);
            a->cert_stage_tab[tb + t] = R[t];
            a->cert_stage_lex[tb + t] = lexs[t];
        }
        if (go && t == 0) a->cert_stage_src[slot] = src;
        wave_sync();
    }

    // Segment h solves source base + h (none past the end, `total`): indices past nsrc
    // name the sources the lane kernel relisted (KArgs::relist).
    __device__ __forceinline__ void solve(uint32_t base, uint32_t total) {
        const DevParams &p = P;
        const uint32_t t = seg_lane();
        const uint32_t s_raw = base + lane_id() / LPS, nsrc = a->nsrc;
        const bool have = s_raw < total;
        const uint32_t r_raw = have ? s_raw : base;
        const uint32_t s_idx = r_raw < nsrc ? r_raw : a->relist[r_raw - nsrc];
        const uint32_t si = s_idx;
        const bool mine = have && t >= 1 && t <= p.NS;
        src = a->src_v[si];
        src_rk = rank[src];
        const int sx = int(src % p.S) - int(p.H), sy = int(src / p.S) - int(p.H);
        const uint32_t ts = sinfo[src] & kNone10;
        const SpecialStatic ss = sp[t <= p.NS ? t : 0u];
        View st0;
        view_start(st0);
        RLab my = compact(st0);
        uint32_t st = 0, bwh = 0, b0 = 0, b1 = 0, b2 = 0, unc = 0, nbk = 0;
        if (t == 0) {
            write_rec(0, st0, 2);
            bnd[0] = 0;
        }
        if (p.use_soe && t < nreg) {
            const uint2 e = reinterpret_cast<const uint2 *>(a->near)[(unsigned long long)src * nreg + t];
            srow[2 * t] = e.x;
            srow[2 * t + 1] = e.y;
        }
        wave_sync();
        improve_reg(mine && t == ts, st, my, st0, ss.rk);
        {  // SHQ / SFm: only the source's own edges can be minimal
            View c = st0;
            c.m1 = p.shq_cost;
            c.t0 = Cmd{kSHQ << 29, src_rk, ss.rk};
            improve_reg(mine && t == p.hq_t, st, my, c, ss.rk);
            c.m1 = p.sfm_cost;
            c.t0 = Cmd{kSFm << 29, src_rk, sp[1].rk};
            improve_reg(mine && p.use_sfm && t == 1, st, my, c, ss.rk);
        }
        uint32_t nb = 1;
        MR_HSTAMP(3);
        {
            View l0;
            view_start(l0);
            l0.len = 0;  // unused for b = 0 (walks from the source start the list)
            relax_boundary(mine && src != p.vc, l0, 0, sx, sy, t, st, my, ss, bwh, b0, b1, b2);
        }
        wave_sync();
        MR_HSTAMP(6);
        MR_HCOUNT(0, 1);
        for (uint32_t it = 0; it <= p.NS; ++it) {
            const uint32_t s = select_reg(mine && st == 1, my, ss.rk);
            if (__all(s == kNone32)) break;
            MR_HCOUNT(1, 1);
            const bool act = s != kNone32;  // this segment settles a special
            const uint32_t sc = act ? s : 0u;
            if (act && t == s) {
                st = 2;
                write_rec(s, expand(my, ss.rk), 2);
            }
            wave_sync();
            View ls;  // the settled label, from the table
            view_rec(sc, ls);
            const SpecialStatic sS = sp[sc];
            const Cmd last = ls.ntail == 2 ? ls.t1 : ls.t0;
            const uint32_t lk = last.kp >> 29;
            const bool boundary = act && lk != kNoMove && lk != kStandard;
            // a boundary that tied a walk becomes a blocker
            const bool tie = act && t == s && boundary && bwh && b0 == my.m0 && b1 == my.m1 && b2 == my.m2;
            if (tie) blk[nbk] = s;
            nbk += seg_bits<LPS>(__ballot(tie)) != 0 ? 1u : 0u;
            MR_HSTAMP(4);
            {  // CentralMove / caravan / SoE edges s -> t (skipped when no segment needs an edge kind)
                const bool live = mine && act && st != 2;
                const bool central_s = act && (sS.flags & (kSpCenter | kSpBorder1));
                if (__any(central_s)) {
                    View c;
                    ext_view(ls, sc, sS.rk, kCentral, 1, 0, 10, ss.rk, c);
                    const uint32_t want = (sS.flags & kSpCenter) ? kSpBorder1 : kSpCenter;
                    improve_reg(live && central_s && (ss.flags & want), st, my, c, ss.rk);
                }
                const bool hub_s = act && p.use_caravans && (sS.flags & kSpHub);
                if (__any(hub_s)) {
                    View c;
                    const uint32_t d = uint32_t(abs(sS.x - ss.x) + abs(sS.y - ss.y));
                    const uint32_t coef = ss.coef5 ? 5u : 2u;
                    ext_view(ls, sc, sS.rk, kCaravan, (d << 1) | ss.coef5, coef * d, p.rgt * d, ss.rk, c);
                    improve_reg(live && hub_s && (ss.flags & kSpHub), st, my, c, ss.rk);
                }
                const bool soe_s = act && p.use_soe && sS.region != kNone10 && sS.region != sc;
                if (__any(soe_s)) {
                    View c;
                    ext_view(ls, sc, sS.rk, kSoE, 0, p.soe_cost, 0, ss.rk, c);
                    improve_reg(live && soe_s && sS.region == t, st, my, c, ss.rk);
                }
            }
            MR_HSTAMP(5);
            const bool walks = boundary && sc != 1;  // a new walk source (entry 1, the Center, has none)
            if (__any(walks)) {
                relax_boundary(mine && walks, ls, sc, sS.x, sS.y, t, st, my, ss, bwh, b0, b1, b2);
                if (walks && t == 0) bnd[nb] = sc;
                nb += walks ? 1u : 0u;
                MR_HCOUNT(2, 1);
            }
            wave_sync();
            MR_HSTAMP(6);
        }
#ifdef MR_HUBDUMP
        if (a->dbg && have && src == uint32_t(a->dbg_blocks)) {  // diagnostics: settled table of one source
            unsigned int *d = reinterpret_cast<unsigned int *>(a->dbg);
            const uint32_t *rw = reinterpret_cast<const uint32_t *>(&R[t]);
            if (t <= p.NS)
                for (int i = 0; i < 7; ++i) d[t * 16 + i] = rw[i];
            d[t * 16 + 11] = st;
            d[t * 16 + 12] = my.m0;
            d[t * 16 + 13] = my.m1;
            d[t * 16 + 14] = my.m2;
            d[t * 16 + 15] = 0xABCD0000u | nb;
        }
#endif
        // Every settled label must be certain.  Checked after the loop against all the
        // blockers (one settled after t cannot lie on t's shortest walk, its label being
        // larger, so the extra ones only make the check more careful).  A label that may
        // miss a blocker hands the source to the SSSP kernel (in all-destinations mode
        // any blocker does: the fill kernel cannot check cells).  No early return: the
        // wave must stay converged.
        wave_sync();
        if (__any(nbk != 0) && mine && st == 2 && !label_avail(expand(my, ss.rk), nbk, ss.x, ss.y, sx, sy)) unc = 1;
        if (!ff_linear() && !(a->dbg_flags & 4u) && mine && st == 2 &&
            !label_certain(expand(my, ss.rk), nb, ss.x, ss.y, sx, sy))
            unc = 1;
        const bool unc_sp = seg_bits<LPS>(__ballot(unc != 0)) != 0;
        const uint32_t qa = a->q_begin[si];
        bool fallback = have && (unc_sp || a->fb_all || (a->all_mode && nbk != 0));
        if (a->all_mode) {
            if (t == 0 && have && !fallback) written += a->q_begin[si + 1] - qa;
            export_table(have && !fallback, have, fallback, s_idx, nb);
        } else {
            const uint32_t qb = (!have || fallback) ? qa : a->q_begin[si + 1];
            const bool unc_q = emit_all(qa, qb, nb, nbk, sx, sy, st0);
            fallback = fallback || (have && seg_bits<LPS>(__ballot(unc_q)) != 0);
            if (t == 0 && have && !fallback) written += qb - qa;
        }
        // A query-mode fallback source stages its label table and boundary ranks under
        // its fallback entry; cert_select_kernel then gives the certificate slots to the
        // staged sources in source order, and the fill + check launches decide whether
        // the SSSP kernel is needed at all
        uint32_t entry = kNone32;
        if (fallback && t == 0) entry = push_fallback(a, counter, s_idx, kNone32);
        entry = uint32_t(__shfl(int(entry), int(lane_id() & ~(LPS - 1u))));  // segment lane 0's
        const bool stage = fallback && !a->all_mode && a->cert_cap && entry < a->cert_stage_cap;
        if (__any(stage)) export_cert(stage, entry, nb);
        if (stage && t == 0) a->fb_cert[entry] = kFbStaged;
        MR_HSTAMP(7);
    }
};

__host__ __device__ constexpr uint32_t align16h(uint32_t x) { return (x + 15u) & ~15u; }

// per-source LDS slots: 4 waves x SPW segments
struct HubLayout {
    uint32_t off_sp, off_hubs, off_near, off_srow, off_R, off_bnd, off_lex, off_blk, rstride, bstride, sstride, total;
};
__host__ __device__ inline HubLayout hub_layout(uint32_t NS, uint32_t nreg, uint32_t spw) {
    HubLayout L{};
    const uint32_t T = NS + 1, slots = 4 * spw;
    uint32_t o = 0;
    L.off_sp = o;
    o = align16h(o + T * uint32_t(sizeof(SpecialStatic)));
    L.off_hubs = o;
    o = align16h(o + T * 2);
    L.off_near = o;  // region rows of the specials (row 0 unused)
    o = align16h(o + T * nreg * 8);
    L.sstride = align16h(nreg * 8);
    L.off_srow = o;  // per slot: its source's region row
    o += slots * L.sstride;
    L.rstride = align16h(T * uint32_t(sizeof(Rec)));
    L.off_R = o;
    o += slots * L.rstride;
    L.bstride = align16h((T + 1) * 4);
    L.off_bnd = o;
    o += slots * L.bstride;
    L.off_lex = o;  // per slot: all-destinations mode, the boundaries' ranks (bstride words)
    o += slots * L.bstride;
    L.off_blk = o;  // per slot: blocking specials (bstride words)
    o += slots * L.bstride;
    L.total = o;
    return L;
}

// PERM = comparator order c1 c2 c3 as metric indices (9*c1 + 3*c2 + c3): a compile-time
// constant here, so every metric selection and comparison folds.  SPW = sources per wave.
#ifndef MR_HUB_WAVES
#define MR_HUB_WAVES 5  // waves per SIMD the register budget is cut for: 6 ran c4 3 % faster but its
                        // larger scratch spill (64 B/lane) overflowed L2: 0.6 GB of HBM traffic per launch
#endif
// the hub kernel's work as workgroup `block` of `nblocks` (a launch of its own, or the
// first workgroups of a fused hub + fill launch, hub_fill_kernel)
template <uint32_t PERM, uint32_t SPW, bool NONLIN>
__device__ __forceinline__ void hub_body(const KArgs *__restrict__ a, char *smem, uint32_t block, uint32_t nblocks) {
    const uint32_t NS = a->p.NS, nreg = a->nreg;
    const HubLayout L = hub_layout(NS, nreg, SPW);
    SpecialStatic *spl = reinterpret_cast<SpecialStatic *>(smem + L.off_sp);
    uint16_t *hubl = reinterpret_cast<uint16_t *>(smem + L.off_hubs);
    uint2 *nearl = reinterpret_cast<uint2 *>(smem + L.off_near);
    for (uint32_t t = threadIdx.x; t <= NS; t += kBS) spl[t] = a->sp[t];
    for (uint32_t h = threadIdx.x; h < a->p.n_hubs; h += kBS) hubl[h] = a->hubs[h];
    for (uint32_t i = threadIdx.x; i < NS * nreg; i += kBS) {
        const uint32_t t = 1 + i / nreg, r = i % nreg;
        nearl[t * nreg + r] = reinterpret_cast<const uint2 *>(a->near)[(unsigned long long)a->sp[t].v * nreg + r];
    }
    __syncthreads();
    const uint32_t slot = (threadIdx.x >> 6) * SPW + lane_id() / (64 / SPW);
    HubSolver<SPW> H;
    H.a = a;
    H.P = a->p;
    H.P.perm[0] = PERM / 9;
    H.P.perm[1] = (PERM / 3) % 3;
    H.P.perm[2] = PERM % 3;
    // linear run times need no near-tie certification (the compiler folds it away)
    if (!NONLIN) H.P.ff_num = H.P.ff_den = 1;
    H.rank = a->rank;
    H.sinfo = a->sinfo;
    H.counter = a->counter;
    H.sh = nullptr;
    H.R = reinterpret_cast<Rec *>(smem + L.off_R + slot * L.rstride);
    H.state = nullptr;
    H.sp = spl;
    H.hubs = hubl;
    H.dst = nullptr;
    H.src = 0;
    H.src_rk = 0;
    H.bnd = reinterpret_cast<uint32_t *>(smem + L.off_bnd + slot * L.bstride);
    H.lexs = reinterpret_cast<uint32_t *>(smem + L.off_lex + slot * L.bstride);
    H.blk = reinterpret_cast<uint32_t *>(smem + L.off_blk + slot * L.bstride);
    H.nearS = reinterpret_cast<const uint32_t *>(smem + L.off_near);
    H.srow = reinterpret_cast<uint32_t *>(smem + L.off_srow + slot * L.sstride);
    H.nreg = nreg;
#ifdef MR_STAMPS
    H.hs_last = __builtin_amdgcn_s_memtime();
#endif
    // sources are strided over the launch's waves (no dequeue atomics: one word
    // would saturate at ~88 dequeues/us, MI355X_MICROARCH.md)
    const uint32_t waves = nblocks * (kBS / 64), wid = block * (kBS / 64) + (threadIdx.x >> 6);
    // the sources [src_off, nsrc), then those the lane kernel of this pass relisted (its
    // launch precedes this one on the stream; the count is reset only by the pass's last
    // kernel's last workgroup, after every workgroup here has read it)
    const uint32_t total = a->nsrc + (a->relist ? __hip_atomic_load(a->counter + kCtrRelist, __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT)
                                                : 0u);
    for (uint32_t k = 0;; ++k) {
        const unsigned long long base = a->src_off + ((unsigned long long)k * waves + wid) * SPW;
#ifdef MR_STAMPS
        H.hmark(8);
#endif
        if (base >= total) break;
        H.solve(uint32_t(base), total);
    }
    H.flush_err();
    __shared__ uint32_t wsum;
    if (threadIdx.x == 0) wsum = 0;
    __syncthreads();
    if (H.written) atomicAdd(&wsum, H.written);
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, wsum, nblocks);
#ifdef MR_STAMPS
    if (lane_id() == 0 && a->dbg) {
        unsigned long long *h = a->dbg + (unsigned long long)a->dbg_blocks * 10;
        for (int i = 0; i < 9; ++i) atomicAdd(h + i, H.hs[i]);
    }
#endif
}
template <uint32_t PERM, uint32_t SPW, bool NONLIN>
__global__ __launch_bounds__(kBS, MR_HUB_WAVES) void hub_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    hub_body<PERM, SPW, NONLIN>(a, smem, blockIdx.x, gridDim.x);
}

// ===================================================================================
// Wide hub solver: more specials than one wave has lanes (NS + 1 up to 64 * SPL;
// c5 has 262 with 64 campfires per homeland), or a grid whose V x regions table
// would not fit.  One source per wave; lane j owns specials j, j + 64, ... with
// their tentative labels in registers.  A settle picks each lane's best owned
// label (full comparator) and then the wave's best on the DPP network, exactly
// as the one-lane-per-special kernel does; the relaxations are the same per
// special.  The source's region row {distance, rank} is computed in the kernel
// from the per-region boundary cells (the nearest cell of a region seen from
// outside it lies on its boundary), the specials' rows come from a per-plan table.
// =====================================================================================
__device__ __forceinline__ void sel_view(bool take, View &d, const View &s) {
    d.m0 = take ? s.m0 : d.m0;
    d.m1 = take ? s.m1 : d.m1;
    d.m2 = take ? s.m2 : d.m2;
    d.len = take ? s.len : d.len;
    d.parent = take ? s.parent : d.parent;
    d.ntail = take ? s.ntail : d.ntail;
    d.t0.kp = take ? s.t0.kp : d.t0.kp;
    d.t0.from = take ? s.t0.from : d.t0.from;
    d.t0.to = take ? s.t0.to : d.t0.to;
    d.t1.kp = take ? s.t1.kp : d.t1.kp;
    d.t1.from = take ? s.t1.from : d.t1.from;
    d.t1.to = take ? s.t1.to : d.t1.to;
}

#ifndef MR_WIDE_REG_STATIC
#define MR_WIDE_REG_STATIC 0  // owned specials' static records in registers up to this SPL: at 3 waves per
                              // SIMD they spilled 156 B per lane; read from LDS the kernel spills none (c5 -0.5 %)
#endif
template <uint32_t SPL>
struct HubWide : HubSolver<1> {
    using B = HubSolver<1>;
    using B::a;
    using B::P;
    using B::rank;
    using B::sinfo;
    using B::counter;
    using B::sp;
    using B::src;
    using B::src_rk;
    using B::bnd;
    using B::srow;
    using B::nreg;
    using B::written;

    // srow[2r], srow[2r+1] = distance and rank of the region-r cell nearest to the
    // source (walks avoid the Center; ties by rank), as the host BFS table defines it
    __device__ __forceinline__ void near_rows(int sx, int sy) const {
        const DevParams &p = P;
        const uint32_t lane = lane_id();
        if (a->near) {  // the grid's V x regions table
            const uint2 *row = reinterpret_cast<const uint2 *>(a->near) + (unsigned long long)src * nreg;
            for (uint32_t r = lane; r < nreg; r += 64) {
                const uint2 e = row[r];
                srow[2 * r] = e.x;
                srow[2 * r + 1] = e.y;
            }
            return;
        }
        const uint32_t rs = region_of(src);  // table index of the source's nearest campfire
        const uint32_t rid_src = rs != kNone10 ? sp[rs].rid : kNone10;
        const uint2 *cells = reinterpret_cast<const uint2 *>(a->rb_cell);
        for (uint32_t r = 0; r < nreg; ++r) {
            uint32_t bd = kNone32, br = kNone32;
            if (src != p.vc) {
                const uint32_t e = a->rb_off[r + 1];
                for (uint32_t i = a->rb_off[r] + lane; i < e; i += 64) {
                    const uint2 c = cells[i];
                    const int ux = int(int16_t(c.x & 0xFFFFu)), uy = int(int16_t(c.x >> 16));
                    const uint32_t d = walk_dist(sx, sy, ux, uy);
                    const bool take = d < bd || (d == bd && c.y < br);
                    bd = take ? d : bd;
                    br = take ? c.y : br;
                }
            }
            const uint32_t md = wave_min_u32(bd);
            const uint32_t mr = wave_min_u32(bd == md ? br : kNone32);
            if (lane == 0) {
                const bool inside = src != p.vc && rid_src == r;
                srow[2 * r] = inside ? 0u : md;
                srow[2 * r + 1] = inside ? src_rk : mr;
            }
        }
    }

    // full comparator of two register labels (own: their specials' ranks)
    __device__ __forceinline__ int cmp_rlab(const RLab &x, uint32_t ox, const RLab &y, uint32_t oy) const {
        const int r = cmp_metrics(x.m0, x.m1, x.m2, y.m0, y.m1, y.m2);
        if (r) return r;
        if (rl_len(x) != rl_len(y)) return rl_len(x) < rl_len(y) ? -1 : 1;
        return cmp_list(expand(x, ox), kOwn, expand(y, oy), kOwn);
    }
    // the wave's best tentative label over every lane's owned specials; returns its
    // table index (wave-uniform) or kNone32
    template <class SSF>
    __device__ __forceinline__ uint32_t select_wide(const bool (&c)[SPL], const RLab (&my)[SPL], SSF SS) const {
        const DevParams &p = P;
        const uint32_t j = lane_id();
        bool any = false;
        RLab bv = my[0];
        uint32_t bt = kNone32, bown = 0;
#pragma unroll
        for (uint32_t i = 0; i < SPL; ++i) {
            const uint32_t own = SS(i).rk;
#ifdef MR_WIDE_SETTLE_TIES
            const bool take = c[i] && (!any || cmp_rlab(my[i], own, bv, bown) < 0);
#else
            // Exact (metrics, length) ties at a settle need no list compare: either entry
            // may settle first (every candidate out of a settled entry is strictly greater
            // than its label in (metrics, length); LaneHub::solve)
            int r = cmp_metrics(my[i].m0, my[i].m1, my[i].m2, bv.m0, bv.m1, bv.m2);
            if (r == 0 && rl_len(my[i]) != rl_len(bv)) r = rl_len(my[i]) < rl_len(bv) ? -1 : 1;
            const bool take = c[i] && (!any || r < 0);
#endif
            sel_rlab(take, bv, my[i]);
            bt = take ? j + 64u * i : bt;
            bown = take ? own : bown;
            any = any || c[i];
        }
        bool cand = any;
        if (__ballot(cand) == 0) return kNone32;
        const unsigned long long m =
            p.perm[0] == 2u ? seg_narrow<64, 20u>(cand, metric(bv, p.perm[0]), metric(bv, p.perm[1]), metric(bv, p.perm[2]), rl_len(bv))
                            : seg_narrow<64, 16u>(cand, metric(bv, p.perm[0]), metric(bv, p.perm[1]), metric(bv, p.perm[2]), rl_len(bv));
#ifdef MR_WIDE_SETTLE_TIES
        if (__popcll(m) == 1) return bcast(bt, uint32_t(__ffsll((long long)m) - 1));
#else
        return bcast(bt, uint32_t(__ffsll((long long)m) - 1));  // (several lanes tied: the lowest)
#endif
        // equal metrics and length in several lanes: compare the command lists
        if (cand) write_rec(bt, expand(bv, bown), 1);
        wave_sync();
        uint32_t mm = cand ? bt : kNone32;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t o = __shfl_xor(mm, off, 64);
            if (o != kNone32 && (mm == kNone32 || cmp_entries(o, mm) < 0)) mm = o;
        }
        return mm;
    }

    // destinations of the source: with few, each query at a time over all lanes
    // (lane j scans boundaries j, j + 64, ...); with many, a query per lane
    __device__ __forceinline__ bool emit_wide(uint32_t qa, uint32_t qb, uint32_t nb, uint32_t nbk, int sx, int sy,
                                              const View &st0) const {
        const DevParams &p = P;
        bool unc = false;
        const uint32_t j = lane_id();
        const uint32_t nq = qb - qa;
        if (nq <= B::kEmitWaveMax) {
            for (uint32_t i = 0; i < nq; ++i) {
                const uint32_t qi = qa + i;
                const uint32_t w = a->q_dst[qi];
                const uint32_t tw = sinfo[w] & kNone10;
                const bool plain = w != src && tw == kNone10;
                View x;
                if (plain) {
                    const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
                    const uint32_t wr = rank[w];
                    bool any = false;
                    View bv;
                    view_start(bv);
                    uint32_t bp = kNone32;
                    for (uint32_t k = j; k < nb; k += 64) {
                        const uint32_t b = bnd[k];
                        if (vert_of(b) == p.vc) continue;
                        View c;
                        walk_to(b, sx, sy, wx, wy, wr, c);
                        const bool take = !any || cmp_view(c, kOwn, bv, kOwn) < 0;
                        sel_view(take, bv, c);
                        bp = take ? k : bp;
                        any = true;
                    }
                    bool cand = any;
                    narrow(cand, metric(bv, p.perm[0]));
                    narrow(cand, metric(bv, p.perm[1]));
                    narrow(cand, metric(bv, p.perm[2]));
                    narrow(cand, bv.len);
                    const unsigned long long m = __ballot(cand);
                    uint32_t win = kNone32;
                    if (__popcll(m) == 1) {
                        win = bcast(bp, uint32_t(__ffsll((long long)m) - 1));
                    } else {
                        uint32_t mm = cand ? bp : kNone32;
#pragma unroll
                        for (int off = 32; off >= 1; off >>= 1) {
                            const uint32_t o = __shfl_xor(mm, off, 64);
                            if (o == kNone32) continue;
                            if (mm == kNone32) {
                                mm = o;
                                continue;
                            }
                            View co, cm;
                            walk_to(bnd[o], sx, sy, wx, wy, wr, co);
                            walk_to(bnd[mm], sx, sy, wx, wy, wr, cm);
                            if (cmp_view(co, kOwn, cm, kOwn) < 0) mm = o;
                        }
                        win = mm;
                    }
                    walk_to(bnd[win], sx, sy, wx, wy, wr, x);
                    if (j == 0 && !B::dest_avail(nbk, bnd[win], w, sx, sy)) unc = true;
                } else if (w == src) {
                    x = st0;
                } else {
                    view_rec(tw, x);
                }
                if (j == 0) emit(x, qi);
            }
        } else {
            for (uint32_t i = qa + j; i < qb; i += 64) {
                const uint32_t w = a->q_dst[i];
                View x;
                const uint32_t tw = sinfo[w] & kNone10;
                if (w == src) {
                    x = st0;
                } else if (tw != kNone10) {
                    view_rec(tw, x);
                } else {
                    const uint32_t b = B::plain_label_serial(w, nb, sx, sy, x);
                    if (!B::dest_avail(nbk, b, w, sx, sy)) unc = true;
                }
                emit(x, i);
            }
        }
        wave_sync();
        return unc;
    }

    __device__ __forceinline__ void solve(uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t j = lane_id();
        src = a->src_v[s_idx];
        src_rk = rank[src];
        const int sx = int(src % p.S) - int(p.H), sy = int(src / p.S) - int(p.H);
        const uint32_t ts = sinfo[src] & kNone10;
        View st0;
        view_start(st0);
        RLab my[SPL];
        uint32_t st[SPL], bwh[SPL], b0[SPL], b1[SPL], b2[SPL];
        bool mine[SPL];
        uint32_t unc = 0, nbk = 0;
        // the owned specials' static records: re-read from LDS (MR_WIDE_REG_STATIC: held
        // in registers up to that many per lane)
        constexpr bool kRegStatic = SPL <= MR_WIDE_REG_STATIC;
        SpecialStatic ssr[kRegStatic ? SPL : 1];
#pragma unroll
        for (uint32_t i = 0; i < SPL; ++i)
            if constexpr (kRegStatic) ssr[i] = sp[j + 64u * i <= p.NS ? j + 64u * i : 0u];
        auto SS = [&](uint32_t i) -> SpecialStatic {
            if constexpr (kRegStatic) return ssr[i];
            else return sp[j + 64u * i <= p.NS ? j + 64u * i : 0u];
        };
        if (j == 0) {
            write_rec(0, st0, 2);
            bnd[0] = 0;
        }
        if (p.use_soe) near_rows(sx, sy);
        wave_sync();
        View l0;
        view_start(l0);
        l0.len = 0;
#pragma unroll
        for (uint32_t i = 0; i < SPL; ++i) {
            const uint32_t t = j + 64u * i;
            mine[i] = t >= 1 && t <= p.NS;
            const SpecialStatic ss = SS(i);
            my[i] = compact(st0);
            st[i] = bwh[i] = b0[i] = b1[i] = b2[i] = 0;
            improve_reg(mine[i] && t == ts, st[i], my[i], st0, ss.rk);
            View c = st0;
            c.m1 = p.shq_cost;
            c.t0 = Cmd{kSHQ << 29, src_rk, ss.rk};
            improve_reg(mine[i] && t == p.hq_t, st[i], my[i], c, ss.rk);
            c.m1 = p.sfm_cost;
            c.t0 = Cmd{kSFm << 29, src_rk, sp[1].rk};
            improve_reg(mine[i] && p.use_sfm && t == 1, st[i], my[i], c, ss.rk);
            relax_boundary(mine[i] && src != p.vc, l0, 0, sx, sy, t, st[i], my[i], ss, bwh[i], b0[i], b1[i], b2[i]);
        }
        wave_sync();
        uint32_t nb = 1;
        for (uint32_t it = 0; it <= p.NS; ++it) {
            bool c[SPL];
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i) c[i] = mine[i] && st[i] == 1;
            const uint32_t s = select_wide(c, my, SS);
            if (s == kNone32) break;
            const uint32_t so = s & 63u, si = s >> 6;
            // s's region-row entries for the owned specials' regions, read before the
            // settle so their latency overlaps it (used if s turns out a boundary)
            uint32_t ed[SPL], eu[SPL];
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i) {
                const uint32_t rid = SS(i).rid;
                ed[i] = kNone32;
                eu[i] = 0;
                if (p.use_soe && mine[i] && st[i] == 1 && rid != kNone10) {
                    const uint2 e = reinterpret_cast<const uint2 *>(B::nearS)[s * nreg + rid];
                    ed[i] = e.x;
                    eu[i] = e.y;
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i)
                if (j == so && i == si) {
                    st[i] = 2;
                    write_rec(s, expand(my[i], SS(i).rk), 2);
                }
            wave_sync();
            View ls;
            view_rec(s, ls);
            const SpecialStatic sS = sp[s];
            const Cmd last = ls.ntail == 2 ? ls.t1 : ls.t0;
            const uint32_t lk = last.kp >> 29;
            const bool boundary = lk != kNoMove && lk != kStandard;
            // a boundary that tied a walk becomes a blocker
            bool tie = false;
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i)
                if (j == so && i == si)
                    tie = boundary && bwh[i] && b0[i] == my[i].m0 && b1[i] == my[i].m1 && b2[i] == my[i].m2;
            if (tie) B::blk[nbk] = s;
            nbk += __ballot(tie) != 0 ? 1u : 0u;
            const bool central_s = (sS.flags & (kSpCenter | kSpBorder1)) != 0;
            const bool hub_s = p.use_caravans && (sS.flags & kSpHub);
            const bool soe_s = p.use_soe && sS.region != kNone10 && sS.region != s;
            const bool walks = boundary && s != 1;
            View cc;
            if (central_s) ext_view(ls, s, sS.rk, kCentral, 1, 0, 10, 0, cc);
            const uint32_t want = (sS.flags & kSpCenter) ? kSpBorder1 : kSpCenter;
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i) {
                const uint32_t t = j + 64u * i;
                const bool live = mine[i] && st[i] != 2;
                if (!__any(live)) continue;  // a row whose specials all settled
                const SpecialStatic ss = SS(i);
                if (central_s) {
                    View c = cc;
                    c.t0.to = ss.rk;
                    improve_reg(live && (ss.flags & want), st[i], my[i], c, ss.rk);
                }
                if (hub_s) {
                    View c;
                    const uint32_t d = uint32_t(abs(sS.x - ss.x) + abs(sS.y - ss.y));
                    const uint32_t coef = ss.coef5 ? 5u : 2u;
                    ext_view(ls, s, sS.rk, kCaravan, (d << 1) | ss.coef5, coef * d, p.rgt * d, ss.rk, c);
                    improve_reg(live && (ss.flags & kSpHub), st[i], my[i], c, ss.rk);
                }
                if (soe_s) {
                    View c;
                    ext_view(ls, s, sS.rk, kSoE, 0, p.soe_cost, 0, ss.rk, c);
                    improve_reg(live && sS.region == t, st[i], my[i], c, ss.rk);
                }
                if (walks) {
                    B::relax_walk(live, ls, s, sS.x, sS.y, t, st[i], my[i], ss, bwh[i], b0[i], b1[i], b2[i]);
                    if (p.use_soe) B::relax_soe(live, ls, s, t, st[i], my[i], ss, ed[i], eu[i]);
                }
            }
            if (walks && j == 0) bnd[nb] = s;
            nb += walks ? 1u : 0u;
            wave_sync();
        }
        wave_sync();
        if (nbk != 0) {  // every settled label must be certain (as in HubSolver::solve)
#pragma unroll
            for (uint32_t i = 0; i < SPL; ++i) {
                const SpecialStatic ss = SS(i);
                if (mine[i] && st[i] == 2 && !B::label_avail(B::expand(my[i], ss.rk), nbk, ss.x, ss.y, sx, sy)) unc = 1;
            }
        }
        bool fallback = __ballot(unc != 0) != 0 || a->fb_all;
        const uint32_t qa = a->q_begin[s_idx], qb = fallback ? qa : a->q_begin[s_idx + 1];
        fallback = __ballot(emit_wide(qa, qb, nb, nbk, sx, sy, st0)) != 0 || fallback;
        if (j == 0 && !fallback) written += qb - qa;
        if (fallback && j == 0) push_fallback(a, counter, s_idx, kNone32);
    }
};

// per-wave LDS slots of the wide kernel (4 waves, one source each)
struct WideLayout {
    uint32_t off_sp, off_hubs, off_srow, off_R, off_bnd, off_blk, rstride, bstride, sstride, total;
};
__host__ __device__ inline WideLayout wide_layout(uint32_t NS, uint32_t nreg) {
    WideLayout L{};
    const uint32_t T = NS + 1;
    uint32_t o = 0;
    L.off_sp = o;
    o = align16h(o + T * uint32_t(sizeof(SpecialStatic)));
    L.off_hubs = o;
    o = align16h(o + T * 2);
    L.sstride = align16h(nreg * 8 + 8);
    L.off_srow = o;
    o += 4 * L.sstride;
    L.rstride = align16h(T * uint32_t(sizeof(Rec)));
    L.off_R = o;
    o += 4 * L.rstride;
    L.bstride = align16h((T + 1) * 4);
    L.off_bnd = o;
    o += 4 * L.bstride;
    L.off_blk = o;
    o += 4 * L.bstride;
    L.total = o;
    return L;
}

#ifndef MR_WIDE_WAVES
#define MR_WIDE_WAVES 3  // waves per SIMD the wide kernel's register budget is cut for: 3 ran c5 27 %
                         // faster than 2 (LDS holds 3 workgroups of 28 B label tables); 4 spilled 480 B
#endif
template <uint32_t PERM, uint32_t SPL>
__global__ __launch_bounds__(kBS, MR_WIDE_WAVES) void hub_wide_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t NS = a->p.NS, nreg = a->nreg;
    const WideLayout L = wide_layout(NS, nreg);
    SpecialStatic *spl = reinterpret_cast<SpecialStatic *>(smem + L.off_sp);
    uint16_t *hubl = reinterpret_cast<uint16_t *>(smem + L.off_hubs);
    for (uint32_t t = threadIdx.x; t <= NS; t += kBS) spl[t] = a->sp[t];
    for (uint32_t h = threadIdx.x; h < a->p.n_hubs; h += kBS) hubl[h] = a->hubs[h];
    __syncthreads();
    const uint32_t slot = threadIdx.x >> 6;
    HubWide<SPL> H;
    H.a = a;
    H.P = a->p;
    H.P.perm[0] = PERM / 9;
    H.P.perm[1] = (PERM / 3) % 3;
    H.P.perm[2] = PERM % 3;
    H.P.ff_num = H.P.ff_den = 1;
    H.rank = a->rank;
    H.sinfo = a->sinfo;
    H.counter = a->counter;
    H.sh = nullptr;
    H.R = reinterpret_cast<Rec *>(smem + L.off_R + slot * L.rstride);
    H.state = nullptr;
    H.sp = spl;
    H.hubs = hubl;
    H.dst = nullptr;
    H.src = 0;
    H.src_rk = 0;
    H.bnd = reinterpret_cast<uint32_t *>(smem + L.off_bnd + slot * L.bstride);
    H.lexs = nullptr;
    H.blk = reinterpret_cast<uint32_t *>(smem + L.off_blk + slot * L.bstride);
    H.nearS = a->near_sp;  // specials' region rows (global, (NS+1) x nreg x 2 words)
    H.srow = reinterpret_cast<uint32_t *>(smem + L.off_srow + slot * L.sstride);
    H.nreg = nreg;
    const uint32_t waves = gridDim.x * (kBS / 64), wid = blockIdx.x * (kBS / 64) + slot;
    for (uint32_t s = wid; s < a->nsrc; s += waves) H.solve(s);
    H.flush_err();
    __shared__ uint32_t wsum;
    if (threadIdx.x == 0) wsum = 0;
    __syncthreads();
    if (H.written) atomicAdd(&wsum, H.written);
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, wsum);
}

// ===================================================================================
// All-destinations fill: the record of every cell of every
// hub-solved source is the best walk from its boundaries — metrics in comparator
// order, then the boundary's rank (precomputed by the hub kernel).
//
// Work is (source, 64x16 tile) items, one per wave, no workgroup barriers.  The
// waves form groups; a group takes a run of sources one after another, and its
// waves interleave each source's tiles (wave j of the group takes tiles j, j + G,
// ...).  Waves running side by side then write neighbouring tiles, whose 1 KB rows
// join into long runs: on gfx950 that shape stores at ~4.1 TB/s against ~2.6-3.0
// for 32x32 tiles taken in order (tools/probes/store_probe.hip).  A wave's LDS
// tables (the boundaries by rank, the specials' own labels by table index) are
// reloaded only when its source changes; the item loop makes no global load (on
// gfx950 vmcnt also counts stores, so a load there would wait for earlier stores).
//
// Per tile the wave prunes the boundaries whose leading metric is beaten everywhere
// in it (wave min + ballot).  Lane l owns column l and rows i < 16.  When the three
// metrics fit one 63-bit key (fields sized per source from the table's maxima) and
// the tile does not touch the axes through the Center (no detours), a walk's key is
// K_b + d * slope, so down a column it moves by +-slope per row: the sweep over a
// boundary's 16 cells is a 64-bit add, a compare and three selects per cell.
// Otherwise the cell's walk distance and the three-metric compare are evaluated in
// full.  The specials of the tile and the source then overwrite their cells.
// =====================================================================================
__device__ __forceinline__ uint32_t bit_width64(unsigned long long x) { return x ? 64u - uint32_t(__clzll(x)) : 0u; }

// the fill kernel's rare path: a tile whose source's keys do not fit 32 bits.  Row
// by row, each cell's walk distance in full and the three-metric compare.
// AggregatedCost::time of a StandardMove run of d legs at Fleetfoot ratio fn/fd (the
// ceil of src/skill.rs:21-30; fn == fd: linear)
__device__ __forceinline__ uint32_t run_time_ff(uint32_t d, uint32_t fn, uint32_t fd) {
    return fn == fd ? 180u * d : uint32_t(floor_div(180ll * d * fn + fd - 1, fd));
}

template <uint32_t PERM>
__device__ __forceinline__ void fill_tile_rows(const uint32_t (*B)[64], unsigned long long live, int wx,
                                                      int y0, int ty0, int cx, uint32_t S, uint32_t pitch, CellWord *outs,
                                                      uint32_t fn, uint32_t fd) {
    constexpr uint32_t q0 = PERM / 9, q1 = (PERM / 3) % 3, q2 = PERM % 3;
#pragma unroll 1
    for (int i = 0; i < int(kFillTH); ++i) {
        uint32_t r0 = 0xFFFFFFFFu, r1 = 0xFFFFFFFFu, r2 = 0xFFFFFFFFu, rv = 0xFFFFFFFFu;
        for (unsigned long long m = live; m; m &= m - 1) {  // rank order: the first of equal metrics wins
            const uint32_t rr = uint32_t(__ffsll((long long)m) - 1);
            const uint32_t d = walk_dist(int(B[0][rr]), int(B[1][rr]), wx, y0 + i);
            const uint32_t b0 = B[2][rr], b1 = B[3][rr], b2 = B[4][rr];
            const uint32_t mm0 = b0 + d, mm2 = b2 + run_time_ff(d, fn, fd);
            const uint32_t c1 = q0 == 0 ? mm0 : (q0 == 1 ? b1 : mm2);
            const uint32_t c2 = q1 == 0 ? mm0 : (q1 == 1 ? b1 : mm2);
            const uint32_t c3 = q2 == 0 ? mm0 : (q2 == 1 ? b1 : mm2);
            const uint32_t k1 = q0 == 0 ? r0 : (q0 == 1 ? r1 : r2);
            const uint32_t k2 = q1 == 0 ? r0 : (q1 == 1 ? r1 : r2);
            const uint32_t k3 = q2 == 0 ? r0 : (q2 == 1 ? r1 : r2);
            const bool better = c1 < k1 || (c1 == k1 && (c2 < k2 || (c2 == k2 && c3 < k3)));
            r0 = better ? mm0 : r0;
            r1 = better ? b1 : r1;
            r2 = better ? mm2 : r2;
            rv = better ? B[5][rr] : rv;
        }
        // the cell word b << 20 | k: B[5] holds (b << 20) - legs(b), r0 = legs(b) + k
        const int cy = ty0 + i;
        if (cy < int(S) && cx < int(pitch)) outs[uint32_t(cy) * pitch + uint32_t(cx)] = rv + r0;  // (pad columns too)
    }
}

#ifndef MR_FILL_WAVES
#define MR_FILL_WAVES 6  // waves per SIMD the fill kernel is register-bounded to
#endif
// the fill's work as workgroup `block` of `nblocks` (its own launch, or the workgroups
// after the hub's in a fused hub + fill launch)
template <uint32_t PERM>
__device__ __forceinline__ void fill_body(const KArgs *__restrict__ a, uint32_t block, uint32_t nblocks) {
    constexpr uint32_t q0 = PERM / 9, q1 = (PERM / 3) % 3, q2 = PERM % 3;
    // per unit of walk distance: legs 1, money 0, time 180 s
    constexpr uint32_t sl[3] = {1u, 0u, 180u};
    constexpr int kTW = int(kFillTW), kTH = int(kFillTH), kCPL = kTW / 64;  // kCPL columns per lane
    // per wave: boundaries by rank (x, y, m0, m1, m2, key), the cell word's parts by
    // srank (or by rank for the full compare), specials by table index (x, y; entry 0 =
    // the source)
    __shared__ uint32_t btab[kBS / 64][10][64];
    // the wave index through readfirstlane: everything derived from it (tile origins,
    // key fields, slopes) then lives in SGPRs
    const uint32_t lane = threadIdx.x & 63u, wv = uint32_t(__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)));
    uint32_t(*B)[64] = btab[wv];
    uint32_t(*P)[64] = btab[wv] + 8;
    // (certificate slots: as many sources as the hub kernel exported this pass)
    const uint32_t NS = a->p.NS, T = NS + 1, S = a->p.S, pitch = a->rec_pitch;
    const uint32_t nsrc = a->nsrc_dev ? min(a->nsrc, *a->nsrc_dev) : a->nsrc;
    // Fleetfoot 1..3 (certificate slots only): walk times through the ceil, so the
    // full-compare path, and prune bounds from run_time_ff
    const uint32_t fn = a->p.ff_num, fd = a->p.ff_den;
    const bool nonlin = fn != fd;
    const int H = int(a->p.H);
    const uint32_t tpx = (S + kTW - 1) / kTW, tpy = (S + kTH - 1) / kTH, ntile = tpx * tpy;
    const bool no_prune = (a->dbg_flags & 1u) != 0, no_pack = (a->dbg_flags & 2u) != 0;
    if ((a->dbg_flags & kDbgInjectFlag) && block == 0 && threadIdx.x == 0) atomicOr(a->counter + kCtrFlags, kErrChain);
    const uint32_t nwaves = nblocks * (kBS / 64), gw = block * (kBS / 64) + wv;
    // At least kFillMinG waves share a source: with one wave per source, as many
    // sources' 4 MB output regions as waves are written at once, and the stores slow
    // down (4096 sources a pass: 5.3 ms with one wave per source, 4.1 ms with four).
    // MR_DBG_FLAGS bit 5 lifts the bound (experiments).
    constexpr uint32_t kFillMinG = 4;
    const uint32_t gcap = (a->dbg_flags & 32u) ? nwaves : max(1u, nwaves / kFillMinG);
    const uint32_t ngroups = max(1u, min(nsrc, gcap)), G = nwaves / ngroups, g = gw / G, j = gw % G;
    // Group g takes sources g, g + ngroups, ...: the groups work through the plan's
    // sources side by side, so the words being written at any time span about ngroups
    // sources (~5 GB at 1025^2), not the whole output (4096 sources a pass: 3.8 ms
    // against 4.9 with a contiguous run of sources per group, which MR_DBG_FLAGS bit 6
    // keeps for experiments).
    const bool runs = (a->dbg_flags & 64u) != 0;
    const uint32_t s_begin = g >= ngroups ? nsrc : (runs ? uint32_t(uint64_t(g) * nsrc / ngroups) : g);
    const uint32_t s_end = g >= ngroups ? nsrc : (runs ? uint32_t(uint64_t(g + 1) * nsrc / ngroups) : nsrc);
    const uint32_t s_step = runs ? 1u : ngroups;
    for (uint32_t s = s_begin; s < s_end; s += s_step) {
        if (a->src_state[s] != 1) continue;  // solved by the SSSP kernel, which wrote its records
        // ---- this source's tables -------------------------------------------------
        const unsigned long long tb = (unsigned long long)s * T;
        const uint32_t src = a->src_v[s];
        wave_sync();  // the previous source's tables have been read
        uint32_t r = kNone32, e0 = 0, e1 = 0, e2 = 0;
        if (lane < T) {
            r = a->out_lex[tb + lane];
            const Rec &e = a->out_tab[tb + lane];
            e0 = e.m[0];
            e1 = e.m[1];
            e2 = e.m[2];
            const uint32_t x = lane == 0 ? uint32_t(int(src % S) - H) : uint32_t(a->sp[lane].x);
            const uint32_t y = lane == 0 ? uint32_t(int(src / S) - H) : uint32_t(a->sp[lane].y);
            P[0][lane] = x;
            P[1][lane] = y;
            if (r != kNone32) {
                B[0][r] = x;
                B[1][r] = y;
                B[2][r] = e0;
                B[3][r] = e1;
                B[4][r] = e2;
            }
        }
        const bool isb = lane < T && r != kNone32;
        const uint32_t nb = uint32_t(__popcll(__ballot(isb)));
        const uint64_t dmax = 2ull * S + 2;  // the longest walk (round the Center)
        const uint64_t em[3] = {e0, e1, e2};
        // The lead metric: the first in comparator order that grows along a walk.  With
        // Money first every walk keeps its boundary's money, so only the boundaries of
        // the least money can win anywhere ("kept"); the lead is then the second metric.
        // Where two walks tie on the lead, their distances differ by a fixed amount, so
        // every metric after it compares as a per-boundary constant c_q = sL * base_q -
        // s_q * base_L, then the boundary's rank: (c, rank) order the tied walks exactly
        // like the comparator.  A walk's key is therefore lead << rbs | srank, srank the
        // boundary's position in that constant order: 32 bits, one add and one min per
        // cell and boundary.
        constexpr uint32_t L = q0 == 1 ? q1 : q0, T1 = q0 == 1 ? q2 : q1, T2 = q0 == 1 ? 3u : q2;
        constexpr uint32_t sL = sl[L];
        bool kept = isb;
        if (q0 == 1) {
            uint32_t mmin = isb ? e1 : 0xFFFFFFFFu;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) mmin = min(mmin, uint32_t(__shfl_xor(int(mmin), o)));
            kept = isb && e1 == mmin;
        }
        const unsigned long long keptm = __ballot(kept);
        const uint32_t nk = uint32_t(__popcll(keptm));
        // the kept boundaries below this one in (c_T1, c_T2, rank) order (every lane takes
        // part in the shuffles)
        uint32_t srank = 0;
        const long long c1 = (long long)sL * (long long)em[T1] - (long long)sl[T1] * (long long)em[L];
        const long long c2 = T2 < 3u ? (long long)sL * (long long)em[T2 % 3u] - (long long)sl[T2 % 3u] * (long long)em[L] : 0;
        for (unsigned long long m = keptm; m; m &= m - 1) {
            const int o = __ffsll((long long)m) - 1;  // table index of a kept boundary
            const uint32_t ro = uint32_t(__shfl(int(r), o));
            const long long o1 = __shfl(c1, o), o2 = __shfl(c2, o);
            srank += (o1 < c1 || (o1 == c1 && (o2 < c2 || (o2 == c2 && ro < r)))) ? 1u : 0u;
        }
        uint64_t mxL = kept ? em[L] + sL * dmax : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mxL = max(mxL, (uint64_t)__shfl_xor((unsigned long long)mxL, o));
        const uint32_t rbs = max(1u, bit_width64(nk - 1));
        const uint32_t wL = uint32_t(__builtin_amdgcn_readfirstlane(int(max(1u, bit_width64(mxL)))));
        // keys wider than 32 bits (or MR_DBG_FLAGS bit 1): the rare full-compare path
        const bool packable = !no_pack && !nonlin && wL + rbs <= 32u;
        const uint32_t stepL = packable ? sL << rbs : 0u, maskr = (1u << rbs) - 1u;
        if (packable) {
            if (isb) B[6][r] = kept ? uint32_t(em[L] << rbs) | srank : 0xFFFFFFFFu;  // by rank
            if (kept) {  // by srank: the cell word's table index and the lead's base
                // (sL = 1: one word, (b << 20) - base, + the lead = b << 20 | k)
                B[5][srank] = sL == 1u ? (lane << kStBShift) - uint32_t(em[L]) : lane << kStBShift;
                B[7][srank] = uint32_t(em[L]);
            }
        } else if (isb) {
            B[5][r] = (lane << kStBShift) - e0;  // full compare (fill_tile_rows): + the cell's legs
        }
        wave_sync();
        // rank `lane`'s boundary position and key in registers: the boundary loop reads
        // them with v_readlane (no LDS round trip per boundary and tile)
        const uint32_t bx_l = lane < nb ? B[0][lane] : 0u, by_l = lane < nb ? B[1][lane] : 0u;
        const uint32_t px_l = lane < T ? P[0][lane] : 0u, py_l = lane < T ? P[1][lane] : 0u;  // specials by table index
        const uint32_t bk_l = lane < nb && packable ? B[6][lane] : 0u;
        // prune on the lead metric (the full compare: on the first one, every boundary);
        // whether rank `lane`'s boundary is kept (Money first) is read off its key
        const uint32_t PL = packable ? L : q0;
        const uint64_t sP = packable ? sL : sl[q0];
        const uint32_t pb_l = lane < nb ? B[2 + PL][lane] : 0u;
        const bool cnd = lane < nb && (!packable || bk_l != 0xFFFFFFFFu);
        // ---- this wave's tiles of the source ---------------------------------------
        CellWord *const outs = a->out_rec + (unsigned long long)s * S * pitch;
        for (uint32_t tile = j; tile < ntile; tile += G) {
            const int tx0 = int(tile % tpx) * kTW, ty0 = int(tile / tpx) * kTH;
            const int x0 = tx0 - H, y0 = ty0 - H;
            const int x1 = min(tx0 + kTW - 1, int(S) - 1) - H, y1 = min(ty0 + kTH - 1, int(S) - 1) - H;
            // Prune the boundaries whose lead metric is beaten everywhere in the tile:
            // lo_b > min over b' of hi_b' (walks are at least the L1 distance to the tile
            // and at most the farthest corner's plus the 2-cell detour round the Center).
            const int bxx_l = int(bx_l), byy_l = int(by_l);
            const int dx = bxx_l < x0 ? x0 - bxx_l : (bxx_l > x1 ? bxx_l - x1 : 0);
            const int dy = byy_l < y0 ? y0 - byy_l : (byy_l > y1 ? byy_l - y1 : 0);
            const int fx = max(abs(bxx_l - x0), abs(bxx_l - x1)), fy = max(abs(byy_l - y0), abs(byy_l - y1));
            unsigned long long live;
            if (packable) {  // the lead fits 32 bits (<= mxL): DPP wave mins, no LDS round trips
                const uint32_t sP32 = uint32_t(sP);
                const uint32_t lo = pb_l + sP32 * uint32_t(dx + dy);
                const uint32_t hi = cnd ? pb_l + sP32 * uint32_t(fx + fy + 2) : 0xFFFFFFFFu;
                const uint32_t hmin = wave_min_u32(hi);
                // Corner dominance: L1(b*, c) - L1(b, c) splits into an x and a y term, each
                // monotone in its coordinate, so over the tile its maximum sits at a corner.
                // A boundary b* whose lead, with the 2-cell Center detour as slack, beats b's
                // at all four corners beats it at every cell of the tile (strictly, on the
                // lead), and b is dropped.  b* = the least lead at the tile's centre.
                const int cxm = (x0 + x1) >> 1, cym = (y0 + y1) >> 1;
                const uint32_t vc = cnd ? pb_l + sP32 * uint32_t(abs(bxx_l - cxm) + abs(byy_l - cym)) : 0xFFFFFFFFu;
                const uint32_t vmin = wave_min_u32(vc);
                const unsigned long long bs = __ballot(cnd && vc == vmin);
                const int star = bs ? __ffsll((long long)bs) - 1 : 0;
                const uint32_t c00 = pb_l + sP32 * uint32_t(abs(bxx_l - x0) + abs(byy_l - y0));
                const uint32_t c10 = pb_l + sP32 * uint32_t(abs(bxx_l - x1) + abs(byy_l - y0));
                const uint32_t c01 = pb_l + sP32 * uint32_t(abs(bxx_l - x0) + abs(byy_l - y1));
                const uint32_t c11 = pb_l + sP32 * uint32_t(abs(bxx_l - x1) + abs(byy_l - y1));
                const uint32_t slack = 2u * sP32;
                // b*'s corners read with every lane active (a v_readlane of a value computed
                // under a narrower exec mask reads a stale register), then compared without
                // short-circuit branches
                const uint32_t s00 = uint32_t(__builtin_amdgcn_readlane(int(c00), star)) + slack;
                const uint32_t s10 = uint32_t(__builtin_amdgcn_readlane(int(c10), star)) + slack;
                const uint32_t s01 = uint32_t(__builtin_amdgcn_readlane(int(c01), star)) + slack;
                const uint32_t s11 = uint32_t(__builtin_amdgcn_readlane(int(c11), star)) + slack;
                const bool dom = (bs != 0ull) & (s00 < c00) & (s10 < c10) & (s01 < c01) & (s11 < c11);
                live = __ballot(cnd && ((lo <= hmin && !dom) || no_prune));
            } else {
                unsigned long long lo = ~0ull, hi = ~0ull;
                if (cnd) {
                    const bool tl = PL == 2u;  // a time lead grows by the run time
                    lo = pb_l + (tl ? uint64_t(run_time_ff(uint32_t(dx + dy), fn, fd)) : sP * uint64_t(dx + dy));
                    hi = pb_l + (tl ? uint64_t(run_time_ff(uint32_t(fx + fy + 2), fn, fd)) : sP * uint64_t(fx + fy + 2));
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long h2 = __shfl_xor(hi, o);
                    hi = h2 < hi ? h2 : hi;
                }
                live = __ballot(cnd && (lo <= hi || no_prune));
            }
            // the specials (and the source) inside this tile
            const int px = int(px_l) - x0, py = int(py_l) - y0;
            const unsigned long long sp_in = __ballot(lane < T && px >= 0 && px < kTW && py >= 0 && py < kTH);
            const bool axis = (x0 <= 0 && x1 >= 0) || (y0 <= 0 && y1 >= 0);
            if (packable) {
                // the least key per cell (column c = lane + 64k, row i at k * kTH + i)
                uint32_t kb[kCPL * kTH];
#pragma unroll
                for (int i = 0; i < kCPL * kTH; ++i) kb[i] = 0xFFFFFFFFu;
                // boundaries on an axis through the Center, in a tile on an axis, take
                // walk_dist's 2-cell detour to cells on the same axis across the Center:
                // they get a loop of their own after the others
                unsigned long long axm = 0;
                if (axis) {
                    const bool on = lane < nb && (bx_l == 0u || by_l == 0u);
                    axm = __ballot(on) & live;
                }
                for (unsigned long long m = live & ~axm; m; m &= m - 1) {
                    const uint32_t rr = uint32_t(__ffsll((long long)m) - 1);
                    // wave-uniform values in SGPRs
                    const int bxx = __builtin_amdgcn_readlane(int(bx_l), int(rr));
                    const int istar = __builtin_amdgcn_readlane(int(by_l), int(rr)) - y0;  // the boundary's row in the tile
                    const uint32_t K = uint32_t(__builtin_amdgcn_readlane(int(bk_l), int(rr)));
                    const uint32_t up = stepL, down = 0u - stepL;
                    // down a column the walk distance moves by +-1 per row, so the key by
                    // +-stepL; a boundary above (below) the tile's rows steps every row the
                    // same way, which needs no per-row select
                    if (istar <= 0 || istar >= kTH - 1) {
                        const uint32_t step = istar <= 0 ? up : down;
#pragma unroll
                        for (int k = 0; k < kCPL; ++k) {
                            const int wx = x0 + 64 * k + int(lane);
                            uint32_t key = K + stepL * (uint32_t(abs(bxx - wx)) + uint32_t(abs(istar)));
#pragma unroll
                            for (int i = 0; i < kTH; ++i) {
                                if (i > 0) key += step;
                                kb[k * kTH + i] = min(kb[k * kTH + i], key);
                            }
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < kCPL; ++k) {
                            const int wx = x0 + 64 * k + int(lane);
                            uint32_t key = K + stepL * (uint32_t(abs(bxx - wx)) + uint32_t(abs(istar)));
#pragma unroll
                            for (int i = 0; i < kTH; ++i) {
                                if (i > 0) key += i > istar ? up : down;
                                kb[k * kTH + i] = min(kb[k * kTH + i], key);
                            }
                        }
                    }
                }
                for (unsigned long long m = axm; m; m &= m - 1) {
                    const uint32_t rr = uint32_t(__ffsll((long long)m) - 1);
                    const int bxx = __builtin_amdgcn_readlane(int(bx_l), int(rr));
                    const int byy = __builtin_amdgcn_readlane(int(by_l), int(rr));
                    const int istar = byy - y0, i0 = -y0;  // i0: the tile's row y = 0
                    const uint32_t K = uint32_t(__builtin_amdgcn_readlane(int(bk_l), int(rr)));
                    const uint32_t up = stepL, down = 0u - stepL, det2 = 2u * stepL;
#pragma unroll
                    for (int k = 0; k < kCPL; ++k) {
                        const int wx = x0 + 64 * k + int(lane);
                        uint32_t key = K + stepL * (uint32_t(abs(bxx - wx)) + uint32_t(abs(istar)));
                        const bool detx = byy == 0 && wx != 0 && bxx != 0 && ((wx < 0) != (bxx < 0));
                        const bool dety = bxx == 0 && wx == 0 && byy != 0;
#pragma unroll
                        for (int i = 0; i < kTH; ++i) {
                            if (i > 0) key += i > istar ? up : down;
                            const bool det = (i == i0 && detx) || (dety && i != i0 && ((i < i0) != (byy < 0)));
                            kb[k * kTH + i] = min(kb[k * kTH + i], key + (det ? det2 : 0u));
                        }
                    }
                }
                // The cell words first: every row's LDS read issued before one wait (kb's
                // unused cells hold all ones, a valid srank).  Then buffer stores off one
                // per-tile base: the lane's offset in a VGPR, the row's (i * S * 4 B) in an
                // SGPR, so no per-row 64-bit address; a row's kCPL stores are one
                // contiguous run of kTW cell words.  A tile inside the grid stores with no
                // per-row mask.
                uint32_t wd[kCPL * kTH];
#pragma unroll
                for (int i = 0; i < kCPL * kTH; ++i) {
                    // the cell word b << 20 | k: k = (lead - the boundary's lead) / sL
                    const uint32_t kv = kb[i], sr = kv & maskr;
                    wd[i] = sL == 1u ? B[5][sr] + (kv >> rbs) : B[5][sr] + ((kv >> rbs) - B[7][sr]) / sL;
                }
                // Rows are padded to a multiple of 32 cells (rec_pitch: 128 B, one line), so
                // every tile row is whole aligned lines, pad columns included: no store ever
                // writes part of a line (partial lines, from one wave or from two XCDs' L2s,
                // halve the HBM write rate once the output outgrows the Infinity Cache).
                // Only the grid's last tile row masks rows, and its last tile column the
                // lanes past the pitch (a 32-cell line).
                const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                    outs + (size_t(ty0) * pitch + size_t(tx0)), 0, int(4u * kTH * pitch), 0x00020000);  // the tile's rows
                if (ty0 + kTH <= int(S) && tx0 + kTW <= int(pitch)) {
                    // (row offsets stepped in a VGPR: per-row SGPR offsets ran out of SGPRs)
                    uint32_t vo = lane * 4u;
#pragma unroll
                    for (int i = 0; i < kTH; ++i) {
#pragma unroll
                        for (int k = 0; k < kCPL; ++k)
                            __builtin_amdgcn_raw_buffer_store_b32(wd[k * kTH + i], rsrc, int(vo + 256u * k), 0, 0);
                        vo += pitch * 4u;
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < kTH; ++i) {
#pragma unroll
                        for (int k = 0; k < kCPL; ++k) {
                            if (ty0 + i < int(S) && tx0 + 64 * k + int(lane) < int(pitch))
                                __builtin_amdgcn_raw_buffer_store_b32(wd[k * kTH + i], rsrc, int((64u * k + lane) * 4u),
                                                                      int(uint32_t(i) * pitch * 4u), 0);
                        }
                    }
                }
            } else {
                for (int k = 0; k < kCPL; ++k) {  // keys too wide for 32 bits
                    const int cx = tx0 + 64 * k + int(lane);
                    fill_tile_rows<PERM>(B, live, x0 + 64 * k + int(lane), y0, ty0, cx, S, pitch, outs, fn, fd);
                }
            }
            // specials' cells hold their own labels, the source's cell (last: it may also
            // be a special) the start label.  These stores follow the lane's own store to
            // the same cell, so they are the ones that land.
            for (unsigned long long m = sp_in; m;) {
                uint32_t t;
                if (m & ~1ull) {
                    t = uint32_t(__ffsll((long long)(m & ~1ull)) - 1);
                    m &= ~(1ull << t);
                } else {
                    t = 0;
                    m = 0;
                }
                const int px = int(P[0][t]) - x0, py = int(P[1][t]) - y0;
                if (lane == uint32_t(px) % 64u)
                    outs[uint32_t(ty0 + py) * pitch + uint32_t(tx0 + px)] = t == 0 ? kViaSource : (kViaSpecial | t);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, 0, nblocks);
}
template <uint32_t PERM>
__global__ __launch_bounds__(kBS, MR_FILL_WAVES) void fill_kernel(const KArgs *__restrict__ a) {
    fill_body<PERM>(a, blockIdx.x, gridDim.x);
}
// All destinations, one launch per pass: the first hub_blocks workgroups solve the
// specials of the NEXT pass into its slot (hub_a), the others fill this pass's cell
// words from the tables the previous launch left (fill_a).  The specials' solve (~85 us
// for 64 sources on 32 waves) then runs beside the fill with no cross-stream events.
template <uint32_t PERM, uint32_t SPW>
__global__ __launch_bounds__(kBS, MR_HUB_WAVES) void hub_fill_kernel(const KArgs *__restrict__ hub_a,
                                                                     const KArgs *__restrict__ fill_a,
                                                                     uint32_t hub_blocks) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (blockIdx.x < hub_blocks) hub_body<PERM, SPW, false>(hub_a, smem, blockIdx.x, hub_blocks);
    else fill_body<PERM>(fill_a, blockIdx.x - hub_blocks, gridDim.x - hub_blocks);
}

// ===================================================================================
// LDS layout and kernels
// ===================================================================================
__host__ __device__ constexpr uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

struct LdsLayout {
    uint32_t off_R, off_a, off_b, off_c, off_d, off_sp, off_hubs, off_dst, off_state, off_l[4], total;
};

// per-table arrays (NS+1 entries each): a 8 B (legs: best64), b/c/d 4 B
// (legs: prio, bnd, fired; generic: best, -, fired); grid part (LDS regime):
// state 4 B/vertex + 2 (legs) or 4 (generic) u16 lists.
__host__ __device__ inline LdsLayout lds_layout(uint32_t NS, uint32_t V, bool grid_in_lds, uint32_t algo) {
    LdsLayout L{};
    const uint32_t T = NS + 1;
    uint32_t o = align16(sizeof(Shared));
    L.off_R = o;
    o = align16(o + T * uint32_t(sizeof(Rec)));
    L.off_a = o;
    o = align16(o + T * 8);
    L.off_b = o;
    o = align16(o + T * 4);
    L.off_c = o;
    o = align16(o + T * 4);
    L.off_d = o;
    o = align16(o + T * 4);
    L.off_sp = o;
    o = align16(o + T * uint32_t(sizeof(SpecialStatic)));
    L.off_hubs = o;
    o = align16(o + T * 2);
    L.off_dst = o;
    o = align16(o + 64 * 4);
    if (grid_in_lds) {
        L.off_state = o;
        o = align16(o + V * 4);
        const uint32_t nl = algo == kAlgoLegs ? 2u : 4u;
        for (uint32_t i = 0; i < 4; ++i) {
            L.off_l[i] = o;
            if (i < nl) o = align16(o + V * 2);
        }
    }
    L.total = o;
    return L;
}

// next source index for a workgroup: every source in order, or (fallback launch
// after the hub solver) the sources it listed
__device__ __forceinline__ uint32_t next_source(const KArgs *__restrict__ a, uint32_t &slot, uint32_t &entry) {
    slot = kNone32;
    entry = kNone32;
    if (a->fb_mode) {
        const uint32_t n = __hip_atomic_load(a->counter + kCtrFbCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t i = atomicAdd(a->counter + kCtrFbDequeue, 1u);
        if (i >= n) return kNone32;
        if (a->fb_cert) slot = a->fb_cert[i];
        if (slot >= a->cert_cap) slot = kNone32;  // none, or staged without a slot
        entry = i;
        return a->fb_list[i] & ~kFbCertified;
    }
    const uint32_t i = atomicAdd(a->counter + kCtrDequeue, 1u);
    return i < a->nsrc ? i : kNone32;
}

template <bool G, class IdxT, uint32_t ALGO>
__global__ __launch_bounds__(kBS) void solve_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // fallback launch after the hub solver: nothing to do unless it listed sources
    if (a->fb_mode && __hip_atomic_load(a->counter + kCtrFbCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (threadIdx.x == 0) finish_launch(a, 0);
        return;
    }
    const uint32_t V = a->p.V, NS = a->p.NS;
    const LdsLayout L = lds_layout(NS, V, !G, ALGO);
    Shared *sh = reinterpret_cast<Shared *>(smem);
    Rec *R = reinterpret_cast<Rec *>(smem + L.off_R);
    uint32_t *state;
    IdxT *l0, *l1, *l2, *l3;
    if constexpr (G) {
        uint32_t *slot = a->ws + (unsigned long long)blockIdx.x * 5ull * V;
        state = slot;
        l0 = reinterpret_cast<IdxT *>(slot + V);
        l1 = reinterpret_cast<IdxT *>(slot + 2ull * V);
        l2 = reinterpret_cast<IdxT *>(slot + 3ull * V);
        l3 = reinterpret_cast<IdxT *>(slot + 4ull * V);
    } else {
        state = reinterpret_cast<uint32_t *>(smem + L.off_state);
        l0 = reinterpret_cast<IdxT *>(smem + L.off_l[0]);
        l1 = reinterpret_cast<IdxT *>(smem + L.off_l[1]);
        l2 = reinterpret_cast<IdxT *>(smem + L.off_l[2]);
        l3 = reinterpret_cast<IdxT *>(smem + L.off_l[3]);
    }
    SpecialStatic *spl = reinterpret_cast<SpecialStatic *>(smem + L.off_sp);
    uint16_t *hubl = reinterpret_cast<uint16_t *>(smem + L.off_hubs);
    uint32_t *dstl = reinterpret_cast<uint32_t *>(smem + L.off_dst);
    for (uint32_t t = threadIdx.x; t <= NS; t += kBS) spl[t] = a->sp[t];
    for (uint32_t h = threadIdx.x; h < a->p.n_hubs; h += kBS) hubl[h] = a->hubs[h];
    __syncthreads();
    uint32_t written = 0;  // result records of this workgroup's sources (thread 0 reports them)
    if constexpr (ALGO == kAlgoLegs) {
        LegsSolver<G, IdxT> S;
        S.a = a;
        S.P = a->p;
        S.rank = a->rank;
        S.sinfo = a->sinfo;
        S.counter = a->counter;
        S.sh = sh;
        S.R = R;
        S.state = state;
        S.sp = spl;
        S.hubs = hubl;
        S.dst = dstl;
        S.src = 0;
        S.src_rk = 0;
        S.F0 = l0;
        S.F1 = l1;
        S.best64 = reinterpret_cast<unsigned long long *>(smem + L.off_a);
        S.prio = reinterpret_cast<uint32_t *>(smem + L.off_b);
        S.bnd = reinterpret_cast<uint32_t *>(smem + L.off_c);
        S.fired = reinterpret_cast<uint32_t *>(smem + L.off_d);
        (void)l2;
        (void)l3;
        Stamps stamps;
        stamps.start();
        S.stamps = &stamps;
        uint32_t nsolved = 0;
        for (;;) {
            if (threadIdx.x == 0) sh->sidx = next_source(a, sh->sslot, sh->sentry);
            __syncthreads();
            const uint32_t s = sh->sidx, slot = sh->sslot;
            __syncthreads();
            if (s == kNone32) break;
            if (slot != kNone32 && S.cert_emit(s, slot)) {
                if (threadIdx.x == 0) {
                    atomicAdd(a->counter + kCtrCertDone, 1u);
                    a->fb_list[sh->sentry] |= kFbCertified;  // answered without a search
                }
            } else {
                S.solve(s);
            }
            written += a->q_begin[s + 1] - a->q_begin[s];
            ++nsolved;
        }
        S.flush_err();
#ifdef MR_STAMPS
        if (threadIdx.x == 0 && a->dbg) {
            for (int i = 0; i < 8; ++i) a->dbg[blockIdx.x * 10 + i] = stamps.acc[i];
            a->dbg[blockIdx.x * 10 + 8] = nsolved;
        }
#else
        (void)nsolved;
#endif
    } else {
        GenericSolver<G, IdxT> S;
        S.a = a;
        S.P = a->p;
        S.rank = a->rank;
        S.sinfo = a->sinfo;
        S.counter = a->counter;
        S.sh = sh;
        S.R = R;
        S.state = state;
        S.sp = spl;
        S.hubs = hubl;
        S.dst = dstl;
        S.src = 0;
        S.src_rk = 0;
        S.L0b = l0;
        S.lstride = uint32_t(l1 - l0);
        S.dirty = l3;
        S.best = reinterpret_cast<uint32_t *>(smem + L.off_b);
        S.fired = reinterpret_cast<uint32_t *>(smem + L.off_d);
        for (;;) {
            if (threadIdx.x == 0) sh->sidx = next_source(a, sh->sslot, sh->sentry);
            __syncthreads();
            const uint32_t s = sh->sidx, slot = sh->sslot;
            __syncthreads();
            if (s == kNone32) break;
            if (slot != kNone32 && S.cert_emit(s, slot)) {
                if (threadIdx.x == 0) {
                    atomicAdd(a->counter + kCtrCertDone, 1u);
                    a->fb_list[sh->sentry] |= kFbCertified;  // answered without a search
                }
            } else {
                S.solve(s);
            }
            written += a->q_begin[s + 1] - a->q_begin[s];
        }
        S.flush_err();
    }
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, written);
}

}  // namespace mr
