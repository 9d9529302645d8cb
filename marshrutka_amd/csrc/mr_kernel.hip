// mr_kernel.hip — gfx950 single-source solves for the pathfinder hot path.
//
// Replaces the body of FindPath::eval (src/pathfinder.rs:199-248): the binary
// heap frontier (src/binary_heap.rs) becomes bucketed parallel settling, the
// per-pop edge generator (Inflight::edges, src/pathfinder.rs:24-180) becomes
// implicit grid neighbours + a small table of teleport edges, and the ~240 B
// cloned labels (src/cost.rs:187-315) become one 32-bit word per grid vertex.
// See mr_engine.hpp for the layout and DESIGN.md §3 for the exactness argument.
//
// One 256-thread workgroup solves one source at a time (sources are dequeued
// from a global counter).  Per bucket B:
//   1. settle   — every plain vertex listed for B is final: mark it, feed the
//                 Scroll-of-Escape region argmin, mark its 4 neighbours dirty;
//   2. specials — wave 0: fire SoE candidates, then an exact Dijkstra over the
//                 specials whose tentative label lies in bucket B (wave argmin);
//   3. pull     — every dirty vertex recomputes its best walk label from its
//                 settled neighbours (deterministic, no label atomics); a plain
//                 vertex is appended to the list of bucket B+1 or B+2 on first touch;
//   4. next     — B' = min(non-empty list buckets, tentative specials).
// Grid state lives in LDS when it fits (G=false) and in a per-workgroup HBM
// slot otherwise (G=true; cross-thread words then go through sc1 loads).
#include <hip/hip_runtime.h>

#include "mr_engine.hpp"

namespace mr {

struct Shared {
    unsigned long long B;        // current bucket key
    uint32_t cnt[3];             // list counts per buffer
    uint32_t lb;                 // list rotation base: L0 = buf[lb]
    uint32_t nd;                 // dirty count
    uint32_t sidx;
    uint32_t done;
    uint32_t pad[3];
};

constexpr int kBS = 256;
constexpr uint32_t kOwn = 0xFFFFu;
constexpr uint32_t kNone32 = 0xFFFFFFFFu;
constexpr unsigned long long kInf64 = ~0ull;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A label viewed for comparison: metrics, length and the last <= 2 commands
// plus the prefix pointer (table index; 0 = empty prefix).
struct View {
    uint32_t m[3];
    uint32_t len;
    uint32_t parent;
    uint32_t ntail;
    Cmd tail[2];
};

template <bool G, class IdxT>
struct Solver {
    const KArgs &a;
    const DevParams &p;
    Shared *sh;
    Rec *R;
    uint32_t *best;
    uint32_t *fired;
    uint32_t *state;
    IdxT *lbuf[3];
    IdxT *dirty;
    uint32_t src;

    __device__ Solver(const KArgs &a_, Shared *sh_, Rec *R_, uint32_t *best_, uint32_t *fired_,
                      uint32_t *state_, IdxT *l0, IdxT *l1, IdxT *l2, IdxT *dirty_)
        : a(a_), p(a_.p), sh(sh_), R(R_), best(best_), fired(fired_), state(state_), dirty(dirty_), src(0) {
        lbuf[0] = l0;
        lbuf[1] = l1;
        lbuf[2] = l2;
    }

    // ---- memory helpers ---------------------------------------------------
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
    __device__ __forceinline__ uint32_t ld_idx(const IdxT *l, uint32_t i) const {
        if constexpr (G) return __hip_atomic_load(l + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return l[i];
    }
    __device__ __forceinline__ void st_idx(IdxT *l, uint32_t i, uint32_t v) const {
        if constexpr (G) __hip_atomic_store(l + i, IdxT(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else l[i] = IdxT(v);
    }
    __device__ __forceinline__ void flag(uint32_t e) const { atomicOr(a.counter + 1, e); }

    __device__ __forceinline__ uint32_t special_of(uint32_t v) const { return a.sinfo[v] & kNone10; }
    __device__ __forceinline__ uint32_t region_of(uint32_t v) const { return (a.sinfo[v] >> 10) & kNone10; }
    __device__ __forceinline__ uint32_t vert_of(uint32_t t) const { return t == 0 ? src : a.sp[t].v; }

    // ---- arithmetic (u32 like the reference; overflow is reported, not wrapped)
    __device__ __forceinline__ uint32_t add32(uint32_t x, uint32_t y) const {
        uint32_t r = x + y;
        if (r < x) flag(kErrMetricOverflow);
        return r;
    }
    // AggregatedCost::time of a StandardMove run of k legs: Fleetfoot ceil of
    // 180k seconds (src/cost.rs:122-124, src/skill.rs:21-30)
    __device__ __forceinline__ uint32_t run_time(uint32_t k) const {
        unsigned long long t = 180ull * k;
        if (p.ff_num != p.ff_den) t = (t * p.ff_num + p.ff_den - 1) / p.ff_den;
        if (t > 0xFFFFFFFFull) flag(kErrMetricOverflow);
        return uint32_t(t);
    }
    __device__ __forceinline__ unsigned long long key_of(const uint32_t *m) const {
        switch (p.bucket_mode) {
            case kBucketLegs: return m[0];
            case kBucketTime: return m[2] / p.W;
            case kBucketMoneyLegs: return (unsigned long long)m[1] << 32 | m[0];
            default: return (unsigned long long)m[1] << 32 | (m[2] / p.W);
        }
    }

    // ---- views ------------------------------------------------------------
    __device__ __forceinline__ void view_rec(uint32_t t, View &x) const {
        const Rec &r = R[t];
        x.m[0] = r.m[0];
        x.m[1] = r.m[1];
        x.m[2] = r.m[2];
        x.len = r.len;
        x.parent = r.parent;
        x.ntail = r.ntail;
        x.tail[0] = r.tail[0];
        x.tail[1] = r.tail[1];
    }
    // the start label TotalCost::new(src) (src/cost.rs:196-205)
    __device__ __forceinline__ void view_start(View &x) const {
        x.m[0] = x.m[1] = x.m[2] = 0;
        x.len = 1;
        x.parent = 0;
        x.ntail = 1;
        x.tail[0] = Cmd{kNoMove << 29, src, src};
        x.tail[1] = Cmd{0, 0, 0};
    }
    // walk label of v: full(b) ++ [StandardMove{k} vert(b) -> v]
    __device__ __forceinline__ void view_walk(uint32_t b, uint32_t k, uint32_t v, View &x) const {
        if (b == 0 && k == 0) {
            view_start(x);
            return;
        }
        const Rec &rb = R[b];
        x.m[0] = add32(rb.m[0], k);
        x.m[1] = rb.m[1];
        x.m[2] = add32(rb.m[2], run_time(k));
        x.len = (b == 0 ? 0u : rb.len) + 1u;
        x.parent = b;
        x.ntail = 1;
        x.tail[0] = Cmd{(kStandard << 29) | k, vert_of(b), v};
        x.tail[1] = Cmd{0, 0, 0};
    }

    // ---- comparator: CostComparator::and_then (src/cost.rs:411-426) --------
    __device__ __forceinline__ int cmp_cmd(const Cmd &x, const Cmd &y) const {
        if (x.kp != y.kp) return x.kp < y.kp ? -1 : 1;
        if (x.from != y.from) return a.rank[x.from] < a.rank[y.from] ? -1 : 1;
        if (x.to != y.to) return a.rank[x.to] < a.rank[y.to] ? -1 : 1;
        return 0;
    }
    // lexicographic compare of two command lists of equal length; xid/yid are
    // the table entries the views were read from (kOwn for built views).
    __device__ int cmp_list(const View &x, uint32_t xid, const View &y, uint32_t yid) const {
        uint32_t xe = xid, ye = yid;
        int xt = int(x.ntail) - 1, yt = int(y.ntail) - 1;
        int res = 0;
        for (uint32_t guard = 0; guard < 4096u; ++guard) {
            if (xe != kOwn && xe == ye && xt == yt) return res;  // shared prefix node
            const Cmd &cx = (xe == kOwn) ? x.tail[xt] : R[xe].tail[xt];
            const Cmd &cy = (ye == kOwn) ? y.tail[yt] : R[ye].tail[yt];
            int r = cmp_cmd(cx, cy);
            if (r) res = r;
            // step to the previous command
            if (xt > 0) --xt;
            else {
                uint32_t pp = (xe == kOwn) ? x.parent : R[xe].parent;
                if (pp == 0) return res;
                xe = pp;
                xt = int(R[pp].ntail) - 1;
            }
            if (yt > 0) --yt;
            else {
                uint32_t pp = (ye == kOwn) ? y.parent : R[ye].parent;
                if (pp == 0) return res;
                ye = pp;
                yt = int(R[pp].ntail) - 1;
            }
        }
        flag(kErrChain);
        return res;
    }
    __device__ __forceinline__ int cmp_metrics(const uint32_t *x, const uint32_t *y) const {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint32_t u = x[p.perm[i]], w = y[p.perm[i]];
            if (u != w) return u < w ? -1 : 1;
        }
        return 0;
    }
    __device__ int cmp_view(const View &x, uint32_t xid, const View &y, uint32_t yid) const {
        int r = cmp_metrics(x.m, y.m);
        if (r) return r;
        if (x.len != y.len) return x.len < y.len ? -1 : 1;
        return cmp_list(x, xid, y, yid);
    }
    __device__ __forceinline__ int cmp_entries(uint32_t s, uint32_t t) const {
        View x, y;
        view_rec(s, x);
        view_rec(t, y);
        return cmp_view(x, s, y, t);
    }

    // ---- special table updates ---------------------------------------------
    __device__ __forceinline__ void try_improve(uint32_t t, const View &c) const {
        Rec &r = R[t];
        if (r.state == 2) return;
        if (r.state == 1) {
            View cur;
            view_rec(t, cur);
            if (cmp_view(c, kOwn, cur, t) >= 0) return;
        }
        r.m[0] = c.m[0];
        r.m[1] = c.m[1];
        r.m[2] = c.m[2];
        r.len = uint16_t(c.len);
        r.ntail = uint8_t(c.ntail);
        r.parent = uint16_t(c.parent);
        r.tail[0] = c.tail[0];
        r.tail[1] = c.tail[1];
        r.state = 1;
    }
    // extend the settled label of special s by a non-Standard edge to t
    // (TotalCost += edge, src/cost.rs:208-315)
    __device__ __forceinline__ void ext_special(uint32_t s, uint32_t kind, uint32_t payload,
                                                uint32_t dm_money, uint32_t dm_time, uint32_t t, View &c) const {
        const Rec &r = R[s];
        const Cmd &last = r.tail[r.ntail - 1];
        uint32_t lk = last.kp >> 29;
        uint32_t vt = a.sp[t].v;
        if (lk == kNoMove) {  // the start label: NoMove is replaced, from kept
            c.m[0] = 0;
            c.m[1] = dm_money;
            c.m[2] = dm_time;
            c.len = 1;
            c.parent = 0;
            c.ntail = 1;
            c.tail[0] = Cmd{(kind << 29) | payload, last.from, vt};
        } else if (kind == kCentral && lk == kCentral) {  // central moves merge
            c.m[0] = r.m[0];
            c.m[1] = r.m[1];
            c.m[2] = add32(r.m[2], dm_time);
            c.len = r.len;
            c.parent = r.parent;
            c.ntail = r.ntail;
            c.tail[0] = r.tail[0];
            c.tail[1] = r.tail[1];
            c.tail[c.ntail - 1] = Cmd{last.kp + 1u, last.from, vt};
        } else {
            c.m[0] = r.m[0];
            c.m[1] = add32(r.m[1], dm_money);
            c.m[2] = add32(r.m[2], dm_time);
            c.len = r.len + 1u;
            c.parent = s;
            c.ntail = 1;
            c.tail[0] = Cmd{(kind << 29) | payload, a.sp[s].v, vt};
        }
        if (c.ntail == 1) c.tail[1] = Cmd{0, 0, 0};
    }

    // ---- grid helpers --------------------------------------------------------
    // geometric neighbour d (0:-x 1:+x 2:-y 3:+y) of v, or kNone32
    __device__ __forceinline__ uint32_t nbr(uint32_t v, int d) const {
        uint32_t x = v % p.S;
        switch (d) {
            case 0: return x == 0 ? kNone32 : v - 1;
            case 1: return x + 1 == p.S ? kNone32 : v + 1;
            case 2: return v < p.S ? kNone32 : v - p.S;
            default: return v + p.S >= p.V ? kNone32 : v + p.S;
        }
    }
    // mark the StandardMove out-neighbours of a freshly settled vertex dirty
    // (edges touching the Center are CentralMoves and are handled by the table)
    __device__ __forceinline__ void mark_dirty(uint32_t v, uint32_t n) const {
        if (n == kNone32 || v == p.vc || n == p.vc) return;
        uint32_t old = or_state(n, kStDirty);
        if (old & (kStSettled | kStDirty)) return;
        uint32_t i = atomicAdd(&sh->nd, 1u);
        st_idx(dirty, i, n);
    }

    // ---- phase 1: settle plain vertices of bucket B ---------------------------
    __device__ void region_offer(uint32_t r, uint32_t v) const {
        uint32_t cur = best[r];
        for (;;) {
            if (cur != kNone32) {
                uint32_t su = ld_state(cur), sv = ld_state(v);
                View xu, xv;
                view_walk((su >> kStBShift) & kNone10, su & kStKMask, cur, xu);
                view_walk((sv >> kStBShift) & kNone10, sv & kStKMask, v, xv);
                if (cmp_view(xu, kOwn, xv, kOwn) <= 0) return;
            }
            uint32_t prev = atomicCAS(best + r, cur, v);
            if (prev == cur) return;
            cur = prev;
        }
    }
    __device__ void settle_plain(uint32_t v) const {
        or_state(v, kStSettled);
        if (p.use_soe) {
            uint32_t r = region_of(v);
            if (r != kNone10 && !fired[r]) region_offer(r, v);
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) mark_dirty(v, nbr(v, d));
    }

    // ---- phase 2: specials (one wave) -----------------------------------------
    __device__ void fire_regions() const {
        for (uint32_t t = 1 + lane_id(); t <= p.NS; t += 64) {
            uint32_t u = best[t];
            if (u == kNone32) continue;
            best[t] = kNone32;
            fired[t] = 1;
            if (R[t].state == 2) continue;
            uint32_t su = ld_state(u);
            uint32_t b = (su >> kStBShift) & kNone10, k = su & kStKMask;
            View c;
            uint32_t vt = a.sp[t].v;
            if (b == 0 && k == 0) {  // u is the source: [SoE src->c]
                c.m[0] = 0;
                c.m[1] = p.soe_cost;
                c.m[2] = 0;
                c.len = 1;
                c.parent = 0;
                c.ntail = 1;
                c.tail[0] = Cmd{kSoE << 29, src, vt};
                c.tail[1] = Cmd{0, 0, 0};
            } else {  // full(b) ++ [Std{k} b->u, SoE u->c]
                view_walk(b, k, u, c);
                c.m[1] = add32(c.m[1], p.soe_cost);
                c.len += 1;
                c.ntail = 2;
                c.tail[1] = Cmd{kSoE << 29, u, vt};
            }
            try_improve(t, c);
        }
        wave_sync();
    }

    __device__ void settle_special(uint32_t s) const {
        const uint32_t lane = lane_id();
        const uint32_t vs = a.sp[s].v;
        if (lane == 0) {
            Rec &r = R[s];
            r.state = 2;
            const Cmd &last = r.tail[r.ntail - 1];
            uint32_t lk = last.kp >> 29, seed;
            if (lk == kNoMove) seed = 0;  // the source itself
            else if (lk == kStandard) seed = (uint32_t(r.parent) << kStBShift) | (last.kp & kStKMask);
            else seed = s << kStBShift;   // a boundary: walks restart here
            st_state(vs, kStSettled | seed);
        }
        wave_sync();
        if (lane < 4) mark_dirty(vs, nbr(vs, int(lane)));
        const uint32_t fl = a.sp[s].flags;
        // CentralMove edges (src/pathfinder.rs:30-53)
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
        // caravans between Center and campfires (src/pathfinder.rs:140-160, 251-273)
        if (p.use_caravans && (fl & kSpHub)) {
            const SpecialStatic &ss = a.sp[s];
            for (uint32_t h = lane; h < p.n_hubs; h += 64) {
                uint32_t t = a.hubs[h];
                if (t == s || R[t].state == 2) continue;
                const SpecialStatic &st = a.sp[t];
                uint32_t d = uint32_t(abs(ss.x - st.x) + abs(ss.y - st.y));
                uint32_t coef = st.coef5 ? 5u : 2u;
                View c;
                ext_special(s, kCaravan, (d << 1) | st.coef5, coef * d, p.rgt * d, t, c);
                try_improve(t, c);
            }
        }
        wave_sync();
        // Scroll of Escape to this cell's nearest campfire (src/pathfinder.rs:162-170)
        if (p.use_soe && lane == 0) {
            uint32_t t = a.sp[s].region;
            if (t != kNone10 && t != s) {
                View c;
                ext_special(s, kSoE, 0, p.soe_cost, 0, t, c);
                try_improve(t, c);
            }
        }
        wave_sync();
    }

    __device__ void specials_in_bucket(unsigned long long B) const {
        const uint32_t lane = lane_id();
        for (uint32_t iter = 0; iter <= p.NS + 1; ++iter) {
            uint32_t mine = kNone32;
            for (uint32_t t = 1 + lane; t <= p.NS; t += 64) {
                if (R[t].state != 1) continue;
                unsigned long long k = key_of(R[t].m);
                if (k < B) flag(kErrBucket);
                if (k > B) continue;
                if (mine == kNone32 || cmp_entries(t, mine) < 0) mine = t;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                uint32_t other = __shfl_xor(mine, off, 64);
                if (other != kNone32 && (mine == kNone32 || cmp_entries(other, mine) < 0)) mine = other;
            }
            if (mine == kNone32) return;
            settle_special(mine);
        }
    }

    // ---- phase 3: pull -----------------------------------------------------------
    __device__ void pull(uint32_t w) const {
        // a vertex marked dirty may have been settled later in the same bucket
        // (a plain vertex of bucket B, or a special settled by the table)
        if (ld_state(w) & kStSettled) return;
        const uint32_t t = special_of(w);
        uint32_t bb = kNone10, bk = 0;
        if (w != p.vc) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t n = nbr(w, d);
                if (n == kNone32 || n == p.vc) continue;
                uint32_t sn = ld_state(n);
                if (!(sn & kStSettled)) continue;
                uint32_t b = (sn >> kStBShift) & kNone10, k = (sn & kStKMask) + 1u;
                if (k > kStKMask) {
                    flag(kErrKOverflow);
                    continue;
                }
                if (bb == kNone10) {
                    bb = b;
                    bk = k;
                } else if (b == bb) {
                    if (k < bk) bk = k;  // same boundary: fewer legs is smaller in every order
                } else {
                    View xc, xb;
                    view_walk(b, k, w, xc);
                    view_walk(bb, bk, w, xb);
                    if (cmp_view(xc, kOwn, xb, kOwn) < 0) {
                        bb = b;
                        bk = k;
                    }
                }
            }
        }
        if (t != kNone10) {
            st_state(w, kStUntouched);
            if (bb != kNone10) {
                View c;
                view_walk(bb, bk, w, c);
                try_improve(t, c);
            }
            return;
        }
        uint32_t old = ld_state(w);
        if (bb == kNone10) {  // cannot happen: a dirty vertex has a settled StandardMove neighbour
            st_state(w, old & ~kStDirty);
            flag(kErrBucket);
            return;
        }
        st_state(w, (bb << kStBShift) | bk);
        if (((old >> kStBShift) & kNone10) == kNone10) {  // first touch: list it
            View c;
            view_walk(bb, bk, w, c);
            unsigned long long X = key_of(c.m), B = sh->B;
            uint32_t j;
            if (X == B + 1) j = 1;
            else if (X == B + 2) j = 2;
            else {
                flag(kErrBucket);
                return;
            }
            uint32_t buf = (sh->lb + j) % 3u;
            uint32_t i = atomicAdd(&sh->cnt[buf], 1u);
            st_idx(lbuf[buf], i, w);
        }
    }

    // ---- phase 4: next bucket ----------------------------------------------------
    __device__ void next_bucket(uint32_t s) const {
        const uint32_t lane = lane_id();
        unsigned long long smin = kInf64;
        for (uint32_t t = 1 + lane; t <= p.NS; t += 64)
            if (R[t].state == 1) {
                unsigned long long k = key_of(R[t].m);
                if (k < smin) smin = k;
            }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            unsigned long long o = __shfl_xor(smin, off, 64);
            if (o < smin) smin = o;
        }
        // early exit once every destination of this source is settled
        uint32_t all_done = 0;
        const uint32_t q0 = a.q_begin[s], q1 = a.q_begin[s + 1];
        if (q1 - q0 <= a.early_exit_max) {
            bool ok = true;
            if (lane < q1 - q0) ok = (ld_state(a.q_dst[q0 + lane]) & kStSettled) != 0;
            all_done = __all(ok) ? 1u : 0u;
        }
        if (lane == 0) {
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

    // ---- outputs -----------------------------------------------------------------
    __device__ void write_output(uint32_t w, uint32_t qid) const {
        OutResult &o = a.out_res[qid];
        const uint32_t sw = ld_state(w);
        if (!(sw & kStSettled)) {
            o = OutResult{0, 0, 0, uint32_t(16 + 1) << 16};  // MR_NOT_FOUND
            return;
        }
        View x;
        uint32_t xid = kOwn;
        const uint32_t t = special_of(w);
        if (t != kNone10) {
            view_rec(t, x);
            xid = t;
        } else {
            view_walk((sw >> kStBShift) & kNone10, sw & kStKMask, w, x);
        }
        if (x.len > p.max_cmds) {  // MR_ERR_CAPACITY: caller re-runs with more slots
            o = OutResult{x.m[0], x.m[1], x.m[2], (uint32_t(16 - 4) << 16) | (x.len & 0xFFFFu)};
            return;
        }
        OutCmd *oc = a.out_cmd + (unsigned long long)qid * p.max_cmds;
        int pos = int(x.len) - 1;
        for (int j = int(x.ntail) - 1; j >= 0 && pos >= 0; --j, --pos)
            oc[pos] = OutCmd{x.tail[j].kp, x.tail[j].from, x.tail[j].to, 0};
        uint32_t pp = x.parent;
        while (pp != 0 && pos >= 0) {
            const Rec &r = R[pp];
            for (int j = int(r.ntail) - 1; j >= 0 && pos >= 0; --j, --pos)
                oc[pos] = OutCmd{r.tail[j].kp, r.tail[j].from, r.tail[j].to, 0};
            pp = r.parent;
        }
        if (pos != -1 || pp != 0) flag(kErrChain);
        (void)xid;
        o = OutResult{x.m[0], x.m[1], x.m[2], (uint32_t(16) << 16) | (x.len & 0xFFFFu)};
    }

    // ---- one source ----------------------------------------------------------------
    __device__ void solve(uint32_t s) {
        const uint32_t tid = threadIdx.x;
        src = a.src_v[s];
        for (uint32_t v = tid; v < p.V; v += kBS) st_state(v, kStUntouched);
        for (uint32_t t = tid; t <= p.NS; t += kBS) {
            R[t].state = 0;
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
            View st;
            view_start(st);
            // entry 0 = the source (root of every command chain)
            R[0].m[0] = R[0].m[1] = R[0].m[2] = 0;
            R[0].len = 1;
            R[0].ntail = 1;
            R[0].parent = 0;
            R[0].tail[0] = st.tail[0];
            R[0].state = 2;
            const uint32_t ts = special_of(src);
            if (ts != kNone10) {
                try_improve(ts, st);
            } else {
                st_state(src, 0u);  // walk label (0,0) = the start label
                sh->cnt[0] = 1;
                st_idx(lbuf[0], 0, src);
            }
            // SHQ / SFm: only the source's own edges can be minimal (a prefix only
            // adds metrics and length), src/pathfinder.rs:172-178
            if (p.hq_t) {
                View c;
                view_start(c);
                c.m[1] = p.shq_cost;
                c.tail[0] = Cmd{kSHQ << 29, src, a.sp[p.hq_t].v};
                try_improve(p.hq_t, c);
            }
            if (p.use_sfm) {
                View c;
                view_start(c);
                c.m[1] = p.sfm_cost;
                c.tail[0] = Cmd{kSFm << 29, src, p.vc};
                try_improve(1, c);
            }
        }
        __syncthreads();
        for (uint32_t guard = 0;; ++guard) {
            // 1. settle
            {
                const uint32_t lb = sh->lb;
                const uint32_t n0 = sh->cnt[lb];
                const IdxT *L0 = lbuf[lb];
                for (uint32_t i = tid; i < n0; i += kBS) settle_plain(ld_idx(L0, i));
            }
            __syncthreads();
            // 2. specials
            if (tid < 64) {
                if (p.use_soe) fire_regions();
                specials_in_bucket(sh->B);
            }
            __syncthreads();
            // 3. pull
            {
                const uint32_t nd = sh->nd;
                for (uint32_t i = tid; i < nd; i += kBS) pull(ld_idx(dirty, i));
            }
            __syncthreads();
            // 4. next bucket
            if (tid < 64) next_bucket(s);
            __syncthreads();
            if (sh->done) break;
            if (guard > p.V + p.NS + 64u) {
                flag(kErrBucket);
                break;
            }
        }
        const uint32_t q0 = a.q_begin[s], q1 = a.q_begin[s + 1];
        for (uint32_t i = q0 + tid; i < q1; i += kBS) write_output(a.q_dst[i], a.q_id[i]);
        __syncthreads();
    }
};

__host__ __device__ constexpr uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

struct LdsLayout {
    uint32_t off_R, off_best, off_fired, off_state, off_l0, off_l1, off_l2, off_dirty, total;
};

__host__ __device__ inline LdsLayout lds_layout(uint32_t NS, uint32_t V, bool grid_in_lds) {
    LdsLayout L{};
    uint32_t o = align16(sizeof(Shared));
    L.off_R = o;
    o = align16(o + (NS + 1) * sizeof(Rec));
    L.off_best = o;
    o = align16(o + (NS + 1) * 4);
    L.off_fired = o;
    o = align16(o + (NS + 1) * 4);
    if (grid_in_lds) {
        L.off_state = o;
        o = align16(o + V * 4);
        L.off_l0 = o;
        o = align16(o + V * 2);
        L.off_l1 = o;
        o = align16(o + V * 2);
        L.off_l2 = o;
        o = align16(o + V * 2);
        L.off_dirty = o;
        o = align16(o + V * 2);
    }
    L.total = o;
    return L;
}

template <bool G, class IdxT>
__global__ __launch_bounds__(kBS) void sssp_kernel(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const LdsLayout L = lds_layout(a.p.NS, a.p.V, !G);
    Shared *sh = reinterpret_cast<Shared *>(smem);
    Rec *R = reinterpret_cast<Rec *>(smem + L.off_R);
    uint32_t *best = reinterpret_cast<uint32_t *>(smem + L.off_best);
    uint32_t *fired = reinterpret_cast<uint32_t *>(smem + L.off_fired);
    uint32_t *state;
    IdxT *l0, *l1, *l2, *dirty;
    if constexpr (G) {
        uint32_t *slot = a.ws + (unsigned long long)blockIdx.x * 5ull * a.p.V;
        state = slot;
        l0 = reinterpret_cast<IdxT *>(slot + a.p.V);
        l1 = reinterpret_cast<IdxT *>(slot + 2ull * a.p.V);
        l2 = reinterpret_cast<IdxT *>(slot + 3ull * a.p.V);
        dirty = reinterpret_cast<IdxT *>(slot + 4ull * a.p.V);
    } else {
        state = reinterpret_cast<uint32_t *>(smem + L.off_state);
        l0 = reinterpret_cast<IdxT *>(smem + L.off_l0);
        l1 = reinterpret_cast<IdxT *>(smem + L.off_l1);
        l2 = reinterpret_cast<IdxT *>(smem + L.off_l2);
        dirty = reinterpret_cast<IdxT *>(smem + L.off_dirty);
    }
    Solver<G, IdxT> S(a, sh, R, best, fired, state, l0, l1, l2, dirty);
    for (;;) {
        if (threadIdx.x == 0) sh->sidx = atomicAdd(a.counter, 1u);
        __syncthreads();
        const uint32_t s = sh->sidx;
        __syncthreads();
        if (s >= a.nsrc) break;
        S.solve(s);
    }
}

// ---- host-side launch helpers (called from mr_api.cpp) -------------------------
uint32_t lds_bytes(uint32_t NS, uint32_t V, bool grid_in_lds) { return lds_layout(NS, V, grid_in_lds).total; }

hipError_t launch_sssp(const KArgs &a, bool grid_in_lds, uint32_t blocks, hipStream_t stream) {
    const uint32_t bytes = lds_bytes(a.p.NS, a.p.V, grid_in_lds);
    if (grid_in_lds) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&sssp_kernel<false, uint16_t>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
        hipLaunchKernelGGL((sssp_kernel<false, uint16_t>), dim3(blocks), dim3(kBS), bytes, stream, a);
    } else {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&sssp_kernel<true, uint32_t>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
        hipLaunchKernelGGL((sssp_kernel<true, uint32_t>), dim3(blocks), dim3(kBS), bytes, stream, a);
    }
    return hipGetLastError();
}

int max_blocks_per_cu(bool grid_in_lds, uint32_t bytes) {
    int n = 0;
    if (grid_in_lds)
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sssp_kernel<false, uint16_t>, kBS, bytes);
    else
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sssp_kernel<true, uint32_t>, kBS, bytes);
    return n;
}

}  // namespace mr
