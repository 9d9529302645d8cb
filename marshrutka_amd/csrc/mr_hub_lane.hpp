// mr_hub_lane.hpp — the hub solver with one SOURCE per lane (hub_lane_kernel).
//
// Same algorithm and results as hub_kernel (mr_device.hpp): an exact
// Dijkstra over the specials (Center, border-1 cells, campfires, HQ) whose edges are
// the closed-form walks from settled boundaries, CentralMove / caravan / Scroll-of-
// Escape edges and SoE edges from each region's nearest cell; plain destinations are
// read off as the best walk from a boundary (FindPath::eval, src/pathfinder.rs:199-248;
// uniqueness of the result: SURVEY.md §8a).
//
// The mapping is what differs.  hub_kernel gives one special per lane, so every
// settle is a cross-lane reduction (DPP minima, readlane, ballots) over ~21 useful
// lanes, and each wave instruction advances one or two sources.  Here lane l owns
// source l of its wave and keeps ALL of that source's tentative labels in registers
// (entries 1..TM-1, fully unrolled loops, so nothing is indexed at run time): a
// settle is a per-lane scan, a relaxation a per-lane compare-and-select, and every
// wave instruction advances 64 sources.  No LDS traffic beyond the specials' static
// table, no cross-lane operation in the loop.
//
// Exactness follows hub_kernel step for step:
//   * candidates into an entry from one settled special s share chain(s), so among
//     them (metrics, length) ties are decided by the last command's kp (= the list
//     order); the best of them is compared with the entry's tentative label, and only
//     an exact (metrics, length) tie there walks the command lists (cmp_list, rare,
//     out of the unrolled code);
//   * blockers: a boundary special whose settled label some walk candidate tied on
//     all three metrics (hub_kernel's note_walk).  One bit per entry keeps "a walk
//     candidate so far has the tentative label's metrics" — every candidate is >= the
//     tentative label, so when the tentative metrics drop no earlier walk can tie;
//   * the blocker certification (avail) and the SSSP fallback of uncertain sources
//     are hub_kernel's.
// Sources with more than kLaneMaxQ queries stay on hub_kernel (a lane per query).
#pragma once
#include "mr_device.hpp"

namespace mr {

#ifndef MR_LANE_WAVES
#define MR_LANE_WAVES 2  // waves per SIMD the register budget is cut for
#endif

// a label of a table entry: metrics, len | parent << 16 | (ntail - 1) << 31, and the
// first tail command's kp.  Its tail commands are {kp, rank(parent), u} and, when
// ntail = 2, {SoE, u, own rank}; u is the entry's own rank unless ntail = 2, when it is
// the region cell nearest to the parent (the parent's region row at the entry's region).
struct LLab {
    uint32_t m0, m1, m2, lpn, kp;
};
__device__ __forceinline__ uint32_t ll_len(uint32_t lpn) { return lpn & 0xFFFFu; }
__device__ __forceinline__ uint32_t ll_par(uint32_t lpn) { return (lpn >> 16) & kNone10; }
__device__ __forceinline__ uint32_t ll_nt(uint32_t lpn) { return (lpn >> 31) + 1u; }
__device__ __forceinline__ uint32_t ll_pack(uint32_t len, uint32_t par, uint32_t nt) {
    return (len & 0xFFFFu) | (par << 16) | ((nt - 1u) << 31);
}
__device__ __forceinline__ LLab ll_start() { return LLab{0, 0, 0, ll_pack(1, 0, 1), kNoMove << 29}; }
__device__ __forceinline__ void ll_sel(bool take, LLab &d, const LLab &c) {
    d.m0 = take ? c.m0 : d.m0;
    d.m1 = take ? c.m1 : d.m1;
    d.m2 = take ? c.m2 : d.m2;
    d.lpn = take ? c.lpn : d.lpn;
    d.kp = take ? c.kp : d.kp;
}

template <uint32_t PERM, uint32_t TM>
struct LaneHub {
    static constexpr uint32_t C1 = PERM / 9, C2 = (PERM / 3) % 3, C3 = PERM % 3;
    const KArgs *__restrict__ a;
    DevParams P;
    const SpecialStatic *spl;  // LDS copy of a->sp
    const uint2 *nearS;        // LDS: region rows of the specials, row t at t * nreg
    const uint32_t *rank, *sinfo, *rank_inv;
    uint32_t *counter;
    uint32_t nreg;
    uint32_t err = 0;
    // this lane's source
    uint32_t src = 0, src_rk = 0, ts = kNone10;
    int sx = 0, sy = 0;
    const uint2 *srow = nullptr;  // global: the source's region row
    // tentative / settled labels of entries 1..TM-1 (entry 0, the source, is the start label)
    LLab L[TM];
    uint32_t tent = 0, done = 0, wt = 0, bndm = 0, blk = 0;

    template <uint32_t I>
    __device__ __forceinline__ static uint32_t met(const LLab &x) {
        return I == 0 ? x.m0 : (I == 1 ? x.m1 : x.m2);
    }
    // (c1, c2, c3, length) in comparator order: -1, 0, 1
    __device__ __forceinline__ static int cmp4(const LLab &x, const LLab &y) {
        if (met<C1>(x) != met<C1>(y)) return met<C1>(x) < met<C1>(y) ? -1 : 1;
        if (met<C2>(x) != met<C2>(y)) return met<C2>(x) < met<C2>(y) ? -1 : 1;
        if (met<C3>(x) != met<C3>(y)) return met<C3>(x) < met<C3>(y) ? -1 : 1;
        const uint32_t lx = ll_len(x.lpn), ly = ll_len(y.lpn);
        if (lx != ly) return lx < ly ? -1 : 1;
        return 0;
    }
    __device__ __forceinline__ static bool eq3(const LLab &x, const LLab &y) {
        return x.m0 == y.m0 && x.m1 == y.m1 && x.m2 == y.m2;
    }
    __device__ __forceinline__ uint32_t add32(uint32_t x, uint32_t y) {
        const uint32_t r = x + y;
        err |= r < x ? kErrMetricOverflow : 0u;
        return r;
    }
    // a StandardMove run of k legs: 180 k s (linear run times only on this kernel)
    __device__ __forceinline__ uint32_t run_time(uint32_t k) {
        const unsigned long long t = 180ull * k;
        err |= t > 0xFFFFFFFFull ? kErrMetricOverflow : 0u;
        return uint32_t(t);
    }
    __device__ __forceinline__ uint32_t rk(uint32_t e) const { return e == 0 ? src_rk : spl[e].rk; }
    // the rank of the region cell nearest to entry p's cell in region r
    __device__ __forceinline__ uint32_t near_rank(uint32_t p, uint32_t r) const {
        return p == 0 ? srow[r].y : nearS[p * nreg + r].y;
    }
    __device__ __forceinline__ uint32_t u_of(const LLab &x, uint32_t own_rk, uint32_t own_rid) const {
        return ll_nt(x.lpn) == 2 ? near_rank(ll_par(x.lpn), own_rid) : own_rk;
    }
    // entry e's label (run-time e; a select per entry: the rare paths only)
    __device__ __forceinline__ LLab get(uint32_t e) const {
        LLab r = ll_start();
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) ll_sel(e == t, r, L[t]);
        return r;
    }
    __device__ __forceinline__ void put(uint32_t e, const LLab &c) {
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) ll_sel(e == t, L[t], c);
    }

    // ---- label builders (TotalCost += edge, src/cost.rs:208-315) ---------------------
    // the settled label ls of special s extended by a non-Standard edge (ext_view)
    __device__ __forceinline__ LLab ext(const LLab &ls, uint32_t s, uint32_t kind, uint32_t payload, uint32_t dm,
                                        uint32_t dt) {
        const uint32_t lk = ll_nt(ls.lpn) == 2 ? kSoE : (ls.kp >> 29);
        LLab c;
        if (lk == kNoMove) {  // the start label: NoMove is replaced, its from kept
            c = LLab{0, dm, dt, ll_pack(1, 0, 1), (kind << 29) | payload};
        } else if (kind == kCentral && lk == kCentral) {  // CentralMoves merge
            c = LLab{ls.m0, ls.m1, add32(ls.m2, dt), ll_pack(ll_len(ls.lpn), ll_par(ls.lpn), 1), ls.kp + 1u};
        } else {
            c = LLab{ls.m0, add32(ls.m1, dm), add32(ls.m2, dt), ll_pack(ll_len(ls.lpn) + 1u, s, 1), (kind << 29) | payload};
        }
        return c;
    }
    // full(b) ++ [StandardMove{k} b -> .] from the settled special b (k > 0)
    __device__ __forceinline__ LLab walk(const LLab &lb, uint32_t b, uint32_t k) {
        return LLab{add32(lb.m0, k), lb.m1, add32(lb.m2, run_time(k)), ll_pack(ll_len(lb.lpn) + 1u, b, 1),
                    (kStandard << 29) | k};
    }
    // ... and then its Scroll of Escape from the walk's end (ntail 2)
    __device__ __forceinline__ LLab walk_soe(const LLab &lb, uint32_t b, uint32_t k) {
        LLab c = walk(lb, b, k);
        c.m1 = add32(c.m1, P.soe_cost);
        c.lpn = ll_pack(ll_len(lb.lpn) + 2u, b, 2);
        return c;
    }

    // ---- the command-list order (src/cost.rs:423-424), rare --------------------------
    __device__ __forceinline__ static int cmp_cmd(const Cmd &x, const Cmd &y) {
        if (x.kp != y.kp) return x.kp < y.kp ? -1 : 1;
        if (x.from != y.from) return x.from < y.from ? -1 : 1;
        if (x.to != y.to) return x.to < y.to ? -1 : 1;
        return 0;
    }
    __device__ __forceinline__ Cmd tail(const LLab &x, uint32_t own_rk, uint32_t own_rid, int i) const {
        const uint32_t u = u_of(x, own_rk, own_rid);
        if (i == 0) return Cmd{x.kp, rk(ll_par(x.lpn)), u};
        return Cmd{kSoE << 29, u, own_rk};
    }
    // lexicographic compare of two equal-length command lists, walking from the last
    // command towards the first (hub_kernel's cmp_list); xid/yid name the table entries
    // the labels are (kOwn for built ones), so a shared prefix stops the walk
    __device__ __forceinline__ int cmp_list(LLab x, uint32_t xid, uint32_t xrk, uint32_t xrid, LLab y, uint32_t yid, uint32_t yrk,
                            uint32_t yrid) const {
        int xt = int(ll_nt(x.lpn)) - 1, yt = int(ll_nt(y.lpn)) - 1;
        int res = 0;
        for (uint32_t guard = 0; guard < 4096u; ++guard) {
            if (xid != kOwn && xid == yid && xt == yt) return res;
            const int r = cmp_cmd(tail(x, xrk, xrid, xt), tail(y, yrk, yrid, yt));
            if (r) res = r;
            if (xt > 0) {
                --xt;
            } else {
                const uint32_t p = ll_par(x.lpn);
                if (p == 0) return res;
                xid = p;
                x = get(p);
                xrk = spl[p].rk;
                xrid = spl[p].rid;
                xt = int(ll_nt(x.lpn)) - 1;
            }
            if (yt > 0) {
                --yt;
            } else {
                const uint32_t p = ll_par(y.lpn);
                if (p == 0) return res;
                yid = p;
                y = get(p);
                yrk = spl[p].rk;
                yrid = spl[p].rid;
                yt = int(ll_nt(y.lpn)) - 1;
            }
        }
        atomicOr(counter + kCtrFlags, kErrChain);
        return res;
    }

    // ---- candidates from one settled special s into entry t ------------------------
    // The best of the CentralMove, caravan, SoE, walk and SoE-region candidates from s
    // (they share chain(s): (metrics, length) ties go to the smaller last kp), and the
    // walk candidate itself (for the blocker bit).  `live`: t is an unsettled entry.
    struct FromS {
        LLab c, w;
        bool any, won;
    };
    __device__ __forceinline__ void consider(FromS &f, bool on, const LLab &c) const {
        bool take = on;
        if (on && f.any) {
            const int r = cmp4(c, f.c);
            take = r < 0 || (r == 0 && c.kp < f.c.kp);
        }
        ll_sel(take, f.c, c);
        f.any = f.any || on;
    }
    __device__ __forceinline__ FromS from_s(bool live, const LLab &ls, uint32_t s, const SpecialStatic &sS, bool walks,
                                            uint32_t t, const SpecialStatic &tS) {
        const DevParams &p = P;
        FromS f;
        f.any = false;
        f.won = false;
        f.c = ls;
        f.w = ls;
        if (tS.flags & (kSpCenter | kSpBorder1)) {  // CentralMove: Center <-> border-1 cells
            const bool on = live && (((sS.flags & kSpCenter) && (tS.flags & kSpBorder1)) ||
                                     ((sS.flags & kSpBorder1) && (tS.flags & kSpCenter)));
            consider(f, on, ext(ls, s, kCentral, 1, 0, 10));
        }
        if (p.use_caravans && (tS.flags & kSpHub)) {  // caravans between hubs (src/pathfinder.rs:140-160)
            const bool on = live && (sS.flags & kSpHub);
            const uint32_t d = uint32_t(abs(sS.x - tS.x) + abs(sS.y - tS.y));
            const uint32_t coef = tS.coef5 ? 5u : 2u;
            consider(f, on, ext(ls, s, kCaravan, (d << 1) | tS.coef5, coef * d, p.rgt * d));
        }
        if (p.use_soe && tS.rid != kNone10) {
            // Scroll of Escape from s to its region's campfire (src/pathfinder.rs:162-170)
            const bool on_e = live && sS.region == t && sS.region != s;
            consider(f, on_e, ext(ls, s, kSoE, 0, p.soe_cost, 0));
            // ... and from the region cell nearest to boundary s: [Std{d} s -> u, SoE u -> t]
            const uint2 e = nearS[s * nreg + tS.rid];
            const bool on_r = live && walks && e.x != kNone32 && e.x != 0;
            consider(f, on_r, walk_soe(ls, s, on_r ? e.x : 1u));
        }
        if (t != 1) {  // walks from boundary s (not into the Center)
            const bool on = live && walks;
            const LLab c = walk(ls, s, walk_dist(sS.x, sS.y, tS.x, tS.y));
            consider(f, on, c);
            f.w = c;
            f.won = on;
        }
        return f;
    }
    // the best candidate into entry t against its tentative label: a strict win takes,
    // an exact (metrics, length) tie is left to the list compare (bit t of *ties)
    __device__ __forceinline__ void offer(uint32_t t, const FromS &f, uint32_t &ties) {
        if (!f.any) return;
        LLab &T = L[t];
        const uint32_t bit = 1u << t;
        const bool have = (tent & bit) != 0;
        const int r = have ? cmp4(f.c, T) : -1;
        const bool same3 = have && eq3(f.c, T);
        ll_sel(r < 0, T, f.c);
        tent |= bit;
        // blocker bit: a walk candidate with the (new) tentative metrics
        const bool keep = same3 || (have && r > 0);
        const bool wtie = f.won && eq3(f.w, T);
        wt = (wt & ~bit) | (((keep && (wt & bit)) || wtie) ? bit : 0u);
        ties |= r == 0 ? bit : 0u;
    }

    // ---- certification (hub_kernel's avail / label_avail) ----------------------------
    __device__ __forceinline__ void bpos(uint32_t b, int &bx, int &by) const {
        bx = b == 0 ? sx : spl[b].x;
        by = b == 0 ? sy : spl[b].y;
    }
    __device__ __forceinline__ bool avail(uint32_t b, int bx, int by, int vx, int vy) const {
        if (blk == 0) return true;
        const int x0 = min(bx, vx), x1 = max(bx, vx), y0 = min(by, vy), y1 = max(by, vy);
        const bool detour = walk_dist(bx, by, vx, vy) != uint32_t(x1 - x0 + y1 - y0);
        uint32_t inside = 0;
        for (uint32_t m = blk; m; m &= m - 1u) {
            const uint32_t k = uint32_t(__builtin_ctz(m));
            if (k == b) continue;
            const int kx = spl[k].x, ky = spl[k].y;
            if (kx >= x0 && kx <= x1 && ky >= y0 && ky <= y1) inside += 1;
            else if (detour && kx >= x0 - 1 && kx <= x1 + 1 && ky >= y0 - 1 && ky <= y1 + 1) inside += 2;
        }
        if (inside == 0) return true;
        if (inside > 1 || detour) return false;
        if (x0 <= 0 && 0 <= x1 && y0 <= 0 && 0 <= y1) return false;
        return x0 != x1 && y0 != y1;
    }
    __device__ __forceinline__ bool label_avail(const LLab &x, uint32_t t) const {
        if ((x.kp >> 29) != kStandard) return true;
        const uint32_t b = ll_par(x.lpn);
        int bx, by;
        bpos(b, bx, by);
        if (ll_nt(x.lpn) == 1) return avail(b, bx, by, spl[t].x, spl[t].y);
        const uint32_t u = rank_inv[near_rank(b, spl[t].rid)];
        return avail(b, bx, by, int(u % P.S) - int(P.H), int(u / P.S) - int(P.H));
    }

    // ---- output (Core::emit) --------------------------------------------------------
    __device__ __forceinline__ void emit(const LLab &x, uint32_t own_rk, uint32_t own_rid, uint32_t qi) {
        const DevParams &p = P;
        OutResult &o = a->out_res[qi];
        OutCmd *oc = a->out_cmd + (unsigned long long)qi * p.max_cmds;
        const uint32_t len = ll_len(x.lpn);
        uint32_t status = 16;
        if (len > p.max_cmds) {  // the overflow pool, else MR_ERR_CAPACITY
            const uint32_t off = atomicAdd(counter + kCtrOvf, len);
            if (p.max_cmds == 0 || off + len > a->ovf_cap || off + len < off) {
                o = OutResult{x.m0, x.m1, x.m2, (uint32_t(16 - 4) << 16) | (len & 0xFFFFu)};
                return;
            }
            oc[0] = OutCmd{kOvfTag, off, len, 0};
            oc = a->ovf + off;
            status = 16 + kStatusOverflow;
        }
        int pos = int(len) - 1;
        LLab e = x;
        uint32_t erk = own_rk, erid = own_rid, eid = kOwn;
        for (uint32_t guard = 0; pos >= 0 && guard <= TM + 1; ++guard) {
            for (int j = int(ll_nt(e.lpn)) - 1; j >= 0 && pos >= 0; --j, --pos) {
                const Cmd c = tail(e, erk, erid, j);
                oc[pos] = OutCmd{c.kp, c.from, c.to, 0};
            }
            eid = ll_par(e.lpn);
            if (eid == 0) break;
            e = get(eid);
            erk = spl[eid].rk;
            erid = spl[eid].rid;
        }
        if (pos != -1 || eid != 0) atomicOr(counter + kCtrFlags, kErrChain);
        o = OutResult{x.m0, x.m1, x.m2, (status << 16) | (len & 0xFFFFu)};
    }

    // ---- one source per lane ----------------------------------------------------------
    // returns the records this lane wrote (0 when the source went to the SSSP kernel)
    __device__ __forceinline__ uint32_t solve(bool have, uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t NS = p.NS;
        src = a->src_v[s_idx];
        src_rk = rank[src];
        sx = int(src % p.S) - int(p.H);
        sy = int(src / p.S) - int(p.H);
        ts = sinfo[src] & kNone10;
        srow = reinterpret_cast<const uint2 *>(a->near) + (unsigned long long)src * nreg;
        // the source's own edges: its start label if it is a special, SHQ, SFm, the
        // walks from it and the SoE edges from its region rows (src/pathfinder.rs:162-178)
        const bool walks0 = have && src != p.vc;
        const LLab st0 = ll_start();
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) {
            if (t > NS) continue;
            const SpecialStatic tS = spl[t];
            FromS f;
            f.any = false;
            f.won = false;
            f.c = st0;
            f.w = st0;
            consider(f, have && t == ts, st0);
            consider(f, have && t == p.hq_t, LLab{0, p.shq_cost, 0, ll_pack(1, 0, 1), kSHQ << 29});
            consider(f, have && p.use_sfm && t == 1, LLab{0, p.sfm_cost, 0, ll_pack(1, 0, 1), kSFm << 29});
            if (p.use_soe && tS.rid != kNone10) {  // [SoE src -> t], or [Std{d} src -> u, SoE u -> t]
                const uint2 e = have ? srow[tS.rid] : make_uint2(kNone32, 0);
                const bool on = walks0 && e.x != kNone32;
                const LLab c = e.x == 0 ? LLab{0, p.soe_cost, 0, ll_pack(1, 0, 1), kSoE << 29}
                                        : LLab{e.x, p.soe_cost, run_time(e.x), ll_pack(2, 0, 2), (kStandard << 29) | e.x};
                consider(f, on, c);
            }
            if (t != 1) {
                const bool on = walks0 && tS.v != src;
                const uint32_t k = walk_dist(sx, sy, tS.x, tS.y);
                const LLab c{k, 0, run_time(k), ll_pack(1, 0, 1), (kStandard << 29) | k};
                consider(f, on, c);
                f.w = c;
                f.won = on;
            }
            if (f.any) {
                L[t] = f.c;
                tent |= 1u << t;
                wt |= (f.won && eq3(f.w, f.c)) ? (1u << t) : 0u;
            } else {
                L[t] = st0;
            }
        }
        // ---- Dijkstra over the specials, one settle per lane per iteration ----------
        for (uint32_t it = 0; it < NS; ++it) {
            const uint32_t cand = tent & ~done;
            if (!__any(cand != 0)) break;
            // the settle candidate: least (c1, c2, c3, length)
            LLab ls = st0;
            uint32_t s = 0;
            bool tie = false;
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
                const bool c = (cand >> t) & 1u;
                const int r = s == 0 ? -1 : cmp4(L[t], ls);
                const bool take = c && r < 0;
                tie = take ? false : (tie || (c && r == 0));
                ll_sel(take, ls, L[t]);
                s = take ? t : s;
            }
            if (tie) {  // exact (metrics, length) ties: the command lists decide (rare)
                for (uint32_t m = cand & ~(1u << s); m; m &= m - 1u) {
                    const uint32_t t = uint32_t(__builtin_ctz(m));
                    const LLab lt = get(t);
                    if (cmp4(lt, ls) != 0) continue;
                    if (cmp_list(lt, t, spl[t].rk, spl[t].rid, ls, s, spl[s].rk, spl[s].rid) < 0) {
                        ls = lt;
                        s = t;
                    }
                }
            }
            const bool act = s != 0;
            const uint32_t sc = act ? s : 1u;
            const SpecialStatic sS = spl[sc];
            done |= act ? (1u << s) : 0u;
            const uint32_t lk = ll_nt(ls.lpn) == 2 ? kSoE : (ls.kp >> 29);
            const bool boundary = act && lk != kNoMove && lk != kStandard;
            blk |= (boundary && ((wt >> s) & 1u)) ? (1u << s) : 0u;  // a walk tied it: a blocker
            const bool walks = boundary && s != 1;                     // the Center starts no walks
            bndm |= walks ? (1u << s) : 0u;
            uint32_t ties = 0;
            const bool any_walks = __any(walks);
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
                if (t > NS || !__any(act && !((done >> t) & 1u))) continue;  // settled in every lane
                const SpecialStatic tS = spl[t];
                const bool live = act && !((done >> t) & 1u);
                FromS f;
                if (any_walks) f = from_s(live, ls, sc, sS, walks, t, tS);
                else f = from_s(live, ls, sc, sS, false, t, tS);
                offer(t, f, ties);
            }
            // exact ties with a tentative label: the candidate is rebuilt and its command
            // list compared (rare; run-time t)
            for (; ties; ties &= ties - 1u) {
                const uint32_t t = uint32_t(__builtin_ctz(ties));
                const SpecialStatic tS = spl[t];
                const FromS f = from_s(true, ls, sc, sS, walks, t, tS);
                const LLab cur = get(t);
                if (cmp4(f.c, cur) == 0 && cmp_list(f.c, kOwn, tS.rk, tS.rid, cur, t, tS.rk, tS.rid) < 0) put(t, f.c);
            }
        }
        if (!have) return 0;
        // ---- certification: with blockers, every settled walk label must be certain ----
        bool unc = false;
        if (blk != 0) {
            for (uint32_t m = done; m; m &= m - 1u) {
                const uint32_t t = uint32_t(__builtin_ctz(m));
                if (!label_avail(get(t), t)) unc = true;
            }
        }
        const uint32_t qa = a->q_begin[s_idx], qb = a->q_begin[s_idx + 1];
        const bool fb_sp = unc || a->fb_all;
        // ---- destinations: the source, a special's own label, or the best walk ------------
        const bool walk0 = src != p.vc;
        for (uint32_t qi = fb_sp ? qb : qa; qi < qb; ++qi) {
            const uint32_t w = a->q_dst[qi];
            const uint32_t tw = sinfo[w] & kNone10;
            const uint32_t wr = rank[w];
            if (w == src) {
                emit(st0, src_rk, kNone10, qi);
                continue;
            }
            if (tw != kNone10) {
                emit(get(tw), spl[tw].rk, spl[tw].rid, qi);
                continue;
            }
            const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
            LLab x = st0;
            uint32_t bx = kNone32;
            bool tie = false;
            if (walk0) {
                const uint32_t k = walk_dist(sx, sy, wx, wy);
                x = LLab{k, 0, run_time(k), ll_pack(1, 0, 1), (kStandard << 29) | k};
                bx = 0;
            }
#pragma unroll
            for (uint32_t t = 2; t < TM; ++t) {
                if (!__any((bndm >> t) & 1u)) continue;
                const bool on = (bndm >> t) & 1u;
                const LLab c = walk(L[t], t, walk_dist(spl[t].x, spl[t].y, wx, wy));
                const int r = bx == kNone32 ? -1 : cmp4(c, x);
                const bool take = on && r < 0;
                tie = take ? false : (tie || (on && r == 0));
                ll_sel(take, x, c);
                bx = take ? t : bx;
            }
            if (tie) {  // equal metrics and length from several boundaries: the lists decide
                for (uint32_t m = (bndm | (walk0 ? 1u : 0u)) & ~(1u << bx); m; m &= m - 1u) {
                    const uint32_t b = uint32_t(__builtin_ctz(m));
                    int px, py;
                    bpos(b, px, py);
                    const uint32_t k = walk_dist(px, py, wx, wy);
                    const LLab c = b == 0 ? LLab{k, 0, run_time(k), ll_pack(1, 0, 1), (kStandard << 29) | k}
                                          : walk(get(b), b, k);
                    if (cmp4(c, x) == 0 && cmp_list(c, kOwn, wr, kNone10, x, kOwn, wr, kNone10) < 0) {
                        x = c;
                        bx = b;
                    }
                }
            }
            if (bx == kNone32) {  // no boundary can walk here: cannot happen on a connected grid
                a->out_res[qi] = OutResult{0, 0, 0, uint32_t(16 + 1) << 16};
                continue;
            }
            emit(x, wr, kNone10, qi);
            if (blk != 0) {
                int px, py;
                bpos(bx, px, py);
                if (!avail(bx, px, py, wx, wy)) unc = true;
            }
        }
        const bool fallback = fb_sp || unc;
        if (fallback) a->fb_list[atomicAdd(counter + kCtrFbCount, 1u)] = s_idx;
        return fallback ? 0u : qb - qa;
    }
};

template <uint32_t PERM, uint32_t TM>
__global__ __launch_bounds__(kBS, MR_LANE_WAVES) void hub_lane_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t NS = a->p.NS, nreg = a->nreg;
    SpecialStatic *spl = reinterpret_cast<SpecialStatic *>(smem);
    uint2 *nearl = reinterpret_cast<uint2 *>(smem + align16h((NS + 1) * uint32_t(sizeof(SpecialStatic))));
    for (uint32_t t = threadIdx.x; t <= NS; t += kBS) spl[t] = a->sp[t];
    for (uint32_t i = threadIdx.x; i < NS * nreg; i += kBS) {
        const uint32_t t = 1 + i / nreg, r = i % nreg;
        nearl[t * nreg + r] = reinterpret_cast<const uint2 *>(a->near)[(unsigned long long)a->sp[t].v * nreg + r];
    }
    __syncthreads();
    LaneHub<PERM, TM> H;
    H.a = a;
    H.P = a->p;
    H.P.perm[0] = PERM / 9;
    H.P.perm[1] = (PERM / 3) % 3;
    H.P.perm[2] = PERM % 3;
    H.spl = spl;
    H.nearS = nearl;
    H.rank = a->rank;
    H.sinfo = a->sinfo;
    H.rank_inv = a->rank_inv;
    H.counter = a->counter;
    H.nreg = nreg;
    // lane l of wave w: source 64 w + l of the lane kernel's sources [0, n_lane)
    const uint32_t s_idx = (blockIdx.x * (kBS / 64) + (threadIdx.x >> 6)) * 64u + lane_id();
    const uint32_t n = a->n_lane;
    const bool have = s_idx < n;
    uint32_t written = 0;
    if (__any(have)) written = H.solve(have, have ? s_idx : (n ? n - 1 : 0));
    if (H.err) atomicOr(a->counter + kCtrFlags, H.err);
    __shared__ uint32_t wsum;
    if (threadIdx.x == 0) wsum = 0;
    __syncthreads();
    if (written) atomicAdd(&wsum, written);
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, wsum);
}

}  // namespace mr
