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
// wave instruction advances 64 sources.  No cross-lane operation in the loop.
//
// A label is 4 registers: (c1, c2) as one 64-bit key, c3, and a meta word (length,
// parent entry, tail count, the first tail command's kind and CentralMove count); the
// command payloads (walk / caravan / SoE-region distances) follow from the parent's
// and the entry's cells, so they are rebuilt where a command is written or compared.
// The host only gives this kernel plans whose metric sums provably stay below 2^32
// (lane_bounds_ok, mr_host.cpp), so a 64-bit add of packed deltas never carries.
//
// Exactness follows hub_kernel step for step:
//   * candidates into an entry from one settled special s share chain(s), so among
//     them (metrics, length) ties are decided by the last command's kind (the list
//     order; their kinds differ); the best of them is compared with the entry's
//     tentative label, and only an exact (metrics, length) tie there walks the command
//     lists (cmp_list, rare, out of the unrolled code);
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
// a scheduling fence between the unrolled entries: without it the scheduler interleaves
// all of them and runs out of (scalar lane-mask) registers
#ifndef MR_LANE_NOFENCE
#define MR_LANE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define MR_LANE_FENCE() do {} while (0)
#endif

// meta: kind of the first tail command (3 b) | length (8 b) << 3 | parent entry (5 b)
// << 11 | (tail count - 1) << 16 | CentralMove count (2 b) << 17.  (meta & 0x7FF)
// orders by (length, kind): the tie-break among candidates from one settled special.
__device__ __forceinline__ uint32_t lm_kind(uint32_t m) { return m & 7u; }
__device__ __forceinline__ uint32_t lm_len(uint32_t m) { return (m >> 3) & 0xFFu; }
__device__ __forceinline__ uint32_t lm_lk(uint32_t m) { return m & 0x7FFu; }
__device__ __forceinline__ uint32_t lm_par(uint32_t m) { return (m >> 11) & 31u; }
__device__ __forceinline__ uint32_t lm_nt(uint32_t m) { return ((m >> 16) & 1u) + 1u; }
__device__ __forceinline__ uint32_t lm_cj(uint32_t m) { return (m >> 17) & 3u; }
__device__ __forceinline__ uint32_t lm_pack(uint32_t len, uint32_t par, uint32_t nt, uint32_t kind, uint32_t cj = 0) {
    return kind | (len << 3) | (par << 11) | ((nt - 1u) << 16) | (cj << 17);
}
constexpr unsigned long long kInfK = ~0ull;  // a label that is not there (no metrics reach 2^32 - 1 here)
// the pair table word of specials (s, t): walk distance | detour << 14 | SoE-region
// distance from s into t's region << 15 (kPtNoSd: none) | t's caravan coefficient bit
// << 29; Manhattan = walk - 2 detour
constexpr uint32_t kPtNoSd = 0x3FFFu;
__device__ __forceinline__ uint32_t pt_wd(uint32_t w) { return w & 0x3FFFu; }
__device__ __forceinline__ uint32_t pt_md(uint32_t w) { return (w & 0x3FFFu) - ((w >> 13) & 2u); }
__device__ __forceinline__ uint32_t pt_sd(uint32_t w) { return (w >> 15) & 0x3FFFu; }
__device__ __forceinline__ uint32_t pt_c5(uint32_t w) { return (w >> 29) & 1u; }  // a caravan into t costs 5 per unit

struct LLab {
    unsigned long long K;  // c1 << 32 | c2
    uint32_t c3, meta;
};
// A per-lane bit as a plain VGPR value.  Without the empty asm the compiler keeps
// every such boolean of the unrolled loops as a 64-bit lane mask in SGPRs, runs out of
// them and spills (hundreds of SGPRs, 60 VGPRs of spill lanes).
__device__ __forceinline__ uint32_t vbit(bool b, uint32_t bit) {
    uint32_t v = b ? bit : 0u;
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ void ll_sel(bool take, LLab &d, const LLab &c) {
    d.K = take ? c.K : d.K;
    d.c3 = take ? c.c3 : d.c3;
    d.meta = take ? c.meta : d.meta;
}

template <uint32_t PERM, uint32_t TM>
struct LaneHub {
    static constexpr uint32_t C1 = PERM / 9, C2 = (PERM / 3) % 3, C3 = PERM % 3;
    const KArgs *__restrict__ a;
    DevParams P;
    const SpecialStatic *spl;  // LDS copy of a->sp
    const uint2 *nearS;        // LDS: region rows of the specials, row t at t * nreg
    const uint32_t *PT;        // LDS: the pair table, row s at s * TM
    const uint32_t *rank, *sinfo, *rank_inv;
    uint32_t *counter;
    uint32_t nreg;
    uint32_t hubm, c5m, regm;  // entries that are caravan hubs / cost 5 per unit to reach / region campfires
    uint32_t validm;           // entries 1..NS
    // this lane's source
    uint32_t src = 0, src_rk = 0, ts = kNone10;
    int sx = 0, sy = 0;
    const uint2 *srow = nullptr;  // global: the source's region row
    // tentative / settled labels of entries 1..TM-1 (entry 0, the source, is the start label)
    LLab L[TM];
    uint32_t tent = 0, done = 0, wt = 0, bndm = 0, blk = 0;

    // ---- metrics in comparator order -------------------------------------------------
    __device__ __forceinline__ static uint32_t pick(uint32_t i, uint32_t legs, uint32_t money, uint32_t time) {
        return i == 0 ? legs : (i == 1 ? money : time);
    }
    // a (legs, money, time) delta packed as the key's (c1, c2) part
    __device__ __forceinline__ static unsigned long long dK(uint32_t legs, uint32_t money, uint32_t time) {
        return ((unsigned long long)pick(C1, legs, money, time) << 32) | pick(C2, legs, money, time);
    }
    __device__ __forceinline__ static uint32_t d3(uint32_t legs, uint32_t money, uint32_t time) {
        return pick(C3, legs, money, time);
    }
    __device__ __forceinline__ static uint32_t metric(const LLab &x, uint32_t i) {  // i: 0 legs, 1 money, 2 time
        return i == C1 ? uint32_t(x.K >> 32) : (i == C2 ? uint32_t(x.K) : x.c3);
    }
    __device__ __forceinline__ static LLab mk(unsigned long long K, uint32_t c3, uint32_t meta) { return LLab{K, c3, meta}; }
    __device__ __forceinline__ static LLab start() { return LLab{0ull, 0u, lm_pack(1, 0, 1, kNoMove)}; }
    // (c1, c2, c3, length): -1, 0, 1
    __device__ __forceinline__ static int cmp4(const LLab &x, const LLab &y) {
        if (x.K != y.K) return x.K < y.K ? -1 : 1;
        if (x.c3 != y.c3) return x.c3 < y.c3 ? -1 : 1;
        const uint32_t lx = lm_len(x.meta), ly = lm_len(y.meta);
        if (lx != ly) return lx < ly ? -1 : 1;
        return 0;
    }
    __device__ __forceinline__ static bool eq3(const LLab &x, const LLab &y) { return (x.K == y.K) & (x.c3 == y.c3); }
    // the same as two flags, without branches (bitwise, so nothing short-circuits into
    // divergent control flow in the unrolled loops)
    struct Cmp {
        bool lt, eq;
    };
    __device__ __forceinline__ static Cmp cmpx(const LLab &x, const LLab &y) {
        const bool kl = x.K < y.K, ke = x.K == y.K, cl = x.c3 < y.c3, ce = x.c3 == y.c3;
        const uint32_t lx = lm_len(x.meta), ly = lm_len(y.meta);
        return Cmp{bool(kl | (ke & (cl | (ce & (lx < ly))))), bool(ke & ce & (lx == ly))};
    }

    __device__ __forceinline__ uint32_t rk(uint32_t e) const { return e == 0 ? src_rk : spl[e].rk; }
    __device__ __forceinline__ void pos(uint32_t e, int &x, int &y) const {
        x = e == 0 ? sx : spl[e].x;
        y = e == 0 ? sy : spl[e].y;
    }
    // region row entry r of entry p's cell (p = 0: the source)
    __device__ __forceinline__ uint2 near_of(uint32_t p, uint32_t r) const { return p == 0 ? srow[r] : nearS[p * nreg + r]; }
    // entry e's label (run-time e; a select per entry: the rare paths only)
    __device__ __forceinline__ LLab get(uint32_t e) const {
        LLab r = start();
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) ll_sel(e == t, r, L[t]);
        return r;
    }
    __device__ __forceinline__ void put(uint32_t e, const LLab &c) {
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) ll_sel(e == t, L[t], c);
    }

    // ---- commands of a label (rare paths: list compares and output) -----------------
    // The label x ends at a cell at (ox, oy) of rank ork, region orid (kNone10: none).
    // Its first tail command's payload follows from its parent's cell: a walk's or a
    // caravan's distance, the SoE-region distance, or the CentralMove count.
    struct Own {
        int x, y;
        uint32_t rk, rid, c5;  // c5: a caravan into this cell costs 5 per unit
    };
    __device__ __forceinline__ Own own_of(uint32_t e) const {
        int x, y;
        pos(e, x, y);
        return Own{x, y, rk(e), e == 0 ? kNone10 : spl[e].rid, (c5m >> e) & 1u};
    }
    __device__ __forceinline__ Cmd tail(uint32_t meta, const Own &o, int i) const {
        const uint32_t p = lm_par(meta), kind = lm_kind(meta), nt = lm_nt(meta);
        int px, py;
        pos(p, px, py);
        uint32_t pay = 0, u = o.rk;
        if (nt == 2) {  // [Std{d} p -> u, SoE u -> own]: u is p's nearest cell of own's region
            const uint2 e = near_of(p, o.rid);
            pay = e.x;
            u = e.y;
        } else if (kind == kStandard) {
            pay = walk_dist(px, py, o.x, o.y);
        } else if (kind == kCaravan) {
            pay = (uint32_t(abs(px - o.x) + abs(py - o.y)) << 1) | o.c5;
        } else if (kind == kCentral) {
            pay = lm_cj(meta);
        }
        if (i == 0) return Cmd{(kind << 29) | pay, rk(p), u};
        return Cmd{kSoE << 29, u, o.rk};
    }
    __device__ __forceinline__ static int cmp_cmd(const Cmd &x, const Cmd &y) {
        if (x.kp != y.kp) return x.kp < y.kp ? -1 : 1;
        if (x.from != y.from) return x.from < y.from ? -1 : 1;
        if (x.to != y.to) return x.to < y.to ? -1 : 1;
        return 0;
    }
    // The rare paths read the entries' meta words from a per-wave LDS copy (M: entry t of
    // lane l at t * 64 + l), written by dump_meta() right before them, so they walk
    // command chains with LDS reads instead of selects over the register-held table.
    uint32_t *M;
    __device__ __forceinline__ void dump_meta() const {
        const uint32_t l = lane_id();
        M[l] = start().meta;
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) M[t * 64u + l] = L[t].meta;
    }
    __device__ __forceinline__ uint32_t meta_of(uint32_t e) const { return M[e * 64u + lane_id()]; }
    // lexicographic compare of two equal-length command lists (metas x and y), walking
    // from the last command towards the first (hub_kernel's cmp_list); xid/yid name the
    // table entries the labels are (kOwn for built ones), so a shared prefix stops the walk
    __device__ __forceinline__ int cmp_list(uint32_t x, uint32_t xid, Own xo, uint32_t y, uint32_t yid, Own yo) const {
        int xt = int(lm_nt(x)) - 1, yt = int(lm_nt(y)) - 1;
        int res = 0;
        for (uint32_t guard = 0; guard < 4096u; ++guard) {
            if (xid != kOwn && xid == yid && xt == yt) return res;
            const int r = cmp_cmd(tail(x, xo, xt), tail(y, yo, yt));
            if (r) res = r;
            if (xt > 0) {
                --xt;
            } else {
                const uint32_t pp = lm_par(x);
                if (pp == 0) return res;
                xid = pp;
                x = meta_of(pp);
                xo = own_of(pp);
                xt = int(lm_nt(x)) - 1;
            }
            if (yt > 0) {
                --yt;
            } else {
                const uint32_t pp = lm_par(y);
                if (pp == 0) return res;
                yid = pp;
                y = meta_of(pp);
                yo = own_of(pp);
                yt = int(lm_nt(y)) - 1;
            }
        }
        atomicOr(counter + kCtrFlags, kErrChain);
        return res;
    }

    // the walk of k legs from table entry b (label lb) to a plain cell
    __device__ __forceinline__ static LLab walk_to(const LLab &lb, uint32_t b, uint32_t k) {
        return mk(lb.K + dK(k, 0, 180u * k), lb.c3 + d3(k, 0, 180u * k), lm_pack(lm_len(lb.meta) + 1u, b, 1, kStandard));
    }

    // ---- candidates from one settled special s into entry t ------------------------
    // The best of the CentralMove, caravan, SoE, walk and SoE-region candidates from s;
    // they share chain(s), so (metrics, length) ties go to the smaller last-command kind.
    // Also the walk candidate itself (for the blocker bit).
    // A candidate that does not apply has K = kInfK, so choosing among candidates is a
    // plain minimum and no per-entry flag outlives its compare.
    struct FromS {
        LLab c, w;  // the best candidate from s; the walk candidate (for the blocker bit)
    };
    __device__ __forceinline__ static LLab opt(bool on, const LLab &c) { return LLab{on ? c.K : kInfK, c.c3, c.meta}; }
    // c replaces f.c if smaller by (c1, c2, c3, length, kind)
    __device__ __forceinline__ static void consider(LLab &f, const LLab &c) {
        const bool lt = (c.K < f.K) | ((c.K == f.K) & ((c.c3 < f.c3) | ((c.c3 == f.c3) & (lm_lk(c.meta) < lm_lk(f.meta)))));
        ll_sel(lt, f, c);
    }
    // Per-iteration context of the settled special s: its label ls; `base` = ls with an
    // appended command (length + 1, parent s; the zero label when ls is the start label,
    // whose NoMove is replaced); merge = ls ends in a CentralMove (one more merges).
    // Which candidate kinds apply to which entries is a set of per-lane bit masks.
    struct Settle {
        LLab ls, base;
        uint32_t s;
        bool merge;
        uint32_t cen, car, soe, reg, walk;  // entries a CentralMove / caravan / SoE / SoE-region / walk reaches
    };
    __device__ __forceinline__ FromS from_s(const Settle &z, uint32_t t, uint32_t w) const {
        const DevParams &p = P;
        const uint32_t wd = pt_wd(w), md = pt_md(w), sd = pt_sd(w);
        const uint32_t s = z.s, len = lm_len(z.ls.meta);
        FromS f;
        // the walk from boundary s (not into the Center)
        f.w = opt((z.walk >> t) & 1u, mk(z.ls.K + dK(wd, 0, 180u * wd), z.ls.c3 + d3(wd, 0, 180u * wd),
                                          lm_pack(len + 1u, s, 1, kStandard)));
        f.c = f.w;
        // CentralMove: the Center (entry 1) <-> the border-1 cells (entries 2..5)
        if (t <= 5) {
            const LLab c = z.merge ? mk(z.ls.K + dK(0, 0, 10), z.ls.c3 + d3(0, 0, 10),
                                        lm_pack(len, lm_par(z.ls.meta), 1, kCentral, lm_cj(z.ls.meta) + 1u))
                                   : mk(z.base.K + dK(0, 0, 10), z.base.c3 + d3(0, 0, 10),
                                        z.base.meta | lm_pack(0, 0, 1, kCentral, 1));
            consider(f.c, opt((z.cen >> t) & 1u, c));
        }
        // caravans between hubs (src/pathfinder.rs:140-160, caravan_cost :251-273)
        {
            const uint32_t money = (2u + 3u * pt_c5(w)) * md, time = p.rgt * md;
            consider(f.c, opt((z.car >> t) & 1u, mk(z.base.K + dK(0, money, time), z.base.c3 + d3(0, money, time),
                                                    z.base.meta | lm_pack(0, 0, 1, kCaravan))));
        }
        // s's Scroll of Escape to its region's campfire (src/pathfinder.rs:162-170)
        consider(f.c, opt((z.soe >> t) & 1u, mk(z.base.K + dK(0, p.soe_cost, 0), z.base.c3 + d3(0, p.soe_cost, 0),
                                                z.base.meta | lm_pack(0, 0, 1, kSoE))));
        // from the region cell nearest to boundary s: [Std{d} s -> u, SoE u -> t]
        consider(f.c, opt(((z.reg >> t) & 1u) & (sd != kPtNoSd) & (sd != 0u),
                          mk(z.ls.K + dK(sd, p.soe_cost, 180u * sd), z.ls.c3 + d3(sd, p.soe_cost, 180u * sd),
                             lm_pack(len + 2u, s, 2, kStandard))));
        return f;
    }
    // the best candidate into entry t against its tentative label (K = kInfK: none):
    // a strict win takes, an exact (metrics, length) tie is left to the list compare
    // (bit t of *ties)
    __device__ __forceinline__ void offer(uint32_t t, const FromS &f, uint32_t &ties) {
        LLab &T = L[t];
        const uint32_t bit = 1u << t;
        const bool any = f.c.K != kInfK;
        const bool ke = f.c.K == T.K, ce = f.c.c3 == T.c3;
        const uint32_t lf = lm_len(f.c.meta), lt_ = lm_len(T.meta);
        const bool lt = any & ((f.c.K < T.K) | (ke & ((f.c.c3 < T.c3) | (ce & (lf < lt_)))));
        const bool same3 = any & ke & ce;
        ll_sel(lt, T, f.c);
        tent |= vbit(lt, bit);
        // blocker bit: a walk candidate with the (new) tentative metrics; kept while the
        // tentative metrics stay (an unchanged label, or a win on length / commands)
        const bool keep = !lt | same3;
        const bool wtie = (f.w.K != kInfK) & (f.w.K == T.K) & (f.w.c3 == T.c3);
        wt = (wt & ~bit) | vbit((keep & ((wt & bit) != 0)) | wtie, bit);
        ties |= vbit(same3 & (lf == lt_), bit);
    }

    // ---- certification (hub_kernel's avail / label_avail) ----------------------------
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
    // entry t's settled label x: its walk, or the walk to the cell its SoE is read from
    __device__ __forceinline__ bool label_avail(uint32_t meta, uint32_t t) const {
        if (lm_kind(meta) != kStandard) return true;
        const uint32_t b = lm_par(meta);
        int bx, by;
        pos(b, bx, by);
        if (lm_nt(meta) == 1) return avail(b, bx, by, spl[t].x, spl[t].y);
        const uint32_t u = rank_inv[near_of(b, spl[t].rid).y];
        return avail(b, bx, by, int(u % P.S) - int(P.H), int(u / P.S) - int(P.H));
    }

    // ---- output (Core::emit) --------------------------------------------------------
    __device__ __forceinline__ void emit(const LLab &x, uint32_t xid, const Own &xo, uint32_t qi) const {
        const DevParams &p = P;
        OutResult &o = a->out_res[qi];
        OutCmd *oc = a->out_cmd + (unsigned long long)qi * p.max_cmds;
        const uint32_t len = lm_len(x.meta);
        const uint32_t legs = metric(x, 0), money = metric(x, 1), time = metric(x, 2);
        uint32_t status = 16;
        if (len > p.max_cmds) {  // the overflow pool, else MR_ERR_CAPACITY
            const uint32_t off = atomicAdd(counter + kCtrOvf, len);
            if (p.max_cmds == 0 || off + len > a->ovf_cap || off + len < off) {
                o = OutResult{legs, money, time, (uint32_t(16 - 4) << 16) | (len & 0xFFFFu)};
                return;
            }
            oc[0] = OutCmd{kOvfTag, off, len, 0};
            oc = a->ovf + off;
            status = 16 + kStatusOverflow;
        }
        int at = int(len) - 1;
        uint32_t e = x.meta;
        Own eo = xo;
        uint32_t eid = xid;
        for (uint32_t guard = 0; at >= 0 && guard <= TM + 1; ++guard) {
            for (int j = int(lm_nt(e)) - 1; j >= 0 && at >= 0; --j, --at) {
                const Cmd c = tail(e, eo, j);
                oc[at] = OutCmd{c.kp, c.from, c.to, 0};
            }
            eid = lm_par(e);
            if (eid == 0) break;
            e = meta_of(eid);
            eo = own_of(eid);
        }
        if (at != -1 || eid != 0) atomicOr(counter + kCtrFlags, kErrChain);
        o = OutResult{legs, money, time, (status << 16) | (len & 0xFFFFu)};
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
        const LLab st0 = start(), inf = LLab{kInfK, 0u, 0u};
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) {
            const bool valid = have && t <= NS;
            const SpecialStatic tS = spl[t <= NS ? t : 1u];
            LLab c = opt(valid && t == ts, st0);
            consider(c, opt(valid && t == p.hq_t, mk(dK(0, p.shq_cost, 0), d3(0, p.shq_cost, 0), lm_pack(1, 0, 1, kSHQ))));
            consider(c, opt(valid && p.use_sfm && t == 1,
                            mk(dK(0, p.sfm_cost, 0), d3(0, p.sfm_cost, 0), lm_pack(1, 0, 1, kSFm))));
            {  // [SoE src -> t], or [Std{d} src -> u, SoE u -> t]
                const bool reg = valid && p.use_soe && tS.rid != kNone10;
                const uint32_t e = reg ? srow[reg ? tS.rid : 0u].x : kNone32;
                const bool on = walks0 && reg && e != kNone32;
                const uint32_t d = on ? e : 1u;
                consider(c, opt(on, d == 0 ? mk(dK(0, p.soe_cost, 0), d3(0, p.soe_cost, 0), lm_pack(1, 0, 1, kSoE))
                                           : mk(dK(d, p.soe_cost, 180u * d), d3(d, p.soe_cost, 180u * d),
                                                lm_pack(2, 0, 2, kStandard))));
            }
            LLab w = inf;
            if (t != 1) {
                const uint32_t k = walk_dist(sx, sy, tS.x, tS.y);
                w = opt(valid && walks0 && tS.v != src, mk(dK(k, 0, 180u * k), d3(k, 0, 180u * k), lm_pack(1, 0, 1, kStandard)));
                consider(c, w);
            }
            L[t] = c;
            tent |= c.K != kInfK ? (1u << t) : 0u;
            wt |= ((w.K != kInfK) & eq3(w, c)) ? (1u << t) : 0u;
        }
        // ---- Dijkstra over the specials, one settle per lane per iteration ----------
        for (uint32_t it = 0; it < NS; ++it) {
            const uint32_t cand = tent & ~done;
            if (!__any(cand != 0)) break;
            // the settle candidate: least (c1, c2, c3, length), two interleaved chains
            // (odd and even entries) for the latency, then merged
            LLab la = inf, lb = inf;
            uint32_t sa = 0, sb = 0;
            bool ta = false, tb = false;
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
                LLab &lx = (t & 1u) ? la : lb;
                uint32_t &sx_ = (t & 1u) ? sa : sb;
                bool &tx = (t & 1u) ? ta : tb;
                const LLab c = opt((cand >> t) & 1u, L[t]);
                const bool ke = c.K == lx.K, ce = c.c3 == lx.c3;
                const uint32_t lc = lm_len(c.meta), ll = lm_len(lx.meta);
                const bool lt = (c.K < lx.K) | (ke & ((c.c3 < lx.c3) | (ce & (lc < ll))));
                tx = lt ? false : (tx | ((c.K != kInfK) & ke & ce & (lc == ll)));
                ll_sel(lt, lx, c);
                sx_ = lt ? t : sx_;
            }
            Settle z;
            z.ls = la;
            uint32_t s = sa;
            bool tie = ta;
            {
                const bool ke = lb.K == la.K, ce = lb.c3 == la.c3;
                const uint32_t l1 = lm_len(lb.meta), l0 = lm_len(la.meta);
                const bool lt = (lb.K < la.K) | (ke & ((lb.c3 < la.c3) | (ce & (l1 < l0))));
                ll_sel(lt, z.ls, lb);
                s = lt ? sb : sa;
                tie = lt ? tb : (ta | ((lb.K != kInfK) & ke & ce & (l1 == l0)));
            }
            if (__any(tie)) {  // exact (metrics, length) ties: the command lists decide (rare)
                uint32_t tied = 0;  // the entries with the winner's metrics and length
#pragma unroll
                for (uint32_t t = 1; t < TM; ++t)
                    tied |= (((cand >> t) & 1u) & eq3(L[t], z.ls) & (lm_len(L[t].meta) == lm_len(z.ls.meta))) ? (1u << t)
                                                                                                            : 0u;
                dump_meta();
                if (tie) {
                    for (uint32_t m = tied & ~(1u << s); m; m &= m - 1u) {
                        const uint32_t t = uint32_t(__builtin_ctz(m));
                        const uint32_t mt = meta_of(t);
                        if (cmp_list(mt, t, own_of(t), z.ls.meta, s, own_of(s)) < 0) {
                            z.ls.meta = mt;  // (same metrics)
                            s = t;
                        }
                    }
                }
            }
            const bool act = s != 0;
            z.s = act ? s : 1u;
            done |= act ? (1u << s) : 0u;
            const uint32_t lk = lm_nt(z.ls.meta) == 2 ? kSoE : lm_kind(z.ls.meta);
            const bool boundary = act && lk != kNoMove && lk != kStandard;
            blk |= (boundary && ((wt >> s) & 1u)) ? (1u << s) : 0u;  // a walk tied it: a blocker
            const bool walks = boundary && s != 1;                     // the Center starts no walks
            bndm |= walks ? (1u << s) : 0u;
            const bool nomove = lk == kNoMove;  // the start label: its NoMove is replaced
            z.base = mk(nomove ? 0ull : z.ls.K, nomove ? 0u : z.ls.c3,
                        nomove ? lm_pack(1, 0, 1, 0) : lm_pack(lm_len(z.ls.meta) + 1u, z.s, 1, 0));
            z.merge = lk == kCentral;
            const uint32_t live = act ? (validm & ~done) : 0u;  // unsettled entries
            const uint32_t rg = spl[z.s].region;
            z.cen = live & (z.s == 1 ? 0x3Cu : ((z.s >= 2 && z.s <= 5) ? 0x2u : 0u));
            z.car = (p.use_caravans && ((hubm >> z.s) & 1u)) ? (live & hubm) : 0u;
            z.soe = (p.use_soe && rg != kNone10 && rg != z.s) ? (live & (1u << rg)) : 0u;
            z.reg = (walks && p.use_soe) ? (live & regm) : 0u;
            z.walk = walks ? (live & ~0x2u) : 0u;
            const uint32_t *row = PT + z.s * TM;
            uint32_t ties = 0;
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
                const FromS f = from_s(z, t, row[t]);
                offer(t, f, ties);
                MR_LANE_FENCE();
            }
            // exact ties with a tentative label: the candidate is rebuilt and its command
            // list compared (rare; run-time t)
            // (same metrics: only the meta word can change; the new ones go through LDS)
            if (__any(ties != 0)) {
                dump_meta();
                uint32_t repl = 0;
                for (; ties; ties &= ties - 1u) {
                    const uint32_t t = uint32_t(__builtin_ctz(ties));
                    const FromS f = from_s(z, t, row[t]);
                    const uint32_t cur = meta_of(t);
                    if (cmp_list(f.c.meta, kOwn, own_of(t), cur, t, own_of(t)) < 0) {
                        M[t * 64u + lane_id()] = f.c.meta;
                        repl |= 1u << t;
                    }
                }
#pragma unroll
                for (uint32_t t = 1; t < TM; ++t)
                    if ((repl >> t) & 1u) L[t].meta = M[t * 64u + lane_id()];
            }
        }
        if (!have) return 0;
        // ---- certification: with blockers, every settled walk label must be certain ----
        bool unc = false;
        dump_meta();  // (certification and the destinations' command chains)
        if (blk != 0) {
            for (uint32_t m = done; m; m &= m - 1u) {
                const uint32_t t = uint32_t(__builtin_ctz(m));
                if (!label_avail(meta_of(t), t)) unc = true;
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
                emit(st0, kOwn, Own{sx, sy, src_rk, kNone10, 0u}, qi);
                continue;
            }
            if (tw != kNone10) {
                emit(get(tw), tw, own_of(tw), qi);
                continue;
            }
            const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
            const Own wo{wx, wy, wr, kNone10, 0u};
            LLab x = inf;
            uint32_t bx = kNone32;
            bool tie = false;
            {
                const uint32_t k = walk_dist(sx, sy, wx, wy);
                x = opt(walk0, mk(dK(k, 0, 180u * k), d3(k, 0, 180u * k), lm_pack(1, 0, 1, kStandard)));
                bx = walk0 ? 0u : kNone32;
            }
#pragma unroll
            for (uint32_t t = 2; t < TM; ++t) {
                const uint32_t k = walk_dist(spl[t].x, spl[t].y, wx, wy);
                const LLab c = opt((bndm >> t) & 1u, walk_to(L[t], t, k));
                const bool ke = c.K == x.K, ce = c.c3 == x.c3;
                const uint32_t lc = lm_len(c.meta), lx = lm_len(x.meta);
                const bool lt = (c.K < x.K) | (ke & ((c.c3 < x.c3) | (ce & (lc < lx))));
                tie = lt ? false : (tie | ((c.K != kInfK) & ke & ce & (lc == lx)));
                ll_sel(lt, x, c);
                bx = lt ? t : bx;
            }
            if (tie) {  // equal metrics and length from several boundaries: the lists decide
                for (uint32_t m = (bndm | (walk0 ? 1u : 0u)) & ~(1u << bx); m; m &= m - 1u) {
                    const uint32_t b = uint32_t(__builtin_ctz(m));
                    int px, py;
                    pos(b, px, py);
                    const uint32_t k = walk_dist(px, py, wx, wy);
                    const LLab c = b == 0 ? mk(dK(k, 0, 180u * k), d3(k, 0, 180u * k), lm_pack(1, 0, 1, kStandard))
                                          : walk_to(get(b), b, k);
                    if (cmp4(c, x) == 0 && cmp_list(c.meta, kOwn, wo, x.meta, kOwn, wo) < 0) {
                        x = c;
                        bx = b;
                    }
                }
            }
            if (bx == kNone32) {  // no boundary can walk here: cannot happen on a connected grid
                a->out_res[qi] = OutResult{0, 0, 0, uint32_t(16 + 1) << 16};
                continue;
            }
            emit(x, kOwn, wo, qi);
            if (blk != 0) {
                int px, py;
                pos(bx, px, py);
                if (!avail(bx, px, py, wx, wy)) unc = true;
            }
        }
        const bool fallback = fb_sp || unc;
        if (fallback) a->fb_list[atomicAdd(counter + kCtrFbCount, 1u)] = s_idx;
        return fallback ? 0u : qb - qa;
    }
};

// the lane kernel's LDS: the specials' static records, their region rows and the pair table
__host__ __device__ inline uint32_t lane_off_near(uint32_t NS) { return align16h((NS + 1) * uint32_t(sizeof(SpecialStatic))); }
__host__ __device__ inline uint32_t lane_off_pt(uint32_t NS, uint32_t nreg) {
    return align16h(lane_off_near(NS) + (NS + 1) * nreg * 8u);
}
// then the pair table (TM x TM words) and per wave the meta copy of the rare paths (TM x 64 words)
__host__ __device__ inline uint32_t lane_off_meta(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return align16h(lane_off_pt(NS, nreg) + TM * TM * 4u);
}
__host__ __device__ inline uint32_t lane_lds_total(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_meta(NS, nreg, TM) + (kBS / 64) * TM * 64u * 4u;
}

template <uint32_t PERM, uint32_t TM>
__global__ __launch_bounds__(kBS, MR_LANE_WAVES) void hub_lane_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t NS = a->p.NS, nreg = a->nreg;
    SpecialStatic *spl = reinterpret_cast<SpecialStatic *>(smem);
    uint2 *nearl = reinterpret_cast<uint2 *>(smem + lane_off_near(NS));
    uint32_t *pt = reinterpret_cast<uint32_t *>(smem + lane_off_pt(NS, nreg));
    const uint2 *nearg = reinterpret_cast<const uint2 *>(a->near);
    for (uint32_t t = threadIdx.x; t <= NS; t += kBS) spl[t] = a->sp[t];
    for (uint32_t i = threadIdx.x; i < NS * nreg; i += kBS) {
        const uint32_t t = 1 + i / nreg, r = i % nreg;
        nearl[t * nreg + r] = nearg[(unsigned long long)a->sp[t].v * nreg + r];
    }
    // the pair table (LaneHub::from_s): walk / Manhattan / SoE-region distances of (s, t)
    for (uint32_t i = threadIdx.x; i < TM * TM; i += kBS) {
        const uint32_t s = i / TM, t = i % TM;
        uint32_t e = kPtNoSd << 15;
        if (s >= 1 && s <= NS && t >= 1 && t <= NS) {
            const SpecialStatic ss = a->sp[s], st = a->sp[t];
            const uint32_t wd = walk_dist(ss.x, ss.y, st.x, st.y);
            const uint32_t md = uint32_t(abs(ss.x - st.x) + abs(ss.y - st.y));
            uint32_t sd = kPtNoSd;
            if (st.rid != kNone10) {
                const uint32_t d = nearg[(unsigned long long)ss.v * nreg + st.rid].x;
                sd = d == kNone32 ? kPtNoSd : d;
            }
            e = wd | ((wd != md ? 1u : 0u) << 14) | (sd << 15) | ((st.coef5 ? 1u : 0u) << 29);
        }
        pt[i] = e;
    }
    __syncthreads();
    LaneHub<PERM, TM> H;
    H.a = a;
    H.P = a->p;
    H.spl = spl;
    H.nearS = nearl;
    H.PT = pt;
    H.M = reinterpret_cast<uint32_t *>(smem + lane_off_meta(NS, nreg, TM)) + (threadIdx.x >> 6) * (TM * 64u);
    H.rank = a->rank;
    H.sinfo = a->sinfo;
    H.rank_inv = a->rank_inv;
    H.counter = a->counter;
    H.nreg = nreg;
    uint32_t hubm = 0, c5m = 0, regm = 0;
    for (uint32_t t = 1; t <= NS && t < TM; ++t) {
        const SpecialStatic st = spl[t];
        hubm |= (st.flags & kSpHub) ? (1u << t) : 0u;
        c5m |= st.coef5 ? (1u << t) : 0u;
        regm |= st.rid != kNone10 ? (1u << t) : 0u;
    }
    H.hubm = __builtin_amdgcn_readfirstlane(hubm);
    H.c5m = __builtin_amdgcn_readfirstlane(c5m);
    H.regm = __builtin_amdgcn_readfirstlane(regm);
    H.validm = __builtin_amdgcn_readfirstlane(((2u << min(NS, TM - 1u)) - 1u) & ~1u);
    // lane l of wave w: source 64 w + l of the lane kernel's sources [0, n_lane)
    const uint32_t s_idx = (blockIdx.x * (kBS / 64) + (threadIdx.x >> 6)) * 64u + lane_id();
    const uint32_t n = a->n_lane;
    const bool have = s_idx < n;
    uint32_t written = 0;
    if (__any(have)) written = H.solve(have, have ? s_idx : (n ? n - 1 : 0));
    __shared__ uint32_t wsum;
    if (threadIdx.x == 0) wsum = 0;
    __syncthreads();
    if (written) atomicAdd(&wsum, written);
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, wsum);
}

}  // namespace mr
