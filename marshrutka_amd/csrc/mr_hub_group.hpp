// mr_hub_group.hpp — the hub solver with one SOURCE per group of G lanes (hub_group_kernel).
//
// Same algorithm and results as hub_kernel / hub_lane_kernel (DESIGN.md §3a, §3a‴): an
// exact Dijkstra over the specials whose edges are closed-form walks from settled
// boundaries plus the CentralMove / caravan / Scroll-of-Escape edges, and destinations
// read off as the best walk from a boundary (FindPath::eval, src/pathfinder.rs:199-248).
//
// hub_lane_kernel runs a whole source per lane: 64 sources a wave, so a plan needs tens
// of thousands of sources before its waves fill the GPU, and one wave's serial Dijkstra
// (~50k instructions) is the latency of the whole pass.  hub_kernel (a lane per special)
// pays a cross-lane reduction with exec-mask bookkeeping on every settle.  Here G lanes
// (8 or 16, one DPP row or half row) share a source: lane j of the group holds entries
// j, j + G, j + 2G, ... (E slots), so
//   * a settle is a per-lane scan of E slots, then log2(G) DPP rounds in which every lane
//     takes the lesser of its own and its partner's (c1, c2, c3, length, entry): five DPP
//     moves, a four-step borrow chain and five selects a round, and every lane of the
//     group ends with the winner;
//   * a relaxation is E compare-and-selects per lane, with the entries' roles (Center,
//     border, hub, region) as run-time bits of the settle's masks, so any table layout
//     up to 32 entries runs here;
//   * destinations are read off one query per lane from the settled labels in LDS.
// A source's Dijkstra is ~G times shorter in wave instructions than on the lane kernel,
// which is what small plans (configs[0] / configs[1], one query) are bound by.
//
// Exact (metrics, length) ties between candidates into one entry go to the command-list
// compares exactly as in the lane kernel (LaneHub::cmp_list); ties between two entries at
// a settle need none (either may settle first, LaneHub::solve).
#pragma once
#include "mr_hub_lane.hpp"

namespace mr {

// One DPP round of the group minimum: (c1, c2, c3, k) of this lane against the partner's
// (k = length << 24 | entry), the lesser kept with the m word riding along.  The
// partner's words come over by v_mov_b32_dpp; then the borrow chain mine - partner leaves
// VCC = mine < partner and five VOP2 selects keep mine or take the partner's.  (The DPP
// forms of the carry ops themselves, v_subrev_co / v_subbrev_co _dpp, assemble but do not
// compute this on gfx950: tools/micro/group_min.hip.)  s_nop 1: a DPP read of a VGPR
// written by the previous VALU instruction needs two wait states.
#define MR_GRP_ROUND(DPP)                                                                         \
    asm("s_nop 1\n\t"                                                                             \
        "v_mov_b32_dpp %6, %1 " DPP " row_mask:0xf bank_mask:0xf\n\t"                             \
        "v_mov_b32_dpp %7, %2 " DPP " row_mask:0xf bank_mask:0xf\n\t"                             \
        "v_mov_b32_dpp %8, %3 " DPP " row_mask:0xf bank_mask:0xf\n\t"                             \
        "v_mov_b32_dpp %9, %4 " DPP " row_mask:0xf bank_mask:0xf\n\t"                             \
        "v_mov_b32_dpp %10, %5 " DPP " row_mask:0xf bank_mask:0xf\n\t"                            \
        "v_sub_co_u32_e32 %0, vcc, %5, %10\n\t"                                                   \
        "v_subb_co_u32_e32 %0, vcc, %3, %8, vcc\n\t"                                              \
        "v_subb_co_u32_e32 %0, vcc, %2, %7, vcc\n\t"                                              \
        "v_subb_co_u32_e32 %0, vcc, %1, %6, vcc\n\t"                                              \
        "v_cndmask_b32_e32 %1, %6, %1, vcc\n\t"                                                   \
        "v_cndmask_b32_e32 %2, %7, %2, vcc\n\t"                                                   \
        "v_cndmask_b32_e32 %3, %8, %3, vcc\n\t"                                                   \
        "v_cndmask_b32_e32 %4, %9, %4, vcc\n\t"                                                   \
        "v_cndmask_b32_e32 %5, %10, %5, vcc"                                                      \
        : "=&v"(t_), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(m), "+v"(k), "=&v"(p1), "=&v"(p2),          \
          "=&v"(p3), "=&v"(pm), "=&v"(pk)                                                         \
        :                                                                                         \
        : "vcc")

// the same round with the partner's words already in p1..pk (the cross-row round)
__device__ __forceinline__ void grp_take(uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t &m, uint32_t &k, uint32_t p1,
                                         uint32_t p2, uint32_t p3, uint32_t pm, uint32_t pk) {
    uint32_t t_;
    asm("v_sub_co_u32_e32 %0, vcc, %5, %10\n\t"
        "v_subb_co_u32_e32 %0, vcc, %3, %8, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %2, %7, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %1, %6, vcc\n\t"
        "v_cndmask_b32_e32 %1, %6, %1, vcc\n\t"
        "v_cndmask_b32_e32 %2, %7, %2, vcc\n\t"
        "v_cndmask_b32_e32 %3, %8, %3, vcc\n\t"
        "v_cndmask_b32_e32 %4, %9, %4, vcc\n\t"
        "v_cndmask_b32_e32 %5, %10, %5, vcc"
        : "=&v"(t_), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(m), "+v"(k)
        : "v"(p1), "v"(p2), "v"(p3), "v"(pm), "v"(pk)
        : "vcc");
}

// the least (c1, c2, c3, k) over each group of G lanes, in every lane of the group: DPP
// rounds inside a row of 16 lanes, and for 32-lane groups one more through the LDS
// crossbar (ds_swizzle, lane ^ 16: no memory access)
template <uint32_t G>
__device__ __forceinline__ void group_min(uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t &m, uint32_t &k) {
    static_assert(G == 4 || G == 8 || G == 16 || G == 32, "groups are quads, half rows, rows or half waves");
    uint32_t t_, p1, p2, p3, pm, pk;
    MR_GRP_ROUND("quad_perm:[1,0,3,2]");
    MR_GRP_ROUND("quad_perm:[2,3,0,1]");
    if constexpr (G >= 8) MR_GRP_ROUND("row_half_mirror");
    if constexpr (G >= 16) MR_GRP_ROUND("row_mirror");
    if constexpr (G >= 32) {
        constexpr int kXor16 = 0x1F | (0x10 << 10);  // bitmask mode: and 0x1f, or 0, xor 0x10
        grp_take(c1, c2, c3, m, k, __builtin_amdgcn_ds_swizzle(int(c1), kXor16), __builtin_amdgcn_ds_swizzle(int(c2), kXor16),
                 __builtin_amdgcn_ds_swizzle(int(c3), kXor16), __builtin_amdgcn_ds_swizzle(int(m), kXor16),
                 __builtin_amdgcn_ds_swizzle(int(k), kXor16));
    }
}

// bit e of w as a 0 / ~0 mask, e a run-time value (one v_bfe_i32)
__device__ __forceinline__ uint32_t bitv(uint32_t w, uint32_t e) {
    uint32_t r;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(w), "v"(e));
    return r;
}

// diagnostic builds (-DMR_STAMPS): phase cycles per wave (s_memtime), summed into
// a->dbg[dbg_blocks * 10 + 9 ..] by each wave's lane 0 (mr_plan_destroy prints them)
#ifdef MR_STAMPS
#define MR_GSTAMP(i)                                                        \
    do {                                                                    \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();       \
        gst[i] += now_ - gst_last;                                          \
        gst_last = now_;                                                    \
    } while (0)
#else
#define MR_GSTAMP(i) \
    do {             \
    } while (0)
#endif

// NL: Fleetfoot 1..3 (LaneHub's run times and walk certification, the group's lanes
// sharing the boundaries)
template <uint32_t PERM, uint32_t G, uint32_t E, bool NL = false>
struct GroupHub : LaneHub<PERM, G * E, NL> {
#ifdef MR_STAMPS
    unsigned long long gst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, gst_last = 0;
#endif
    static constexpr uint32_t TM = G * E;  // table entries (slot i of lane j: entry i * G + j)
    using Base = LaneHub<PERM, TM, NL>;
    using Base::a;
    using Base::P;
    using Base::spl;
    using Base::PA;
    using Base::PB;
    using Base::M;
    using Base::counter;
    using Base::src;
    using Base::src_rk;
    using Base::ts;
    using Base::sx;
    using Base::sy;
    using Base::srow;
    using Base::nreg;
    using Base::tent;
    using Base::done;
    using Base::wt;
    using Base::bndm;
    using Base::blk;
    using Base::add;
    using Base::mk;
    using Base::opt;
    using Base::inf;
    using Base::start;
    using Base::consider;
    using Base::own_of;
    using Base::pos;
    using Base::cmp_list;
    using Base::cmp4;
    using Base::emit;
    using Base::avail;
    using Base::label_avail;
    using Base::cell_word;
    using Base::settle_ctx;
    using Base::walk_to;
    using Base::meta_of;
    using Base::rtime;
    using Base::mstride;
    using Base::mcolumn;
    using Own = typename Base::Own;
    using Settle = typename Base::Settle;
    using FromS = typename Base::FromS;

    LLab Ls[E];      // labels of this lane's slots
    int ex[E], ey[E];  // their cells (the read-off's walks)
    uint32_t *W = nullptr;  // LDS: this group's destinations of the current batch (G words)
    uint32_t gj = 0, gbase = 0;
    uint4 *LT = nullptr;  // LDS: this group's settled labels, entry e at LT[e]
    uint2 *SR = nullptr;  // LDS: this group's copy of the source's region row (nreg entries)
    // LDS: per settled entry e of this group its meta word and tail commands,
    // CT[2e] = {meta, cmd0}, CT[2e + 1] = {cmd1 (a SoE after a walk), -}: written once after
    // the Dijkstra (every lane its own entries), read by the emission's chain walk
    uint4 *CT = nullptr;

    // a label's record and commands: the last command wc when `last` (a destination's
    // walk, or the start label's NoMove), then the tail commands of entry e and of its
    // parents up to the source (LaneHub::emit with the commands precomputed in CT)
    __device__ __forceinline__ void emit_ct(const LLab &x, uint32_t e, bool last, const Cmd &wc, uint32_t qi) const {
        const DevParams &p = P;
        OutResult &o = a->out_res[qi];
        OutCmd *oc = a->out_cmd + (unsigned long long)qi * p.max_cmds;
        const uint32_t len = lm_len(x.m);
        const uint32_t legs = Base::metric(x, 0), money = Base::metric(x, 1), time = Base::metric(x, 2);
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
        if (last && at >= 0) oc[at--] = OutCmd{wc.kp, wc.from, wc.to, 0};
        for (uint32_t guard = 0; e != 0 && at >= 0 && guard <= TM; ++guard) {
            const uint4 h = CT[2 * e];
            if (lm_nt(h.x) == 2) {
                const uint4 t2 = CT[2 * e + 1];
                oc[at--] = OutCmd{t2.x, t2.y, t2.z, 0};
            }
            if (at >= 0) oc[at--] = OutCmd{h.y, h.z, h.w, 0};
            e = lm_par(h.x);
        }
        if (at != -1 || e != 0) atomicOr(counter + kCtrFlags, kErrChain);
        o = OutResult{legs, money, time, (status << 16) | (len & 0xFFFFu)};
    }

    __device__ __forceinline__ uint32_t ent(uint32_t i) const { return i * G + gj; }
    // some lane of this lane's group has f
    __device__ __forceinline__ bool group_any(bool f) const {
        const unsigned long long b = __ballot(f);
        return ((b >> gbase) & ((1ull << G) - 1ull)) != 0;
    }
    // the group's flags as entry bits of slot i (bit i * G + j: lane j's flag)
    __device__ __forceinline__ uint32_t group_bits(bool f, uint32_t i) const {
        const unsigned long long b = __ballot(f);
        return uint32_t((b >> gbase) & ((1ull << G) - 1ull)) << (i * G);
    }
    // x and y agree on (c1, c2, c3, length)
    __device__ __forceinline__ static bool eq4(const LLab &x, const LLab &y) {
        return ((x.c1 ^ y.c1) | (x.c2 ^ y.c2) | (x.c3 ^ y.c3) | ((x.m ^ y.m) & 0xFFu)) == 0;
    }
    __device__ __forceinline__ LLab lt_get(uint32_t e) const {
        const uint4 v = LT[e];
        return LLab{v.x, v.y, v.z, v.w};
    }

    // candidates from the settled special into entry e (LaneHub::from_s with the entry's
    // role a run-time bit of the settle's masks): CentralMove, walk, caravan, then SoE or
    // the SoE-region pair, a later one replacing the best only when strictly smaller
    __device__ __forceinline__ FromS from_s_rt(const Settle &z, uint32_t e, const uint4 A, const uint2 B) const {
        FromS f;
        f.won = bitv(z.walk, e);  // (z.walk never has the Center's bit)
        f.w = opt(f.won, add(z.ls, A.x, 0, A.y, z.mW));
        const uint32_t oc = bitv(z.cenm, e);
        f.c = opt(oc, z.cen);
        consider(f.c, f.w);
        f.any = f.won | oc;
        const uint32_t on = bitv(z.car, e);
        consider(f.c, opt(on, add(z.ls, 0, A.z, A.w, z.mCar)));
        f.any |= on;
        const uint32_t so = bitv(z.soe, e), onr = so | bitv(z.reg, e);
        consider(f.c, opt(onr, add(z.ls, B.x, P.soe_cost, B.y, msel(so, z.mSoE, z.mR))));
        f.any |= onr;
        return f;
    }
    // LaneHub::offer for slot i (entry bit eb)
    __device__ __forceinline__ void offer_rt(LLab &T, uint32_t eb, const FromS &f, uint32_t &ties) {
        const uint32_t gt = ltm(T, f.c);
        const uint32_t drop = ltm3(f.c, T);
        uint32_t dummy = 0;
        const uint32_t lt = ltm_take_idx(f.c, T, 0u, dummy);
        tent |= lt & eb;
        const uint32_t wtie = f.won & ~ltm3(T, f.w);
        wt = (wt & ~(drop & eb)) | (wtie & eb);
        ties |= f.any & ~(lt | gt) & eb;
    }

    // The source, its query range, this lane's first destination and its entry of the
    // source's region row: global loads issued before the workgroup's setup, so that their
    // latency hides behind the table copy (the kernel calls this first).
    uint32_t qa = 0, qb = 0, w_first = 0;
    uint2 sr0 = make_uint2(0, 0);
    __device__ __forceinline__ void prefetch(uint32_t s_idx) {
        gj = lane_id() & (G - 1u);
        gbase = lane_id() & ~(G - 1u);
        src = a->src_v[s_idx];
        qa = a->q_begin[s_idx];
        qb = a->q_begin[s_idx + 1];
        w_first = qa + gj < qb ? a->q_dst[qa + gj] : 0u;
        if (gj < a->nreg) sr0 = reinterpret_cast<const uint2 *>(a->near)[(unsigned long long)src * a->nreg + gj];
    }

    // ---- non-linear run times (NL): LaneHub::walk_certain with the group's lanes sharing
    // the boundaries: each lane checks the boundaries among its own slots (their labels in
    // registers), the group combines the clean paths.  Group-uniform: every lane of the
    // group calls it with the same target.
    __device__ __forceinline__ bool cert_group(uint32_t b, int vx, int vy) const {
        int bx, by;
        pos(b, bx, by);
        if ((by == 0 && vy == 0 && bx != 0 && vx != 0 && (bx < 0) != (vx < 0)) ||
            (bx == 0 && vx == 0 && by != 0 && vy != 0 && (by < 0) != (vy < 0)))
            return false;  // shortest walks detour round the Center
        const LLab xb = b == 0 ? start() : lt_get(b);
        uint32_t paths = 3u;
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
            const uint32_t e = ent(i);
            const bool isq = e == 0 ? src != P.vc : (e != 1 && ((bndm >> e) & 1u));  // (the Center starts no walks)
            if (!isq || e == b) continue;
            const LLab xq = e == 0 ? start() : Ls[i];
            if (!Base::near_tie(xq, ex[i], ey[i], xb, bx, by, vx, vy)) continue;
            int lists = 0;  // the order of q's and b's command lists when their lengths tie
            if (e != 0 && b != 0 && lm_len(xq.m) == lm_len(xb.m))
                lists = cmp_list(meta_of(e), e, own_of(e), meta_of(b), b, own_of(b));
            uint32_t clean = 0;
            for (uint32_t xf = 0; xf < 2; ++xf)
                clean |= Base::path_tie(xq, e, ex[i], ey[i], xb, b, bx, by, vx, vy, xf == 0, lists) ? 0u : (1u << xf);
            paths &= clean;
        }
        return !(group_any((paths & 1u) == 0u) && group_any((paths & 2u) == 0u));
    }

    // ---- one source per group; every lane of the group calls it with the same source ---
    // returns the records this lane wrote (lane 0 of the group reports the source's)
    __device__ __forceinline__ uint32_t solve(bool have, uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t NS = p.NS;
        MR_GSTAMP(0);  // (0: kernel start to here: the prefetch and the table copy)
        sx = int(src % p.S) - int(p.H);
        sy = int(src / p.S) - int(p.H);
        cell_word(src, sx, sy, ts, src_rk);
        {  // the source's region row, copied into LDS (the list compares read it)
            const uint2 *rg = reinterpret_cast<const uint2 *>(a->near) + (unsigned long long)src * nreg;
            if (gj < nreg) SR[gj] = sr0;
            for (uint32_t r = gj + G; r < nreg; r += G) SR[r] = rg[r];
            srow = SR;
        }
        const LLab st0 = start();
        {
            const LLab x = inf();
#pragma unroll
            for (uint32_t i = 0; i < E; ++i) LT[ent(i)] = make_uint4(x.c1, x.c2, x.c3, x.m);
        }
        // the source's own edges (LaneHub::solve's first loop, entry per slot)
        const bool walks0 = have && src != p.vc;
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
            const uint32_t e = ent(i);
            const bool valid = have && e >= 1 && e <= NS;
            const SpecialStatic tS = spl[valid ? e : 1u];
            ex[i] = e == 0 ? sx : tS.x;
            ey[i] = e == 0 ? sy : tS.y;
            const uint32_t m0 = vmask(valid && e == ts);
            LLab c = opt(m0, st0);
            uint32_t any = m0;
            const uint32_t k = walk_dist(sx, sy, tS.x, tS.y);
            const uint32_t won = vmask(valid && walks0 && tS.v != src && e != 1);  // no walks into the Center
            const LLab w = opt(won, mk(k, 0, rtime(k), lm_pack(1, 0, 1, kStandard)));
            consider(c, w);
            any |= won;
            {  // [SoE src -> e], or [Std{d} src -> u, SoE u -> e]
                const bool reg = valid && p.use_soe && tS.rid != kNone10;
                const uint32_t ev = reg ? srow[reg ? tS.rid : 0u].x : kNone32;
                const bool on = walks0 && reg && ev != kNone32;
                const uint32_t d = on ? ev : 0u;
                const uint32_t om = vmask(on);
                consider(c, opt(om, mk(d, p.soe_cost, rtime(d),
                                       d == 0 ? lm_pack(1, 0, 1, kSoE) : lm_pack(2, 0, 2, kStandard))));
                any |= om;
            }
            {
                const uint32_t om = vmask(valid && e == p.hq_t);
                consider(c, opt(om, mk(0, p.shq_cost, 0, lm_pack(1, 0, 1, kSHQ))));
                any |= om;
            }
            {
                const uint32_t om = vmask(valid && p.use_sfm && e == 1);
                consider(c, opt(om, mk(0, p.sfm_cost, 0, lm_pack(1, 0, 1, kSFm))));
                any |= om;
            }
            Ls[i] = opt(any, c);
            const uint32_t eb = 1u << e;
            tent |= any & eb;
            wt |= won & ~ltm3(c, w) & eb;
        }
        // ---- Dijkstra over the specials, one settle per group per iteration -----------
        uint32_t *mcol = M + mcolumn;  // this group's column of the meta copy
        MR_GSTAMP(1);  // (1: the source's own edges)
        const uint32_t n_it = (a->dbg_flags & kDbgGroupNoSolve) ? 0u : NS;  // (timing experiments)
        for (uint32_t it = 0; it < n_it; ++it) {
            const uint32_t cand = tent & ~done;  // (this lane's entries only)
            if (!__any(cand != 0)) break;
            // this lane's least candidate
            LLab lx = inf();
            uint32_t sl = 0;
#pragma unroll
            for (uint32_t i = 0; i < E; ++i) {
                const uint32_t cm = bitv(cand, ent(i));
                ltm_take_i(opt(cm, Ls[i]), lx, ent(i), sl);
            }
            // the group's least on (c1, c2, c3, length, entry): every lane gets it.  Exact
            // (metrics, length) ties between entries settle in entry order: which one
            // settles first changes no label (LaneHub::solve, MR_LANE_SETTLE_TIES).
            Settle z;
            z.ls = lx;
            uint32_t k = (lx.m << 24) | sl;
            group_min<G>(z.ls.c1, z.ls.c2, z.ls.c3, z.ls.m, k);
            const uint32_t s = k & 0xFFu;
            MR_GSTAMP(2);  // (2: scan and group minimum)
            // the pair-table words of s into this lane's slots, read before the settle's
            // bookkeeping so that their latency overlaps it
            uint4 pa_[E];
            uint2 pb_[E];
            {
                const uint32_t zs = s != 0 ? s : 1u;
#pragma unroll
                for (uint32_t i = 0; i < E; ++i) {
                    pa_[i] = PA[zs * TM + ent(i)];
                    pb_[i] = PB[zs * TM + ent(i)];
                }
            }
            // the blocker bit of s lives with the lane that owns it
            const bool wts = group_any(s != 0 && (s & (G - 1u)) == gj && ((wt >> s) & 1u));
            settle_ctx(z, s, wts);
            if (s != 0) {  // publish the settled label (the chains and the read-off)
                mcol[s * mstride] = z.ls.m;
                if (gj == 0) LT[s] = make_uint4(z.ls.c1, z.ls.c2, z.ls.c3, z.ls.m);
            }
            MR_GSTAMP(3);  // (3: the settle's bookkeeping and its LDS reads)
            // no candidate out of any group's settle (the last settles): nothing to relax
            if (!__any((z.walk | z.cenm | z.car | z.soe | z.reg) != 0)) continue;
            // relaxations into this lane's slots
            uint32_t ties = 0, fcm[E];
#pragma unroll
            for (uint32_t i = 0; i < E; ++i) {
                const uint32_t e = ent(i);
                const FromS f = from_s_rt(z, e, pa_[i], pb_[i]);
                fcm[i] = f.c.m;
                offer_rt(Ls[i], 1u << e, f, ties);
            }
            // exact (metrics, length) ties with a tentative label: the lists decide (rare)
            if (__any(ties != 0) && !(a->dbg_flags & kDbgGroupNoTies)) {
#pragma unroll
                for (uint32_t i = 0; i < E; ++i) {
                    const uint32_t e = ent(i);
                    if (((ties >> e) & 1u) && cmp_list(fcm[i], kOwn, own_of(e), Ls[i].m, e, own_of(e)) < 0)
                        Ls[i].m = fcm[i];
                }
            }
            MR_GSTAMP(4);
        }
        MR_GSTAMP(4);  // (4: relaxations and their ties, from the last stamp of each iteration)
        if (!have) return 0;
        // ---- the settled entries' tail commands, every lane its own (emit_ct) ------------
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
            const uint32_t e = ent(i);
            if (e >= 1 && e <= NS && ((done >> e) & 1u)) {
                const uint32_t m = Ls[i].m;
                const Own o = own_of(e);
                const Cmd c0 = Base::tail(m, o, 0);
                const Cmd c1 = lm_nt(m) == 2 ? Base::tail(m, o, 1) : Cmd{0, 0, 0};
                CT[2 * e] = make_uint4(m, c0.kp, c0.from, c0.to);
                CT[2 * e + 1] = make_uint4(c1.kp, c1.from, c1.to, 0u);
            }
        }
        // ---- certification: with blockers, every settled walk label must be certain ----
        bool unc = false;
        if (blk != 0) {
#pragma unroll
            for (uint32_t i = 0; i < E; ++i) {
                const uint32_t e = ent(i);
                if (e >= 1 && e <= NS && ((done >> e) & 1u) && !label_avail(Ls[i].m, e)) unc = true;
            }
        }
        // non-linear run times: every settled walk label must also be certain against near
        // ties of the time gap (LaneHub::label_certain, the group's lanes sharing the
        // boundaries; done and bndm are the group's)
        if (NL && !group_any(unc) && !(a->dbg_flags & 4u)) {
            for (uint32_t m = done & ~1u; m; m &= m - 1u) {
                const uint32_t t = uint32_t(__builtin_ctz(m));
                const uint32_t mt = meta_of(t);
                if (lm_kind(mt) != kStandard) continue;
                const uint32_t b = lm_par(mt);
                int vx = spl[t].x, vy = spl[t].y;
                if (lm_nt(mt) != 1) {
                    const uint32_t u = Base::rank_inv[Base::near_of(b, spl[t].rid).y];
                    vx = int(u % p.S) - int(p.H);
                    vy = int(u / p.S) - int(p.H);
                }
                if (!cert_group(b, vx, vy)) {
                    unc = true;
                    break;
                }
            }
        }
        const bool fb_sp = group_any(unc) || a->fb_all || (a->dbg_flags & kDbgGroupNoReadoff);
        MR_GSTAMP(6);  // (6: the tail commands and the certification of settled labels)
        // ---- destinations: each query by the whole group, its record by one lane --------
        // A plain destination's label is the best walk from a boundary (the source's walk
        // included): every lane prices the walks from its own slots, the group minimum
        // picks the boundary (exact ties: the lists decide, below); queries go G at a time,
        // query j's label kept by lane j, then every lane emits its own.
        const bool walk0 = src != p.vc;
        bool uncd = false;
        const uint32_t nq = fb_sp ? 0u : qb - qa;
        for (uint32_t j0 = 0; j0 < nq; j0 += G) {
            W[gj] = j0 == 0 ? w_first : (j0 + gj < nq ? a->q_dst[qa + j0 + gj] : 0u);
            const uint32_t nb = min(G, nq - j0);
            uint32_t rk_ = 0, rw = 0, rbx = 0, rtie = 0;  // this lane's record: kind, destination, boundary, tie
            uint32_t fbx = 0;                              // its final boundary (after the list compares)
            LLab rx = inf();
            for (uint32_t j = 0; j < nb; ++j) {
                const uint32_t w = W[j];
                const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
                uint32_t tw, wr;
                cell_word(w, wx, wy, tw, wr);
                uint32_t kind = 3, bx = 0, tie = 0;
                LLab x = inf();
                if (w == src) {
                    kind = 1;
                } else if (tw != kNone10) {
                    kind = 2;
                    bx = tw;
                } else {
                    // candidates compared on the boundary's own meta (length - 1; the source's walk: 0)
                    LLab lx = inf(), cs[E];
                    uint32_t sl = 0;
#pragma unroll
                    for (uint32_t i = 0; i < E; ++i) {
                        const uint32_t e = ent(i);
                        const bool on = e == 0 ? walk0 : ((bndm >> e) & 1u) != 0;
                        const uint32_t kk = walk_dist(ex[i], ey[i], wx, wy);
                        const LLab b0 = e == 0 ? LLab{0u, 0u, 0u, 0u} : Ls[i];
                        cs[i] = opt(vmask(on), add(b0, kk, 0, rtime(kk), b0.m));
                        ltm_take_i(cs[i], lx, e, sl);
                    }
                    x = lx;
                    uint32_t k = (lx.m << 24) | sl;
                    group_min<G>(x.c1, x.c2, x.c3, x.m, k);
                    bx = k & 0xFFu;
                    // the other boundaries with the winner's metrics and length (entry bits)
#pragma unroll
                    for (uint32_t i = 0; i < E; ++i)
                        tie |= group_bits(ent(i) != bx && cs[i].c1 != kInf1 && eq4(cs[i], x), i);
                    if (x.c1 == kInf1) kind = 0;  // no boundary can walk here: cannot happen on a connected grid
                }
                if (j == gj) {
                    rk_ = kind;
                    rw = w;
                    rbx = bx;
                    rtie = tie;
                    rx = x;
                }
            }
            // every lane its own query's record and commands
            const uint32_t qi = qa + j0 + gj;
            if (gj < nb) {
                const uint32_t w = rw;
                const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
                if (rk_ == 1) {  // the start label: [NoMove src]
                    emit_ct(st0, 0u, true, Cmd{kNoMove << 29, src_rk, src_rk}, qi);
                } else if (rk_ == 2) {
                    emit_ct(lt_get(rbx), rbx, false, Cmd{0, 0, 0}, qi);
                } else if (rk_ == 0) {
                    a->out_res[qi] = OutResult{0, 0, 0, uint32_t(16 + 1) << 16};
                } else {
                    uint32_t tw, wr;
                    cell_word(w, wx, wy, tw, wr);
                    const Own wo{wx, wy, wr, kNone10, 0u};
                    LLab x = rx;
                    uint32_t bx = rbx;
                    x.m = lm_pack(lm_len(x.m) + 1u, bx, 1, kStandard);
                    if (rtie && !(a->dbg_flags & kDbgGroupNoTies)) {  // equal metrics and length: the lists decide
                        for (uint32_t mm = rtie; mm; mm &= mm - 1u) {
                            const uint32_t b = uint32_t(__builtin_ctz(mm));
                            int px, py;
                            pos(b, px, py);
                            const uint32_t kk = walk_dist(px, py, wx, wy);
                            const LLab c = b == 0 ? mk(kk, 0, rtime(kk), lm_pack(1, 0, 1, kStandard)) : walk_to(lt_get(b), b, kk);
                            if (cmp4(c, x) == 0 && cmp_list(c.m, kOwn, wo, x.m, kOwn, wo) < 0) {
                                x = c;
                                bx = b;
                            }
                        }
                    }
                    int px, py;
                    pos(bx, px, py);
                    emit_ct(x, bx, true, Cmd{(kStandard << 29) | walk_dist(px, py, wx, wy), Base::rk(bx), wr}, qi);
                    if (blk != 0 && !avail(bx, px, py, wx, wy)) uncd = true;
                    fbx = bx;
                }
            }
            // non-linear run times: each plain destination's winning walk must be certain,
            // checked by the whole group (the queries' winners come over from their lanes)
            if (NL && !(a->dbg_flags & 8u)) {
                for (uint32_t j = 0; j < nb; ++j) {
                    const uint32_t kj = uint32_t(__shfl(int(rk_), int(gbase + j), 64));
                    const uint32_t bj = uint32_t(__shfl(int(fbx), int(gbase + j), 64));
                    const uint32_t wj = uint32_t(__shfl(int(rw), int(gbase + j), 64));
                    if (kj != 3 || group_any(uncd)) continue;
                    if (!cert_group(bj, int(wj % p.S) - int(p.H), int(wj / p.S) - int(p.H))) uncd = true;
                }
            }
        }
        const bool fallback = fb_sp || group_any(uncd);
        // (an uncertain source goes to hub_kernel when the plan relaunches it, as on the lane kernel)
        if (fallback && gj == 0 && a->relist && !a->fb_all) a->relist[atomicAdd(counter + kCtrRelist, 1u)] = s_idx;
        else if (fallback && gj == 0) push_fallback(a, counter, s_idx, kNone32);
        MR_GSTAMP(5);  // (5: certification and the destinations)
        return (fallback || gj != 0) ? 0u : qb - qa;
    }
};

// LDS: the lane kernels' block (TM = G * E), then per group its meta column (TM words:
// the group shares one, LaneHub::mstride / mcolumn), its settled labels, the source's
// region row, the tail commands and the batch's destinations
__host__ __device__ inline uint32_t group_off_m(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return lane_off_meta(NS, nreg, G * E);
}
__host__ __device__ inline uint32_t group_off_lt(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return align16h(group_off_m(NS, nreg, G, E) + (kBS / G) * G * E * 4u);
}
__host__ __device__ inline uint32_t group_off_sr(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return group_off_lt(NS, nreg, G, E) + (kBS / G) * G * E * 16u;
}
__host__ __device__ inline uint32_t group_off_ct(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return align16h(group_off_sr(NS, nreg, G, E) + (kBS / G) * nreg * 8u);
}
__host__ __device__ inline uint32_t group_off_w(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return group_off_ct(NS, nreg, G, E) + (kBS / G) * G * E * 32u;
}
__host__ __device__ inline uint32_t group_lds_total(uint32_t NS, uint32_t nreg, uint32_t G, uint32_t E) {
    return group_off_w(NS, nreg, G, E) + kBS * 4u;
}

template <uint32_t PERM, uint32_t G, uint32_t E, bool NL = false>
__global__ __launch_bounds__(kBS) void hub_group_kernel(const KArgs *__restrict__ a) {
    constexpr uint32_t TM = G * E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    GroupHub<PERM, G, E, NL> H;
    // group q of wave w: source (64 / G) w + q of the sources [0, n_lane)
    const uint32_t grp = (blockIdx.x * (kBS / 64) + (threadIdx.x >> 6)) * (64u / G) + lane_id() / G;
    const uint32_t n = a->n_lane;
    const bool have = grp < n;
    const uint32_t s_idx = have ? grp : (n ? n - 1 : 0);
    H.a = a;
#ifdef MR_STAMPS
    H.gst_last = __builtin_amdgcn_s_memtime();
#endif
    H.prefetch(s_idx);
    lane_setup<TM>(a, smem, H);
    H.M = reinterpret_cast<uint32_t *>(smem + group_off_m(a->p.NS, a->nreg, G, E)) + (threadIdx.x / G) * TM;
    H.mstride = 1u;  // (one meta column per group)
    H.mcolumn = 0u;
    H.LT = reinterpret_cast<uint4 *>(smem + group_off_lt(a->p.NS, a->nreg, G, E)) + (threadIdx.x / G) * TM;
    H.SR = reinterpret_cast<uint2 *>(smem + group_off_sr(a->p.NS, a->nreg, G, E)) + (threadIdx.x / G) * a->nreg;
    H.CT = reinterpret_cast<uint4 *>(smem + group_off_ct(a->p.NS, a->nreg, G, E)) + (threadIdx.x / G) * (2 * TM);
    H.W = reinterpret_cast<uint32_t *>(smem + group_off_w(a->p.NS, a->nreg, G, E)) + (threadIdx.x / G) * G;
    uint32_t written = 0;
    if (__any(have)) written = H.solve(have, s_idx);
#ifdef MR_STAMPS
    if (a->dbg && lane_id() == 0) {
        unsigned long long *h = a->dbg + (unsigned long long)a->dbg_blocks * 10 + 9;
        atomicAdd(h, 1ull);
        for (int i = 0; i < 6; ++i) atomicAdd(h + 1 + i, H.gst[i]);
        atomicAdd(h - 2, H.gst[6]);  // (the hub words h[7], h[8]: unused by this kernel)
        atomicAdd(h - 1, H.gst[7]);
    }
#endif
    __shared__ uint32_t wsum;
    if (threadIdx.x == 0) wsum = 0;
    __syncthreads();
    if (written) atomicAdd(&wsum, written);
    __syncthreads();
    if (threadIdx.x == 0) finish_launch(a, wsum);
}

}  // namespace mr
