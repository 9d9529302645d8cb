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
// A label is 4 registers: the metrics in comparator order (c1, c2, c3) and a meta word
// (length in byte 0, the first tail command's kind, parent entry, tail count and
// CentralMove count); the command payloads (walk / caravan / SoE-region distances)
// follow from the parent's and the entry's cells, so they are rebuilt where a command
// is written or compared.  The host only gives this kernel plans whose metric sums
// provably stay below 2^32 - 1 (lane_bounds_ok, mr_host.cpp): c1 = 2^32 - 1 marks a
// label that is not there, and no add carries.
//
// The order on (c1, c2, c3, length) is one borrow chain (ltm: byte-0 SDWA subtract,
// three subtract-with-borrow) whose borrow becomes a 0 / ~0 VGPR mask, and every
// selection is a bitwise select on such masks (one v_bitop3 per word): no compare
// result lives in a 64-bit scalar lane mask, so the unrolled loops are pure VALU.
//
// Exactness follows hub_kernel step for step:
//   * candidates into an entry from one settled special s share chain(s), so among
//     them (metrics, length) ties are decided by the last command's kind (the list
//     order; their kinds differ): they are visited in kind order and a later one
//     replaces the best only when strictly smaller; the best is compared with the
//     entry's tentative label, and only an exact (metrics, length) tie there walks the
//     command lists (cmp_list, rare, out of the unrolled code);
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

// waves per SIMD the register budget is cut for: two for the 22-entry table (256
// VGPRs, no spill), one for 24 and 32 entries (256 VGPRs + AGPRs, no scratch)
#ifndef MR_LANE_WAVES
#define MR_LANE_WAVES 2
#endif
__host__ __device__ constexpr uint32_t lane_waves(uint32_t TM) { return TM <= 22 ? MR_LANE_WAVES : 1u; }
// a scheduling fence after every MR_LANE_FENCE_EVERY unrolled entries (0: none), so the
// scheduler does not interleave all of them and run out of registers
#ifndef MR_LANE_FENCE_EVERY
#define MR_LANE_FENCE_EVERY 0  // none: c4 0.975 ms against 1.033 with a fence after every entry (r04 A/B)
#endif
#define MR_LANE_FENCE_AT(t)                                                              \
    do {                                                                                 \
        if (MR_LANE_FENCE_EVERY > 0 && ((t) % (MR_LANE_FENCE_EVERY > 0 ? MR_LANE_FENCE_EVERY : 1)) == 0) \
            __builtin_amdgcn_sched_barrier(0);                                           \
    } while (0)
#define MR_LANE_FENCE() MR_LANE_FENCE_AT(t)

// pair-table reads issued this many entries ahead of their use in the relax loop (round 6:
// 0, in the entry's own step, 0.460 / 0.460 ms at c4 against 0.470 / 0.469 one entry ahead,
// tools/r06/gpu_final_b.sh; round 5 had measured the opposite before the skips)
#ifndef MR_LANE_PF
#define MR_LANE_PF 0
#endif
// relaxations of entries with no candidate in any lane of the wave skipped (1) or run as
// no-ops (0)
#ifndef MR_LANE_SKIP
#define MR_LANE_SKIP 1
#endif
// OR of v over the wave (uniform): four DPP rounds within each row of 16 lanes, then the
// four rows' words by readlane.  Exact only with every lane active (the DPP reads of an
// inactive lane give 0 with bound_ctrl off, and lanes 0/16/32/48 are read whatever EXEC
// says); the relax loop's callers keep EXEC full (MR_LANE_SKIP: lanes without a source run
// the loop to its end), and with EXEC not full the result is ~0 — every entry treated as
// needed, so a skip can only be lost, never taken wrongly
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    const bool full = __builtin_amdgcn_read_exec() == ~0ull;
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xF, 0xF, false));  // row_mirror
    const uint32_t r = uint32_t(__builtin_amdgcn_readlane(int(v), 0) | __builtin_amdgcn_readlane(int(v), 16) |
                                __builtin_amdgcn_readlane(int(v), 32) | __builtin_amdgcn_readlane(int(v), 48));
    return full ? r : ~0u;
}
// meta: length (8 b) | kind of the first tail command (3 b) << 8 | parent entry (5 b)
// << 11 | (tail count - 1) << 16 | CentralMove count (2 b) << 17
__device__ __forceinline__ uint32_t lm_len(uint32_t m) { return m & 0xFFu; }
__device__ __forceinline__ uint32_t lm_kind(uint32_t m) { return (m >> 8) & 7u; }
__device__ __forceinline__ uint32_t lm_par(uint32_t m) { return (m >> 11) & 31u; }
__device__ __forceinline__ uint32_t lm_nt(uint32_t m) { return ((m >> 16) & 1u) + 1u; }
__device__ __forceinline__ uint32_t lm_cj(uint32_t m) { return (m >> 17) & 3u; }
__device__ __host__ __forceinline__ constexpr uint32_t lm_pack(uint32_t len, uint32_t par, uint32_t nt, uint32_t kind,
                                                              uint32_t cj = 0) {
    return len | (kind << 8) | (par << 11) | ((nt - 1u) << 16) | (cj << 17);
}
constexpr uint32_t kInf1 = ~0u;  // c1 of a label that is not there
// the specials' cells by hash (kLaneHash slots of {vertex, entry}, linear probing)
constexpr uint32_t kLaneHash = 64;
__host__ __device__ __forceinline__ uint32_t lane_hash(uint32_t v) { return (v * 0x9E3779B1u) >> 26; }

struct LLab {
    uint32_t c1, c2, c3, m;
};


// ---- masks: 0 / ~0 per lane, kept in VGPRs ---------------------------------------------
// An empty asm makes the value opaque: without it the compiler turns every such mask
// back into a 64-bit scalar lane mask (v_cmp + s_and/s_or), runs out of SGPRs and spills.
__device__ __forceinline__ uint32_t vopaque(uint32_t v) {
    asm("" : "+v"(v));
    return v;
}
// a wave-uniform value re-read where it is used: the uniform branches of the unrolled
// loops test bits of it, and without this the compiler hoists all their conditions out
// of the iteration loop as 64-bit lane masks (SGPR spills)
__device__ __forceinline__ uint32_t sopaque(uint32_t v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ uint32_t vvolatile(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t vmask(bool b) { return vopaque(b ? ~0u : 0u); }
// bit t of w as a mask (t is a constant in the unrolled loops: one v_bfe_i32)
__device__ __forceinline__ uint32_t bitm(uint32_t w, uint32_t t) { return vopaque(uint32_t(int32_t(w << (31u - t)) >> 31)); }
// k ? a : b per bit (one v_bfi_b32; written out, the compiler often makes it and/and/or/not)
__device__ __forceinline__ uint32_t msel(uint32_t k, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(k), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ void ll_sel(uint32_t k, LLab &d, const LLab &c) {
    d.c1 = msel(k, c.c1, d.c1);
    d.c2 = msel(k, c.c2, d.c2);
    d.c3 = msel(k, c.c3, d.c3);
    d.m = msel(k, c.m, d.m);
}
// x < y on (c1, c2, c3, length): the borrow of x - y, from the length byte up
__device__ __forceinline__ uint32_t ltm(const LLab &x, const LLab &y) {
    uint32_t t, r;
    asm("v_sub_co_u32_sdwa %0, vcc, %2, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %4, %5, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %6, %7, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %9, vcc\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, vcc"
        : "=&v"(t), "=v"(r)
        : "v"(x.m), "v"(y.m), "v"(x.c3), "v"(y.c3), "v"(x.c2), "v"(y.c2), "v"(x.c1), "v"(y.c1)
        : "vcc");
    return r;
}
// d = c when c < d on (c1, c2, c3, length): the borrow chain leaves the order in VCC and
// four v_cndmask_b32_e32 select on it directly (4-byte VOP2 selects, no mask register,
// and one asm block instead of six, so no s_nop between them).  The in-out operands are
// early clobbers: a select writes d before the block has read all of c, and an input
// holding the same value as a d word may otherwise share its register.
__device__ __forceinline__ void ltm_take(const LLab &c, LLab &d) {
    uint32_t t;
    asm("v_sub_co_u32_sdwa %0, vcc, %5, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %6, %2, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %7, %3, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %4, vcc\n\t"
        "v_cndmask_b32_e32 %4, %4, %8, vcc\n\t"
        "v_cndmask_b32_e32 %3, %3, %7, vcc\n\t"
        "v_cndmask_b32_e32 %2, %2, %6, vcc\n\t"
        "v_cndmask_b32_e32 %1, %1, %5, vcc"
        : "=&v"(t), "+&v"(d.m), "+&v"(d.c3), "+&v"(d.c2), "+&v"(d.c1)
        : "v"(c.m), "v"(c.c3), "v"(c.c2), "v"(c.c1)
        : "vcc");
}
// the same with an index word riding along (i = ci when c is taken); returns the mask
__device__ __forceinline__ uint32_t ltm_take_idx(const LLab &c, LLab &d, uint32_t ci, uint32_t &i) {
    uint32_t t, k;
    asm("v_sub_co_u32_sdwa %0, vcc, %8, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %9, %4, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %10, %5, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %11, %6, vcc\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, vcc\n\t"
        "v_cndmask_b32_e32 %6, %6, %11, vcc\n\t"
        "v_cndmask_b32_e32 %5, %5, %10, vcc\n\t"
        "v_cndmask_b32_e32 %4, %4, %9, vcc\n\t"
        "v_cndmask_b32_e32 %3, %3, %8, vcc\n\t"
        "v_cndmask_b32_e32 %2, %2, %7, vcc"
        : "=&v"(t), "=&v"(k), "+&v"(i), "+&v"(d.m), "+&v"(d.c3), "+&v"(d.c2), "+&v"(d.c1)
        : "v"(ci), "v"(c.m), "v"(c.c3), "v"(c.c2), "v"(c.c1)
        : "vcc");
    return k;
}
// the same with the mask and no index (offer: the index word was a dummy kept in a register)
__device__ __forceinline__ uint32_t ltm_take_m(const LLab &c, LLab &d) {
    uint32_t t, k;
    asm("v_sub_co_u32_sdwa %0, vcc, %6, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %7, %3, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %4, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %9, %5, vcc\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, vcc\n\t"
        "v_cndmask_b32_e32 %5, %5, %9, vcc\n\t"
        "v_cndmask_b32_e32 %4, %4, %8, vcc\n\t"
        "v_cndmask_b32_e32 %3, %3, %7, vcc\n\t"
        "v_cndmask_b32_e32 %2, %2, %6, vcc"
        : "=&v"(t), "=&v"(k), "+&v"(d.m), "+&v"(d.c3), "+&v"(d.c2), "+&v"(d.c1)
        : "v"(c.m), "v"(c.c3), "v"(c.c2), "v"(c.c1)
        : "vcc");
    return k;
}
// c when c < d on (c1, c2, c3, length), else d, into new registers.  For the first two
// candidates of an entry, whose words are shared across the unrolled entries (the settled
// label's, the meta constants): ltm_take would first copy d (up to four v_mov an entry).
__device__ __forceinline__ LLab ltm_min(const LLab &c, const LLab &d) {
    uint32_t t;
    LLab r;
    asm("v_sub_co_u32_sdwa %0, vcc, %5, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %6, %10, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %7, %11, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %12, vcc\n\t"
        "v_cndmask_b32_e32 %1, %9, %5, vcc\n\t"
        "v_cndmask_b32_e32 %2, %10, %6, vcc\n\t"
        "v_cndmask_b32_e32 %3, %11, %7, vcc\n\t"
        "v_cndmask_b32_e32 %4, %12, %8, vcc"
        : "=&v"(t), "=&v"(r.m), "=&v"(r.c3), "=&v"(r.c2), "=&v"(r.c1)
        : "v"(c.m), "v"(c.c3), "v"(c.c2), "v"(c.c1), "v"(d.m), "v"(d.c3), "v"(d.c2), "v"(d.c1)
        : "vcc");
    return r;
}
// the same without the mask (the scans: only the index is wanted)
__device__ __forceinline__ void ltm_take_i(const LLab &c, LLab &d, uint32_t ci, uint32_t &i) {
    uint32_t t;
    asm("v_sub_co_u32_sdwa %0, vcc, %7, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %3, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %9, %4, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %10, %5, vcc\n\t"
        "v_cndmask_b32_e32 %5, %5, %10, vcc\n\t"
        "v_cndmask_b32_e32 %4, %4, %9, vcc\n\t"
        "v_cndmask_b32_e32 %3, %3, %8, vcc\n\t"
        "v_cndmask_b32_e32 %2, %2, %7, vcc\n\t"
        "v_cndmask_b32_e32 %1, %1, %6, vcc"
        : "=&v"(t), "+&v"(i), "+&v"(d.m), "+&v"(d.c3), "+&v"(d.c2), "+&v"(d.c1)
        : "v"(ci), "v"(c.m), "v"(c.c3), "v"(c.c2), "v"(c.c1)
        : "vcc");
}
// x < y on the metrics (c1, c2, c3) alone
__device__ __forceinline__ uint32_t ltm3(const LLab &x, const LLab &y) {
    uint32_t t, r;
    asm("v_sub_co_u32_e32 %0, vcc, %2, %3\n\t"
        "v_subb_co_u32_e32 %0, vcc, %4, %5, vcc\n\t"
        "v_subb_co_u32_e32 %0, vcc, %6, %7, vcc\n\t"
        "v_cndmask_b32_e64 %1, 0, -1, vcc"
        : "=&v"(t), "=v"(r)
        : "v"(x.c3), "v"(y.c3), "v"(x.c2), "v"(y.c2), "v"(x.c1), "v"(y.c1)
        : "vcc");
    return r;
}

// the pair table of specials (s, t), row s at s * TM: walk legs, walk time, caravan
// money, caravan time (uint4), SoE-region distance from s into t's region and its walk
// time (uint2; 0 where there is none), and per row s the entries t whose SoE-region
// candidate applies (distance known and nonzero)
// diagnostic builds (-DMR_STAMPS): the lane kernel's phase cycles per wave (s_memtime),
// summed like the group kernel's (mr_hub_group.hpp MR_GSTAMP; mr_plan_destroy prints them)
#ifdef MR_STAMPS
#define MR_LSTAMP(i)                                                  \
    do {                                                              \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        lst[i] += now_ - lst_last;                                    \
        lst_last = now_;                                              \
    } while (0)
#else
#define MR_LSTAMP(i) \
    do {             \
    } while (0)
#endif

template <uint32_t PERM, uint32_t TM, bool NL = false>
struct LaneHub {
#ifdef MR_STAMPS
    unsigned long long lst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lst_last = 0;
#endif
    static constexpr uint32_t C1 = PERM / 9, C2 = (PERM / 3) % 3, C3 = PERM % 3;
    const KArgs *__restrict__ a;
    DevParams P;
    const SpecialStatic *spl;  // LDS copy of a->sp
    const uint2 *nearS;        // LDS: region rows of the specials, row t at t * nreg
    const uint4 *PA;           // LDS: pair table, walk / caravan words
    const uint2 *PB;           // LDS: pair table, SoE-region words
    const uint32_t *RM;        // LDS: per row, the entries with a SoE-region candidate
    const uint32_t *rank, *sinfo, *rank_inv;
    const uint2 *cell;  // {sinfo, rank} per cell: the source's and destinations' words in one line
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
    // b + (legs, money, time), with meta word m (a zero delta folds away)
    __device__ __forceinline__ static LLab add(const LLab &b, uint32_t legs, uint32_t money, uint32_t time, uint32_t m) {
        return LLab{b.c1 + pick(C1, legs, money, time), b.c2 + pick(C2, legs, money, time),
                    b.c3 + pick(C3, legs, money, time), m};
    }
    __device__ __forceinline__ static LLab mk(uint32_t legs, uint32_t money, uint32_t time, uint32_t m) {
        return LLab{pick(C1, legs, money, time), pick(C2, legs, money, time), pick(C3, legs, money, time), m};
    }
    __device__ __forceinline__ static uint32_t metric(const LLab &x, uint32_t i) {  // i: 0 legs, 1 money, 2 time
        return i == C1 ? x.c1 : (i == C2 ? x.c2 : x.c3);
    }
    __device__ __forceinline__ static LLab start() { return LLab{0u, 0u, 0u, lm_pack(1, 0, 1, kNoMove)}; }
    __device__ __forceinline__ static LLab inf() { return LLab{kInf1, 0u, 0u, 0u}; }
    __device__ __forceinline__ static LLab opt(uint32_t on, const LLab &c) { return LLab{c.c1 | ~on, c.c2, c.c3, c.m}; }
    // c replaces f when strictly smaller (callers visit candidates in kind order)
#ifdef MR_LANE_CLASSIC
    __device__ __forceinline__ static void consider(LLab &f, const LLab &c) { ll_sel(ltm(c, f), f, c); }
#else
    __device__ __forceinline__ static void consider(LLab &f, const LLab &c) { ltm_take(c, f); }
#endif
    // (c1, c2, c3, length): -1, 0, 1 (rare paths)
    __device__ __forceinline__ static int cmp4(const LLab &x, const LLab &y) {
        if (x.c1 != y.c1) return x.c1 < y.c1 ? -1 : 1;
        if (x.c2 != y.c2) return x.c2 < y.c2 ? -1 : 1;
        if (x.c3 != y.c3) return x.c3 < y.c3 ? -1 : 1;
        const uint32_t lx = lm_len(x.m), ly = lm_len(y.m);
        if (lx != ly) return lx < ly ? -1 : 1;
        return 0;
    }

    // (branchless: row 0 of the LDS copy exists and is read anyway, then the source's
    // values are selected; divergent branches around each LDS read cost more)
    __device__ __forceinline__ uint32_t rk(uint32_t e) const {
        const uint32_t r = spl[e].rk;
        return e == 0 ? src_rk : r;
    }
    __device__ __forceinline__ void pos(uint32_t e, int &x, int &y) const {
        const int rx = spl[e].x, ry = spl[e].y;
        x = e == 0 ? sx : rx;
        y = e == 0 ? sy : ry;
    }
    // region row entry r of entry p's cell (p = 0: the source)
    __device__ __forceinline__ uint2 near_of(uint32_t p, uint32_t r) const { return p == 0 ? srow[r] : nearS[p * nreg + r]; }
    // entry e's label (run-time e; a select per entry: the rare paths only)
    __device__ __forceinline__ LLab get(uint32_t e) const {
        LLab r = start();
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) ll_sel(vmask(e == t), r, L[t]);
        return r;
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
        const uint32_t rid = spl[e].rid;
        return Own{x, y, rk(e), e == 0 ? kNone10 : rid, (c5m >> e) & 1u};
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
    const uint2 *HT;     // LDS: the specials' cells by hash (lane_hash)
    uint32_t ht_probes;  // the longest probe sequence in HT
    __device__ __forceinline__ void dump_meta() const {
        const uint32_t l = lane_id();
        M[mcolumn] = start().m;
        (void)l;
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) M[t * mstride + mcolumn] = L[t].m;
    }
    __device__ __forceinline__ uint32_t meta_of(uint32_t e) const { return M[e * mstride + mcolumn]; }
    // the meta copy's layout: entry t of this lane's column at t * mstride + mcolumn (the
    // lane kernel: a column per lane; the group kernel: one per group)
    uint32_t mstride = 64u, mcolumn = 0u;
    // per wave: each relaxation's best candidate meta into entry t (t * 64 + lane), read
    // by the relaxation ties; M holds the settled entries' metas (written at their settle)
    uint32_t *MC = nullptr;
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

    // The time of a run of k StandardMove legs (AggregatedCost, src/cost.rs:122-124): 180 k
    // s, or with Fleetfoot 1..3 (NL) ceil(180 k num / den) (src/skill.rs:65-71) as a
    // multiply-high by the plan's magic, exact for k <= 2 S + 256 (checked on the host,
    // ff_magic in mr_host.cpp: every walk on the grid is shorter, and path_tie's period
    // check reads f at most 2 den + 1 past a walk's length)
    __device__ __forceinline__ uint32_t rtime(uint32_t k) const {
        if (!NL) return 180u * k;
        return __umulhi(P.ff_c * k + P.ff_den - 1u, P.ff_magic) >> P.ff_shift;
    }
    // the walk of k legs from table entry b (label lb) to a plain cell
    __device__ __forceinline__ LLab walk_to(const LLab &lb, uint32_t b, uint32_t k) const {
        return add(lb, k, 0, rtime(k), lm_pack(lm_len(lb.m) + 1u, b, 1, kStandard));
    }

    // ---- candidates from one settled special s into entry t ------------------------
    // Per-iteration context of the settled special s: its label ls, the meta words of the
    // candidates from it (walk, SoE-region, caravan, SoE: length + 1 resp. + 2, parent
    // s; a NoMove start label is replaced, not extended), the CentralMove candidate, and
    // which entries each candidate kind reaches (bit masks).
    struct Settle {
        LLab ls, cen;
        uint32_t s, mW, mR, mCar, mSoE;
        uint32_t cenm, car, soe, reg, walk;
    };
    struct FromS {
        LLab c, w;         // the best candidate from s; the walk candidate (for the blocker bit)
        uint32_t any, won;  // masks: some candidate applies; the walk applies
    };
    // candidates in command-kind order: CentralMove, walk, caravan, then SoE or the
    // SoE-region pair [Std{d} s -> u, SoE u -> t] (one candidate: the SoE is the d = 0
    // case, s in t's region; the pair is one command longer than the others)
    __device__ __forceinline__ FromS from_s(const Settle &z, uint32_t t, const uint4 A, const uint2 B) const {
        FromS f;
        if (t == 1) {  // no walks into the Center
            f.w = inf();
            f.won = 0;
        } else {
            f.won = bitm(z.walk, t);
            f.w = opt(f.won, add(z.ls, A.x, 0, A.y, z.mW));
        }
        f.c = f.w;
        f.any = f.won;
        // (the first two candidates combine into new registers: ltm_min)
        if (t <= 5) {  // CentralMove: the Center (entry 1) <-> the border-1 cells (entries 2..5)
            const uint32_t on = bitm(z.cenm, t);
            f.c = t != 1 ? ltm_min(f.w, opt(on, z.cen)) : opt(on, z.cen);
            f.any |= on;
        }
        // Which entries are hubs / region campfires is known from the table layout the
        // host guarantees (lane_layout_ok, mr_host.cpp): no hub among the border-1 cells
        // 2..5, region campfires in 6 .. 6 + kLaneRegs - 1.  (Run-time branches per entry
        // instead cost ~80 VGPRs of split live ranges in the unrolled loop.)
        if (t == 1 || t >= 6) {  // caravans between hubs (src/pathfinder.rs:140-160, :251-273)
            const uint32_t on = bitm(z.car, t);
            f.c = ltm_min(opt(on, add(z.ls, 0, A.z, A.w, z.mCar)), f.c);
            f.any |= on;
        }
        if (t >= 6 && t < 6 + kLaneRegs) {  // Scroll of Escape (src/pathfinder.rs:162-170)
            const uint32_t so = bitm(z.soe, t), on = so | bitm(z.reg, t);
            consider(f.c, opt(on, add(z.ls, B.x, P.soe_cost, B.y, msel(so, z.mSoE, z.mR))));
            f.any |= on;
        }
        return f;
    }
    // the best candidate into entry t against its tentative label: a strict win takes,
    // an exact (metrics, length) tie is left to the list compare (bit t of ties)
    __device__ __forceinline__ void offer(uint32_t t, const FromS &f, uint32_t &ties) {
        LLab &T = L[t];
        const uint32_t bit = 1u << t;
        // (an absent candidate, c1 = 2^32 - 1, is below neither a present label nor an
        // absent one: no `& f.any` on lt and drop)
        const uint32_t gt = ltm(T, f.c);
        const uint32_t drop = ltm3(f.c, T);  // the tentative metrics drop
#ifdef MR_LANE_CLASSIC
        const uint32_t lt = ltm(f.c, T);
        ll_sel(lt, T, f.c);
#else
        const uint32_t lt = ltm_take_m(f.c, T);
#endif
        tent |= lt & bit;
        // blocker bit: a walk candidate with the (new) tentative metrics; the walk is >= the
        // new tentative label, so it ties unless the label's metrics are strictly smaller
        const uint32_t wtie = f.won & ~ltm3(T, f.w);
        wt = (wt & ~(drop & bit)) | (wtie & bit);
        ties |= f.any & ~(lt | gt) & bit;
    }

    // Bookkeeping of the settle of entry s (0: none this iteration) with label z.ls: the
    // settled and boundary masks, the blocker bit (wts: some walk candidate had s's
    // metrics) and the per-iteration context of the candidates from s.
    __device__ __forceinline__ void settle_ctx(Settle &z, uint32_t s, bool wts) {
        const DevParams &p = P;
        const bool act = s != 0;
        z.s = act ? s : 1u;
        done |= act ? (1u << s) : 0u;
        const uint32_t lm = z.ls.m, len = lm_len(lm);
        const uint32_t lk = lm_nt(lm) == 2 ? kSoE : lm_kind(lm);
        const bool boundary = act && lk != kNoMove && lk != kStandard;
        blk |= (boundary && wts) ? (1u << s) : 0u;  // a walk tied it: a blocker
        const bool walks = boundary && s != 1;  // the Center starts no walks
        bndm |= walks ? (1u << s) : 0u;
        // the start label (the source's own special; metrics 0): its NoMove is replaced
        const uint32_t bm = lk == kNoMove ? lm_pack(1, 0, 1, 0) : lm_pack(len + 1u, z.s, 1, 0);
        z.mW = lm_pack(len + 1u, z.s, 1, kStandard);
        z.mR = lm_pack(len + 2u, z.s, 2, kStandard);
        z.mCar = bm | (kCaravan << 8);
        z.mSoE = bm | (kSoE << 8);
        // a CentralMove after a CentralMove merges into it
        z.cen = add(z.ls, 0, 0, 10u,
                    lk == kCentral ? lm_pack(len, lm_par(lm), 1, kCentral, lm_cj(lm) + 1u)
                                   : (bm | lm_pack(0, 0, 1, kCentral, 1)));
        const uint32_t live = act ? (validm & ~done) : 0u;  // unsettled entries
        const uint32_t rg = spl[z.s].region, rmr = RM[z.s];  // (both read up front: one LDS round trip)
        z.cenm = live & (z.s == 1 ? 0x3Cu : ((z.s >= 2 && z.s <= 5) ? 0x2u : 0u));
        z.car = (p.use_caravans && ((hubm >> z.s) & 1u)) ? (live & hubm) : 0u;
        z.soe = (p.use_soe && rg != kNone10 && rg != z.s) ? (live & (1u << rg)) : 0u;
        z.reg = (walks && p.use_soe) ? (live & rmr) : 0u;
        z.walk = walks ? (live & ~0x2u) : 0u;
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

    // ---- non-linear run times (NL): hub_kernel's walk certification -----------------
    // near_tie / path_tie / walk_clear of mr_device.hpp (DESIGN.md §3a'') over this lane's
    // table.  The comparator order is a compile-time constant here.
    static constexpr bool kLegsBefore = C1 == 0 || (C2 == 0 && C1 != 2);
    static constexpr bool kMoneyBefore = C1 == 1 || (C2 == 1 && C1 != 2);
    static constexpr uint32_t kAfter = C1 == 2 ? C2 : (C2 == 2 ? C3 : 3u);  // the metric after Time (3: none)
    // the gap f(k + m) - f(k) takes one of {lo, hi} for every k: hi = ceil(180 |m| num / den)
    // (rtime), lo = floor(...); negated and swapped for m < 0
    __device__ __forceinline__ bool gap_hits(int d0, int m) const {
        const uint32_t am = uint32_t(m < 0 ? -m : m);
        const uint32_t h = rtime(am);
        const int hi0 = int(h), lo0 = int(h) - (h * P.ff_den != P.ff_c * am ? 1 : 0);
        const int lo = m < 0 ? -hi0 : lo0, hi = m < 0 ? -lo0 : hi0;
        return d0 + lo == -1 || d0 + lo == 0 || d0 + hi == -1 || d0 + hi == 0;
    }
    // Can boundary q (label xq at qx, qy) beat walk(b, .) non-isotonically somewhere on a
    // shortest b-path to (vx, vy)?  m = d_q(u) - d_b(u) runs within [L1(q, v) - L1(b, v),
    // L1(q, b) + 2] on those paths; the metrics before Time must be able to tie and the
    // time gap d0 + (f(k + m) - f(k)) reach -1 or 0.  A time difference beyond 2^22 s is
    // past any walk's gap (|gap| <= 180 (2 S + 2) + 1 < 2^21), so the rest is 32-bit.
    __device__ __forceinline__ bool near_tie(const LLab &xq, int qx, int qy, const LLab &xb, int bx, int by, int vx,
                                             int vy) const {
        const uint32_t tq = metric(xq, 2), tb = metric(xb, 2);
        if (kMoneyBefore && metric(xq, 1) != metric(xb, 1)) return false;
        if ((tq > tb ? tq - tb : tb - tq) > (1u << 22)) return false;
        const int d0 = int(tq - tb);
        const int mlo = abs(qx - vx) + abs(qy - vy) - abs(bx - vx) - abs(by - vy);
        const int mhi = abs(qx - bx) + abs(qy - by) + 2;
        if (kLegsBefore) {  // the legs tie where m = L_b - L_q
            const int m = int(metric(xb, 0)) - int(metric(xq, 0));
            return m != 0 && m >= mlo && m <= mhi && gap_hits(d0, m);
        }
        // d0 + 180 m num / den within (-2, 1): m next to -d0 den / (180 num).  The quotient
        // of two integers below 2^31 and 2^15 in double precision floors exactly.
        const int m0 = int(floor(double((-2 - d0) * int(P.ff_den)) / double(P.ff_c)));
        bool hit = false;
        for (int m = m0 - 1; m <= m0 + 2; ++m) hit = hit || (m != 0 && m >= mlo && m <= mhi && gap_hits(d0, m));
        return hit;
    }
    // Along one L-shaped shortest path from b to v (x first, or y first), is there a cell u
    // (v excluded) where walk(q, .) beats walk(b, .) and the next leg flips their order?
    // hub_kernel's path_tie step for step, with the periodic skip (tests/test_path_tie_skip.py).
    __device__ __forceinline__ bool path_tie(const LLab &xq, uint32_t q, int qx, int qy, const LLab &xb, uint32_t b, int bx, int by,
                             int vx, int vy, bool x_first, int lists) const {
        const long long tb = metric(xb, 2), tq = metric(xq, 2), lb = metric(xb, 0), lq = metric(xq, 0);
        const long long mb = metric(xb, 1), mq = metric(xq, 1);
        if (kMoneyBefore && mq != mb) return false;
        const int sxd = vx > bx ? 1 : -1, syd = vy > by ? 1 : -1;
        const int K = abs(vx - bx) + abs(vy - by), kx = abs(vx - bx), ky = K - kx;
        // the walks' lengths (the source's walk replaces its NoMove: length 1)
        const long long nq0 = q == 0 ? 1 : lm_len(xq.m), nq1 = q == 0 ? 1 : lm_len(xq.m) + 1;
        const long long nb0 = b == 0 ? 1 : lm_len(xb.m), nb1 = b == 0 ? 1 : lm_len(xb.m) + 1;
        auto cell = [&](int k, int &ux, int &uy) {
            if (x_first) {
                ux = k < kx ? bx + sxd * k : vx;
                uy = k < kx ? by : by + syd * (k - kx);
            } else {
                uy = k < ky ? by + syd * k : vy;
                ux = k < ky ? bx : bx + sxd * (k - ky);
            }
        };
        auto tail = [&](long long dd, long long kk) -> int {  // -1 q ahead, +1 b ahead, 0 the lists
            if (kAfter == 0) {
                if (lq + dd != lb + kk) return lq + dd < lb + kk ? -1 : 1;
            } else if (kAfter == 1) {
                if (mq != mb) return mq < mb ? -1 : 1;
            }
            const long long nq = dd > 0 ? nq1 : nq0, nbb = kk > 0 ? nb1 : nb0;
            if (nq != nbb) return nq < nbb ? -1 : 1;
            return (dd > 0 && kk > 0) ? lists : 0;
        };
        const int den = int(P.ff_den);
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
                const int c0 = ax ? ux : uy, qc = ax ? qx : qy, sd = ax ? sxd : syd;
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
            const bool tie_before = !kLegsBefore || lq + dq == lb + k;
            if (tie_before && dqn > dq) {
                const long long fq = rtime(dq), fb = rtime(uint32_t(k));
                const long long delta = ((long long)rtime(dqn) - fq) - ((long long)rtime(uint32_t(k) + 1) - fb);
                const long long gap = tq + fq - tb - fb;
                if ((gap == -1 || gap == 0) && delta >= 0) {
                    const bool q_beats_u = gap == -1 || tail(dq, k) != 1;
                    const long long gw = gap + delta;
                    const bool b_beats_w = gw > 0 || (gw == 0 && tail(dqn, k + 1) != -1);
                    if (q_beats_u && b_beats_w) return true;
                }
            }
            const bool along_x = x_first ? k < kx : k >= ky;
            const bool plain = k >= 1 && (along_x ? (ux != 0 && wx != 0 && sxd * (ux - qx) >= 0)
                                                  : (uy != 0 && wy != 0 && syd * (uy - qy) >= 0));
            // the next step that is not plain: the segment's end, or the step before the one
            // whose cell lies on the axis being crossed
            int j = along_x ? (x_first ? kx : K) : (x_first ? K : ky);
            {
                const int c0 = along_x ? ux : uy, sd = along_x ? sxd : syd;
                if (c0 * sd < 0) j = min(j, k + abs(c0) - 1);
            }
            // A plain run of at least den steps from here (q off the walk, so the tail is
            // the run's): its steps see every residue of k mod den, and the time gaps at a
            // step and the next are d0 + F(r), d0 + F(r + 1), F(r) = f(r + m) - f(r) with m
            // = dq - k constant on the run.  One period of F decides whether some step of
            // the run flips; the run is then skipped whole (tests/test_path_tie_skip.py).
            if (plain && tie_before && dq > 0 && j - k >= den) {
                const int m = int(dq) - k, T = tail(dq, k);
                const long long d0 = tq - tb;
                const int base = den * ((max(0, -m) + den - 1) / den);  // (r + m >= 0)
                for (int i = 0; i < den; ++i) {
                    const uint32_t r = uint32_t(base + i);
                    const long long g = d0 + (long long)rtime(uint32_t(int(r) + m)) - (long long)rtime(r);
                    const long long gw = d0 + (long long)rtime(uint32_t(int(r) + 1 + m)) - (long long)rtime(r + 1u);
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
    // Is the closed-form walk(b, d_b(v)) (b's label xb) the reference's label of v?  One
    // L-path must be clean for every boundary (hub_kernel's walk_certain / walk_clear).  The
    // near_tie filter runs over the register-held table (static entries); the few
    // boundaries that pass it get the path scans.
    __device__ __forceinline__ bool walk_certain(uint32_t b, const LLab &xb, int vx, int vy) const {
        int bx, by;
        pos(b, bx, by);
        if ((by == 0 && vy == 0 && bx != 0 && vx != 0 && (bx < 0) != (vx < 0)) ||
            (bx == 0 && vx == 0 && by != 0 && vy != 0 && (by < 0) != (vy < 0)))
            return false;  // shortest walks detour round the Center
        uint32_t need = 0;
        if (b != 0 && src != P.vc && near_tie(start(), sx, sy, xb, bx, by, vx, vy)) need = 1u;
#pragma unroll
        for (uint32_t t = 2; t < TM; ++t)  // (entry 1, the Center, starts no walks)
            if (((bndm >> t) & 1u) && t != b && near_tie(L[t], spl[t].x, spl[t].y, xb, bx, by, vx, vy)) need |= 1u << t;
        uint32_t paths = 3u;
        for (uint32_t m = need; m && paths; m &= m - 1u) {
            const uint32_t q = uint32_t(__builtin_ctz(m));
            const LLab xq = get(q);
            int qx, qy;
            pos(q, qx, qy);
            int lists = 0;  // the order of q's and b's command lists when their lengths tie
            if (q != 0 && b != 0 && lm_len(xq.m) == lm_len(xb.m))
                lists = cmp_list(meta_of(q), q, own_of(q), meta_of(b), b, own_of(b));
            uint32_t clean = 0;
            for (uint32_t xf = 0; xf < 2; ++xf)
                clean |= path_tie(xq, q, qx, qy, xb, b, bx, by, vx, vy, xf == 0, lists) ? 0u : (1u << xf);
            paths &= clean;
        }
        return paths != 0;
    }
    // entry t's settled label (meta): its walk, or the walk to the cell its SoE is read from
    __device__ __forceinline__ bool label_certain(uint32_t meta, uint32_t t) const {
        if (lm_kind(meta) != kStandard) return true;
        const uint32_t b = lm_par(meta);
        int vx = spl[t].x, vy = spl[t].y;
        if (lm_nt(meta) != 1) {
            const uint32_t u = rank_inv[near_of(b, spl[t].rid).y];
            vx = int(u % P.S) - int(P.H);
            vy = int(u / P.S) - int(P.H);
        }
        return walk_certain(b, get(b), vx, vy);
    }

    // ---- output (Core::emit) --------------------------------------------------------
    __device__ __forceinline__ void emit(const LLab x, uint32_t xid, const Own xo, uint32_t qi) const {
        const DevParams &p = P;
        OutResult &o = a->out_res[qi];
        OutCmd *oc = a->out_cmd + (unsigned long long)qi * p.max_cmds;
        const uint32_t len = lm_len(x.m);
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
        uint32_t e = x.m;
        // the current label's own cell, as scalars (an Own copied along the loop went to
        // scratch memory)
        int ox = xo.x, oy = xo.y;
        uint32_t ork = xo.rk, orid = xo.rid, oc5 = xo.c5;
        uint32_t eid = xid;
        for (uint32_t guard = 0; at >= 0 && guard <= TM + 1; ++guard) {
            const Own eo{ox, oy, ork, orid, oc5};
            if (lm_nt(e) == 2 && at >= 0) {
                const Cmd c = tail(e, eo, 1);
                oc[at--] = OutCmd{c.kp, c.from, c.to, 0};
            }
            if (at >= 0) {
                const Cmd c = tail(e, eo, 0);
                oc[at--] = OutCmd{c.kp, c.from, c.to, 0};
            }
            eid = lm_par(e);
            if (eid == 0) break;
            e = meta_of(eid);
            const Own n = own_of(eid);
            ox = n.x;
            oy = n.y;
            ork = n.rk;
            orid = n.rid;
            oc5 = n.c5;
        }
        if (at != -1 || eid != 0) atomicOr(counter + kCtrFlags, kErrChain);
        o = OutResult{legs, money, time, (status << 16) | (len & 0xFFFFu)};
    }

    // A cell's special entry (kNone10: plain) and CellIndex rank.  On a grid in the
    // standard layout (mr_grid rank_std: every cell's rank is the closed form of its
    // position) the rank is arithmetic and the entry a scan of the specials' cells in
    // LDS, so a source or destination costs no random HBM line; else the grid's
    // {sinfo, rank} record.
    __device__ __forceinline__ void cell_word(uint32_t v, int x, int y, uint32_t &t, uint32_t &r) const {
        if (a->rank_std) {
            r = std_rank(x, y, P.H);
            t = kNone10;
            const uint32_t h = lane_hash(v);
            for (uint32_t k = 0; k < ht_probes; ++k) {  // (uniform bound)
                const uint2 e = HT[(h + k) & (kLaneHash - 1u)];
                t = e.x == v ? e.y : t;
            }
        } else {
            const uint2 c = cell[v];  // {sinfo, rank}
            t = c.x & kNone10;
            r = c.y;
        }
    }

    // ---- one source per lane ----------------------------------------------------------
    // returns the records this lane wrote (0 when the source went to the SSSP kernel)
    __device__ __forceinline__ uint32_t solve(bool have, uint32_t s_idx) {
        const DevParams &p = P;
        const uint32_t NS = p.NS;
        src = a->src_v[s_idx];
        sx = int(src % p.S) - int(p.H);
        sy = int(src / p.S) - int(p.H);
        cell_word(src, sx, sy, ts, src_rk);
        srow = reinterpret_cast<const uint2 *>(a->near) + (unsigned long long)src * nreg;
        // the source's own edges, in command-kind order: its start label if it is a
        // special, the walks from it, the SoE edges from its region rows, SHQ, SFm
        // (src/pathfinder.rs:162-178)
        const bool walks0 = have && src != p.vc;
        const LLab st0 = start();
        // The source's region row (at most kLaneRegs regions on this kernel's layout,
        // lane_layout_ok), loaded at once.  Read per entry below, each load sat in its own
        // branch and was waited for: a row of dependent round trips to memory per source.
        // (A lane without a source has s_idx of a real one: its row is readable.)
        uint32_t rowx[kLaneRegs];
        {
            const uint32_t nr = min(nreg, kLaneRegs);
#pragma unroll
            for (uint32_t r = 0; r < kLaneRegs; ++r) rowx[r] = r < nr ? srow[r].x : kNone32;
        }
#pragma unroll
        for (uint32_t t = 1; t < TM; ++t) {
            const bool valid = have && t <= NS;
            const SpecialStatic tS = spl[t <= NS ? t : 1u];
            const uint32_t m0 = vmask(valid && t == ts);
            LLab c = opt(m0, st0);
            uint32_t any = m0, won = 0;
            LLab w = inf();
            if (t != 1) {
                const uint32_t k = walk_dist(sx, sy, tS.x, tS.y);
                won = vmask(valid && walks0 && tS.v != src);
                w = opt(won, mk(k, 0, rtime(k), lm_pack(1, 0, 1, kStandard)));
                consider(c, w);
                any |= won;
            }
            {  // [SoE src -> t], or [Std{d} src -> u, SoE u -> t]
                const bool reg = valid && p.use_soe && tS.rid != kNone10;
                // (tS is a static record: the same in every lane)
                const uint32_t rid = __builtin_amdgcn_readfirstlane(tS.rid);
                uint32_t ev = kNone32;
#pragma unroll
                for (uint32_t r = 0; r < kLaneRegs; ++r) ev = rid == r ? rowx[r] : ev;
                const uint32_t e = reg ? ev : kNone32;
                const bool on = walks0 && reg && e != kNone32;
                const uint32_t d = on ? e : 0u;
                const uint32_t om = vmask(on);
                consider(c, opt(om, mk(d, p.soe_cost, rtime(d),
                                       d == 0 ? lm_pack(1, 0, 1, kSoE) : lm_pack(2, 0, 2, kStandard))));
                any |= om;
            }
            {
                const uint32_t om = vmask(valid && t == p.hq_t);
                consider(c, opt(om, mk(0, p.shq_cost, 0, lm_pack(1, 0, 1, kSHQ))));
                any |= om;
            }
            {
                const uint32_t om = vmask(valid && p.use_sfm && t == 1);
                consider(c, opt(om, mk(0, p.sfm_cost, 0, lm_pack(1, 0, 1, kSFm))));
                any |= om;
            }
            L[t] = opt(any, c);
            tent |= any & (1u << t);
            wt |= won & ~ltm3(c, w) & (1u << t);
            MR_LANE_FENCE();
        }
        MR_LSTAMP(1);  // (1: the source's own edges)
        // ---- Dijkstra over the specials, one settle per lane per iteration ----------
        for (uint32_t it = 0; it < NS; ++it) {
            const uint32_t cand = tent & ~done;
            if (!__any(cand != 0)) break;
#if MR_LANE_SKIP
            const uint32_t cand_w = wave_or_u32(cand);  // (entries no lane can settle: skipped)
#endif
            // the settle candidate: least (c1, c2, c3, length), two interleaved chains
            // (odd and even entries) for the latency, then merged; ta / tb: the chain's
            // best has an exact tie (MR_LANE_SETTLE_TIES only)
            LLab la = inf(), lb = inf();
            uint32_t sa = 0, sb = 0, ta = 0, tb = 0;
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
#if MR_LANE_SKIP
                if (!((cand_w >> t) & 1u)) continue;
#endif
                LLab &lx = (t & 1u) ? la : lb;
                uint32_t &sx_ = (t & 1u) ? sa : sb;
                uint32_t &tx = (t & 1u) ? ta : tb;
                const uint32_t cm = bitm(cand, t);
                const LLab c = opt(cm, L[t]);
#ifdef MR_LANE_SETTLE_TIES
                const uint32_t gt = ltm(lx, c);
                const uint32_t lt = ltm_take_idx(c, lx, t, sx_);
                tx = ~lt & (tx | (cm & ~gt));
#else
                (void)tx;
                ltm_take_i(c, lx, t, sx_);
#endif
                MR_LANE_FENCE();
            }
            MR_LSTAMP(2);  // (2: the settle scan)
            Settle z;
            z.ls = la;
            uint32_t s, tie = 0;
            {
                const uint32_t lt = ltm(lb, la);
                ll_sel(lt, z.ls, lb);
                s = msel(lt, sb, sa);
#ifdef MR_LANE_SETTLE_TIES
                const uint32_t gt = ltm(la, lb);
                tie = msel(lt, tb, ta | (vmask(sb != 0) & ~gt));
#endif
            }
            // Exact (metrics, length) ties between two entries need no list compare here:
            // whichever settles first, both labels and every relaxation come out the same
            // (a candidate from one tied entry into the other is one command longer, and
            // candidates into a third entry that tie are ordered by their lists in offer).
            // MR_LANE_SETTLE_TIES keeps the reference's pop order (tests: equal results).
            if (__any(tie != 0)) {  // exact (metrics, length) ties: the command lists decide (rare)
                uint32_t tied = 0;  // the entries with the winner's metrics and length
#pragma unroll
                for (uint32_t t = 1; t < TM; ++t)
                    tied |= bitm(cand, t) & ~(ltm(L[t], z.ls) | ltm(z.ls, L[t])) & (1u << t);
                dump_meta();
                if (tie) {
                    for (uint32_t m = tied & ~(1u << s); m; m &= m - 1u) {
                        const uint32_t t = uint32_t(__builtin_ctz(m));
                        const uint32_t mt = meta_of(t);
                        if (cmp_list(mt, t, own_of(t), z.ls.m, s, own_of(s)) < 0) {
                            z.ls.m = mt;  // (same metrics and length)
                            s = t;
                        }
                    }
                }
            }
            settle_ctx(z, s, ((wt >> s) & 1u) != 0);
            if (s != 0) M[s * mstride + mcolumn] = z.ls.m;  // (the settled meta, for the chains)
            MR_LSTAMP(3);  // (3: the settle's ties and bookkeeping)
            // no candidate out of any lane's settle (the last settles): nothing to relax
            if (!__any((z.walk | z.cenm | z.car | z.soe | z.reg) != 0)) continue;
#if MR_LANE_SKIP
            // the entries some lane of the wave has a candidate into (a wave-uniform mask):
            // the others' relaxations are no-ops in every lane and are skipped
            const uint32_t live_w = wave_or_u32(z.walk | z.cenm | z.car | z.soe | z.reg);
#endif
            const uint4 *rowa = PA + z.s * TM;
            const uint2 *rowb = PB + z.s * TM;
            // Each step also stores into the per-wave LDS copy MC the meta of this
            // iteration's best candidate, which the tie path below reads instead of
            // rebuilding the candidate.
            // The pair-table words of entry t are read MR_LANE_PF entries ahead: the fences
            // keep each entry's code in place, so a read issued in its own entry left the
            // wave parked on it (SQ: ~31 % of the kernel's wave cycles waiting).
            uint32_t ties = 0;
            uint32_t *ml = MC + lane_id();
            uint4 pa[MR_LANE_PF + 1];
            uint2 pb[MR_LANE_PF + 1];
#pragma unroll
            for (uint32_t j = 0; j < MR_LANE_PF; ++j) {
                if (1 + j < TM) pa[j] = rowa[1 + j];
                if (1 + j >= 6 && 1 + j < 6 + kLaneRegs && 1 + j < TM) pb[j] = rowb[1 + j];
            }
#pragma unroll
            for (uint32_t t = 1; t < TM; ++t) {
                constexpr uint32_t R = MR_LANE_PF + 1;
                const uint32_t ahead = t + MR_LANE_PF;
                if (ahead < TM) {
                    pa[(ahead - 1) % R] = rowa[ahead];
                    if (ahead >= 6 && ahead < 6 + kLaneRegs) pb[(ahead - 1) % R] = rowb[ahead];
                }
#if MR_LANE_SKIP
                if (!((live_w >> t) & 1u)) continue;
#endif
                const uint2 B = (t >= 6 && t < 6 + kLaneRegs) ? pb[(t - 1) % R] : make_uint2(0, 0);
                const FromS f = from_s(z, t, pa[(t - 1) % R], B);
                offer(t, f, ties);
                ml[t * 64u] = f.c.m;
                MR_LANE_FENCE();
            }
            // exact (metrics, length) ties with a tentative label: the command lists decide
            // (rare; run-time t; only the meta word can change)
            if (__any(ties != 0)) {
                uint32_t repl = 0;
                for (; ties; ties &= ties - 1u) {
                    const uint32_t t = uint32_t(__builtin_ctz(ties));
                    uint32_t cur = 0;  // entry t's meta
#pragma unroll
                    for (uint32_t e = 1; e < TM; ++e) cur = msel(vmask(e == t), L[e].m, cur);
                    if (cmp_list(ml[t * 64u], kOwn, own_of(t), cur, t, own_of(t)) < 0) repl |= 1u << t;
                }
#pragma unroll
                for (uint32_t t = 1; t < TM; ++t) L[t].m = msel(bitm(repl, t), ml[t * 64u], L[t].m);
            }
            MR_LSTAMP(4);  // (4: the relaxations and their ties)
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
        // non-linear run times: every settled walk label must also be certain against
        // near ties of the time gap (hub_kernel's label_certain)
        if (NL && !unc && !(a->dbg_flags & 4u)) {
            for (uint32_t m = done; m && !unc; m &= m - 1u) {
                const uint32_t t = uint32_t(__builtin_ctz(m));
                if (!label_certain(meta_of(t), t)) unc = true;
            }
        }
        MR_LSTAMP(6);  // (6: the certification of settled labels)
        const uint32_t qa = a->q_begin[s_idx], qb = a->q_begin[s_idx + 1];
        const bool fb_sp = unc || a->fb_all;
        // ---- destinations: the source, a special's own label, or the best walk ------------
        const bool walk0 = src != p.vc;
        for (uint32_t qi = fb_sp ? qb : qa; qi < qb; ++qi) {
            const uint32_t w = a->q_dst[qi];
            const int wx = int(w % p.S) - int(p.H), wy = int(w / p.S) - int(p.H);
            uint32_t tw, wr;
            cell_word(w, wx, wy, tw, wr);
            if (w == src) {
                emit(st0, kOwn, Own{sx, sy, src_rk, kNone10, 0u}, qi);
                continue;
            }
            if (tw != kNone10) {
                emit(get(tw), tw, own_of(tw), qi);
                continue;
            }
            const Own wo{wx, wy, wr, kNone10, 0u};
            // Every candidate is a boundary's label plus one walk command, so they are
            // compared on the boundary's own meta word (length - 1; the source's walk:
            // 0) and the walk's meta is built for the winner.  The clobber and the
            // volatile copy of bndm keep the per-entry terms inside the query loop
            // (hoisted out of it they would hold ~170 VGPRs for the whole kernel).
            asm volatile("" ::: "memory");
            const uint32_t bq = vvolatile(bndm);
            LLab x = inf();
            uint32_t bx = walk0 ? 0u : kNone32;
            uint32_t tie = 0;  // the boundaries whose walk ties the best so far exactly (entry bits)
            {
                const uint32_t k = walk_dist(sx, sy, wx, wy);
                ll_sel(vmask(walk0), x, mk(k, 0, rtime(k), 0u));
            }
#pragma unroll
            for (uint32_t t = 2; t < TM; ++t) {
                const uint32_t k = walk_dist(spl[t].x, spl[t].y, wx, wy);
                const uint32_t cm = bitm(bq, t);
                const LLab c = opt(cm, add(L[t], k, 0, rtime(k), L[t].m));
#ifdef MR_LANE_CLASSIC
                const uint32_t lt = ltm(c, x), gt = ltm(x, c);
                tie = ~lt & (tie | (cm & ~gt & (1u << t)));
                ll_sel(lt, x, c);
                bx = msel(lt, t, bx);
#else
                const uint32_t gt = ltm(x, c);
                const uint32_t lt = ltm_take_idx(c, x, t, bx);
                tie = ~lt & (tie | (cm & ~gt & (1u << t)));
#endif
                MR_LANE_FENCE();
            }
            x.m = lm_pack(lm_len(x.m) + 1u, bx == kNone32 ? 0u : bx, 1, kStandard);
            // Equal metrics and length from several boundaries: the lists decide, among the
            // boundaries that tied the final best only (a strictly better walk cleared the
            // set; the source's walk, visited first, is never taken on a tie)
            if (tie) {
                for (uint32_t m = tie; m; m &= m - 1u) {
                    const uint32_t b = uint32_t(__builtin_ctz(m));
                    int px, py;
                    pos(b, px, py);
                    const uint32_t k = walk_dist(px, py, wx, wy);
                    const LLab c = b == 0 ? mk(k, 0, rtime(k), lm_pack(1, 0, 1, kStandard)) : walk_to(get(b), b, k);
                    if (cmp4(c, x) == 0 && cmp_list(c.m, kOwn, wo, x.m, kOwn, wo) < 0) {
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
            if (NL && !unc && !(a->dbg_flags & 8u) && !walk_certain(bx, get(bx), wx, wy)) unc = true;
        }
        const bool fallback = fb_sp || unc;
        // an uncertain source goes to hub_kernel when the plan relaunches it for such
        // sources (its fallback reaches the certificate), else to the SSSP kernel
        if (fallback && a->relist && !a->fb_all) a->relist[atomicAdd(counter + kCtrRelist, 1u)] = s_idx;
        else if (fallback) push_fallback(a, counter, s_idx, kNone32);
        return fallback ? 0u : qb - qa;
    }
};

// The lane kernels' LDS.  Its first part is a per-plan block the host builds once
// (lane_blob, mr_host.cpp) and every workgroup copies in one pass: the specials' static
// records, their region rows, the pair table (TM x TM uint4 + uint2), its row masks (TM
// words), the specials' cells by hash (kLaneHash slots) and a header {longest probe
// sequence, hub mask, cost-5 mask, region mask}.  Then per wave the meta copy of the
// rare paths (TM x 64 words).
__host__ __device__ inline uint32_t lane_off_near(uint32_t NS) { return align16h((NS + 1) * uint32_t(sizeof(SpecialStatic))); }
__host__ __device__ inline uint32_t lane_off_pt(uint32_t NS, uint32_t nreg) {
    return align16h(lane_off_near(NS) + (NS + 1) * nreg * 8u);
}
__host__ __device__ inline uint32_t lane_off_pb(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_pt(NS, nreg) + TM * TM * 16u;
}
__host__ __device__ inline uint32_t lane_off_rm(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_pb(NS, nreg, TM) + TM * TM * 8u;
}
__host__ __device__ inline uint32_t lane_off_hash(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return align16h(lane_off_rm(NS, nreg, TM) + TM * 4u);
}
__host__ __device__ inline uint32_t lane_off_hdr(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_hash(NS, nreg, TM) + kLaneHash * 8u;
}
// the host-built block (a multiple of 16 bytes)
__host__ __device__ inline uint32_t lane_blob_bytes(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_hdr(NS, nreg, TM) + 16u;
}
__host__ __device__ inline uint32_t lane_off_meta(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_blob_bytes(NS, nreg, TM);
}
__host__ __device__ inline uint32_t lane_lds_total(uint32_t NS, uint32_t nreg, uint32_t TM) {
    return lane_off_meta(NS, nreg, TM) + (kBS / 64) * TM * 64u * 4u;
}

// The lane kernels' workgroup setup: the plan's block copied into LDS (16 B a thread per
// step; the same block for every workgroup, so after the first ones it comes from L2),
// and the solver's fields.
template <uint32_t TM, class Hub>
__device__ __forceinline__ void lane_setup(const KArgs *__restrict__ a, char *smem, Hub &H) {
    const uint32_t NS = a->p.NS, nreg = a->nreg;
    {
        const uint4 *blob = a->lane_blob;
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        const uint32_t n16 = lane_blob_bytes(NS, nreg, TM) / 16u;
        for (uint32_t i = threadIdx.x; i < n16; i += kBS) dst[i] = blob[i];
    }
    __syncthreads();
    H.a = a;
    H.P = a->p;
    H.spl = reinterpret_cast<const SpecialStatic *>(smem);
    H.nearS = reinterpret_cast<const uint2 *>(smem + lane_off_near(NS));
    H.PA = reinterpret_cast<const uint4 *>(smem + lane_off_pt(NS, nreg));
    H.PB = reinterpret_cast<const uint2 *>(smem + lane_off_pb(NS, nreg, TM));
    H.RM = reinterpret_cast<const uint32_t *>(smem + lane_off_rm(NS, nreg, TM));
    H.M = reinterpret_cast<uint32_t *>(smem + lane_off_meta(NS, nreg, TM)) + (threadIdx.x >> 6) * (TM * 64u);
    H.mstride = 64u;
    H.mcolumn = lane_id();
    H.HT = reinterpret_cast<const uint2 *>(smem + lane_off_hash(NS, nreg, TM));
    const uint4 hdr = *reinterpret_cast<const uint4 *>(smem + lane_off_hdr(NS, nreg, TM));
    H.ht_probes = __builtin_amdgcn_readfirstlane(hdr.x);
    H.hubm = __builtin_amdgcn_readfirstlane(hdr.y);
    H.c5m = __builtin_amdgcn_readfirstlane(hdr.z);
    H.regm = __builtin_amdgcn_readfirstlane(hdr.w);
    H.validm = __builtin_amdgcn_readfirstlane(((2u << min(NS, TM - 1u)) - 1u) & ~1u);
    H.rank = a->rank;
    H.sinfo = a->sinfo;
    H.rank_inv = a->rank_inv;
    H.cell = a->cell;
    H.counter = a->counter;
    H.nreg = nreg;
}

// NL: Fleetfoot 1..3 (non-linear run times, the walk certification above)
template <uint32_t PERM, uint32_t TM, bool NL = false>
__global__ __launch_bounds__(kBS, lane_waves(TM)) void hub_lane_kernel(const KArgs *__restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LaneHub<PERM, TM, NL> H;
#ifdef MR_STAMPS
    H.lst_last = __builtin_amdgcn_s_memtime();
#endif
    lane_setup<TM>(a, smem, H);
    H.MC = reinterpret_cast<uint32_t *>(smem + lane_lds_total(a->p.NS, a->nreg, TM)) + (threadIdx.x >> 6) * (TM * 64u);
#ifdef MR_STAMPS
    {
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();
        H.lst[0] += now_ - H.lst_last;  // (0: the table copy)
        H.lst_last = now_;
    }
#endif
    // lane l of wave w: source 64 w + l of the lane kernel's sources [0, n_lane)
    const uint32_t s_idx = (blockIdx.x * (kBS / 64) + (threadIdx.x >> 6)) * 64u + lane_id();
    const uint32_t n = a->n_lane;
    const bool have = s_idx < n;
    uint32_t written = 0;
    if (__any(have)) written = H.solve(have, have ? s_idx : (n ? n - 1 : 0));
#ifdef MR_STAMPS
    {
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();
        H.lst[5] += now_ - H.lst_last;  // (5: the destinations, from the certification's end)
        if (a->dbg && lane_id() == 0) {
            unsigned long long *h = a->dbg + (unsigned long long)a->dbg_blocks * 10 + 9;
            atomicAdd(h, 1ull);
            for (int i = 0; i < 6; ++i) atomicAdd(h + 1 + i, H.lst[i]);
            atomicAdd(h - 2, H.lst[6]);
        }
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
