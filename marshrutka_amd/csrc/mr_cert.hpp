// mr_cert.hpp — certified fallback: the fixed-point check and the
// sorted repair sweep over a certificate slot's cell words.
//
// A hub source whose closed form the hub kernel cannot certify (hub_kernel, query mode)
// exports its label table into a slot; the fill writes every cell's closed-form word
// (the best geodesic walk over its boundaries, any run time).  Call that assignment C.
// The reference's labels L are the unique fixed point of L(v) = min over in-edges
// extend(L(u), u -> v) with L(src) = start (every edge raises (metrics, length), so a
// least discrepancy cannot exist).  The check tests, at every cell v,
//   pull: C(v) is the extension of some in-neighbour's C (or a special's own label that
//         the hub's exact Dijkstra over the specials built from another special), and
//   push: no in-neighbour's extension is smaller than C(v),
// and the slot's key is the least leading metric c1 of min(C(v), best extension) over
// the cells that fail.  Induction on the least discrepancy w (by min(C(w), L(w))) shows
// that every label with c1 below the key is the reference's: a discrepancy there
// fails one of the two tests at w with a smaller key.  The in-edges of a plain cell are
// the StandardMoves from its grid neighbours; those of a special also come from other
// specials (built by the hub's Dijkstra, so pull and push hold by construction) and from
// scrolls (SoE from a region, SHQ, SFm: the least extension is the region's least C, or
// the source's, which the hub's candidates are).
//
// Where the closed form is wrong (Fleetfoot 1-2: the ceil makes two boundaries' time
// gap alternate by a second, so the winner alternates cell by cell in a band, and the
// reference settles the band in label order), the sweep recomputes the failing cells'
// bounding box (plus a margin) in one pass in order of their leading metric, in
// buckets of the least StandardMove increment (cells of one bucket cannot extend one
// another): each cell from its neighbours' current words.  The check then runs again.
#pragma once
#include "mr_device.hpp"

namespace mr {

// per table entry of a slot (LDS): metrics, length, boundary rank (kNone32: not a
// boundary), and for a walk label its boundary and run length
struct CertEntry {
    uint32_t m0, m1, m2, len, lex, wb, wk, par;  // par: the label's parent entry
    uint32_t sb, sk, su, fl;  // a Scroll-of-Escape-region label: its walk (b, k) and the cell (rank) it ends at;
                              // fl: kCertF* flags of the entry
    uint32_t v;               // the entry's cell (entries >= 1)
    int32_t x, y;             // its position
    uint32_t reg;             // its region's campfire (table index; kNone10: none)
};
// CertEntry::fl: the Center or a border-1 cell (never demoted: CentralMoves merge), a
// caravan hub, the HQ, a caravan into it costs 5 a unit, the label is the start label
constexpr uint32_t kCertFCentral = 1u, kCertFHub = 2u, kCertFHQ = 4u, kCertFCoef5 = 8u, kCertFStart = 16u;
// a walk label (b, k) as comparator keys: c1..c3 in comparator order, length, rank of b
struct CertLab {
    uint32_t c1, c2, c3, len, lex, b, k;
};
constexpr uint32_t kCertNoB = 0xFFFFu;

__device__ __forceinline__ bool cert_less(const CertLab &x, const CertLab &y) {
    if (x.c1 != y.c1) return x.c1 < y.c1;
    if (x.c2 != y.c2) return x.c2 < y.c2;
    if (x.c3 != y.c3) return x.c3 < y.c3;
    if (x.len != y.len) return x.len < y.len;
    return x.lex < y.lex;
}
__device__ __forceinline__ bool cert_same(const CertLab &x, const CertLab &y) {
    return x.c1 == y.c1 && x.c2 == y.c2 && x.c3 == y.c3 && x.len == y.len && x.lex == y.lex;
}
__device__ __forceinline__ uint32_t pick(const DevParams &p, int i, uint32_t m0, uint32_t m1, uint32_t m2) {
    const uint32_t q = p.perm[i];
    return q == 0 ? m0 : (q == 1 ? m1 : m2);
}
// walk(b, k): b's label + k legs, its money, the run's time (from the table FT of nft
// run times when given); the list is b's + one command
__device__ __forceinline__ CertLab cert_walk(const DevParams &p, const CertEntry *E, uint32_t b, uint32_t k,
                                             const uint32_t *FT = nullptr, uint32_t nft = 0) {
    const CertEntry &e = E[b];
    const uint32_t m0 = e.m0 + k, m1 = e.m1, m2 = e.m2 + (k < nft ? FT[k] : run_time_ff(k, p.ff_num, p.ff_den));
    return CertLab{pick(p, 0, m0, m1, m2), pick(p, 1, m0, m1, m2), pick(p, 2, m0, m1, m2), b == 0 ? 1u : e.len + 1u,
                   e.lex, b, k};
}
// the extension by one StandardMove of the label in cell word w (false: not a walk source)
__device__ __forceinline__ bool cert_ext(const DevParams &p, const CertEntry *E, uint32_t w, CertLab &x,
                                         const uint32_t *FT = nullptr, uint32_t nft = 0) {
    if (w == kViaSource) {
        x = cert_walk(p, E, 0, 1, FT, nft);
        return true;
    }
    if (w & kViaSpecial) {
        const uint32_t t = w & kNone10;
        if (E[t].wb != kCertNoB) {  // a walk: the run merges
            x = cert_walk(p, E, E[t].wb, E[t].wk + 1, FT, nft);
            return true;
        }
        if (E[t].lex == kNone32) return false;
        x = cert_walk(p, E, t, 1, FT, nft);
        return true;
    }
    x = cert_walk(p, E, (w >> kStBShift) & kNone10, (w & kStKMask) + 1, FT, nft);
    return true;
}
// a slot's table into LDS (every thread of the block takes part)
__device__ __forceinline__ void cert_load_table(const KArgs *__restrict__ a, uint32_t slot, CertEntry *E) {
    const uint32_t T = a->p.NS + 1;
    for (uint32_t t = threadIdx.x; t < T; t += blockDim.x) {
        const Rec r = a->cert_tab[(unsigned long long)slot * T + t];
        const bool walk = r.ntail() == 1 && (r.kp0 >> 29) == kStandard && t != 0;
        const bool soe = r.ntail() == 2 && (r.kp0 >> 29) == kStandard && t != 0;  // walk, then SoE from its end
        const SpecialStatic ss = a->sp[t != 0 ? t : 1u];
        const uint32_t fl = (t != 0 && (ss.flags & (kSpCenter | kSpBorder1)) ? kCertFCentral : 0u) |
                            (t != 0 && (ss.flags & kSpHub) ? kCertFHub : 0u) |
                            (t != 0 && t == a->p.hq_t ? kCertFHQ : 0u) | (t != 0 && ss.coef5 ? kCertFCoef5 : 0u) |
                            ((r.kp0 >> 29) == kNoMove ? kCertFStart : 0u);
        E[t] = CertEntry{r.m[0], r.m[1], r.m[2], r.len(), a->cert_lex[(unsigned long long)slot * T + t],
                         walk ? r.parent() : kCertNoB, walk ? (r.kp0 & 0x1FFFFFFFu) : 0u, r.parent(),
                         soe ? r.parent() : kCertNoB, soe ? (r.kp0 & 0x1FFFFFFFu) : 0u, soe ? r.u : kNone32, fl,
                         t != 0 ? ss.v : kNone32, t != 0 ? ss.x : 0, t != 0 ? ss.y : 0,
                         t != 0 ? ss.region : kNone10};
    }
}

// the least extension of cell (x, y)'s grid neighbours (the Center has none); false when
// The repair sweep's mark on a plain cell word (bit 30: a plain word is b << 20 | k with a
// 10-bit b): the first check sets it on its failing cells, the sweep on the cells a change
// reaches; a sweep rewrites every cell it marked, so no mark outlives it.
constexpr uint32_t kCertDirty = 1u << 30;
__device__ __forceinline__ uint32_t cert_clean(uint32_t w) {
    return (w == kViaSource || (w & kViaSpecial)) ? w : (w & ~kCertDirty);
}
// a neighbour's label cannot be extended here (counted as a failure)
template <bool ATOMIC>
__device__ __forceinline__ bool cert_best4(const DevParams &p, const CertEntry *E, const CellWord *w, uint32_t pitch,
                                           int x, int y, CertLab &best, bool &any, const uint32_t *FT = nullptr,
                                           uint32_t nft = 0) {
    const int S = int(p.S), H = int(p.H);
    any = false;
    bool ok = true;
    const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (nx[i] < 0 || nx[i] >= S || ny[i] < 0 || ny[i] >= S || (nx[i] == H && ny[i] == H)) continue;
        const CellWord *pw = w + (size_t)ny[i] * pitch + nx[i];
        const uint32_t wu = cert_clean(ATOMIC ? __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : *pw);
        CertLab c;
        if (!cert_ext(p, E, wu, c, FT, nft)) {
            ok = false;
            continue;
        }
        if (!any || cert_less(c, best)) best = c;
        any = true;
    }
    return ok;
}

// cert_best4 for the repair sweep's LDS window: a neighbour inside the window
// [x0, x1] x [y0, y1] is read from its LDS copy (row-major, pool), one outside from w
__device__ __forceinline__ void cert_best4_lds(const DevParams &p, const CertEntry *E, const CellWord *w, uint32_t pitch,
                                               const uint32_t *pool, int x0, int y0, int x1, int y1, int x, int y,
                                               CertLab &best, bool &any, const uint32_t *FT, uint32_t nft) {
    const int S = int(p.S), H = int(p.H), bw = x1 - x0 + 1;
    any = false;
    const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (nx[i] < 0 || nx[i] >= S || ny[i] < 0 || ny[i] >= S || (nx[i] == H && ny[i] == H)) continue;
        const bool in = nx[i] >= x0 && nx[i] <= x1 && ny[i] >= y0 && ny[i] <= y1;
        const uint32_t raw = in ? pool[(ny[i] - y0) * bw + (nx[i] - x0)] : w[(size_t)ny[i] * pitch + nx[i]];
        CertLab c;
        if (!cert_ext(p, E, cert_clean(raw), c, FT, nft)) continue;
        if (!any || cert_less(c, best)) best = c;
        any = true;
    }
}

// One launch over every slot's cells (blockIdx.y = slot): failing cells lower the slot's
// key, count, and widen its box.
//
// Demoted specials.  A special whose hub label is a walk can be
// wrong the way a plain cell's closed form is: a walk that its own boundary cannot
// realise.  The first check (mark) then turns such a failing special (not the Center or a
// border-1 cell, whose CentralMoves merge) into a plain cell: its word becomes its walk
// (b, k), marked, and the sweep recomputes it from its neighbours like any other.  A
// demoted special keeps its other in-edges, so the later check tests them too: no
// caravan from a hub and no SHQ may reach it first, and a Scroll of Escape into it (a
// region campfire) is tested against its new word.  The labels the hub built from a
// demoted special (its caravans, SoE, CentralMoves) were built from its old label: a
// special whose parent was demoted fails its pull test.
__global__ __launch_bounds__(kBS) void cert_check_kernel(const KArgs *__restrict__ a, uint32_t mark) {
    __shared__ CertEntry E[64];
    __shared__ uint32_t dem[64];  // entries whose cell holds a plain (demoted) word: that word, else kNone32
    const uint32_t slot = blockIdx.y;
    const uint32_t nslot = min(a->cert_cap, __hip_atomic_load(a->counter + kCtrCert, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT));
    if (slot >= nslot) return;
    // (the second round: a done slot keeps its state; a slot that only sweeps again skips
    // the check before the sweep)
    if (a->cert_redo && (!a->cert_redo[slot] || (mark && a->cert_redo[slot] != kRedoFill))) return;
    const DevParams p = a->p;
    cert_load_table(a, slot, E);
    const uint32_t S = p.S, pitch = a->rec_pitch, T = p.NS + 1;
    const CellWord *w = a->cert_rec + (unsigned long long)slot * S * pitch;
    uint32_t *win = a->cert_win ? a->cert_win + (unsigned long long)slot * kWinWords : nullptr;
    // Entries promoted this pass (their label is now a caravan, cert_promote_kernel) and
    // every entry built on them: the hub built those from the promoted entries' old labels,
    // so they fail (a label resting on them has a lead metric no smaller: the key bounds it)
    __shared__ unsigned long long taint;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tm = win ? ((unsigned long long)win[kWinProm1] << 32) | win[kWinProm0] : 0ull;
        for (uint32_t it = 0; tm && it < 64u; ++it) {
            bool grew = false;
            for (uint32_t e = 1; e < min(T, 64u); ++e)
                if (!((tm >> e) & 1ull) && E[e].par < 64u && ((tm >> E[e].par) & 1ull)) {
                    tm |= 1ull << e;
                    grew = true;
                }
            if (!grew) break;
        }
        taint = tm;
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < 64; t += kBS) {
        uint32_t d = kNone32;
        if (t >= 1 && t < T && !mark) {  // (the first check demotes; it sees none)
            const uint32_t vv = E[t].v, yy = vv / S;
            const uint32_t raw = cert_clean(w[(size_t)yy * pitch + (vv - yy * S)]);
            if (raw != kViaSource && !(raw & kViaSpecial)) d = raw;
        }
        dem[t] = d;
    }
    __syncthreads();
    // entry h's current label as raw metrics (legs, money, time), length, start label
    auto cur = [&](uint32_t h, uint32_t &l, uint32_t &mo, uint32_t &ti, uint32_t &len, bool &start) {
        if (dem[h] != kNone32) {
            const uint32_t b = (dem[h] >> kStBShift) & kNone10, k = dem[h] & kStKMask;
            l = E[b].m0 + k;
            mo = E[b].m1;
            ti = E[b].m2 + run_time_ff(k, p.ff_num, p.ff_den);
            len = b == 0 ? 1u : E[b].len + 1u;
            start = false;
        } else {
            l = E[h].m0;
            mo = E[h].m1;
            ti = E[h].m2;
            len = E[h].len;
            start = (E[h].fl & kCertFStart) != 0;
        }
    };
    // (c1, c2, c3, length) of o strictly before those of the raw metrics (l, mo, ti), len
    auto before = [&](const CertLab &o, uint32_t l, uint32_t mo, uint32_t ti, uint32_t len) {
        const uint32_t e1 = pick(p, 0, l, mo, ti), e2 = pick(p, 1, l, mo, ti), e3 = pick(p, 2, l, mo, ti);
        return o.c1 != e1 ? o.c1 < e1 : (o.c2 != e2 ? o.c2 < e2 : (o.c3 != e3 ? o.c3 < e3 : o.len < len));
    };
    uint32_t key = 0xFFFFFFFFu, nf = 0, x0 = 0xFFFFFFFFu, x1 = 0, y0 = 0xFFFFFFFFu, y1 = 0;
    __shared__ uint32_t dem_bits[2];  // entries this workgroup demotes (mark: the first check)
    if (threadIdx.x < 2) dem_bits[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t v = blockIdx.x * kBS + threadIdx.x; v < p.V; v += gridDim.x * kBS) {
        const uint32_t y = v / S, x = v - y * S;
        const uint32_t cw = cert_clean(w[(size_t)y * pitch + x]);
        if (cw == kViaSource || v == p.vc) continue;
        CertLab best{};
        bool any;
        bool fail = !cert_best4<false>(p, E, w, pitch, int(x), int(y), best, any);
        uint32_t why = fail ? 1u : 0u;  // (diagnostics: which tests failed, kWinWhy)
        uint32_t own1;
        if (cw & kViaSpecial) {
            const uint32_t t = cw & kNone10;
            const CertEntry &e = E[t];
            if (e.wb != kCertNoB) {  // a walk into a special: supported by a neighbour, beaten by none
                const CertLab o = cert_walk(p, E, e.wb, e.wk);
                own1 = o.c1;
                why |= (!any || !cert_same(o, best)) ? 2u : 0u;
                why |= (e.par < 64u && ((taint >> e.par) & 1ull)) ? 4u : 0u;
                fail = fail || !any || !cert_same(o, best) || (e.par < 64u && ((taint >> e.par) & 1ull));
                // (the first check demotes it: cert_window_kernel writes its walk as a plain
                // word before the sweep; recorded here, so this check's readers all see the
                // special's word)
                // (the last check records one that fails its walk test too: the second round
                // demotes it then and sweeps again, from the repaired words)
                // (not a border-1 cell: the Center's label and through it the other border-1
                // cells' rest on its label, and only a new Dijkstra over the specials would
                // rebuild them — tried: the failure moves to those cells)
                if (fail && !(e.fl & kCertFCentral) && (mark || (why & 2u))) atomicOr(&dem_bits[t >> 5], 1u << (t & 31u));
            } else {  // built over the specials: no neighbour's walk may reach it first (a tie on
                      // metrics and length would need the command lists: counted as a failure),
                      // and its parent must still hold the label the hub built it from
                const uint32_t o1 = pick(p, 0, e.m0, e.m1, e.m2), o2 = pick(p, 1, e.m0, e.m1, e.m2),
                               o3 = pick(p, 2, e.m0, e.m1, e.m2);
                own1 = o1;
                const bool below = o1 != best.c1 ? o1 < best.c1
                                                 : (o2 != best.c2 ? o2 < best.c2 : (o3 != best.c3 ? o3 < best.c3 : e.len < best.len));
                why |= (any && !below) ? 8u : 0u;
                why |= (e.par < 64u && (dem[e.par] != kNone32 || ((taint >> e.par) & 1ull))) ? 16u : 0u;
                fail = fail || (any && !below) || (e.par < 64u && (dem[e.par] != kNone32 || ((taint >> e.par) & 1ull)));
            }
        } else {  // a plain cell: exactly its neighbours' least extension
            const uint32_t b = (cw >> kStBShift) & kNone10, k = cw & kStKMask;
            const CertLab o = cert_walk(p, E, b, k);
            own1 = o.c1;
            why |= (!any || !cert_same(o, best)) ? 32u : 0u;
            fail = fail || !any || !cert_same(o, best);
            // a demoted special: no caravan from a hub and no SHQ may reach it first (ties
            // would need the command lists: counted as failures)
            const uint32_t tv = (mark || p.NS == 0) ? kNone10 : (a->sinfo[v] & kNone10);
            if (tv != kNone10 && tv < T) {
                const CertEntry &et = E[tv];
                if (p.use_caravans && (et.fl & kCertFHub)) {
                    const uint32_t coef = (et.fl & kCertFCoef5) ? 5u : 2u;
                    // the least caravan from a hub whose own label is the hub's (a tie between
                    // two such caravans would need the lists: no promotion)
                    CertLab bc{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0};
                    uint32_t bh = kNone32;
                    bool btie = false;
                    for (uint32_t i = 0; i < p.n_hubs; ++i) {
                        const uint32_t h = a->hubs[i];
                        if (h == tv || h >= T) continue;
                        uint32_t l, mo, ti, len;
                        bool start;
                        cur(h, l, mo, ti, len, start);
                        const uint32_t d = uint32_t(abs(E[h].x - et.x) + abs(E[h].y - et.y));
                        if (start) {
                            l = 0;
                            mo = coef * d;
                            ti = p.rgt * d;
                            len = 1;
                        } else {
                            mo += coef * d;
                            ti += p.rgt * d;
                            len += 1;
                        }
                        if (!before(o, l, mo, ti, len)) {
                            fail = true;
                            why |= 64u;
                        }
                        if (dem[h] != kNone32 || (h < 64u && ((taint >> h) & 1ull))) continue;
                        const CertLab c{pick(p, 0, l, mo, ti), pick(p, 1, l, mo, ti), pick(p, 2, l, mo, ti), len, 0, 0, 0};
                        const bool lt = c.c1 != bc.c1 ? c.c1 < bc.c1
                                                      : (c.c2 != bc.c2 ? c.c2 < bc.c2 : (c.c3 != bc.c3 ? c.c3 < bc.c3 : c.len < bc.len));
                        const bool eq = c.c1 == bc.c1 && c.c2 == bc.c2 && c.c3 == bc.c3 && c.len == bc.len;
                        if (lt) {
                            bc = c;
                            bh = h;
                            btie = false;
                        } else if (eq) {
                            btie = true;
                        }
                    }
                    // the caravan strictly before the repaired walk (metrics, length): the
                    // special's label is that caravan unless something else beats both —
                    // cert_promote_kernel makes it so and the next round checks it all again
                    // (not the HQ, not a Scroll-of-Escape target: their other in-edges are not
                    // rebuilt there)
                    const bool cb = bc.c1 != o.c1 ? bc.c1 < o.c1
                                                  : (bc.c2 != o.c2 ? bc.c2 < o.c2 : (bc.c3 != o.c3 ? bc.c3 < o.c3 : bc.len < o.len));
                    if (win && bh != kNone32 && !btie && cb && !(et.fl & kCertFHQ) && a->sp[tv].rid == kNone10 && tv < 64u)
                        win[kWinPromo + tv] = bh + 1u;
                }
                if ((et.fl & kCertFHQ) && !before(o, 0u, p.shq_cost, 0u, 1u)) {
                    fail = true;
                    why |= 128u;
                }
                // a Scroll of Escape into it from a special of its region, or from the source
                if (p.use_soe) {
                    for (uint32_t h = 1; h < T; ++h) {
                        if (h == tv || E[h].reg != tv) continue;
                        uint32_t l, mo, ti, len;
                        bool start;
                        cur(h, l, mo, ti, len, start);
                        if (start) {
                            l = 0;
                            mo = p.soe_cost;
                            ti = 0;
                            len = 1;
                        } else {
                            mo += p.soe_cost;
                            len += 1;
                        }
                        if (!before(o, l, mo, ti, len)) {
                            fail = true;
                            why |= 256u;
                        }
                    }
                    const uint32_t sv = a->cert_src[slot];
                    if (((a->sinfo[sv] >> 10) & kNone10) == tv && !before(o, 0u, p.soe_cost, 0u, 1u)) {
                        fail = true;
                        why |= 512u;
                    }
                }
            }
            // Its Scroll of Escape into its region's campfire c (the repair sweep may have
            // changed the cell after the hub built c's label from the closed form): c's
            // SoE-region label must start from this cell's word when it names this cell
            // (pull), and no other cell's SoE may reach c first (push; a tie on metrics and
            // length would need the command lists: counted as a failure).
            const uint32_t rc = p.use_soe ? (a->sinfo[v] >> 10) & kNone10 : kNone10;
            if (rc != kNone10 && rc < T && dem[rc] != kNone32) {
                // the campfire was demoted: its label is its walk word's; the scroll from this
                // cell must not reach it first (a tie: the lists would decide, a failure)
                if (rc != (a->sinfo[v] & kNone10)) {
                    const uint32_t wm0 = E[b].m0 + k, wm1 = E[b].m1 + p.soe_cost,
                                   wm2 = E[b].m2 + run_time_ff(k, p.ff_num, p.ff_den);
                    const uint32_t rb = (dem[rc] >> kStBShift) & kNone10, rk = dem[rc] & kStKMask;
                    const CertLab cl = cert_walk(p, E, rb, rk);
                    if (!before(cl, wm0, wm1, wm2, o.len + 1u)) {
                        own1 = min(own1, min(cl.c1, pick(p, 0, wm0, wm1, wm2)));
                        fail = true;
                        why |= 1024u;
                    }
                }
            } else if (rc != kNone10) {
                const CertEntry &e = E[rc];
                const CertLab &w = o;
                // metrics of the walk, then + the scroll's money
                const uint32_t wm0 = E[b].m0 + k, wm1 = E[b].m1 + p.soe_cost,
                               wm2 = E[b].m2 + run_time_ff(k, p.ff_num, p.ff_den);
                const uint32_t x1 = pick(p, 0, wm0, wm1, wm2), x2 = pick(p, 1, wm0, wm1, wm2), x3 = pick(p, 2, wm0, wm1, wm2),
                               xl = w.len + 1u;
                const uint32_t c1 = pick(p, 0, e.m0, e.m1, e.m2), c2 = pick(p, 1, e.m0, e.m1, e.m2),
                               c3 = pick(p, 2, e.m0, e.m1, e.m2);
                bool bad;
                const uint32_t rv = a->rank[v];
                if (e.su == rv) {
                    bad = e.sb != b || e.sk != k;
                } else if (c1 != x1 || c2 != x2 || c3 != x3 || e.len != xl) {  // c strictly first
                    bad = !(c1 != x1 ? c1 < x1 : (c2 != x2 ? c2 < x2 : (c3 != x3 ? c3 < x3 : e.len < xl)));
                } else if (e.sb != kCertNoB) {
                    // equal metrics and length against c's own SoE-region label full(sb) ++
                    // [Std sb -> su] ++ [SoE su -> c]: the lists differ inside the boundaries'
                    // labels (their ranks decide) or, from one boundary, in the walk's end cell
                    bad = b != e.sb ? E[b].lex < E[e.sb].lex : rv < e.su;
                } else {
                    bad = true;  // a tie with another kind of label: the lists would decide
                }
                if (bad) {
                    own1 = min(own1, min(c1, x1));
                    fail = true;
                    why |= 2048u;
                }
            }
        }
        if (fail && !mark && win) {  // (diagnostics: the first few failing cells of the last check)
            const uint32_t at = atomicAdd(win + kWinWhy, 1u);
            if (at < 7u) {
                win[kWinWhy + 1 + 4 * at] = x | (y << 16);
                win[kWinWhy + 2 + 4 * at] = why | ((cw & kViaSpecial) && cw != kViaSource ? 0x80000000u : 0u);
                win[kWinWhy + 3 + 4 * at] = own1;
                win[kWinWhy + 4 + 4 * at] = any ? best.c1 : 0xFFFFFFFFu;
            }
        }
        if (fail) {
            // (the check before the sweep: a failing plain cell seeds its queue; only this
            // thread writes the word, and readers mask the mark)
            if (mark && !(cw & kViaSpecial)) const_cast<CellWord *>(w)[(size_t)y * pitch + x] = cw | kCertDirty;
            key = min(key, any ? min(own1, best.c1) : own1);
            ++nf;
            x0 = min(x0, x);
            x1 = max(x1, x);
            y0 = min(y0, y);
            y1 = max(y1, y);
        }
    }
    // the workgroup's partial state (plain stores: a consumer reduces the workgroups')
    __shared__ uint32_t red[kCertSt];
    if (threadIdx.x < kCertSt) red[threadIdx.x] = (threadIdx.x == kCertKey || threadIdx.x == kCertX0 ||
                                                   threadIdx.x == kCertY0) ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    if (threadIdx.x < 2) red[kCertDem0 + threadIdx.x] = dem_bits[threadIdx.x];
    if (__any(nf != 0)) {
        key = wave_min_u32(key);
        x0 = wave_min_u32(x0);
        y0 = wave_min_u32(y0);
        x1 = ~wave_min_u32(~x1);
        y1 = ~wave_min_u32(~y1);
        uint32_t n = nf;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) n += uint32_t(__shfl_xor(int(n), o));
        if (lane_id() == 0) {
            atomicMin(red + kCertKey, key);
            atomicAdd(red + kCertFails, n);
            atomicMin(red + kCertX0, x0);
            atomicMax(red + kCertX1, x1);
            atomicMin(red + kCertY0, y0);
            atomicMax(red + kCertY1, y1);
        }
    }
    __syncthreads();
    if (threadIdx.x < kCertSt) a->cert_st[((unsigned long long)slot * a->cert_parts + blockIdx.x) * kCertSt + threadIdx.x] = red[threadIdx.x];
}

// One workgroup, after the hub launches: the certificate slots go to the staged fallback
// entries in source order (the cert_cap least source indices), and their staged tables
// are copied into the slots; every other entry gets none.  A pass with more fallback
// entries than the staging holds gives no slots (which entries were staged then
// depended on arrival order).  Sets kCtrCert, which the slot kernels read.
constexpr uint32_t kSelectBS = 1024;
__global__ __launch_bounds__(kSelectBS) void cert_select_kernel(const KArgs *__restrict__ a) {
    __shared__ uint32_t key[kCertStageMax], slot_of[kCertStageMax];
    __shared__ uint32_t nstaged;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = __hip_atomic_load(a->counter + kCtrFbCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t cap = min(a->cert_stage_cap, kCertStageMax);
    if (n > cap) {
        for (uint32_t i = tid; i < n; i += kSelectBS) a->fb_cert[i] = kNone32;
        if (tid == 0) a->counter[kCtrCert] = 0;
        return;
    }
    if (tid == 0) nstaged = 0;
    for (uint32_t i = tid; i < n; i += kSelectBS) key[i] = a->fb_cert[i] == kFbStaged ? a->fb_list[i] : kNone32;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kSelectBS) {
        uint32_t slot = kNone32;
        if (key[i] != kNone32) {
            uint32_t r = 0;  // staged entries of a smaller source (sources are distinct)
            for (uint32_t j = 0; j < n; ++j) r += key[j] < key[i] ? 1u : 0u;
            if (r < a->cert_cap) slot = r;
            atomicAdd(&nstaged, 1u);
        }
        slot_of[i] = slot;
        a->fb_cert[i] = slot;
    }
    __syncthreads();
    const uint32_t T = a->p.NS + 1;
    for (uint32_t k = tid; k < n * T; k += kSelectBS) {
        const uint32_t i = k / T, t = k - i * T, slot = slot_of[i];
        if (slot == kNone32) continue;
        a->cert_tab[(unsigned long long)slot * T + t] = a->cert_stage_tab[(unsigned long long)i * T + t];
        a->cert_lex[(unsigned long long)slot * T + t] = a->cert_stage_lex[(unsigned long long)i * T + t];
        if (t == 0) a->cert_src[slot] = a->cert_stage_src[i];
    }
    if (tid == 0) a->counter[kCtrCert] = min(nstaged, a->cert_cap);
    if (a->cert_win)  // (a new pass: nothing promoted yet)
        for (uint32_t s = tid; s < a->cert_cap; s += kSelectBS) {
            a->cert_win[(unsigned long long)s * kWinWords + kWinProm0] = 0;
            a->cert_win[(unsigned long long)s * kWinWords + kWinProm1] = 0;
        }
}

#ifndef MR_SWEEP_BUCKETS
#define MR_SWEEP_BUCKETS 4096
#endif
#ifndef MR_SWEEP_POOL
#define MR_SWEEP_POOL 16384
#endif
#ifndef MR_SWEEP_BS
#define MR_SWEEP_BS 1024
#endif
constexpr uint32_t kSweepBS = MR_SWEEP_BS;  // threads of the sweep's one workgroup per slot
constexpr uint32_t kSweepBuckets = MR_SWEEP_BUCKETS;  // leading-metric buckets a window may span
constexpr int kSweepMargin = 2;            // cells added round the failing cells' box
constexpr int kSweepMarginAgain = 24;      // the same in a sweep-only second round
#ifndef MR_SWEEP_RT
#define MR_SWEEP_RT 4100
#endif
#ifndef MR_SWEEP_LQ
#define MR_SWEEP_LQ MR_SWEEP_POOL
#endif
constexpr uint32_t kSweepRunTimes = MR_SWEEP_RT;  // run-time table (walks of up to 2 S + 3 legs at S = 2048;
                                           // longer ones divide)
constexpr uint32_t kSweepPool = MR_SWEEP_POOL;  // LDS words: the window's words, or its mark bitmap
static_assert(kSweepPool <= 65536, "an LDS window's queues hold 16-bit cell indices");

// One workgroup per slot: the failing box (+ margin) in order of the leading metric of its
// cells, bucket by bucket (buckets of the least StandardMove increment: a cell never
// extends another of its bucket), each cell recomputed from its neighbours' current words.
// Only the cells that can change are touched: the ones the first check marked (its
// failing plain cells) and those whose neighbour changed in an earlier bucket — any other
// cell's word already is its neighbours' least extension, and stays so while they do.
// Each bucket holds a queue of those cells (its region of the counting-sorted window,
// filled through an LDS counter; a mark keeps a cell queued once), and a bucket with an
// empty queue costs no barrier.  A window of at most kSweepPool cells keeps its words in
// LDS (marks in bit 30) and writes them back at the end; a larger one (up to 32 x
// kSweepPool cells) keeps its marks in an LDS bitmap and its words in the slot's buffer,
// owned by this workgroup (one CU) during the sweep, so workgroup-scope accesses and the
// barrier order the buckets.  An LDS window's queues are in LDS too (16-bit cell indices),
// so its buckets touch no global memory; a bitmap window's are in the slot's list buffer.
// A queued cell's four neighbour words are read once, for its least extension and for
// queueing them (an unmarked neighbour is not rewritten in this bucket).  Wider windows
// are left to the SSSP kernel.  (ff 2 at 1025^2,
// 100k of the window's 441k cells in 810 of its 1 329 buckets.)
__global__ __launch_bounds__(kSweepBS) void cert_sweep_kernel(const KArgs *__restrict__ a) {
    __shared__ CertEntry E[64];
    __shared__ uint32_t off[kSweepBuckets];   // bucket j's queue: list[off[j - 1] ..), off[-1] = 0
    __shared__ uint32_t fill[kSweepBuckets];  // its length so far
    __shared__ uint32_t FT[kSweepRunTimes];   // run times of 0 .. kSweepRunTimes - 1 legs
    __shared__ uint32_t pool[kSweepPool];
    __shared__ uint16_t lq[MR_SWEEP_LQ];  // an LDS window's queues (window cell indices)
    __shared__ uint32_t red[2];
    const uint32_t slot = blockIdx.x, tid = threadIdx.x;
    const uint32_t nslot = min(a->cert_cap, __hip_atomic_load(a->counter + kCtrCert, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT));
    if (slot >= nslot) return;
    // (cert_window_kernel gave this slot to the tile sweep, or to nobody)
    if (a->cert_win && a->cert_win[(unsigned long long)slot * kWinWords + kWinMode] != kWinOld) return;
    if (a->cert_redo && !a->cert_redo[slot]) return;
    // the check's state: the least / greatest over its workgroups' partials
    __shared__ uint32_t st[kCertSt];
    if (tid < kCertSt) st[tid] = (tid == kCertKey || tid == kCertX0 || tid == kCertY0) ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    for (uint32_t j = tid; j < a->cert_parts; j += kSweepBS) {
        const uint32_t *ps = a->cert_st + ((unsigned long long)slot * a->cert_parts + j) * kCertSt;
        if (ps[kCertFails] == 0) continue;
        atomicAdd(st + kCertFails, ps[kCertFails]);
        atomicMin(st + kCertX0, ps[kCertX0]);
        atomicMax(st + kCertX1, ps[kCertX1]);
        atomicMin(st + kCertY0, ps[kCertY0]);
        atomicMax(st + kCertY1, ps[kCertY1]);
    }
    __syncthreads();
    if (st[kCertFails] == 0) return;  // certified as it stands (and nothing was marked)
    const DevParams p = a->p;
    cert_load_table(a, slot, E);
    const uint32_t nft = min(kSweepRunTimes, 2u * p.S + 4u);
    for (uint32_t k = tid; k < nft; k += kSweepBS) FT[k] = run_time_ff(k, p.ff_num, p.ff_den);
    if (tid == 0) {
        red[0] = 0xFFFFFFFFu;
        red[1] = 0;
    }
    const int S = int(p.S), H = int(p.H);
    const int mg = (a->cert_redo && a->cert_redo[slot] == kRedoSweep) ? kSweepMarginAgain : kSweepMargin;
    const int bx0 = max(0, int(st[kCertX0]) - mg), bx1 = min(S - 1, int(st[kCertX1]) + mg);
    const int by0 = max(0, int(st[kCertY0]) - mg), by1 = min(S - 1, int(st[kCertY1]) + mg);
    const uint32_t bw = uint32_t(bx1 - bx0 + 1), area = bw * uint32_t(by1 - by0 + 1);
    const uint32_t pitch = a->rec_pitch;
    CellWord *w = a->cert_rec + (unsigned long long)slot * p.S * pitch;
    uint32_t *list = a->cert_aux + (unsigned long long)slot * p.V;
    const bool in_lds = area <= kSweepPool && !(a->dbg_flags & kDbgSweepNoLds);  // the words in LDS
    const bool fits = in_lds || area <= 32u * kSweepPool;  // else: left to the SSSP kernel
    // the leading metric: the first in comparator order that grows along a walk; its least
    // StandardMove increment is the bucket width
    const uint32_t L = p.perm[0] != 1u ? p.perm[0] : p.perm[1];
    const uint32_t W = L == 0 ? 1u : max(1u, p.W);
    auto lead_of = [&](uint32_t cw) {
        const uint32_t b = (cw >> kStBShift) & kNone10, k = cw & kStKMask;
        return L == 0 ? E[b].m0 + k : E[b].m2 + (k < nft ? FT[k] : run_time_ff(k, p.ff_num, p.ff_den));
    };
    auto plain_word = [&](uint32_t cw) { return cw != kViaSource && !(cw & kViaSpecial); };
    auto gptr = [&](int x, int y) { return w + (size_t)y * pitch + x; };
    auto widx = [&](int x, int y) { return uint32_t(y - by0) * bw + uint32_t(x - bx0); };
    auto inwin = [&](int x, int y) { return x >= bx0 && x <= bx1 && y >= by0 && y <= by1; };
    // a cell's current word (marks off): LDS inside an LDS window, else the slot's buffer
    auto word = [&](int x, int y) -> uint32_t {
        if (in_lds && inwin(x, y)) return cert_clean(pool[widx(x, y)]);
        return cert_clean(__hip_atomic_load(gptr(x, y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    __syncthreads();
    // the window's key range; an LDS window's words come in (with the check's marks)
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0;
    for (uint32_t i = tid; i < area; i += kSweepBS) {
        const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
        const uint32_t raw = *gptr(x, y), cw = cert_clean(raw);
        if (in_lds) pool[i] = raw;
        if (!plain_word(cw)) continue;
        const uint32_t kk = lead_of(cw) / W;
        kmin = min(kmin, kk);
        kmax = max(kmax, kk);
    }
    kmin = wave_min_u32(kmin);
    kmax = ~wave_min_u32(~kmax);
    if (lane_id() == 0) {
        atomicMin(&red[0], kmin);
        atomicMax(&red[1], kmax);
    }
    __syncthreads();
    kmin = red[0];
    kmax = red[1];
    const uint32_t nb = kmax >= kmin ? kmax - kmin + 1 : 0;
    if (nb == 0 || nb > kSweepBuckets || !fits) {  // nothing to sweep / too wide: left to the SSSP kernel
        for (uint32_t i = tid; i < area; i += kSweepBS) {  // (the check's marks come off)
            const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
            const uint32_t cw = *gptr(x, y);
            if (plain_word(cw) && (cw & kCertDirty)) *gptr(x, y) = cw & ~kCertDirty;
        }
        return;
    }
    const bool full = (a->dbg_flags & kDbgSweepFull) != 0;  // (A/B: every window cell queued)
    const bool reread = (a->dbg_flags & kDbgSweepReread) != 0,
               lql = in_lds && !(a->dbg_flags & kDbgSweepGList) && MR_SWEEP_LQ >= kSweepPool;
    for (uint32_t j = tid; j < nb; j += kSweepBS) {
        off[j] = 0;
        fill[j] = 0;
    }
    if (!in_lds)
        for (uint32_t i = tid; i < (area + 31) / 32; i += kSweepBS) pool[i] = 0;  // the mark bitmap
    __syncthreads();
    // marks: test-and-set (true: this thread set it) and test
    auto mark = [&](int x, int y) -> bool {
        const uint32_t i = widx(x, y);
        if (in_lds) return !(atomicOr(&pool[i], kCertDirty) & kCertDirty);
        const uint32_t bit = 1u << (i & 31u);
        return !(atomicOr(&pool[i >> 5], bit) & bit);
    };
    auto marked = [&](int x, int y) -> bool {
        const uint32_t i = widx(x, y);
        return in_lds ? (pool[i] & kCertDirty) != 0 : ((pool[i >> 5] >> (i & 31u)) & 1u) != 0;
    };
    // bucket sizes over the whole window (a queue never outgrows its bucket)
    for (uint32_t i = tid; i < area; i += kSweepBS) {
        const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
        const uint32_t cw = in_lds ? cert_clean(pool[i]) : cert_clean(*gptr(x, y));
        if (plain_word(cw)) atomicAdd(&off[lead_of(cw) / W - kmin], 1u);
    }
    __syncthreads();
    // inclusive prefix sum of the sizes (each thread a run of buckets, then the runs):
    // off[j] ends bucket j's region
    {
        const uint32_t per = (nb + kSweepBS - 1) / kSweepBS, j0 = tid * per, j1 = min(nb, j0 + per);
        uint32_t sum = 0;
        for (uint32_t j = j0; j < j1; ++j) sum += off[j];
        __shared__ uint32_t runs[kSweepBS];
        runs[tid] = sum;
        __syncthreads();
        for (uint32_t d = 1; d < kSweepBS; d <<= 1) {
            const uint32_t v = tid >= d ? runs[tid - d] : 0u;
            __syncthreads();
            runs[tid] += v;
            __syncthreads();
        }
        uint32_t acc = runs[tid] - sum;
        for (uint32_t j = j0; j < j1; ++j) {
            acc += off[j];
            off[j] = acc;
        }
    }
    __syncthreads();
    // the seeds: the cells the first check marked (a bitmap window takes the marks off the
    // words; an LDS window keeps them in its words)
    for (uint32_t i = tid; i < area; i += kSweepBS) {
        const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
        uint32_t raw = in_lds ? pool[i] : *gptr(x, y);
        if (!plain_word(raw)) continue;
        bool seed = (raw & kCertDirty) != 0 || full;
        if (in_lds) {
            if (full) pool[i] = raw | kCertDirty;
        } else {
            if (raw & kCertDirty) *gptr(x, y) = raw & ~kCertDirty;
        }
        if (!seed) continue;
        if (!in_lds) atomicOr(&pool[i >> 5], 1u << (i & 31u));
        const uint32_t j = lead_of(raw & ~kCertDirty) / W - kmin;
        const uint32_t at = (j ? off[j - 1] : 0u) + atomicAdd(&fill[j], 1u);
        if (lql) lq[at] = uint16_t(i);
        else list[at] = uint32_t(y) << 16 | uint32_t(x);
    }
    __syncthreads();
    // bucket j's queue region and a push into it (a full region drops the push: the check
    // after the sweep then finds the stale cell, and the SSSP kernel solves the source)
    auto region = [&](uint32_t j) { return j ? off[j - 1] : 0u; };
    auto push = [&](uint32_t j, int x, int y) {
        const uint32_t at = atomicAdd(&fill[j], 1u);
        if (at >= off[j] - region(j)) return;
        if (lql) lq[region(j) + at] = uint16_t(widx(x, y));
        else list[region(j) + at] = uint32_t(y) << 16 | uint32_t(x);
    };
    // Bucket by bucket: each queued cell takes its neighbours' least extension; a change
    // queues its unmarked neighbours of later buckets.  A cell whose new word lies in a
    // later bucket is queued again there: its label may rest on a neighbour of this
    // bucket that changes concurrently, and only a later bucket's evaluation sees every
    // cell it can rest on final.
    for (uint32_t j = 0; j < nb; ++j) {
        const uint32_t n = min(fill[j], off[j] - region(j));  // (uniform: written before the last barrier)
        if (n == 0) continue;
        const uint32_t beg = region(j);
        for (uint32_t i = beg + tid; i < beg + n; i += kSweepBS) {
            int x, y;
            if (lql) {
                const uint32_t wi = lq[i], r = wi / bw;
                y = by0 + int(r);
                x = bx0 + int(wi - r * bw);
            } else {
                const uint32_t v = list[i];
                y = int(v >> 16);
                x = int(v & 0xFFFFu);
            }
            // the neighbours' least extension (the Center has none), and their words (marks
            // off) for the queueing below.  (The least extension goes through cert_best4*:
            // the same loop written out here left the Fleetfoot 1 test source uncertified
            // on the GPU, test_gpu_cert.py, for reasons not found)
            const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
            uint32_t nwd[4];
            bool on[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                on[q] = nx[q] >= 0 && nx[q] < S && ny[q] >= 0 && ny[q] < S && !(nx[q] == H && ny[q] == H);
                nwd[q] = on[q] ? word(nx[q], ny[q]) : 0u;
            }
            const uint32_t old = word(x, y);
            CertLab best{};
            bool any = false;
            if (in_lds) cert_best4_lds(p, E, w, pitch, pool, bx0, by0, bx1, by1, x, y, best, any, FT, nft);
            else cert_best4<true>(p, E, w, pitch, x, y, best, any, FT, nft);
            const uint32_t nw = any ? ((best.b << kStBShift) | best.k) : old;
            if (nw == old) continue;
            if (in_lds) pool[widx(x, y)] = nw | kCertDirty;  // (the mark stays: never queued again)
            else __hip_atomic_store(gptr(x, y), nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (!on[q] || !inwin(nx[q], ny[q])) continue;  // (outside the window: fixed)
                // (an unmarked neighbour is never processed in this bucket: its word read
                // above is current; a marked one is skipped)
                const uint32_t cu = reread ? word(nx[q], ny[q]) : nwd[q];
                if (!plain_word(cu) || marked(nx[q], ny[q])) continue;  // (queued or processed already)
                const uint32_t ju = lead_of(cu) / W - kmin;           // (an unmarked cell: its initial bucket)
                if (ju <= j || ju >= nb) continue;                    // (an earlier or this bucket: not its reader)
                if (!mark(nx[q], ny[q])) continue;                    // (another thread queued it)
                push(ju, nx[q], ny[q]);
            }
            const uint32_t jn = lead_of(nw) / W - kmin;  // (the mark stays: nobody else queues it)
            if (jn > j && jn < nb) push(jn, x, y);
        }
        __syncthreads();
    }
    // an LDS window's words go back, marks off
    if (in_lds)
        for (uint32_t i = tid; i < area; i += kSweepBS) {
            const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
            const uint32_t raw = pool[i];
            if (plain_word(raw)) *gptr(x, y) = raw & ~kCertDirty;
        }
}

}  // namespace mr
