// mr_cert_tile.hpp — the certificate's repair as a multi-workgroup bucketed relaxation
// (DESIGN.md section 3d, round 6).
//
// The repair window (the first check's failing cells' box plus a margin) is solved as the
// reference's Dijkstra (src/pathfinder.rs:219-246) restricted to it: every plain cell of the
// window (demoted specials included) starts unsettled, every other cell keeps its word and
// is a fixed source.  Cells settle in buckets of the comparator's leading metric G (legs
// or time), W wide, the least StandardMove increment of G: a label of bucket j extends only
// into buckets j + 1 and j + 2 (a run's time grows by floor(c) or floor(c) + 1, c = 180 n / d),
// so a cell of bucket j rests on cells of earlier buckets only, and at step j every
// unsettled cell whose least pushed candidate lies in bucket j is final (the uniqueness
// lemma, DESIGN.md section 2: one pass in label order reproduces the fixed point).  The
// check after the sweep certifies the result as before; nothing here is trusted unchecked.
//
// A label is a 64-bit key whose integer order is the comparator's on walks
// (src/cost.rs:379-426 restricted to StandardMove runs): walk(b, k) has (G, O, money, length,
// list) with G and O the two growing metrics (legs, time) and the rest constant per
// boundary b, so
//     key = (G - B0) << 40 | RM(b) << 34 | O << 6 | id(b)
// where, if the second metric is O, RM = 0 and id = rank of (money, length, list) among the
// boundaries, and if it is money, RM = rank of money and id = rank of (length, list).  id
// is unique, so a key names its boundary; O and G name k.  A cell holds the key of its
// label's one-step extension (what it pushes), with bit 63 clear once settled; an
// unsettled cell holds 1 << 63 | its least pushed candidate, so an atomic 64-bit minimum
// is the relaxation and can never disturb a settled cell.
//
// Work decomposition.  A window of at most kTileN cells (with its ring of fixed cells) is one
// workgroup's LDS: every step is a barrier of that workgroup.  A larger one is cut into
// kTileT x kTileT tiles, one workgroup each (the slot's team), whose LDS region is the tile
// plus a kTileH-cell halo: a team runs kTileH steps between exchanges (temporal blocking —
// an error at the region's edge travels one cell a step, so the tile's own cells stay
// exact for kTileH steps), then each tile publishes its cells (write-through sc1 stores),
// the team meets at a counter barrier, and each tile reloads its halo from its neighbours'
// publications.  The barrier and the exchange are paid once per kTileH buckets.
#pragma once
#include "mr_cert.hpp"

namespace mr {

// (tile and window constants: mr_engine.hpp)

// One workgroup per slot, after the first check: reduces the check's partial states,
// writes the specials it demoted as plain walk words (their cells are in the failing box),
// and sizes the slot's repair: the window, its tiles and the first bucket's base B0 (the
// least G over the fixed cells that border the window, the only ones whose labels enter
// it).  Money-first orders keep the round-5 sweep (walks of different money need not
// settle in time order), and so do windows wider than its limit (left to the SSSP kernel).
__device__ __forceinline__ void cert_window_slot(const KArgs *__restrict__ a, uint32_t slot) {
    __shared__ CertEntry E[64];
    __shared__ uint32_t st[kCertSt];
    __shared__ uint32_t b0;
    const uint32_t tid = threadIdx.x;
    uint32_t *win = a->cert_win + (unsigned long long)slot * kWinWords;
    if (a->cert_redo && !a->cert_redo[slot]) return;  // (the second round: this slot is done)
    for (uint32_t i = tid; i < kWinWords; i += 256)
        if (i != kWinProm0 && i != kWinProm1) win[i] = 0;
    const uint32_t nslot = min(a->cert_cap, __hip_atomic_load(a->counter + kCtrCert, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT));
    if (slot >= nslot) return;
    if (tid < kCertSt) st[tid] = (tid == kCertKey || tid == kCertX0 || tid == kCertY0) ? 0xFFFFFFFFu : 0u;
    if (tid == 0) b0 = 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t j = tid; j < a->cert_parts; j += 256) {
        const uint32_t *ps = a->cert_st + ((unsigned long long)slot * a->cert_parts + j) * kCertSt;
        if (ps[kCertFails] == 0) continue;
        atomicAdd(st + kCertFails, ps[kCertFails]);
        atomicMin(st + kCertX0, ps[kCertX0]);
        atomicMax(st + kCertX1, ps[kCertX1]);
        atomicMin(st + kCertY0, ps[kCertY0]);
        atomicMax(st + kCertY1, ps[kCertY1]);
        atomicOr(st + kCertDem0, ps[kCertDem0]);
        atomicOr(st + kCertDem1, ps[kCertDem1]);
    }
    __syncthreads();
    if (st[kCertFails] == 0) return;  // certified as it stands (kWinNone)
    const DevParams p = a->p;
    cert_load_table(a, slot, E);
    __syncthreads();
    const uint32_t T = p.NS + 1, pitch = a->rec_pitch;
    CellWord *w = a->cert_rec + (unsigned long long)slot * p.S * pitch;
    // the demoted specials become plain cells holding their walk
    for (uint32_t t = 1 + tid; t < min(T, 64u); t += 256) {
        if (!((st[kCertDem0 + (t >> 5)] >> (t & 31u)) & 1u) || E[t].wb == kCertNoB) continue;
        const uint32_t v = E[t].v, y = v / p.S;
        w[(size_t)y * pitch + (v - y * p.S)] = ((E[t].wb << kStBShift) | E[t].wk) | kCertDirty;
    }
    const int S = int(p.S), H = int(p.H);
    // (a sweep-only round repairs what the last sweep's window left: cells just past its
    // edge, downstream of a special demoted late; a wider margin takes them in at once)
    const int mg = (a->cert_redo && a->cert_redo[slot] == kRedoSweep) ? kSweepMarginAgain : kSweepMargin;
    const int bx0 = max(0, int(st[kCertX0]) - mg), bx1 = min(S - 1, int(st[kCertX1]) + mg);
    const int by0 = max(0, int(st[kCertY0]) - mg), by1 = min(S - 1, int(st[kCertY1]) + mg);
    const uint32_t bw = uint32_t(bx1 - bx0 + 1), bh = uint32_t(by1 - by0 + 1);
    const bool money_first = p.perm[0] == 1u;
    uint32_t ntx = 1, nty = 1;
    if (bw + 2 > kTileP || bh + 2 > kTileR) {
        ntx = (bw + kTileT - 1) / kTileT;
        nty = (bh + kTileT - 1) / kTileT;
    }
    // the growing metric after the lead (O) must fit its 28 bits for every walk here
    const uint32_t L = p.perm[0], O = L == 0 ? 2u : 0u, kmax = 2u * p.S + 4u;
    bool fits = true;
    for (uint32_t t = 0; t < min(T, 64u); ++t) {
        if (t != 0 && E[t].lex == kNone32) continue;
        const uint64_t ob = uint64_t(O == 0 ? E[t].m0 : E[t].m2) + (O == 0 ? kmax : run_time_ff(kmax, p.ff_num, p.ff_den));
        fits = fits && ob < (1ull << 28);
    }
    if (T > 64u) fits = false;
    const bool wide = bw * bh > 32u * kSweepPool || ntx * nty > min(a->cert_pub_wgs, kTileMaxTiles) || !fits;
    if (money_first || (wide && bw * bh <= 32u * kSweepPool)) {
        if (tid == 0) win[kWinMode] = kWinOld;  // (the round-5 sweep decides, and strips the marks)
        return;
    }
    if (wide) {  // left to the SSSP kernel: the check's marks come off
        for (uint32_t i = tid; i < bw * bh; i += 256) {
            const int y = by0 + int(i / bw), x = bx0 + int(i % bw);
            const uint32_t cw = w[(size_t)y * pitch + x];
            if (cw != kViaSource && !(cw & kViaSpecial) && (cw & kCertDirty)) w[(size_t)y * pitch + x] = cw & ~kCertDirty;
        }
        if (tid == 0) win[kWinMode] = kWinWide;
        return;
    }
    __syncthreads();  // (the demoted words are in place)
    // B0: the least own G over the fixed cells bordering the window: its ring (inside the
    // grid, the Center excluded) and the fixed cells inside it (the source, the specials
    // that were not demoted)
    auto own_g = [&](uint32_t cw) -> uint32_t {
        if (cw == kViaSource) return 0u;
        if (cw & kViaSpecial) {
            const CertEntry &e = E[(cw & kNone10) < 64u ? (cw & kNone10) : 0u];
            return L == 0 ? e.m0 : e.m2;
        }
        const uint32_t b = (cw >> kStBShift) & kNone10, k = cw & kStKMask;
        const CertEntry &e = E[b < 64u ? b : 0u];
        return L == 0 ? e.m0 + k : e.m2 + run_time_ff(k, p.ff_num, p.ff_den);
    };
    uint32_t g = 0xFFFFFFFFu;
    const uint32_t ring = 2u * (bw + bh);
    for (uint32_t i = tid; i < ring; i += 256) {
        int x, y;
        if (i < bw) { x = bx0 + int(i); y = by0 - 1; }
        else if (i < 2u * bw) { x = bx0 + int(i - bw); y = by1 + 1; }
        else if (i < 2u * bw + bh) { x = bx0 - 1; y = by0 + int(i - 2u * bw); }
        else { x = bx1 + 1; y = by0 + int(i - 2u * bw - bh); }
        if (x < 0 || y < 0 || x >= S || y >= S || (x == H && y == H)) continue;
        g = min(g, own_g(cert_clean(w[(size_t)y * pitch + x])));
    }
    for (uint32_t t = 1 + tid; t < T + 1; t += 256) {
        uint32_t v;
        if (t < T) {
            if (t >= 64u) continue;
            v = E[t].v;
        } else {
            v = a->cert_src[slot];
        }
        const int y = int(v / p.S), x = int(v % p.S);
        if (x < bx0 || x > bx1 || y < by0 || y > by1 || (x == H && y == H)) continue;
        const uint32_t cw = cert_clean(w[(size_t)y * pitch + x]);
        if (cw == kViaSource || (cw & kViaSpecial)) g = min(g, own_g(cw));
    }
    atomicMin(&b0, g);
    __syncthreads();
    if (tid == 0) {
        win[kWinX0] = uint32_t(bx0);
        win[kWinY0] = uint32_t(by0);
        win[kWinX1] = uint32_t(bx1);
        win[kWinY1] = uint32_t(by1);
        win[kWinNtx] = ntx;
        win[kWinNty] = nty;
        win[kWinB0] = b0 == 0xFFFFFFFFu ? 0u : b0;
        win[kWinMode] = kWinTile;
    }
}

// The windows, then (the last workgroup to finish) the choice between the two sweeps.
// The tile sweep buys latency with CUs: a window of T tiles keeps T CUs for about one
// source's label-order chain, where the round-5 sweep keeps one CU about three times as
// long.  So multi-tile windows take the tile sweep only while every tile window of the
// pass fits one round of the persistent grid (a lone handed-over source: the latency
// case); otherwise they keep the round-5 sweep, all in parallel (many handed-over
// sources: the throughput case).  One-tile windows always take the tile sweep.
__global__ __launch_bounds__(256) void cert_window_kernel(const KArgs *__restrict__ a) {
    cert_window_slot(a, blockIdx.x);
    __shared__ bool last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        uint32_t *ctr = a->cert_win + (unsigned long long)a->cert_cap * kWinWords;
        last = atomicAdd(ctr, 1u) == gridDim.x - 1u;
        if (last) {
            __threadfence();
            uint32_t tiles = 0;
            for (uint32_t s = 0; s < gridDim.x; ++s) {
                const uint32_t *win = a->cert_win + (unsigned long long)s * kWinWords;
                if (a->cert_redo && !a->cert_redo[s]) continue;
                if (__hip_atomic_load(win + kWinMode, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kWinTile)
                    tiles += win[kWinNtx] * win[kWinNty];
            }
            if (tiles > a->cert_pub_wgs)
                for (uint32_t s = 0; s < gridDim.x; ++s) {
                    uint32_t *win = a->cert_win + (unsigned long long)s * kWinWords;
                    if (a->cert_redo && !a->cert_redo[s]) continue;
                    if (win[kWinMode] == kWinTile && win[kWinNtx] * win[kWinNty] > 1u) win[kWinMode] = kWinOld;
                }
            *ctr = 0;
            __threadfence();
        }
    }
}

// The tile sweep.  A persistent grid of cert_pub_wgs workgroups (one a CU: the LDS block
// admits no second), so a team's workgroups are resident together and its waits end.
// The slots' teams are packed into rounds of at most that many tiles, in slot order; every
// workgroup computes the same packing and takes position blockIdx.x of each round.  A
// team's tiles are contiguous in its round, so a tile's publish area is the workgroup that
// holds it.
//
// Exchanges are neighbour-to-neighbour: after each kTileH steps a tile publishes its cells
// (two areas, by parity) and raises its flag; before reloading its halo it waits for the
// flags of its (up to eight) neighbours only.  A tile whose own cells are all settled is
// final: it publishes them into both areas, sets its flag to kTileDone and leaves, so a team
// ends without a global step.  Every spin is bounded (a timeout marks the slot failed: the
// check then fails it and the SSSP kernel answers).
__global__ __launch_bounds__(kTileBS) void cert_tile_kernel(const KArgs *__restrict__ a) {
    __shared__ unsigned long long Sx[kTileN];      // the region's cells, kTileP a row (file comment)
    __shared__ uint16_t lst[4][kTileList];         // bucket lists (bucket j in lst[j & 3])
    __shared__ uint32_t cnt[4];
    __shared__ unsigned long long ev[kTileEv];     // fixed cells bordering window cells: own G << 14 | cell
    __shared__ uint16_t FD[kTileFD];               // f(k + 1) - f(k)
    __shared__ CertEntry E[64];
    __shared__ unsigned long long kbase[64];       // per boundary: RM << 34 | O_b << 6 | id
    __shared__ uint32_t gbase[64], legs_id[64];    // per boundary its G; per id its boundary's legs
    __shared__ uint8_t inv[64];                    // id -> table entry
    __shared__ uint32_t fixedb[kTileN / 32];       // cells that are not window plain cells
    __shared__ uint32_t jobs[64][2], njobs, nev, ev_ptr, flag, unset;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, P = gridDim.x;
    const uint32_t nslot = min(a->cert_cap, __hip_atomic_load(a->counter + kCtrCert, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT));
    if (tid == 0) {  // this workgroup's tiles, one a round
        uint32_t used = 0, n = 0;
        for (uint32_t s = 0; s < nslot; ++s) {
            const uint32_t *win = a->cert_win + (unsigned long long)s * kWinWords;
            if (win[kWinMode] != kWinTile || (a->cert_redo && !a->cert_redo[s])) continue;
            const uint32_t nt = win[kWinNtx] * win[kWinNty];
            if (used + nt > P) used = 0;  // the next round
            if (blockIdx.x >= used && blockIdx.x < used + nt && n < 64) {
                jobs[n][0] = s;
                jobs[n][1] = used;
                ++n;
            }
            used += nt;
        }
        njobs = n;
    }
    __syncthreads();
    const DevParams p = a->p;
    const int S = int(p.S), H = int(p.H);
    const uint32_t T = p.NS + 1, pitch = a->rec_pitch;
    const uint32_t L = p.perm[0];                      // the lead: legs (0) or time (2)
    const bool legs_lead = L == 0;
    const bool layout_b = p.perm[1] == 1u;             // money second
    const uint32_t W = legs_lead ? 1u : max(1u, p.W);
    constexpr uint32_t kEvWave = kTileBS / 64u - 1u;   // the wave that activates events (lists go to the others first)
    for (uint32_t i = tid; i < kTileFD; i += kTileBS)
        FD[i] = uint16_t(run_time_ff(i + 1, p.ff_num, p.ff_den) - run_time_ff(i, p.ff_num, p.ff_den));
    for (uint32_t jb = 0; jb < njobs; ++jb) {
        const uint32_t slot = jobs[jb][0], base = jobs[jb][1];
        uint32_t *win = a->cert_win + (unsigned long long)slot * kWinWords;
        const int bx0 = int(win[kWinX0]), by0 = int(win[kWinY0]), bx1 = int(win[kWinX1]), by1 = int(win[kWinY1]);
        const uint32_t ntx = win[kWinNtx], nty = win[kWinNty], nt = ntx * nty, B0 = win[kWinB0];
        const uint32_t ti = blockIdx.x - base, tx = ti % ntx, ty = ti / ntx;
        const bool single = nt == 1;
        CellWord *w = a->cert_rec + (unsigned long long)slot * p.S * pitch;
        // the tile's own cells and its LDS region (halo, clipped to the window's ring)
        const int ix0 = single ? bx0 : bx0 + int(tx * kTileT), iy0 = single ? by0 : by0 + int(ty * kTileT);
        const int ix1 = single ? bx1 : min(bx1, ix0 + int(kTileT) - 1), iy1 = single ? by1 : min(by1, iy0 + int(kTileT) - 1);
        const int hw = single ? 1 : int(kTileH);
        const int rx0 = max(max(0, bx0 - 1), ix0 - hw), rx1 = min(min(S - 1, bx1 + 1), ix1 + hw);
        const int ry0 = max(max(0, by0 - 1), iy0 - hw), ry1 = min(min(S - 1, by1 + 1), iy1 + hw);
        const uint32_t RW = uint32_t(rx1 - rx0 + 1), RH = uint32_t(ry1 - ry0 + 1), N = RH * kTileP;
        const uint32_t iw = uint32_t(ix1 - ix0 + 1), ih = uint32_t(iy1 - iy0 + 1);
        unsigned long long t_step = 0, t_xchg = 0, t_pub = 0, t_wait = 0;
        cert_load_table(a, slot, E);
        if (tid < 4) cnt[tid] = 0;
        if (tid == 0) {
            nev = 0;
            ev_ptr = 0;
            flag = 0;
        }
        __syncthreads();
        // keys: ranks of the boundaries (id unique: the lists differ), money ranks
        if (tid < 64) {
            const uint32_t t = tid;
            const bool bnd = t < T && (t == 0 || E[t].lex != kNone32);
            uint32_t id = 0, rm = 0;
            const uint32_t mo = E[t].m1, ln = t == 0 ? 1u : E[t].len + 1u, lx = E[t].lex;
            if (bnd)
                for (uint32_t u = 0; u < min(T, 64u); ++u) {
                    if (u == t || !(u == 0 || E[u].lex != kNone32)) continue;
                    const uint32_t mu = E[u].m1, lu = u == 0 ? 1u : E[u].len + 1u, xu = E[u].lex;
                    const bool lenlex = lu != ln ? lu < ln : xu < lx;
                    if (layout_b) {
                        id += lenlex ? 1u : 0u;
                        rm += mu < mo ? 1u : 0u;
                    } else {
                        id += (mu != mo ? mu < mo : lenlex) ? 1u : 0u;
                    }
                }
            if (bnd) {
                inv[id] = uint8_t(t);
                legs_id[id] = E[t].m0;
                const uint32_t ob = legs_lead ? E[t].m2 : E[t].m0;
                kbase[t] = ((unsigned long long)rm << 34) | ((unsigned long long)ob << 6) | id;
                gbase[t] = legs_lead ? E[t].m0 : E[t].m2;
            }
        }
        __syncthreads();
        // key of walk(b, k) (kTileNoExt when below B0 or far beyond the window's buckets)
        auto walk_key = [&](uint32_t b, uint32_t k) -> unsigned long long {
            const uint32_t fk = run_time_ff(k, p.ff_num, p.ff_den);
            const unsigned long long g = (unsigned long long)gbase[b] + (legs_lead ? k : fk);
            const unsigned long long o = legs_lead ? fk : k;
            if (g < B0 || g - B0 >= kTileGMax) return kTileNoExt;
            return ((g - B0) << 40) + kbase[b] + (o << 6);
        };
        auto in_win = [&](int x, int y) { return x >= bx0 && x <= bx1 && y >= by0 && y <= by1; };
        auto rid = [&](int x, int y) { return uint32_t(y - ry0) * kTileP + uint32_t(x - rx0); };
        // the region: window plain cells unsettled; every other cell fixed, holding the key
        // of its extension (cert_ext: a walk continues its run, a boundary starts one);
        // pad columns fixed with nothing to push
        for (uint32_t i = tid; i < kTileN / 32; i += kTileBS) fixedb[i] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < N; i += kTileBS) {
            const uint32_t lx = i & (kTileP - 1u);
            const int y = ry0 + int(i / kTileP), x = rx0 + int(lx);
            unsigned long long v = kTileNoExt;
            if (lx < RW && !(x == H && y == H)) {
                const uint32_t cw = cert_clean(w[(size_t)y * pitch + x]);
                const bool plain = cw != kViaSource && !(cw & kViaSpecial);
                if (plain && in_win(x, y)) v = ~0ull;
                else if (cw == kViaSource) v = walk_key(0, 1);
                else if (cw & kViaSpecial) {
                    const uint32_t t = cw & kNone10;
                    if (t < 64u && E[t].wb != kCertNoB) v = walk_key(E[t].wb, E[t].wk + 1u);
                    else if (t < 64u && E[t].lex != kNone32) v = walk_key(t, 1);
                } else {
                    const uint32_t b = (cw >> kStBShift) & kNone10;
                    if (b < 64u) v = walk_key(b, (cw & kStKMask) + 1u);
                }
            }
            Sx[i] = v;
            if (v != ~0ull) atomicOr(&fixedb[i >> 5], 1u << (i & 31u));
        }
        __syncthreads();
        // events: fixed cells with something to push and a window neighbour in the region,
        // by their own G (the extension's G less one step's increment)
        for (uint32_t i = tid; i < N; i += kTileBS) {
            const unsigned long long v = Sx[i];
            if ((v >> 63) || v == kTileNoExt) continue;
            const uint32_t lx = i & (kTileP - 1u), ly = i / kTileP;
            const bool nb = (lx > 0 && (Sx[i - 1] >> 63)) || (lx + 1 < RW && (Sx[i + 1] >> 63)) ||
                            (ly > 0 && (Sx[i - kTileP] >> 63)) || (ly + 1 < RH && (Sx[i + kTileP] >> 63));
            if (!nb) continue;
            const uint32_t gx = uint32_t(v >> 40), id = uint32_t(v & 63u);
            const uint32_t ox = uint32_t((v >> 6) & ((1u << 28) - 1u));
            const uint32_t k1 = (legs_lead ? gx + B0 : ox) - legs_id[id];  // the extension's run length
            const uint32_t d = legs_lead ? 1u : (k1 - 1u < kTileFD ? FD[k1 - 1u]
                                                                   : run_time_ff(k1, p.ff_num, p.ff_den) - run_time_ff(k1 - 1u, p.ff_num, p.ff_den));
            const uint32_t gown = gx >= d ? gx - d : 0u;
            const uint32_t at = atomicAdd(&nev, 1u);
            if (at < kTileEv) ev[at] = ((unsigned long long)gown << 14) | i;
        }
        __syncthreads();
        const uint32_t ne = min(nev, kTileEv);
        if (nev > kTileEv && tid == 0) atomicOr(win + kWinFail, 1u);
        {  // sort the events by own G (rank sort; a few hundred)
            unsigned long long mine[2] = {~0ull, ~0ull};
            uint32_t rk[2] = {0, 0};
            for (uint32_t r = 0; r < 2; ++r) {
                const uint32_t i = tid + r * kTileBS;
                if (i >= ne) continue;
                mine[r] = ev[i];
                for (uint32_t u = 0; u < ne; ++u) rk[r] += ev[u] < mine[r] ? 1u : 0u;
            }
            __syncthreads();
            for (uint32_t r = 0; r < 2; ++r)
                if (tid + r * kTileBS < ne) ev[rk[r]] = mine[r];
        }
        __syncthreads();
        // f(k + 1) - f(k): 180, or the Fleetfoot ceil by the plan's multiply-high (exact for
        // k <= 2 S + 256, checked on the host; ff_magic 1 when it could not be), else the table
        const bool lin = p.ff_num == p.ff_den, magic = p.ff_magic != 1u;
        auto run_inc = [&](uint32_t k) -> uint32_t {
            if (lin) return 180u;
            if (magic)
                return (__umulhi(p.ff_c * (k + 1u) + p.ff_den - 1u, p.ff_magic) >> p.ff_shift) -
                       (__umulhi(p.ff_c * k + p.ff_den - 1u, p.ff_magic) >> p.ff_shift);
            return k < kTileFD ? uint32_t(FD[k]) : run_time_ff(k + 1u, p.ff_num, p.ff_den) - run_time_ff(k, p.ff_num, p.ff_den);
        };
        // extension key x pushed from cell n (settled, or an event at step j) into its four
        // neighbours: the four minima in flight together, then the bucket lists
        auto push4 = [&](uint32_t n, unsigned long long x, uint32_t j) {
            const uint32_t lx = n & (kTileP - 1u), ly = n / kTileP;
            const unsigned long long xv = kTileHi | x;
            const uint32_t nn[4] = {n - 1u, n + 1u, n - kTileP, n + kTileP};
            const bool ok[4] = {lx > 0, lx + 1 < RW, ly > 0, ly + 1 < RH};
            unsigned long long old[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) old[q] = ok[q] ? atomicMin(&Sx[nn[q]], xv) : 0ull;
            const uint32_t gx = uint32_t(x >> 40);
            const uint32_t bx = gx < (j + 2u) * W ? j + 1u : j + 2u;
            bool need[4];
            uint32_t m = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // better, not settled or fixed, and not queued in that bucket already
                const uint32_t go = uint32_t((old[q] & ~kTileHi) >> 40);
                need[q] = ok[q] && xv < old[q] && (old[q] >> 63) &&
                          (old[q] == ~0ull || (go < (j + 2u) * W ? j + 1u : j + 2u) != bx);
                m += need[q] ? 1u : 0u;
            }
            if (m == 0) return;
            uint32_t at = atomicAdd(&cnt[bx & 3u], m);  // (one add for the cell's pushes)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (need[q]) {
                    if (at < kTileList) lst[bx & 3u][at] = uint16_t(nn[q]);
                    ++at;
                }
        };
        // settle region cell n (unsettled, candidate c of bucket j)
        auto settle = [&](uint32_t n, unsigned long long c, uint32_t j) {
            const uint32_t gx = uint32_t(c >> 40), id = uint32_t(c & 63u);
            const uint32_t ox = uint32_t((c >> 6) & ((1u << 28) - 1u));
            const uint32_t k = (legs_lead ? gx + B0 : ox) - legs_id[id];
            const uint32_t d = run_inc(k);
            const uint32_t dg = legs_lead ? 1u : d, dox = legs_lead ? d : 1u;
            unsigned long long x = c + ((unsigned long long)dg << 40) + ((unsigned long long)dox << 6);
            if (gx + dg >= kTileGMax) x = kTileNoExt;
            Sx[n] = x;
            if (x != kTileNoExt) push4(n, x, j);
        };
        uint32_t j = 0, blk = 0;
        bool failed = false;
        const uint32_t kdone = kTileDone, kfin = 0x80000000u;  // flag: exchanges published | final
        bool fin = false;  // this tile's cells are all settled (it only publishes them now)
        for (;;) {
            const uint32_t nsteps = single ? kTileMaxSteps : kTileH;
            bool done = false;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            if (fin) j += nsteps;
            for (uint32_t s = 0; s < nsteps && !fin; ++s, ++j) {
                const uint32_t bound = (j + 1u) * W;  // G - B0 below it: bucket j or earlier
                if (tid == 0) cnt[(j + 3u) & 3u] = 0;  // (the list of step j - 1)
                if ((tid >> 6) == kEvWave) {  // the events of bucket j (sorted: a prefix of those left)
                    uint32_t p0 = ev_ptr;
                    for (;;) {
                        const uint32_t idx = p0 + lane;
                        const bool take = idx < ne && (ev[idx] >> 14) < bound;
                        const unsigned long long bal = __ballot(take);
                        if (take) {
                            const uint32_t n = uint32_t(ev[idx] & 0x3FFFu);
                            push4(n, Sx[n], j);
                        }
                        const uint32_t c = uint32_t(__popcll(bal));
                        p0 += c;
                        if (c < 64u) break;
                    }
                    if (lane == 0) ev_ptr = p0;
                }
                const uint32_t nl = cnt[j & 3u];
                if (nl <= kTileList) {
                    for (uint32_t e = tid; e < nl; e += kTileBS) {
                        const uint32_t n = lst[j & 3u][e];
                        const unsigned long long v = Sx[n];
                        if (!(v >> 63) || v == ~0ull) continue;
                        const unsigned long long c = v & ~kTileHi;
                        if (uint32_t(c >> 40) >= bound) continue;
                        settle(n, c, j);
                    }
                } else {  // the list overflowed: every unsettled cell of the region
                    for (uint32_t n = tid; n < N; n += kTileBS) {
                        const unsigned long long v = Sx[n];
                        if (!(v >> 63) || v == ~0ull) continue;
                        const unsigned long long c = v & ~kTileHi;
                        if (uint32_t(c >> 40) >= bound) continue;
                        settle(n, c, j);
                    }
                }
                __syncthreads();
                if (cnt[(j + 1u) & 3u] == 0 && cnt[(j + 2u) & 3u] == 0) {
                    // nothing pending in the next two buckets: the next work is the next event
                    // (a single tile with none left is done); skip the empty steps up to it,
                    // within this exchange's steps (every read here is uniform)
                    if (single && ev_ptr >= ne) {
                        ++j;
                        done = true;
                        break;
                    }
                    const uint32_t jn = ev_ptr < ne ? uint32_t((ev[ev_ptr] >> 14) / W) : 0xFFFFFFFFu;
                    const uint32_t jend = j + (nsteps - s);  // the first step past this exchange's
                    const uint32_t jt = min(jn, jend);
                    if (jt > j + 1u && jt < kTileMaxSteps) {
                        if (tid == 0) cnt[j & 3u] = 0;  // (the other lists are empty)
                        s += jt - 1u - j;
                        j = jt - 1u;
                    }
                }
                if (j + 1u >= kTileMaxSteps) {
                    failed = true;
                    ++j;
                    break;
                }
            }
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            t_step += t1 - t0;
            if (single || failed) {
                if (!done) failed = true;
                break;
            }
            // are this tile's own cells final (every window cell settled)?
            if (!fin) {
                if (tid == 0) unset = 0;
                __syncthreads();
                uint32_t u = 0;
                for (uint32_t i = tid; i < iw * ih; i += kTileBS) {
                    const int y = iy0 + int(i / iw), x = ix0 + int(i % iw);
                    u |= (Sx[rid(x, y)] >> 63) ? 1u : 0u;
                }
                if (u) unset = 1;
                __syncthreads();
                fin = unset == 0;
            }
            // publish this tile's cells (write-through), then raise its flag behind every
            // wave's stores.  A final tile keeps publishing (its neighbours read each exchange's
            // state in its turn: never a later one) until every neighbour is final too.
            unsigned long long *pub = a->cert_pub + (unsigned long long)blockIdx.x * 2 * kTileT * kTileT;
            auto publish = [&](uint32_t par) {
                for (uint32_t i = tid; i < iw * ih; i += kTileBS) {
                    const int y = iy0 + int(i / iw), x = ix0 + int(i % iw);
                    __hip_atomic_store(pub + par * kTileT * kTileT + uint32_t(y - iy0) * kTileT + uint32_t(x - ix0), Sx[rid(x, y)],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            };
            publish(blk & 1u);
            const unsigned long long tp = __builtin_amdgcn_s_memrealtime();
            t_pub += tp - t1;
            if (tid == 0)
                __hip_atomic_store(win + kWinFlag + ti, (blk + 1u) | (fin ? kfin : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // wait for the neighbours' publications of this exchange (lanes 0..8 of wave 0)
            if (tid == 0) unset = 1;  // (reused: every neighbour final)
            __syncthreads();
            if (tid < 9 && tid != 4) {
                const int dx = int(tid % 3) - 1, dy = int(tid / 3) - 1;
                const int nx = int(tx) + dx, ny = int(ty) + dy;
                if (nx >= 0 && ny >= 0 && nx < int(ntx) && ny < int(nty)) {
                    const uint32_t *f = win + kWinFlag + uint32_t(ny) * ntx + uint32_t(nx);
                    uint32_t spins = 0, fv;
                    while (((fv = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & ~kfin) < blk + 1u) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > (1u << 22)) {  // (seconds: a neighbour never published)
                            flag = 1;
                            break;
                        }
                    }
                    if (!(fv & kfin)) unset = 0;
                }
            }
            __syncthreads();
            t_wait += __builtin_amdgcn_s_memrealtime() - tp;
            if (flag) {
                failed = true;
                if (tid == 0) __hip_atomic_store(win + kWinFlag + ti, kdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            if (fin && unset) {
                // final, and so is every neighbour: the next exchange's area gets this state too
                // (a neighbour reads it only after seeing kTileDone), then leave
                publish((blk + 1u) & 1u);
                if (tid == 0) __hip_atomic_store(win + kWinFlag + ti, kdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                t_xchg += __builtin_amdgcn_s_memrealtime() - t1;
                break;
            }
            if (fin) {  // (no halo to reload: this tile's cells are final)
                ++blk;
                t_xchg += __builtin_amdgcn_s_memrealtime() - t1;
                if (blk >= kTileMaxSteps / kTileH) {
                    failed = true;
                    break;
                }
                continue;
            }
            // reload the halo's window cells from their tiles' areas of this exchange, and
            // list those with a candidate (a stale entry of this tile's own is harmless: a
            // listed cell is settled only if its candidate lies in the step's bucket)
            const unsigned long long *src = a->cert_pub + (blk & 1u) * kTileT * kTileT;
            constexpr uint32_t kB = 8;  // loads in flight per thread
            for (uint32_t i0 = 0; i0 < N; i0 += kTileBS * kB) {
                const unsigned long long *ad[kB];
                uint32_t ci[kB];
#pragma unroll
                for (uint32_t r = 0; r < kB; ++r) {
                    const uint32_t i = i0 + r * kTileBS + tid;
                    const uint32_t lx = i & (kTileP - 1u);
                    const int y = ry0 + int(i / kTileP), x = rx0 + int(lx);
                    ci[r] = kNone32;
                    ad[r] = nullptr;
                    if (i >= N || lx >= RW || !in_win(x, y) || (x >= ix0 && x <= ix1 && y >= iy0 && y <= iy1)) continue;
                    const uint32_t ox = uint32_t(x - bx0) / kTileT, oy = uint32_t(y - by0) / kTileT;
                    ad[r] = src + (unsigned long long)(base + oy * ntx + ox) * 2 * kTileT * kTileT +
                            (uint32_t(y - by0) - oy * kTileT) * kTileT + (uint32_t(x - bx0) - ox * kTileT);
                    ci[r] = i;
                }
                unsigned long long v[kB];
#pragma unroll
                for (uint32_t r = 0; r < kB; ++r)
                    v[r] = ci[r] != kNone32 ? __hip_atomic_load(ad[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
#pragma unroll
                for (uint32_t r = 0; r < kB; ++r) {
                    if (ci[r] == kNone32) continue;
                    Sx[ci[r]] = v[r];
                    if (!(v[r] >> 63) || v[r] == ~0ull) continue;
                    const uint32_t g = uint32_t((v[r] & ~kTileHi) >> 40);
                    const uint32_t bk = g < (j + 1u) * W ? j : j + 1u;
                    const uint32_t at = atomicAdd(&cnt[bk & 3u], 1u);
                    if (at < kTileList) lst[bk & 3u][at] = uint16_t(ci[r]);
                }
            }
            __syncthreads();
            // The halo ring next to this tile's cells was exact only until the block's last
            // step (an error at the region's edge reaches distance H - 1 by step H), so a push
            // it made then into a border cell of this tile may be wrong, and with a Fleetfoot
            // ceil a wrong label can extend to a smaller key.  So every unsettled border cell's
            // candidate is rebuilt from its neighbours, now exact: the settled window cells,
            // and the fixed cells whose event has fired (own bucket before step j).
            {
                const uint32_t per = 2u * (iw + ih);
                for (uint32_t e = tid; e < per; e += kTileBS) {
                    int x, y;
                    if (e < iw) { x = ix0 + int(e); y = iy0; }
                    else if (e < 2u * iw) { x = ix0 + int(e - iw); y = iy1; }
                    else if (e < 2u * iw + ih) { x = ix0; y = iy0 + int(e - 2u * iw); }
                    else { x = ix1; y = iy0 + int(e - 2u * iw - ih); }
                    const uint32_t c = rid(x, y);
                    const unsigned long long cur = Sx[c];
                    if (!(cur >> 63)) continue;  // settled or fixed
                    unsigned long long best = ~0ull;
                    const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (nx[q] < rx0 || nx[q] > rx1 || ny[q] < ry0 || ny[q] > ry1) continue;
                        const uint32_t n = rid(nx[q], ny[q]);
                        const unsigned long long v = Sx[n];
                        if ((v >> 63) || v == kTileNoExt) continue;
                        if ((fixedb[n >> 5] >> (n & 31u)) & 1u) {  // a fixed cell: has its event fired?
                            const uint32_t gx = uint32_t(v >> 40), id = uint32_t(v & 63u);
                            const uint32_t ox = uint32_t((v >> 6) & ((1u << 28) - 1u));
                            const uint32_t k1 = (legs_lead ? gx + B0 : ox) - legs_id[id];
                            const uint32_t d = legs_lead ? 1u : run_inc(k1 - 1u);
                            if ((gx >= d ? gx - d : 0u) >= j * W) continue;
                        }
                        best = min(best, kTileHi | v);
                    }
                    if (best == cur) continue;
                    Sx[c] = best;
                    if (best == ~0ull) continue;
                    const uint32_t g = uint32_t((best & ~kTileHi) >> 40);
                    const uint32_t bk = g < (j + 1u) * W ? j : j + 1u;
                    const uint32_t go = uint32_t((cur & ~kTileHi) >> 40);
                    if (cur != ~0ull && (go < (j + 1u) * W ? j : j + 1u) == bk) continue;  // listed there already
                    const uint32_t at = atomicAdd(&cnt[bk & 3u], 1u);
                    if (at < kTileList) lst[bk & 3u][at] = uint16_t(c);
                }
            }
            __syncthreads();
            ++blk;
            t_xchg += __builtin_amdgcn_s_memrealtime() - t1;
        }
        if (failed && tid == 0) {
            atomicOr(win + kWinFail, 1u);
            __hip_atomic_store(win + kWinFlag + ti, kdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) {
            atomicMax(win + kWinSteps, j);
            if (ti == 0) {
                win[kWinTStep] = uint32_t(t_step);
                win[kWinTXchg] = uint32_t(t_xchg);
                win[kWinNXchg] = blk;
            }
            if (ti < kTileMaxTiles) {
                win[kWinStat + 4 * ti] = uint32_t(t_step);
                win[kWinStat + 4 * ti + 1] = uint32_t(t_xchg);
                win[kWinStat + 4 * ti + 2] = uint32_t(t_pub) << 16 | min(uint32_t(t_wait), 0xFFFFu);
                win[kWinStat + 4 * ti + 3] = j;
            }
        }
        // the tile's settled window cells back as walk words (b, k): the key of the
        // extension names walk(b, k + 1); marks come off, unsettled cells keep their word
        for (uint32_t i = tid; i < iw * ih; i += kTileBS) {
            const int y = iy0 + int(i / iw), x = ix0 + int(i % iw);
            CellWord *pw = w + (size_t)y * pitch + x;
            const uint32_t cw = *pw;
            if (cw == kViaSource || (cw & kViaSpecial) || (x == H && y == H)) continue;
            const unsigned long long v = Sx[rid(x, y)];
            if ((v >> 63) || v == kTileNoExt) {
                *pw = cw & ~kCertDirty;
                continue;
            }
            const uint32_t gx = uint32_t(v >> 40), id = uint32_t(v & 63u), b = inv[id];
            const uint32_t ox = uint32_t((v >> 6) & ((1u << 28) - 1u));
            const uint32_t k1 = (legs_lead ? gx + B0 : ox) - legs_id[id];
            *pw = (b << kStBShift) | (k1 - 1u);
        }
        __syncthreads();
    }
}

// Between the two rounds (one wave per slot): a demoted special whose repaired walk a
// caravan beats (the last check named the hub, kWinPromo) gets that caravan as its label
// (src/pathfinder.rs:141-160, TotalCost += Caravan, src/cost.rs:208-315), becomes a
// boundary (its cell word names its own entry again), and the boundaries' ranks by
// (length, command list) are taken again.  The slot is then redone: closed form, check,
// repair, check (cert_redo[slot] = 1); the check fails every entry the hub built on a
// promoted one.  Other slots keep their result (cert_redo[slot] = 0).
__global__ __launch_bounds__(64) void cert_promote_kernel(const KArgs *__restrict__ a, uint32_t *redo) {
    __shared__ Rec R[64];
    __shared__ uint32_t lex[64];
    __shared__ uint32_t prom_lo, prom_hi;
    const uint32_t slot = blockIdx.x, lane = threadIdx.x;
    uint32_t *win = a->cert_win + (unsigned long long)slot * kWinWords;
    const uint32_t nslot = min(a->cert_cap, __hip_atomic_load(a->counter + kCtrCert, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t T = a->p.NS + 1;
    const uint32_t promo = slot < nslot && T <= 64u && lane < T ? win[kWinPromo + lane] : 0u;
    const unsigned long long any = __ballot(promo != 0u);
    // a slot whose last check still failed sweeps again from its repaired words, over the
    // failing cells' box with a wider margin (specials that check demoted become plain)
    uint32_t nf = 0;
    if (slot < nslot && !any)
        for (uint32_t j = lane; j < a->cert_parts; j += 64)
            nf |= a->cert_st[((unsigned long long)slot * a->cert_parts + j) * kCertSt + kCertFails];
    const bool again = __ballot(nf != 0u) != 0ull;
    if (lane == 0) redo[slot] = any ? kRedoFill : (again ? kRedoSweep : 0u);
    if (!any) return;
    const unsigned long long tb = (unsigned long long)slot * T;
    if (lane < T) {
        R[lane] = a->cert_tab[tb + lane];
        lex[lane] = a->cert_lex[tb + lane];
    }
    if (lane == 0) {
        prom_lo = win[kWinProm0] | uint32_t(any);
        prom_hi = win[kWinProm1] | uint32_t(any >> 32);
    }
    wave_sync();
    const DevParams p = a->p;
    const SpecialStatic *sp = a->sp;
    if (promo) {
        const uint32_t t = lane, h = promo - 1u;
        const Rec rh = R[h];
        const SpecialStatic st = sp[t], sh = sp[h];
        const uint32_t d = uint32_t(abs(sh.x - st.x) + abs(sh.y - st.y)), coef = st.coef5 ? 5u : 2u;
        const uint32_t kp = (kCaravan << 29) | (d << 1) | st.coef5;
        Rec r;
        if ((rh.kp0 >> 29) == kNoMove) {  // from the start label: the NoMove is replaced
            r.m[0] = 0;
            r.m[1] = coef * d;
            r.m[2] = p.rgt * d;
            r.meta = Rec::pack(1, 0, 1, 2);
            r.from0 = rh.from0;
        } else {
            r.m[0] = rh.m[0];
            r.m[1] = rh.m[1] + coef * d;
            r.m[2] = rh.m[2] + p.rgt * d;
            r.meta = Rec::pack(rh.len() + 1u, h, 1, 2);
            r.from0 = sh.rk;
        }
        r.kp0 = kp;
        r.u = st.rk;
        R[t] = r;
        // its cell names its own entry again (a boundary)
        const uint32_t v = st.v, y = v / p.S;
        a->cert_rec[(unsigned long long)slot * p.S * a->rec_pitch + (size_t)y * a->rec_pitch + (v - y * p.S)] = kViaSpecial | t;
    }
    wave_sync();
    // the boundaries' ranks by (length, command list), the source first (export_cert in
    // mr_device.hpp): lists of equal length compare from their first differing command,
    // found walking both chains back from the end
    auto tail = [&](uint32_t e, int i) -> Cmd {
        const Rec &r = R[e];
        return i == 0 ? Cmd{r.kp0, r.from0, r.u} : Cmd{kSoE << 29, r.u, sp[e].rk};
    };
    auto cmp_lists = [&](uint32_t x, uint32_t y) -> int {
        uint32_t xe = x, ye = y;
        int xt = int(R[x].ntail()) - 1, yt = int(R[y].ntail()) - 1, res = 0;
        for (uint32_t guard = 0; guard < 4096u; ++guard) {
            if (xe == ye && xt == yt) return res;
            const Cmd cx = tail(xe, xt), cy = tail(ye, yt);
            if (cx.kp != cy.kp) res = cx.kp < cy.kp ? -1 : 1;
            else if (cx.from != cy.from) res = cx.from < cy.from ? -1 : 1;
            else if (cx.to != cy.to) res = cx.to < cy.to ? -1 : 1;
            if (xt > 0) --xt;
            else {
                const uint32_t pp = R[xe].parent();
                if (pp == 0) return res;
                xe = pp;
                xt = int(R[pp].ntail()) - 1;
            }
            if (yt > 0) --yt;
            else {
                const uint32_t pp = R[ye].parent();
                if (pp == 0) return res;
                ye = pp;
                yt = int(R[pp].ntail()) - 1;
            }
        }
        return res;
    };
    const bool bnd = lane < T && (lane == 0 || lex[lane] != kNone32 || promo != 0u);
    uint32_t r = kNone32;
    if (bnd) {
        r = 0;
        for (uint32_t i = 0; i < T; ++i) {
            if (i == lane || !(i == 0 || lex[i] != kNone32 || ((any >> i) & 1ull))) continue;
            bool less;
            if (i == 0 || lane == 0) less = i == 0;
            else if (R[i].len() != R[lane].len()) less = R[i].len() < R[lane].len();
            else less = cmp_lists(i, lane) < 0;
            r += less ? 1u : 0u;
        }
    }
    wave_sync();
    if (lane < T) {
        a->cert_lex[tb + lane] = r;
        if (promo) a->cert_tab[tb + lane] = R[lane];
    }
    if (lane == 0) {
        win[kWinProm0] = prom_lo;
        win[kWinProm1] = prom_hi;
    }
}

}  // namespace mr
