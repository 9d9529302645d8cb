// mr_oracle.cpp — TEST INFRASTRUCTURE ONLY (see mr_oracle.h).
//
// A line-by-line *semantic* restatement of the reference pathfinder in C++:
// full path labels (TotalCost with its command vector), a binary min-heap of
// labels ordered by the user comparator, a hash map `dist`, lazy deletion and
// early exit — the same algorithm and data-structure shape as
// src/pathfinder.rs:199-248.  Nothing here is used by the product library.
//
// Widening: coordinates/pos/shift are 16-bit (reference: i8/u8) so grids above
// S = 255 can be checked; for S <= 255 behaviour is the reference's.
#include "mr_oracle.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <queue>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace mro {

// ---------------------------------------------------------------- CellIndex
// src/index.rs:41-46.  Derived Ord = (variant, fields...).  We keep the
// canonical form: Center {0,0,0}; Homeland {sub=homeland, x, y}; Border
// {sub=border, x=shift, y=0}; so a tuple compare is the derived Ord.
struct CellIndex {
    uint8_t kind = MR_CELL_CENTER, sub = 0;
    uint16_t x = 0, y = 0;
    auto key() const { return std::make_tuple(kind, sub, x, y); }
    bool operator==(const CellIndex &o) const { return key() == o.key(); }
    bool operator!=(const CellIndex &o) const { return !(*this == o); }
    bool operator<(const CellIndex &o) const { return key() < o.key(); }
};
struct CellIndexHash {
    size_t operator()(const CellIndex &c) const {
        return (size_t(c.kind) << 40) ^ (size_t(c.sub) << 32) ^ (size_t(c.x) << 16) ^ c.y;
    }
};
static CellIndex center() { return CellIndex{}; }
static int cmp_ci(const CellIndex &a, const CellIndex &b) { return a < b ? -1 : (b < a ? 1 : 0); }

enum Homeland : uint8_t { Blue = 0, Red = 1, Green = 2, Yellow = 3 };
enum Border : uint8_t { BR = 0, RG = 1, GY = 2, YB = 3 };
enum Dir : uint8_t { Horizontal = 0, Vertical = 1 };

// CellIndexBuilder::build (src/index.rs:257-312) — canonicalisation.
static CellIndex build_homeland(uint8_t h, int x, int y) {
    CellIndex c;
    if (x == 0 && y == 0) return center();
    if (x == 0) {  // Yellow/Blue -> YB y ; Red/Green -> RG y
        c.kind = MR_CELL_BORDER;
        c.sub = (h == Yellow || h == Blue) ? YB : RG;
        c.x = uint16_t(y);
        return c;
    }
    if (y == 0) {  // Blue/Red -> BR x ; Green/Yellow -> GY x
        c.kind = MR_CELL_BORDER;
        c.sub = (h == Blue || h == Red) ? BR : GY;
        c.x = uint16_t(x);
        return c;
    }
    c.kind = MR_CELL_HOMELAND;
    c.sub = h;
    c.x = uint16_t(x);
    c.y = uint16_t(y);
    return c;
}
static CellIndex build_border(uint8_t b, int shift) {
    if (shift == 0) return center();
    CellIndex c;
    c.kind = MR_CELL_BORDER;
    c.sub = b;
    c.x = uint16_t(shift);
    return c;
}
static CellIndex build_any(const mr_cell_index &m) {
    if (m.kind == MR_CELL_HOMELAND) return build_homeland(m.sub, m.x, m.y);
    if (m.kind == MR_CELL_BORDER) return build_border(m.sub, m.x);
    return center();
}
static bool valid_input(const mr_cell_index &m) {
    if (m.reserved != 0) return false;
    if (m.kind == MR_CELL_CENTER) return m.sub == 0 && m.x == 0 && m.y == 0;
    if (m.kind == MR_CELL_HOMELAND) return m.sub < 4;
    if (m.kind == MR_CELL_BORDER) return m.sub < 4 && m.y == 0;
    return false;
}
static mr_cell_index to_mr(const CellIndex &c) {
    mr_cell_index m;
    m.kind = c.kind;
    m.sub = c.sub;
    m.x = c.x;
    m.y = c.y;
    m.reserved = 0;
    return m;
}

// Border::neighbours / direction (src/index.rs:339-353)
static void border_neighbours(uint8_t b, uint8_t out[2]) {
    static const uint8_t t[4][2] = {{Blue, Red}, {Red, Green}, {Green, Yellow}, {Yellow, Blue}};
    out[0] = t[b][0];
    out[1] = t[b][1];
}
static Dir border_direction(uint8_t b) { return (b == BR || b == GY) ? Horizontal : Vertical; }
// Homeland::border (src/homeland.rs:66-82)
static uint8_t homeland_border(uint8_t h, Dir d) {
    static const uint8_t t[4][2] = {{BR, YB}, {BR, RG}, {GY, RG}, {GY, YB}};
    return t[h][d];
}
static uint8_t homeland_farland(uint8_t h) {  // src/homeland.rs:89-96
    static const uint8_t t[4] = {Green, Yellow, Blue, Red};
    return t[h];
}
static uint8_t homeland_neighbour(uint8_t h, Dir d) {  // src/homeland.rs:66-77,84-87
    static const uint8_t t[4][2] = {{Red, Yellow}, {Blue, Green}, {Yellow, Red}, {Green, Blue}};
    return t[h][d];
}

// ---------------------------------------------------------------- skills
// Skill::time (src/skill.rs:21-30): ratio==1 -> t; else ceil(ratio*t).
// Out-of-range level -> None (callers then use the raw time).
struct Ratio {
    int64_t n, d;
};
static std::optional<Ratio> route_guru_ratio(uint32_t v) {  // src/skill.rs:43-52
    switch (v) {
        case 0: return Ratio{1, 1};
        case 1: return Ratio{19, 24};
        case 2: return Ratio{7, 10};
        case 3: return Ratio{73, 120};
        case 4: return Ratio{31, 60};
        case 5: return Ratio{51, 120};
        default: return std::nullopt;
    }
}
static std::optional<Ratio> fleetfoot_ratio(uint32_t v) {  // src/skill.rs:65-71
    switch (v) {
        case 0: return Ratio{1, 1};
        case 1: return Ratio{50, 53};
        case 2: return Ratio{100, 109};
        case 3: return Ratio{25, 28};
        default: return std::nullopt;
    }
}
static std::optional<int64_t> skill_time(std::optional<Ratio> r, int64_t t) {
    if (!r) return std::nullopt;
    if (r->n == r->d) return t;
    // num-rational 0.4: Ratio * int is exact; ceil() for non-negative = (n+d-1)/d
    int64_t n = r->n * t, d = r->d;
    if (n >= 0) return (n + d - 1) / d;
    return n / d;
}

// ---------------------------------------------------------------- costs
// EdgeCost (src/cost.rs:11-20) and AggregatedCost (src/cost.rs:90-110).
enum Kind : uint8_t { NoMove = 0, Central = 1, Standard = 2, Caravan = 3, SoE = 4, SHQ = 5, SFm = 6 };

struct EdgeCost {
    Kind kind;
    int64_t car_time = 0;   // CaravanCost.time
    uint32_t car_money = 0; // CaravanCost.money
};
// EdgeCost::legs/money/time (src/cost.rs:35-74)
static uint32_t edge_legs(const EdgeCost &e) { return e.kind == Standard ? 1u : 0u; }
static uint32_t edge_money(const EdgeCost &e, uint32_t soe, uint32_t shq, uint32_t sfm) {
    switch (e.kind) {
        case Caravan: return e.car_money;
        case SoE: return soe;
        case SHQ: return shq;
        case SFm: return sfm;
        default: return 0;
    }
}
static int64_t edge_time(const EdgeCost &e) {
    switch (e.kind) {
        case Standard: return 180;
        case Central: return 10;
        case Caravan: return e.car_time;
        default: return 0;
    }
}

struct Agg {
    Kind kind = NoMove;
    int64_t time = 0;
    uint32_t legs = 0, money = 0, fleetfoot = 0;
};
// derived Ord of AggregatedCost: variant, then the variant's fields in order.
static int cmp_agg(const Agg &a, const Agg &b) {
    if (a.kind != b.kind) return a.kind < b.kind ? -1 : 1;
    auto c3 = [](auto x, auto y) { return x < y ? -1 : (y < x ? 1 : 0); };
    int r = 0;
    switch (a.kind) {
        case NoMove: return 0;
        case Central: return c3(a.time, b.time);
        case Standard:
            if ((r = c3(a.time, b.time))) return r;
            if ((r = c3(a.legs, b.legs))) return r;
            return c3(a.fleetfoot, b.fleetfoot);
        case Caravan:
            if ((r = c3(a.time, b.time))) return r;
            return c3(a.money, b.money);
        default: return c3(a.money, b.money);
    }
}
// AggregatedCost::time/money/legs (src/cost.rs:112-151)
static int64_t agg_time(const Agg &a) {
    switch (a.kind) {
        case Central:
        case Caravan: return a.time;
        case Standard: {
            auto t = skill_time(fleetfoot_ratio(a.fleetfoot), a.time);
            return t ? *t : a.time;
        }
        default: return 0;
    }
}
static uint32_t agg_money(const Agg &a) {
    switch (a.kind) {
        case Caravan:
        case SoE:
        case SHQ:
        case SFm: return a.money;
        default: return 0;
    }
}
static uint32_t agg_legs(const Agg &a) { return a.kind == Standard ? a.legs : 0; }

// From<(EdgeCost,u32,u32,u32,Fleetfoot)> for AggregatedCost (src/cost.rs:153-185)
static Agg agg_from_edge(const EdgeCost &e, uint32_t soe, uint32_t shq, uint32_t sfm, uint32_t ff) {
    Agg a;
    a.kind = e.kind;
    switch (e.kind) {
        case NoMove: break;
        case Central: a.time = edge_time(e); break;
        case Standard:
            a.legs = edge_legs(e);
            a.time = edge_time(e);
            a.fleetfoot = ff;
            break;
        case Caravan:
            a.time = e.car_time;
            a.money = e.car_money;
            break;
        case SoE: a.money = soe; break;
        case SHQ: a.money = shq; break;
        case SFm: a.money = sfm; break;
    }
    return a;
}

struct Command {  // src/cost.rs:83-88, derived Ord (agg, from, to)
    Agg agg;
    CellIndex from, to;
};
static int cmp_cmd(const Command &a, const Command &b) {
    int r = cmp_agg(a.agg, b.agg);
    if (r) return r;
    if ((r = cmp_ci(a.from, b.from))) return r;
    return cmp_ci(a.to, b.to);
}

struct TotalCost {  // src/cost.rs:187-206
    uint32_t legs = 0, money = 0;
    int64_t time = 0;
    std::vector<Command> commands;
};
static TotalCost total_new(const CellIndex &from) {  // TotalCost::new
    TotalCost t;
    Command c;
    c.agg.kind = NoMove;
    c.from = from;
    c.to = from;
    t.commands.push_back(c);
    return t;
}

// AddAssign<(EdgeCost,..,from,to)> for TotalCost (src/cost.rs:208-315)
static void total_add_assign(TotalCost &self, const EdgeCost &edge, uint32_t soe, uint32_t shq,
                             uint32_t sfm, uint32_t ff, const CellIndex &from, const CellIndex &to) {
    uint32_t legs = edge_legs(edge);
    uint32_t money = edge_money(edge, soe, shq, sfm);
    int64_t time = edge_time(edge);
    Agg agg;
    CellIndex cfrom;
    const Command *last = self.commands.empty() ? nullptr : &self.commands.back();
    if (last && last->agg.kind == NoMove) {
        agg = agg_from_edge(edge, soe, shq, sfm, ff);
        cfrom = last->from;
        self.commands.pop_back();
    } else if (last && last->agg.kind == Standard && edge.kind == Standard) {
        agg.kind = Standard;
        agg.legs = last->agg.legs + legs;
        agg.time = last->agg.time + time;
        agg.fleetfoot = last->agg.fleetfoot;
        cfrom = last->from;
        self.commands.pop_back();
    } else if (last && last->agg.kind == Central && edge.kind == Central) {
        agg.kind = Central;
        agg.time = last->agg.time + time;
        cfrom = last->from;
        self.commands.pop_back();
    } else {
        agg.kind = edge.kind;
        switch (edge.kind) {
            case NoMove: break;
            case Central: agg.time = time; break;
            case Standard:
                agg.time = time;
                agg.legs = legs;
                agg.fleetfoot = ff;
                break;
            case Caravan:
                agg.time = time;
                agg.money = money;
                break;
            default: agg.money = money; break;
        }
        cfrom = from;
    }
    Command c;
    c.agg = agg;
    c.from = cfrom;
    c.to = to;
    self.commands.push_back(c);
    // recompute (legs, money, time) as sums over all commands (:299-313);
    // u32 sums wrap as in a release build.
    uint32_t l = 0, m = 0;
    int64_t t = 0;
    for (const auto &cmd : self.commands) {
        l += agg_legs(cmd.agg);
        m += agg_money(cmd.agg);
        t += agg_time(cmd.agg);
    }
    self.legs = l;
    self.money = m;
    self.time = t;
}

// ---------------------------------------------------------------- comparator
enum CC : uint8_t { CLegs = 0, CTime = 1, CMoney = 2 };
static CC probable_second_target(CC c) {  // src/cost.rs:379-385
    return c == CLegs ? CTime : CLegs;
}
static void eval_next(CC self, CC c, CC &c2, CC &c3) {  // src/cost.rs:387-405
    c2 = (self == c) ? probable_second_target(c) : c;
    if (self == CLegs && c2 == CTime) c3 = CMoney;
    else if (self == CLegs && c2 == CMoney) c3 = CTime;
    else if (self == CTime && c2 == CLegs) c3 = CMoney;
    else if (self == CTime && c2 == CMoney) c3 = CLegs;
    else if (self == CMoney && c2 == CLegs) c3 = CTime;
    else c3 = CLegs;  // (Money, Time)
}
struct Comparator {  // CostComparator::and_then (src/cost.rs:411-426)
    CC c[3];
    static int metric(const TotalCost &a, const TotalCost &b, CC c) {
        switch (c) {
            case CLegs: return a.legs < b.legs ? -1 : (a.legs > b.legs ? 1 : 0);
            case CMoney: return a.money < b.money ? -1 : (a.money > b.money ? 1 : 0);
            default: return a.time < b.time ? -1 : (a.time > b.time ? 1 : 0);
        }
    }
    int operator()(const TotalCost &a, const TotalCost &b) const {
        for (int i = 0; i < 3; ++i) {
            int r = metric(a, b, c[i]);
            if (r) return r;
        }
        if (a.commands.size() != b.commands.size()) return a.commands.size() < b.commands.size() ? -1 : 1;
        for (size_t i = 0; i < a.commands.size(); ++i) {
            int r = cmp_cmd(a.commands[i], b.commands[i]);
            if (r) return r;
        }
        return 0;
    }
};
static Comparator make_comparator(uint8_t s1, uint8_t s2) {
    Comparator cmp;
    cmp.c[0] = CC(s1);
    eval_next(CC(s1), CC(s2), cmp.c[1], cmp.c[2]);
    return cmp;
}

// ---------------------------------------------------------------- grid
struct Cell {  // src/cell.rs:23-36 (only the path-relevant fields)
    CellIndex index;
    uint8_t poi = MR_POI_NONE;
    int32_t x = 0, y = 0;  // reference: i8 (widened)
    std::optional<CellIndex> nearest_campfire[4];
};
// Cell::distance / manhattan_distance (src/cell.rs:172-190)
static uint64_t distance(const Cell &a, const Cell &b) {
    return uint64_t(std::llabs(int64_t(a.x) - b.x) + std::llabs(int64_t(a.y) - b.y));
}

}  // namespace mro

struct mro_grid {
    uint32_t square_size = 0;
    std::vector<mro::Cell> grid;                                           // row-major
    std::unordered_map<mro::CellIndex, size_t, mro::CellIndexHash> index;  // src/grid.rs:35
    std::unordered_set<mro::CellIndex, mro::CellIndexHash> campfires;      // poi[PoI::Campfire]
    std::vector<mro::CellIndex> campfires_sorted;                          // deterministic iteration
    size_t homeland_size() const { return square_size / 2; }              // src/grid.rs:280-282
    const mro::Cell *at(const mro::CellIndex &c) const {
        auto it = index.find(c);
        return it == index.end() ? nullptr : &grid[it->second];
    }
};

namespace mro {

// nearest_campfire (src/grid.rs:297-325)
static std::optional<CellIndex> nearest_campfire(const CellIndex &from, uint8_t h,
                                                 const std::vector<std::pair<int, int>> &campfires,
                                                 const mro_grid &g) {
    if (from.kind == MR_CELL_HOMELAND && from.sub == h) {
        for (auto &p : campfires)
            if (p.first == from.x && p.second == from.y) return from;
    }
    const Cell *fc = g.at(from);
    std::optional<CellIndex> best;
    std::tuple<uint64_t, bool, uint64_t, uint64_t, uint64_t> best_key;
    for (auto &p : campfires) {
        CellIndex ci = build_homeland(h, p.first, p.second);
        const Cell *cc = g.at(ci);
        uint64_t x = uint64_t(std::llabs(cc->x)), y = uint64_t(std::llabs(cc->y));
        auto key = std::make_tuple(distance(*fc, *cc), x != y, x + y, x, y);
        if (!best || key < best_key) {  // min_by_key: first minimum
            best = cc->index;
            best_key = key;
        }
    }
    return best;
}

static size_t xy_to_i(long hs, size_t s, long x, long y) {  // src/grid.rs:293-295
    return size_t(x + hs) + size_t(y + hs) * s;
}

}  // namespace mro

using namespace mro;

static thread_local std::string g_err;

extern "C" int mro_grid_create(const mr_cell *cells, uint32_t n_cells, mro_grid **out) {
    if (!cells || !out) return MR_ERR_INVALID_ARG;
    *out = nullptr;
    // MapGrid::parse (src/grid.rs:47-237), starting from the parsed cells.
    uint64_t s = 0;
    while ((s + 1) * (s + 1) <= n_cells) ++s;
    if (s * s != n_cells || s == 0) return MR_ERR_INVALID_GRID;  // :60-63
    auto g = new mro_grid();
    g->square_size = uint32_t(s);
    long max_coord = long(s / 2);
    long x = -max_coord, y = -max_coord;  // scan (:68-77)
    g->grid.resize(n_cells);
    for (uint32_t i = 0; i < n_cells; ++i) {
        if (x == max_coord + 1) {
            x = -max_coord;
            y += 1;
        }
        if (!valid_input(cells[i].index) || cells[i].poi > MR_POI_FORUM) {
            delete g;
            return MR_ERR_INVALID_GRID;
        }
        Cell &c = g->grid[i];
        c.index = build_any(cells[i].index);  // CellIndex parse builds canonically
        c.poi = cells[i].poi;
        c.x = int32_t(x);
        c.y = int32_t(y);
        g->index[c.index] = i;  // collect(): a later duplicate wins
        x += 1;
    }
    auto it = g->index.find(center());  // :122-133
    if (it == g->index.end() || g->grid[it->second].x != 0 || g->grid[it->second].y != 0) {
        delete g;
        return MR_ERR_INVALID_GRID;
    }
    // poi sets (:134-154)
    std::vector<std::pair<int, int>> by_h[4];
    for (auto &c : g->grid) {
        if (c.poi != MR_POI_CAMPFIRE) continue;
        g->campfires.insert(c.index);
        if (c.index.kind == MR_CELL_HOMELAND) by_h[c.index.sub].push_back({c.index.x, c.index.y});
    }
    g->campfires_sorted.assign(g->campfires.begin(), g->campfires.end());
    std::sort(g->campfires_sorted.begin(), g->campfires_sorted.end());
    // nearest campfire per homeland via the reference's projection shortcut (:155-230)
    for (uint8_t h = 0; h < 4; ++h) {
        const auto &cf = by_h[h];
        uint8_t farland = homeland_farland(h);
        uint8_t vert_border = homeland_border(h, Vertical), vert_neighbour = homeland_neighbour(h, Vertical);
        uint8_t hor_border = homeland_border(h, Horizontal), hor_neighbour = homeland_neighbour(h, Horizontal);
        std::unordered_map<CellIndex, CellIndex, CellIndexHash> cached;
        auto cache_one = [&](const CellIndex &ci) {
            if (!g->at(ci)) return;
            auto nc = nearest_campfire(ci, h, cf, *g);
            if (nc) cached[ci] = *nc;
        };
        for (uint8_t b : {vert_border, hor_border})
            for (long sh = 1; sh <= max_coord; ++sh) cache_one(build_border(b, int(sh)));
        cache_one(center());
        for (auto &cell : g->grid) {
            std::optional<CellIndex> r;
            auto hit = cached.find(cell.index);
            if (hit != cached.end()) {
                r = hit->second;
            } else {
                long px, py;
                const CellIndex &ci = cell.index;
                if (ci.kind == MR_CELL_HOMELAND && ci.sub == h) { px = cell.x; py = cell.y; }
                else if (ci.kind == MR_CELL_HOMELAND && ci.sub == vert_neighbour) { px = 0; py = cell.y; }
                else if (ci.kind == MR_CELL_HOMELAND && ci.sub == hor_neighbour) { px = cell.x; py = 0; }
                else if (ci.kind == MR_CELL_HOMELAND && ci.sub == farland) { px = 0; py = 0; }
                else if (ci.kind == MR_CELL_BORDER && ci.sub != vert_border && ci.sub != hor_border) { px = 0; py = 0; }
                else {
                    // unreachable!() in the reference (only reachable for inconsistent maps)
                    delete g;
                    return MR_ERR_INVALID_GRID;
                }
                size_t pi = xy_to_i(max_coord, s, px, py);
                CellIndex pidx = g->grid[pi].index;
                auto h2 = cached.find(pidx);
                if (h2 != cached.end()) r = h2->second;
                else r = nearest_campfire(pidx, h, cf, *g);
            }
            cell.nearest_campfire[h] = r;
        }
    }
    *out = g;
    return MR_OK;
}

extern "C" void mro_grid_destroy(mro_grid *g) { delete g; }

extern "C" int mro_grid_nearest_campfire(const mro_grid *g, uint32_t i, uint32_t h, mr_cell_index *out) {
    if (!g || i >= g->grid.size() || h > 3 || !out) return 0;
    auto &nc = g->grid[i].nearest_campfire[h];
    if (!nc) return 0;
    *out = to_mr(*nc);
    return 1;
}

extern "C" int mro_grid_nearest_campfire_direct(const mro_grid *g, uint32_t i, uint32_t h,
                                                mr_cell_index *out) {
    if (!g || i >= g->grid.size() || h > 3 || !out) return 0;
    std::vector<std::pair<int, int>> cf;
    for (auto &c : g->grid)
        if (c.poi == MR_POI_CAMPFIRE && c.index.kind == MR_CELL_HOMELAND && c.index.sub == h)
            cf.push_back({c.index.x, c.index.y});
    auto r = nearest_campfire(g->grid[i].index, uint8_t(h), cf, *g);
    if (!r) return 0;
    *out = to_mr(*r);
    return 1;
}

namespace {

struct Query {
    const mro_grid *g;
    uint32_t soe, shq, sfm;
    bool use_soe, use_sfm, use_caravans;
    std::optional<CellIndex> hq;
    uint32_t route_guru, fleetfoot;
    Comparator cmp;
    uint8_t homeland;
};

// caravan_cost (src/pathfinder.rs:251-273)
static EdgeCost caravan_cost(const Query &q, const CellIndex &from, const CellIndex &to) {
    uint32_t d = uint32_t(distance(*q.g->at(from), *q.g->at(to)));
    uint32_t coef;
    if (to.kind == MR_CELL_CENTER) coef = 2;                                          // CARAVAN_TO_CENTER_MONEY
    else if (to.kind == MR_CELL_HOMELAND && to.sub == q.homeland) coef = 2;           // CARAVAN_TO_HOME_MONEY
    else coef = 5;                                                                    // CARAVAN_MONEY
    auto t = skill_time(route_guru_ratio(q.route_guru), 240);                         // CARAVAN_TIME = 4 min
    int64_t tt = t ? *t : 240;
    EdgeCost e;
    e.kind = Caravan;
    e.car_money = coef * d;
    e.car_time = tt * int64_t(d);
    return e;
}

// Inflight::edges (src/pathfinder.rs:24-180).  Returns false when the
// reference would panic on a grid lookup.
static bool edges(const Query &q, const CellIndex &v, std::vector<std::pair<CellIndex, EdgeCost>> &ret) {
    ret.clear();
    size_t hs = q.g->homeland_size();
    EdgeCost std_e{Standard}, cen_e{Central};
    if (v.kind == MR_CELL_CENTER) {
        for (uint8_t b = 0; b < 4; ++b) ret.push_back({build_border(b, 1), cen_e});
    } else if (v.kind == MR_CELL_BORDER) {
        uint8_t b = v.sub;
        int shift = v.x;
        if (shift == 1) ret.push_back({center(), cen_e});
        else ret.push_back({build_border(b, shift - 1), std_e});
        if (size_t(shift) < hs) ret.push_back({build_border(b, shift + 1), std_e});
        uint8_t nb[2];
        border_neighbours(b, nb);
        for (uint8_t h : nb) {
            // adjacent_pos_u8: Horizontal -> (shift, 1); Vertical -> (1, shift)
            if (border_direction(b) == Horizontal) ret.push_back({build_homeland(h, shift, 1), std_e});
            else ret.push_back({build_homeland(h, 1, shift), std_e});
        }
    } else {
        uint8_t h = v.sub;
        int x = v.x, y = v.y;
        ret.push_back({x == 1 ? build_border(homeland_border(h, Vertical), y) : build_homeland(h, x - 1, y), std_e});
        ret.push_back({y == 1 ? build_border(homeland_border(h, Horizontal), x) : build_homeland(h, x, y - 1), std_e});
        if (size_t(x) < hs) ret.push_back({build_homeland(h, x + 1, y), std_e});
        if (size_t(y) < hs) ret.push_back({build_homeland(h, x, y + 1), std_e});
    }
    if (q.use_caravans) {
        if (v == center() || q.g->campfires.count(v)) {
            if (!q.g->at(v)) return false;
            auto push = [&](const CellIndex &d) {
                if (d == v) return;
                ret.push_back({d, caravan_cost(q, v, d)});
            };
            push(center());
            for (auto &c : q.g->campfires_sorted) push(c);
        }
    }
    if (q.use_soe) {
        const Cell *c = q.g->at(v);
        if (!c) return false;  // grid[&vertex] panics
        if (c->nearest_campfire[q.homeland]) ret.push_back({*c->nearest_campfire[q.homeland], EdgeCost{SoE}});
    }
    if (q.hq) ret.push_back({*q.hq, EdgeCost{SHQ}});
    if (q.use_sfm) ret.push_back({center(), EdgeCost{SFm}});
    return true;
}

// FindPath::eval (src/pathfinder.rs:199-248)
static int eval(const Query &q, const CellIndex &from, const CellIndex &to, TotalCost &out) {
    TotalCost start = total_new(from);
    if (from == to) {
        out = start;
        return MR_OK;
    }
    std::unordered_map<CellIndex, TotalCost, CellIndexHash> dist;
    // BinaryHeap::new_by(|a, b| comparator(b, a)): a max-heap under the reversed
    // order = a min-heap of labels.  The comparator is total, so the
    // pop order does not depend on the heap's internal layout.
    auto heap_less = [&](const TotalCost &a, const TotalCost &b) { return q.cmp(a, b) > 0; };
    std::priority_queue<TotalCost, std::vector<TotalCost>, decltype(heap_less)> heap(heap_less);
    dist[from] = start;
    heap.push(start);
    std::vector<std::pair<CellIndex, EdgeCost>> es;
    while (!heap.empty()) {
        TotalCost cost = heap.top();
        heap.pop();
        CellIndex lowest = cost.commands.back().to;
        if (lowest == to) {
            out = std::move(cost);
            return MR_OK;
        }
        if (q.cmp(cost, dist[lowest]) > 0) continue;
        if (!edges(q, lowest, es)) return MR_ERR_INVALID_INDEX;
        for (auto &[w, e] : es) {
            TotalCost next = cost;
            total_add_assign(next, e, q.soe, q.shq, q.sfm, q.fleetfoot, lowest, w);
            auto it = dist.find(w);
            if (it == dist.end() || q.cmp(next, it->second) < 0) {
                dist[w] = next;
                heap.push(std::move(next));
            }
        }
    }
    return MR_NOT_FOUND;
}

static int make_query(const mro_grid *g, const mr_params *p, Query &q) {
    if (!g || !p) return MR_ERR_INVALID_ARG;
    if (p->sort_by[0] > 2 || p->sort_by[1] > 2 || p->homeland > 3) return MR_ERR_INVALID_ARG;
    q.g = g;
    q.soe = p->scroll_of_escape_cost;
    q.shq = p->scroll_of_escape_hq_cost;
    q.sfm = p->scroll_of_escape_forum_cost;
    q.use_soe = p->use_soe;
    q.use_sfm = p->use_sfm;
    q.use_caravans = p->use_caravans;
    if (p->has_hq) {
        if (!valid_input(p->hq_position)) return MR_ERR_INVALID_INDEX;
        q.hq = build_any(p->hq_position);
        if (!g->at(*q.hq)) return MR_ERR_INVALID_INDEX;
    }
    q.route_guru = p->route_guru;
    q.fleetfoot = p->fleetfoot;
    q.cmp = make_comparator(p->sort_by[0], p->sort_by[1]);
    q.homeland = p->homeland;
    return MR_OK;
}

static void write_result(const TotalCost &t, mr_result *r, mr_command *cmds, uint32_t cap, int status) {
    r->legs = t.legs;
    r->money = t.money;
    r->time_s = t.time;
    r->n_commands = uint32_t(t.commands.size());
    r->status = status;
    if (cmds) {
        for (uint32_t i = 0; i < r->n_commands && i < cap; ++i) {
            const Command &c = t.commands[i];
            mr_command &o = cmds[i];
            std::memset(&o, 0, sizeof(o));
            o.kind = c.agg.kind;
            o.legs = c.agg.legs;
            o.money = c.agg.money;
            o.fleetfoot = c.agg.fleetfoot;
            o.time_s = c.agg.time;
            o.from = to_mr(c.from);
            o.to = to_mr(c.to);
        }
    }
}

static int run_one(const Query &q, const mr_cell_index &from, const mr_cell_index &to, TotalCost &t) {
    if (!valid_input(from) || !valid_input(to)) return MR_ERR_INVALID_INDEX;
    CellIndex f = build_any(from), d = build_any(to);
    // canonical inputs only (a reference CellIndex is always built canonically),
    // and both ends must be grid cells (the reference panics on a missing cell;
    // we return an error instead)
    auto same = [](const CellIndex &c, const mr_cell_index &m) {
        return c.kind == m.kind && c.sub == m.sub && c.x == m.x && c.y == m.y;
    };
    if (!same(f, from) || !same(d, to) || !q.g->at(f) || !q.g->at(d)) return MR_ERR_INVALID_INDEX;
    return eval(q, f, d, t);
}

}  // namespace

extern "C" int mro_find_path(const mro_grid *g, const mr_params *p, mr_cell_index from, mr_cell_index to,
                             mr_result *out, mr_command *cmds, uint32_t cap) {
    if (!out) return MR_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    Query q;
    int st = make_query(g, p, q);
    if (st != MR_OK) {
        out->status = st;
        return st;
    }
    TotalCost t;
    st = run_one(q, from, to, t);
    if (st != MR_OK) {
        out->status = st;
        return st;
    }
    write_result(t, out, cmds, cap, MR_OK);
    if (out->n_commands > cap) {
        out->status = MR_ERR_CAPACITY;
        return MR_ERR_CAPACITY;
    }
    return MR_OK;
}

extern "C" int mro_find_path_batch(const mro_grid *g, const mr_params *p, const mr_query *queries, uint32_t n,
                                   mr_result *results, mr_command *pool, uint64_t pool_cap, uint32_t threads) {
    if (!queries || !results || (n && !pool && pool_cap)) return MR_ERR_INVALID_ARG;
    Query q;
    int st = make_query(g, p, q);
    if (st != MR_OK) return st;
    std::vector<TotalCost> labels(n);
    std::vector<int> status(n);
    std::atomic<uint32_t> next{0};
    auto worker = [&]() {
        for (;;) {
            uint32_t i = next.fetch_add(1);
            if (i >= n) break;
            status[i] = run_one(q, queries[i].from, queries[i].to, labels[i]);
        }
    };
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    threads = std::min<uint32_t>(threads, std::max<uint32_t>(1, n));
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads; ++t) ts.emplace_back(worker);
    worker();
    for (auto &t : ts) t.join();
    uint64_t off = 0;
    int ret = MR_OK;
    for (uint32_t i = 0; i < n; ++i) {
        std::memset(&results[i], 0, sizeof(mr_result));
        results[i].status = status[i];
        if (status[i] != MR_OK) {
            if (status[i] < 0 && ret == MR_OK) ret = status[i];
            continue;
        }
        uint32_t nc = uint32_t(labels[i].commands.size());
        results[i].command_offset = uint32_t(off);
        bool fits = off + nc <= pool_cap;
        write_result(labels[i], &results[i], fits ? pool + off : nullptr, nc, MR_OK);
        results[i].command_offset = uint32_t(off);
        if (!fits) ret = MR_ERR_CAPACITY;
        off += nc;
    }
    return ret;
}

// Every destination of one source (test infrastructure for the all-destinations
// plans): FindPath::eval's Dijkstra (src/pathfinder.rs:199-248) run without the early
// exit.  By SURVEY 8a's uniqueness lemma the final dist[] label of each cell is the
// label eval(from, cell) returns (eval pops `to` with that label and stops).  One
// result per cell in the grid's input (row-major) order; the commands go to pool
// (results[i].command_offset), MR_ERR_CAPACITY if pool_cap is too small.
namespace mro {
// FindPath::eval's loop (src/pathfinder.rs:219-246) without the early exit: the final
// dist[] label of every cell reachable from f.
static int sssp_dist(const Query &q, const CellIndex &f,
                     std::unordered_map<CellIndex, TotalCost, CellIndexHash> &dist) {
    auto heap_less = [&](const TotalCost &a, const TotalCost &b) { return q.cmp(a, b) > 0; };
    std::priority_queue<TotalCost, std::vector<TotalCost>, decltype(heap_less)> heap(heap_less);
    dist[f] = total_new(f);
    heap.push(dist[f]);
    std::vector<std::pair<CellIndex, EdgeCost>> es;
    while (!heap.empty()) {
        TotalCost cost = heap.top();
        heap.pop();
        CellIndex lowest = cost.commands.back().to;
        if (q.cmp(cost, dist[lowest]) > 0) continue;
        if (!edges(q, lowest, es)) return MR_ERR_INVALID_INDEX;
        for (auto &[w, e] : es) {
            TotalCost next = cost;
            total_add_assign(next, e, q.soe, q.shq, q.sfm, q.fleetfoot, lowest, w);
            auto it = dist.find(w);
            if (it == dist.end() || q.cmp(next, it->second) < 0) {
                dist[w] = next;
                heap.push(std::move(next));
            }
        }
    }
    return MR_OK;
}

// The digest of a command list that tests/label_digest.py computes from mr_command
// arrays: each 40 B command as five little-endian u64 words (reserved bytes zero),
// h = Horner over the words with kDigestP, the list H = Horner over the commands'
// h with kDigestQ, all mod 2^64.
static constexpr uint64_t kDigestP = 0x9E3779B97F4A7C15ull, kDigestQ = 0xC2B2AE3D27D4EB4Full;
static uint64_t label_digest(const TotalCost &t) {
    uint64_t H = 0;
    for (const Command &c : t.commands) {
        mr_command o;
        std::memset(&o, 0, sizeof(o));
        o.kind = c.agg.kind;
        o.legs = c.agg.legs;
        o.money = c.agg.money;
        o.fleetfoot = c.agg.fleetfoot;
        o.time_s = c.agg.time;
        o.from = to_mr(c.from);
        o.to = to_mr(c.to);
        uint64_t w[5];
        std::memcpy(w, &o, sizeof(w));
        uint64_t h = 0;
        for (uint64_t x : w) h = h * kDigestP + x;
        H = H * kDigestQ + h;
    }
    return H;
}
}  // namespace mro

// Every destination of each of n sources, on `threads` host threads (test
// infrastructure for full-size parity): per source s and row-major cell i, at
// [s * V + i]: legs, money, time, command count, status (MR_OK / MR_NOT_FOUND) and
// the command-list digest (label_digest above).  Any output pointer may be null.
extern "C" int mro_sssp_digest_batch(const mro_grid *g, const mr_params *p, const mr_cell_index *sources, uint32_t n,
                                     uint32_t threads, uint32_t *legs, uint32_t *money, int64_t *time_s,
                                     uint32_t *n_commands, int32_t *status, uint64_t *digest) {
    if (!g || (n && !sources)) return MR_ERR_INVALID_ARG;
    Query q;
    int st = make_query(g, p, q);
    if (st != MR_OK) return st;
    const size_t V = g->grid.size();
    std::vector<int> res(n, MR_OK);
    std::atomic<uint32_t> next{0};
    auto worker = [&]() {
        for (uint32_t s = next++; s < n; s = next++) {
            if (!valid_input(sources[s])) {
                res[s] = MR_ERR_INVALID_INDEX;
                continue;
            }
            CellIndex f = build_any(sources[s]);
            if (!g->at(f)) {
                res[s] = MR_ERR_INVALID_INDEX;
                continue;
            }
            std::unordered_map<CellIndex, TotalCost, CellIndexHash> dist;
            dist.reserve(V);
            if ((res[s] = sssp_dist(q, f, dist)) != MR_OK) continue;
            for (size_t i = 0; i < V; ++i) {
                const size_t o = size_t(s) * V + i;
                auto it = dist.find(g->grid[i].index);
                const bool ok = it != dist.end();
                if (legs) legs[o] = ok ? it->second.legs : 0;
                if (money) money[o] = ok ? it->second.money : 0;
                if (time_s) time_s[o] = ok ? it->second.time : 0;
                if (n_commands) n_commands[o] = ok ? uint32_t(it->second.commands.size()) : 0;
                if (status) status[o] = ok ? MR_OK : MR_NOT_FOUND;
                if (digest) digest[o] = ok ? label_digest(it->second) : 0;
            }
        }
    };
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    threads = std::min<uint32_t>(threads, std::max<uint32_t>(1, n));
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads; ++t) ts.emplace_back(worker);
    worker();
    for (auto &t : ts) t.join();
    for (int r : res)
        if (r != MR_OK) return r;
    return MR_OK;
}

extern "C" int mro_sssp_all(const mro_grid *g, const mr_params *p, mr_cell_index from, mr_result *results,
                            mr_command *pool, uint64_t pool_cap) {
    if (!g || !results) return MR_ERR_INVALID_ARG;
    Query q;
    int st = make_query(g, p, q);
    if (st != MR_OK) return st;
    if (!valid_input(from)) return MR_ERR_INVALID_INDEX;
    CellIndex f = build_any(from);
    if (!g->at(f)) return MR_ERR_INVALID_INDEX;
    std::unordered_map<CellIndex, TotalCost, CellIndexHash> dist;
    if ((st = sssp_dist(q, f, dist)) != MR_OK) return st;
    const size_t n = g->grid.size();
    for (size_t i = 0; i < n; ++i) {
        std::memset(&results[i], 0, sizeof(mr_result));
        results[i].status = MR_NOT_FOUND;
    }
    int ret = MR_OK;
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
        const CellIndex &c = g->grid[i].index;
        auto it = dist.find(c);
        if (it == dist.end()) continue;
        // from == to: eval returns the start label
        const TotalCost &t = c == f ? dist[f] : it->second;
        uint32_t nc = uint32_t(t.commands.size());
        bool fits = pool && off + nc <= pool_cap;
        write_result(t, &results[i], fits ? pool + off : nullptr, nc, MR_OK);
        results[i].command_offset = uint32_t(off);
        if (!fits) ret = MR_ERR_CAPACITY;
        off += nc;
    }
    return ret;
}

// time 0.3 Duration Display (verbose form): d, h, m, s (whole seconds only)
extern "C" int mro_duration_display(int64_t seconds, char *buf, uint32_t cap) {
    std::string s;
    if (seconds < 0) s += "-";
    uint64_t a = uint64_t(seconds < 0 ? -seconds : seconds);
    if (a == 0) s = "0s";
    else {
        auto item = [&](uint64_t v, const char *name) {
            if (v) s += std::to_string(v) + name;
        };
        item(a / 86400, "d");
        item(a / 3600 % 24, "h");
        item(a / 60 % 60, "m");
        item(a % 60, "s");
    }
    if (buf && cap) {
        size_t k = std::min<size_t>(s.size(), cap - 1);
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return int(s.size());
}

// The hub solver's SoE region table (TEST INFRASTRUCTURE: the checker of the engine's
// device-built mr_grid_region_table).  A region is the set of cells whose nearest
// campfire of the query homeland (src/grid.rs:297-325) is one campfire; walks cannot
// cross the Center (its only edges are CentralMoves, src/pathfinder.rs:30-53).  One
// breadth-first search per region over the grid minus the Center from all of its
// cells, keeping per cell the least (distance, rank of the origin cell).
// region[v]: region index of row-major cell v (0xFFFFFFFF: none), rank[v]: its
// CellIndex rank; out: S*S x nreg x {distance, rank}.
extern "C" int mro_region_table_bfs(uint32_t S, const uint32_t *rank, const uint32_t *region, uint32_t nreg,
                                    uint32_t *out, uint32_t threads) {
    if (S < 3 || !(S & 1u) || !rank || !region || !out) return MR_ERR_INVALID_ARG;
    const uint32_t V = S * S, vc = (S / 2) * S + S / 2, NONE = 0xFFFFFFFFu;
    std::atomic<uint32_t> next{0};
    auto worker = [&]() {
        std::vector<uint32_t> dist(V), org(V), cur, nxt;
        for (uint32_t r = next++; r < nreg; r = next++) {
            std::fill(dist.begin(), dist.end(), NONE);
            cur.clear();
            for (uint32_t v = 0; v < V; ++v)
                if (v != vc && region[v] == r) {
                    dist[v] = 0;
                    org[v] = v;
                    cur.push_back(v);
                }
            for (uint32_t d = 0; !cur.empty(); ++d) {
                nxt.clear();
                for (uint32_t u : cur) {
                    const uint32_t x = u % S, y = u / S;
                    const uint32_t nb[4] = {x > 0 ? u - 1 : NONE, x + 1 < S ? u + 1 : NONE, y > 0 ? u - S : NONE,
                                            y + 1 < S ? u + S : NONE};
                    for (uint32_t w : nb) {
                        if (w == NONE || w == vc) continue;
                        if (dist[w] == NONE) {
                            dist[w] = d + 1;
                            org[w] = org[u];
                            nxt.push_back(w);
                        } else if (dist[w] == d + 1 && rank[org[u]] < rank[org[w]]) {
                            org[w] = org[u];
                        }
                    }
                }
                cur.swap(nxt);
            }
            for (uint32_t v = 0; v < V; ++v) {
                out[(size_t(v) * nreg + r) * 2] = dist[v];
                out[(size_t(v) * nreg + r) * 2 + 1] = dist[v] == NONE ? NONE : rank[org[v]];
            }
        }
    };
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::thread> pool;
    for (uint32_t i = 1; i < std::min(threads, std::max(nreg, 1u)); ++i) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
    return MR_OK;
}
