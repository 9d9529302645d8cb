// mr_engine.hpp — data layout shared by the host planner and the gfx950 kernels.
//
// Algorithm: a single-source solve computes the unique fixed
// point L(v) = min_u extend(L(u), u->v) of the reference's Dijkstra
// (src/pathfinder.rs:199-248; uniqueness: SURVEY.md §8a).  Two facts shape the
// layout:
//  * every vertex that is not a "special" (Center, the four border-1 cells,
//    campfires, HQ) has only StandardMove in-edges, so its label is a walk
//    L(b).commands ++ [StandardMove{k} b->v] from a *boundary* b that is the
//    source or a special (src/cost.rs:246-264 merges the run).  Such a label is
//    stored in ONE 32-bit word: (b, k).
//  * specials (<= ~1000) keep full labels in an LDS table as a parent pointer
//    plus <= 2 tail commands (Rec); command lists compare by walking parents.
// Vertices are settled bucket by bucket on the comparator's leading metric
// (plain vertices of one bucket are independent), specials inside a bucket by
// an exact one-wave Dijkstra.
#pragma once
#include <stdint.h>

namespace mr {

constexpr uint32_t kNone10 = 0x3FFu;          // "no index" in a 10-bit field
constexpr uint32_t kMaxSpecials = 1021u;      // table indices 1..1021 (0 = source)
constexpr uint32_t kStSettled = 0x80000000u;  // grid state word flags
constexpr uint32_t kStDirty = 0x40000000u;
constexpr uint32_t kStBShift = 20u;
constexpr uint32_t kStKMask = 0xFFFFFu;       // walk run length k < 2^20
constexpr uint32_t kStUntouched = kNone10 << kStBShift;

// command kinds = AggregatedCost variant order (src/cost.rs:90-110)
enum : uint32_t { kNoMove = 0, kCentral = 1, kStandard = 2, kCaravan = 3, kSoE = 4, kSHQ = 5, kSFm = 6 };

// A command: kp = kind << 29 | payload.  payload: Standard k (legs of the run),
// Central j (moves merged), Caravan (d << 1 | coef==5), scrolls/NoMove 0.
// Comparing kp as an unsigned integer is the derived Ord of AggregatedCost for
// one query (time = 180k / 10j / d*rgt are monotone in the payload; the
// Caravan money d*coef orders by the coef bit at equal d).
struct Cmd {
    uint32_t kp;
    uint32_t from;  // rank of the cell (position in CellIndex order, src/index.rs:41-46)
    uint32_t to;
};

// A full label of a special (or the source), src/cost.rs:187-206:
//   commands = full(parent) ++ tail[0..ntail)   (parent 0 = empty prefix)
// Stored in 28 B: every label the engine builds (the start label, walks, SoE from a
// region cell, TotalCost += edge, SHQ/SFm) has tail[0] = {kp0, from0 = the rank of
// the parent entry's cell (the source's for parent 0), u} and, when ntail = 2,
// tail[1] = {SoE, u, rank of the entry's own cell}; u is the own cell's rank when
// ntail = 1.
struct Rec {
    uint32_t m[3];  // legs, money, time  (metric index order)
    uint32_t meta;  // len (16 b) | parent (10 b) << 16 | state (2 b) << 26 | (ntail - 1) << 31
    uint32_t kp0;   // tail[0].kp
    uint32_t from0; // tail[0].from
    uint32_t u;     // tail[0].to (= tail[1].from when ntail = 2)
    __host__ __device__ uint32_t len() const { return meta & 0xFFFFu; }
    __host__ __device__ uint32_t parent() const { return (meta >> 16) & 0x3FFu; }
    __host__ __device__ uint32_t state() const { return (meta >> 26) & 3u; }  // 0 none, 1 tentative, 2 settled
    __host__ __device__ uint32_t ntail() const { return (meta >> 31) + 1u; }
    __host__ __device__ void set_state(uint32_t st) { meta = (meta & ~(3u << 26)) | (st << 26); }
    __host__ __device__ static uint32_t pack(uint32_t len, uint32_t parent, uint32_t ntail, uint32_t state) {
        return (len & 0xFFFFu) | ((parent & 0x3FFu) << 16) | ((state & 3u) << 26) | ((ntail - 1u) << 31);
    }
};
static_assert(sizeof(Rec) == 28, "Rec layout");

// Static per-special info (one entry per table index 1..NS; entry 0 unused).
struct SpecialStatic {
    uint32_t v;       // vertex id
    int32_t x, y;     // geometric coordinates
    uint32_t flags;   // bit0 center, bit1 border-1, bit2 caravan hub
    uint32_t region;  // table index of this cell's nearest campfire (query homeland), kNone10 if none
    uint32_t coef5;   // 1 if a caravan INTO this special costs 5/distance (else 2)
    uint32_t rid;     // hub solver: region id if this is a query-homeland campfire, else kNone10
    uint32_t rk;      // rank of v (position in CellIndex order): commands name cells by rank
};
constexpr uint32_t kSpCenter = 1u, kSpBorder1 = 2u, kSpHub = 4u;

// bucket modes: leading comparator metric(s) used as the settle bucket
enum : uint32_t { kBucketLegs = 0, kBucketTime = 1, kBucketMoneyLegs = 2, kBucketMoneyTime = 3 };

struct DevParams {
    uint32_t S, H, V, vc;         // side, half side, vertices, Center vertex id
    uint32_t perm[3];             // comparator metrics c1,c2,c3 as indices into m[] (0 legs, 1 money, 2 time)
    uint32_t bucket_mode;
    uint32_t W;                   // time bucket width = min StandardMove time increment
    uint32_t ff;                  // Fleetfoot level stored in Standard commands
    uint32_t ff_num, ff_den;      // Fleetfoot ratio (1/1 when level 0 or out of range)
    uint32_t ff_c, ff_magic, ff_shift;  // 180 num; ceil(x / den) = umulhi(x + den - 1, magic) >> shift (lane kernel)
    uint32_t rgt;                 // caravan seconds per distance unit (RouteGuru applied)
    uint32_t soe_cost, shq_cost, sfm_cost;
    uint32_t use_soe, use_sfm, use_caravans;
    uint32_t hq_t;                // table index of HQ, 0 if no SHQ
    uint32_t NS;                  // number of specials
    uint32_t n_hubs;              // caravan hubs (Center + campfires), table indices in hubs[]
    uint32_t max_cmds;            // command slots per query in the output
};

// compact per-query output (expanded to mr_result/mr_command on the host)
struct OutResult {
    uint32_t legs, money, time;
    uint32_t ncmd_status;  // low 16 bits: n_commands; high 16 bits: status code + 16
};
struct OutCmd {
    uint32_t kp, from, to, pad;
};
// all-destinations output: one 32-bit cell word per source and cell,
// the label's walk in the grid-state layout above:
//   b << kStBShift | k   the walk of k legs from boundary b (table index; 0 = the
//                        source): commands = table chain of b ++ [StandardMove{k}
//                        b -> v], metrics = the table label's + (k, 0, run_time(k))
//   kViaSpecial | t      special t: its own table label
//   kViaSource           the source: the start label
// The metrics are the table's plus the walk's, so 4 B per cell carry the whole label
// (mr_sssp_records expands them on the host).
typedef uint32_t CellWord;
constexpr uint32_t kViaSpecial = 0x80000000u, kViaSource = 0xFFFFFFFFu;
// all-destinations fill tiles: one wave per kFillTW x kFillTH cells, MR_FILL_CPL
// columns per lane (64 apart), MR_FILL_CELLS cells per lane
#ifndef MR_FILL_CPL
#define MR_FILL_CPL 1
#endif
#ifndef MR_FILL_CELLS
#define MR_FILL_CELLS 16
#endif
constexpr uint32_t kFillTW = 64u * MR_FILL_CPL, kFillTH = MR_FILL_CELLS / MR_FILL_CPL;

// kernel arguments (one solve launch)
struct KArgs {
    DevParams p;
    const uint32_t *sinfo;       // V words: special idx (10b) | region idx << 10
    const uint32_t *rank;        // V words: position in CellIndex order
    const uint32_t *rank_inv;    // V words: vertex of each rank
    const uint2 *cell;           // V x {sinfo, rank}: one line per random cell read (hub_lane_kernel)
    const SpecialStatic *sp;     // NS+1 entries
    const uint16_t *hubs;        // n_hubs caravan endpoints (table indices)
    const uint32_t *src_v;       // nsrc source vertices
    const uint32_t *q_begin;     // nsrc+1 offsets into q_dst/q_id
    const uint32_t *q_dst;       // destinations grouped by source
    const uint32_t *q_id;        // query id of each grouped destination
    OutResult *out_res;          // per query id
    OutCmd *out_cmd;             // per query id * max_cmds
    uint32_t *ws;                // grid-in-HBM mode: per-workgroup slots of 5*V words
    uint32_t *counter;           // kCtr* words (below)
    uint32_t nsrc;
    uint32_t early_exit_max;     // early exit if a source has <= this many destinations (<= 64)
    uint32_t grid_in_lds;        // 1: grid state in LDS, 0: per-workgroup HBM slots
    uint32_t algo;               // kAlgoLegs (Legs-first level-synchronous) or kAlgoGeneric
    unsigned long long *dbg;     // diagnostic builds (-DMR_STAMPS): per-workgroup phase cycles
    // hub solver (linear run time): per vertex and region, the nearest region cell by
    // walk distance avoiding the Center: near[2*(v*nreg + r)] = {distance, rank of the cell}
    const uint32_t *near;
    uint32_t nreg;
    uint32_t *fb_list;           // sources the hub solver hands to the SSSP kernel (counter[2] of them)
    uint32_t *relist;            // non-null: the lane kernel hands an uncertain source to hub_kernel
                                 // (relist[counter[kCtrRelist]++]) instead of the SSSP kernel
    uint32_t fb_mode;            // 1: this SSSP launch solves fb_list[counter[3]++] only
    uint32_t fb_all;             // tests: the hub solver hands every source to the SSSP kernel
    uint32_t dbg_blocks;         // diagnostic builds: SSSP workgroups (hub stamps follow their slots)
    uint32_t last_launch;        // 1: the pass's last kernel; its last workgroup resets the counters
    // all-destinations mode: no per-query outputs; per source, a record per cell, the
    // label table (NS+1 entries), the boundaries' lexicographic ranks and how it was solved
    uint32_t all_mode;
    CellWord *out_rec;           // nsrc * S rows of rec_pitch cell words (rows padded to 64 cells)
    uint32_t rec_pitch;          // cell words per row of out_rec: S rounded up to a multiple of 64
    Rec *out_tab;                // nsrc * (NS+1)
    uint32_t *out_lex;           // nsrc * (NS+1): rank of boundary t by (length, command list), else kNone32
    uint32_t *src_state;         // nsrc: 1 hub solved (records by the fill kernel), 2 SSSP kernel
    uint32_t dbg_flags;          // experiments (MR_DBG_FLAGS); 0 in normal runs
    // wide hub solver (hub_wide_kernel): the specials' region rows ((NS+1) x nreg x
    // {distance, rank}) and each region's boundary cells, {x | y << 16 (int16), rank},
    // region r at rb_cell[rb_off[r] .. rb_off[r+1])
    const uint32_t *near_sp;
    const uint32_t *rb_off;
    const uint32_t *rb_cell;
    // labels longer than max_cmds: their commands in this pool (bump-allocated per pass)
    OutCmd *ovf;
    uint32_t ovf_cap;
    // hub plans: sources [0, n_lane) go to hub_lane_kernel (one source per lane, few
    // queries each), sources [src_off, nsrc) to hub_kernel (src_off = n_lane)
    uint32_t n_lane;
    uint32_t src_off;
    // Certified fallback: the hub kernel exports the label table
    // of up to cert_cap flagged sources into slots (cert_tab / cert_lex / cert_src; the
    // slot of fallback entry i in fb_cert[i], kNone32 for none), the fill writes every
    // cell's closed-form word into cert_rec (rec_pitch words a row), the check kernel
    // the least leading metric of a cell that fails the fixed-point test into
    // cert_key[slot], and the SSSP launch emits a source's labels from its slot when
    // every one of them lies below that key.
    uint32_t cert_cap;
    Rec *cert_tab;
    uint32_t *cert_lex;
    uint32_t *cert_src;
    CellWord *cert_rec;
    uint32_t *cert_st;           // per slot and check workgroup kCertSt words (kCert* below)
    uint32_t cert_parts;         // check workgroups per slot (partial states a consumer reduces)
    uint32_t *cert_aux;          // per slot V words: the repair sweep's cells by bucket
    uint32_t *fb_cert;
    const uint32_t *nsrc_dev;    // fill launches over cert slots: sources = min(nsrc, *nsrc_dev)
    // Slots are given deterministically: the hub kernel stages the table of fallback
    // entry i (while i < cert_stage_cap) and tags fb_cert[i] = kFbStaged; then
    // cert_select_kernel gives the slots to the staged sources in source order (the
    // cert_cap least source indices) and copies their tables into them.  A pass with
    // more fallback entries than cert_stage_cap stages nothing usable: no slots.  So
    // which sources the certificate answers never depends on the order of arrival.
    Rec *cert_stage_tab;         // cert_stage_cap * (NS+1)
    uint32_t *cert_stage_lex;    // cert_stage_cap * (NS+1)
    uint32_t *cert_stage_src;    // cert_stage_cap
    uint32_t cert_stage_cap;
    // 1: every cell's rank is std_rank of its position (mr_hub_lane.hpp; checked at grid
    // creation), so the lane kernel reads no per-cell record
    uint32_t rank_std;
    // lane and group kernels: the plan's LDS block (lane_blob_bytes, mr_hub_lane.hpp), built
    // once on the host (lane_blob_build) and copied by every workgroup
    const uint4 *lane_blob;
    // the certificate's repair (mr_cert_tile.hpp): per slot kWinWords window words
    // (cert_window_kernel), and the tile sweep's publish areas, two kTileT x kTileT keys
    // per workgroup of its launch (cert_pub_wgs of them)
    uint32_t *cert_win;
    unsigned long long *cert_pub;
    uint32_t cert_pub_wgs;
    // the certificate's second round (promoted specials, mr_cert_tile.hpp): non-null in the
    // argument block of the round's kernels, which skip the slots with cert_redo[slot] == 0
    uint32_t *cert_redo;
};
// cert_redo[slot]: kRedoFill — promoted specials: the closed form again, both checks and the
// repair; kRedoSweep — specials the last check demoted: the repair from the current words
// and the last check only
constexpr uint32_t kRedoFill = 1u, kRedoSweep = 2u;
// fb_cert[i] of a staged entry before cert_select_kernel gives it a slot (or none)
constexpr uint32_t kFbStaged = 0xFFFFFFFEu;
// fb_list[i] | kFbCertified: the SSSP launch emitted entry i from its certificate slot
// (mr_plan_fallback_sources leaves such sources out: they cost no search)
constexpr uint32_t kFbCertified = 0x80000000u;
constexpr uint32_t kCertStageMax = 4096u;  // cert_select_kernel's LDS arrays (32 KB)
// counter words: the pass's last workgroup copies the fallback and written counts
// to their "last" slots and zeroes the rest, so no memset precedes a pass
enum : uint32_t {
    kCtrDequeue = 0,      // SSSP source dequeue
    kCtrFlags = 1,        // error flags (sticky until the host collects them)
    kCtrFbCount = 2,      // sources the hub solver handed to the SSSP kernel
    kCtrFbDequeue = 3,    // fallback dequeue
    kCtrLastFb = 4,       // kCtrFbCount of the last completed pass
    kCtrLastWritten = 5,  // kCtrWritten of the last completed pass
    kCtrDone = 6,         // workgroups of the last kernel that finished (low word of one
    kCtrWritten = 7,      // result records written               64-bit counter with this)
    kCtrOvf = 8,          // command-overflow pool: commands allocated in this pass
    kCtrLastOvf = 9,      // kCtrOvf of the last completed pass
    kCtrCert = 10,        // certified-fallback slots given in this pass (cert_select_kernel)
    kCtrCertDone = 11,    // fallback sources the certificate answered in this pass
    kCtrLastCert = 12,    // kCtrCertDone of the last completed pass
    kCtrRelist = 13,      // lane-kernel sources handed to hub_kernel in this pass (KArgs::relist)
    kCtrLastRelist = 14,  // kCtrRelist of the last completed pass
    kCtrWords = 15
};
// per certificate slot and check workgroup: the least leading metric of a failing cell
// (labels below the least over the workgroups are exact), failing cells, their bounding
// box (grid coordinates), and the walk-labelled specials it demoted to plain cells (a
// bit per table entry; applied by cert_window_kernel, so every reader of one check sees
// the same words)
enum : uint32_t {
    kCertKey = 0, kCertFails = 1, kCertX0 = 2, kCertX1 = 3, kCertY0 = 4, kCertY1 = 5, kCertDem0 = 6, kCertDem1 = 7,
    kCertSt = 8
};
// the certificate's tile sweep (mr_cert_tile.hpp)
constexpr uint32_t kTileT = 64;        // a team tile's side
constexpr uint32_t kTileH = 24;        // halo width = steps between exchanges
constexpr uint32_t kTileP = 128;       // LDS row pitch of a region (>= kTileT + 2 kTileH; a power of two)
constexpr uint32_t kTileR = 112;       // LDS rows of a region (>= kTileT + 2 kTileH)
constexpr uint32_t kTileN = kTileP * kTileR;
constexpr uint32_t kTileBS = 512;      // threads of a tile workgroup
constexpr uint32_t kTileList = 2048;   // entries of a bucket list (more: that step scans densely)
constexpr uint32_t kTileEv = 1024;     // fixed cells bordering window cells, per region
constexpr uint32_t kTileFD = 4096;     // run-time increments tabulated (longer runs divide)
constexpr uint32_t kTileMaxSteps = 8192;
constexpr uint32_t kTileMaxTiles = 256;  // tiles of one window (its team)
constexpr unsigned long long kTileHi = 1ull << 63, kTileNoExt = ~kTileHi;  // (fixed, nothing to push)
constexpr uint32_t kTileGMax = 1u << 22;  // G - B0 at or past this: far beyond any step (no push)
constexpr uint32_t kTileDone = 0xFFFFFFFFu;  // a tile's flag once its cells are final

// per slot window words (cert_window_kernel writes them, the sweeps read them)
enum : uint32_t {
    kWinMode = 0,  // kWinNone / kWinTile / kWinOld / kWinWide
    kWinX0 = 1, kWinY0 = 2, kWinX1 = 3, kWinY1 = 4,
    kWinNtx = 5, kWinNty = 6, kWinB0 = 7,
    kWinFail = 8,   // the tile sweep gave up (step cap, a spin timeout, an LDS table too small)
    kWinSteps = 10, // steps of the slot's last tile to finish
    kWinTStep = 11, kWinTXchg = 12, kWinNXchg = 13,  // tile 0: time in steps / exchanges (10 ns), exchanges
    kWinProm0 = 14, kWinProm1 = 15,  // entries promoted this pass (a bit each; zeroed by cert_select_kernel)
    kWinFlag = 16,  // per tile: exchanges published (kTileDone: final)
    kWinStat = 16 + kTileMaxTiles,  // per tile 4 words: time in steps / exchanges (10 ns), settles, steps
    kWinPromo = 16 + 5 * kTileMaxTiles,  // per entry: the hub whose caravan beats its repaired walk, + 1
    kWinWhy = kWinPromo + 64,  // diagnostics: failing cells of the last check (count, 7 x {x | y << 16, tests, keys})
    kWinWords = kWinWhy + 32
};
enum : uint32_t { kWinNone = 0, kWinTile = 1, kWinOld = 2, kWinWide = 3 };
// Wire records (mr_plan_wire_records / mr_decode_wire): a pass's records re-encoded for
// transfer, 1 + 2 max_cmds 32-bit words each, in record order.  Word 0: the rank of the
// first command's `from` cell (kWireRankBits) | code << kWireRankBits, code = n_commands
// for MR_OK (< kWireOvf), kWireOvf for a label whose commands are in the wire pool (slot 0
// = {offset, count}), kWireStatus + 32 + status for any other status.  Then per command
// {kind << 29 | payload, rank of its `to` cell}: a command's `from` is the previous one's
// `to`, and the metrics are the commands' sums (TotalCost::add_assign recomputes them the
// same way, src/cost.rs:299-313), so neither crosses the wire.  The pool: 2 words a command.
constexpr uint32_t kWireRankBits = 25, kWireRankMask = (1u << kWireRankBits) - 1u;
constexpr uint32_t kWireOvf = 64u, kWireStatus = 65u;

// result status (OutResult high half - 16) of a label whose commands went to the
// overflow pool: its first command slot holds {kOvfTag, offset, count}
constexpr uint32_t kStatusOverflow = 64u, kOvfTag = 0xFFFFFFFFu;
enum : uint32_t { kAlgoGeneric = 0, kAlgoLegs = 1 };
// hub plans: sources with at most this many queries run on hub_lane_kernel (one source
// per lane, its queries read off by that lane); sources with more on hub_kernel (a lane
// per query)
constexpr uint32_t kLaneMaxQ = 32;
constexpr uint32_t kLaneRegs = 6;  // hub_lane_kernel: region campfires sit in entries 6 .. 6 + kLaneRegs - 1

// CellIndex rank of the cell at (x, y) in the standard layout (Blue x<0 y<0, Red x<0 y>0,
// Green x>0 y>0, Yellow x>0 y<0; borders BR y=0 x<0, RG x=0 y>0, GY y=0 x>0, YB x=0 y<0):
// the derived Ord Center < Homeland{h, (|x|, |y|)} < Border{b, shift} (src/index.rs:41-46)
// over a complete grid of homeland size H.  mr_grid_create checks it for every cell.
__host__ __device__ inline uint32_t std_rank(int x, int y, uint32_t H) {
    const uint32_t ax = uint32_t(x < 0 ? -x : x), ay = uint32_t(y < 0 ? -y : y);
    if (x == 0 && y == 0) return 0u;
    if (y == 0 || x == 0) {
        const uint32_t b = y == 0 ? (x < 0 ? 0u : 2u) : (y > 0 ? 1u : 3u);
        return 1u + 4u * H * H + b * H + (ax + ay - 1u);
    }
    const uint32_t h = x < 0 ? (y < 0 ? 0u : 1u) : (y > 0 ? 2u : 3u);
    return 1u + h * H * H + (ax - 1u) * H + (ay - 1u);
}

constexpr uint32_t kErrKOverflow = 1u, kErrMetricOverflow = 2u, kErrBucket = 4u, kErrChain = 8u;
// KArgs::dbg_flags bit (tests only): the fill launch raises kErrChain
constexpr uint32_t kDbgInjectFlag = 16u;
// KArgs::dbg_flags bits (timing experiments only, results are not valid): hub_group_kernel
// skips its Dijkstra / its destinations / the list compares of exact ties
constexpr uint32_t kDbgGroupNoSolve = 32u, kDbgGroupNoReadoff = 64u, kDbgGroupNoTies = 128u;
constexpr uint32_t kDbgSweepFull = 256u;   // the repair sweep queues every window cell (A/B)
constexpr uint32_t kDbgSweepNoLds = 512u;  // the repair sweep keeps a small window's words in the slot's buffer
constexpr uint32_t kDbgSweepReread = 1024u, kDbgSweepGList = 2048u;  // (A/B probes of the sweep)

}  // namespace mr
