// The app's command table for a path (src/app.rs:481-561): one row per command
// (NoMove skipped) with the bot command, its duration, the running total and the
// back-scheduled start time-of-day.
//  * command: CentralMove / StandardMove -> "/go_direct_<suffix(to)>", Caravan ->
//    "/car_<suffix(to)>", scrolls -> "/use_soe" | "/use_shq" | "/use_sfm"; suffix
//    (CellIndexCommandSuffix, src/index.rs:378-390): "0_0", "<b|r|g|y>_<x>_<y>",
//    "<br|rg|gy|yb>_<shift>";
//  * duration: AggregatedCost::time (src/cost.rs:118-150): Fleetfoot's ceil on a
//    StandardMove run's raw time for levels 1..3 (src/skill.rs:21-30,65-71);
//  * total: running sum of (duration + pause);
//  * start: arrive_at - sum over this and later commands of (duration + pause),
//    wrapping at midnight like time::Time - Duration;
//  * durations print like time 0.3's Duration Display ("1h3m10s", "0s"), pinned by
//    src/pathfinder.rs:279-285; times as "[hour]:[minute]:[second]".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/marshrutka_pf.h"

namespace {

std::string suffix(const mr_cell_index &c) {
    static const char *hl[4] = {"b", "r", "g", "y"}, *bl[4] = {"br", "rg", "gy", "yb"};
    if (c.kind == MR_CELL_CENTER) return "0_0";
    if (c.kind == MR_CELL_HOMELAND && c.sub < 4)
        return std::string(hl[c.sub]) + "_" + std::to_string(c.x) + "_" + std::to_string(c.y);
    if (c.kind == MR_CELL_BORDER && c.sub < 4) return std::string(bl[c.sub]) + "_" + std::to_string(c.x);
    return "?";
}

std::string duration(int64_t s) {
    if (s == 0) return "0s";
    std::string out = s < 0 ? "-" : "";
    const uint64_t a = s < 0 ? uint64_t(-(s + 1)) + 1 : uint64_t(s);
    const uint64_t parts[4] = {a / 86400, a / 3600 % 24, a / 60 % 60, a % 60};
    static const char *unit[4] = {"d", "h", "m", "s"};
    for (int i = 0; i < 4; ++i)
        if (parts[i]) out += std::to_string(parts[i]) + unit[i];
    return out;
}

}  // namespace

extern "C" int64_t mr_command_time(const mr_command *c) {
    if (!c) return 0;
    static const int64_t num[4] = {1, 50, 100, 25}, den[4] = {1, 53, 109, 28};
    switch (c->kind) {
        case MR_CMD_CENTRAL:
        case MR_CMD_CARAVAN: return c->time_s;
        case MR_CMD_STANDARD:
            if (c->fleetfoot >= 1 && c->fleetfoot <= 3 && c->time_s >= 0) {
                const int64_t n = num[c->fleetfoot], d = den[c->fleetfoot];
                return (c->time_s * n + d - 1) / d;
            }
            return c->time_s;
        default: return 0;
    }
}

extern "C" int mr_duration_display(int64_t seconds, char *buf, uint64_t cap) {
    const std::string s = duration(seconds);
    if (!buf || cap < s.size() + 1) return MR_ERR_CAPACITY;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return MR_OK;
}

extern "C" int mr_render_schedule(const mr_command *cmds, uint32_t n, uint32_t arrive_at_s, uint32_t pause_s, char *buf,
                                  uint64_t cap, uint64_t *len) {
    if ((n && !cmds) || !len || arrive_at_s >= 86400) return MR_ERR_INVALID_ARG;
    std::vector<const mr_command *> rows;
    for (uint32_t i = 0; i < n; ++i)
        if (cmds[i].kind != MR_CMD_NO_MOVE) rows.push_back(&cmds[i]);
    // back-scheduled start of each row
    std::vector<int64_t> at(rows.size());
    int64_t acc = arrive_at_s;
    for (size_t k = rows.size(); k-- > 0;) {
        acc -= mr_command_time(rows[k]) + int64_t(pause_s);
        at[k] = acc;
    }
    std::string out;
    int64_t total = 0;
    for (size_t k = 0; k < rows.size(); ++k) {
        const mr_command &c = *rows[k];
        switch (c.kind) {
            case MR_CMD_CENTRAL:
            case MR_CMD_STANDARD: out += "/go_direct_" + suffix(c.to); break;
            case MR_CMD_CARAVAN: out += "/car_" + suffix(c.to); break;
            case MR_CMD_SOE: out += "/use_soe"; break;
            case MR_CMD_SHQ: out += "/use_shq"; break;
            default: out += "/use_sfm"; break;
        }
        const int64_t t = mr_command_time(&c);
        total += t + int64_t(pause_s);
        const int64_t tod = ((at[k] % 86400) + 86400) % 86400;
        char hms[16];
        std::snprintf(hms, sizeof hms, "%02d:%02d:%02d", int(tod / 3600), int(tod / 60 % 60), int(tod % 60));
        out += "\t" + duration(t) + "\t" + duration(total) + "\t" + hms + "\n";
    }
    *len = out.size();
    if (!buf || cap < out.size() + 1) return MR_ERR_CAPACITY;
    std::memcpy(buf, out.c_str(), out.size() + 1);
    return MR_OK;
}
