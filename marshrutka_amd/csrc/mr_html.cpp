// MapGrid::parse (src/grid.rs:47-133, 337-389; src/cell.rs:45-57,192-201;
// src/index.rs:392-466) restated for the engine's boundary: the reference's HTML
// map format -> row-major mr_cell records (then mr_grid_create).
//
// The reference parses with the `tl` crate (0.7.8) and reads, in order:
//  * the first element whose class list contains "map-grid";
//  * its direct children whose class attribute is exactly "map-cell", row-major,
//    x and y running from -S/2 to S/2 (the count must be a perfect square);
//  * per cell: an optional inline `background-color` (must be a hex colour),
//    the corner texts (first direct child with class exactly "<corner>-text"
//    that has non-empty text) and the centre text (first non-empty direct text
//    child), every text taken raw and trimmed of Unicode white space;
//  * identity from (bottom-right, top-right): "<H> x#y" (H in B R G Y) or
//    "<BR|RG|GY|YB> shift", canonicalised by CellIndexBuilder::build, or no
//    bottom-right with top-right "0#0" for the Center, which must sit at (0,0);
//  * PoI from the centre: a text of one or two characters is an EmojiCode;
//    U+1F525 is a campfire, U+26F2 [U+FE0F] a fountain, U+1F3DB [U+FE0F] a forum.
// Numbers parse like Rust's u8::from_str (optional '+', decimal digits) but up to
// 65535 (the boundary's u16 widths; the reference stops at 255).
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/marshrutka_pf.h"

namespace mr {
mr_cell_index build_index(const mr_cell_index &c);  // CellIndexBuilder::build (mr_host.cpp)
}

namespace {

struct Node {
    bool tag = false;
    std::string_view name, cls, style, text;
    bool has_cls = false, has_style = false;
    std::vector<uint32_t> kids;
};

bool ieq(std::string_view a, std::string_view b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
        char x = a[i], y = b[i];
        if (x >= 'A' && x <= 'Z') x = char(x - 'A' + 'a');
        if (y >= 'A' && y <= 'Z') y = char(y - 'A' + 'a');
        if (x != y) return false;
    }
    return true;
}
bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f'; }
bool is_void(std::string_view n) {
    static const char *v[] = {"area", "base", "br", "col", "embed", "hr", "img", "input",
                              "link", "meta", "param", "source", "track", "wbr"};
    for (const char *x : v)
        if (ieq(n, x)) return true;
    return false;
}

// A tolerant HTML tree: comments, doctypes and processing instructions are
// skipped, void and self-closed elements take no children, script/style bodies
// are skipped, an end tag closes the nearest open element of its name (a stray
// one is ignored) and unclosed elements end with the input.
class Tree {
  public:
    std::vector<Node> nodes;
    explicit Tree(std::string_view s) : s_(s) {
        nodes.emplace_back();  // root
        nodes[0].tag = true;
        build();
    }

  private:
    std::string_view s_;
    void add_child(std::vector<uint32_t> &open, Node &&n) {
        const uint32_t id = uint32_t(nodes.size());
        nodes.push_back(std::move(n));
        nodes[open.back()].kids.push_back(id);
    }
    void build() {
        std::vector<uint32_t> open{0};
        const size_t n = s_.size();
        size_t i = 0;
        while (i < n) {
            if (s_[i] != '<') {
                const size_t j = s_.find('<', i);
                Node t;
                t.text = s_.substr(i, (j == std::string_view::npos ? n : j) - i);
                add_child(open, std::move(t));
                i = j == std::string_view::npos ? n : j;
                continue;
            }
            if (s_.compare(i, 4, "<!--") == 0) {
                const size_t j = s_.find("-->", i + 4);
                i = j == std::string_view::npos ? n : j + 3;
                continue;
            }
            if (i + 1 < n && (s_[i + 1] == '!' || s_[i + 1] == '?')) {
                const size_t j = s_.find('>', i);
                i = j == std::string_view::npos ? n : j + 1;
                continue;
            }
            if (i + 1 < n && s_[i + 1] == '/') {  // end tag
                size_t k = i + 2;
                while (k < n && !is_space(s_[k]) && s_[k] != '>') ++k;
                const std::string_view name = s_.substr(i + 2, k - i - 2);
                const size_t j = s_.find('>', k);
                for (size_t d = open.size(); d-- > 1;)
                    if (ieq(nodes[open[d]].name, name)) {
                        open.resize(d);
                        break;
                    }
                i = j == std::string_view::npos ? n : j + 1;
                continue;
            }
            if (i + 1 >= n || !((s_[i + 1] >= 'a' && s_[i + 1] <= 'z') || (s_[i + 1] >= 'A' && s_[i + 1] <= 'Z'))) {
                Node t;  // a lone '<' is text
                t.text = s_.substr(i, 1);
                add_child(open, std::move(t));
                ++i;
                continue;
            }
            size_t k = i + 1;
            while (k < n && !is_space(s_[k]) && s_[k] != '>' && s_[k] != '/') ++k;
            Node e;
            e.tag = true;
            e.name = s_.substr(i + 1, k - i - 1);
            bool self_close = false;
            while (k < n) {  // attributes
                while (k < n && is_space(s_[k])) ++k;
                if (k >= n) break;
                if (s_[k] == '>') {
                    ++k;
                    break;
                }
                if (s_[k] == '/') {
                    if (k + 1 < n && s_[k + 1] == '>') {
                        self_close = true;
                        k += 2;
                        break;
                    }
                    ++k;
                    continue;
                }
                const size_t a0 = k;
                while (k < n && !is_space(s_[k]) && s_[k] != '=' && s_[k] != '>' && s_[k] != '/') ++k;
                const std::string_view an = s_.substr(a0, k - a0);
                while (k < n && is_space(s_[k])) ++k;
                std::string_view av;
                bool has_v = false;
                if (k < n && s_[k] == '=') {
                    ++k;
                    while (k < n && is_space(s_[k])) ++k;
                    if (k < n && (s_[k] == '"' || s_[k] == '\'')) {
                        const char q = s_[k];
                        const size_t e0 = k + 1, e1 = s_.find(q, e0);
                        av = s_.substr(e0, (e1 == std::string_view::npos ? n : e1) - e0);
                        k = e1 == std::string_view::npos ? n : e1 + 1;
                    } else {
                        const size_t e0 = k;
                        while (k < n && !is_space(s_[k]) && s_[k] != '>') ++k;
                        av = s_.substr(e0, k - e0);
                    }
                    has_v = true;
                }
                if (ieq(an, "class") && !e.has_cls) {
                    e.cls = av;
                    e.has_cls = has_v;
                } else if (ieq(an, "style") && !e.has_style) {
                    e.style = av;
                    e.has_style = has_v;
                }
            }
            const std::string_view name = e.name;
            add_child(open, std::move(e));
            const uint32_t id = uint32_t(nodes.size() - 1);
            i = k;
            if (ieq(name, "script") || ieq(name, "style")) {  // raw text body
                size_t j = i;
                for (;;) {
                    j = s_.find("</", j);
                    if (j == std::string_view::npos || s_.compare(j + 2, name.size(), name) == 0 ||
                        ieq(s_.substr(j + 2, name.size()), name))
                        break;
                    j += 2;
                }
                const size_t e = j == std::string_view::npos ? n : s_.find('>', j);
                i = e == std::string_view::npos ? n : e + 1;
                continue;
            }
            if (!self_close && !is_void(name)) open.push_back(id);
        }
    }
};

// UTF-8 code points of s (invalid bytes become U+FFFD)
std::vector<uint32_t> code_points(std::string_view s) {
    std::vector<uint32_t> out;
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = static_cast<unsigned char>(s[i]);
        uint32_t cp = 0xFFFD;
        size_t len = 1;
        if (c < 0x80) cp = c;
        else if ((c >> 5) == 6 && i + 1 < s.size()) cp = ((c & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu), len = 2;
        else if ((c >> 4) == 14 && i + 2 < s.size())
            cp = ((c & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu), len = 3;
        else if ((c >> 3) == 30 && i + 3 < s.size())
            cp = ((c & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu),
            len = 4;
        out.push_back(cp);
        i += len;
    }
    return out;
}
// char::is_whitespace (Unicode White_Space)
bool uspace(uint32_t c) {
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
// str::trim on a UTF-8 view: drop leading/trailing white space code points
std::string_view trim(std::string_view s) {
    size_t b = 0, e = s.size();
    while (b < e) {
        const auto cp = code_points(s.substr(b, std::min<size_t>(4, e - b)));
        if (cp.empty() || !uspace(cp[0])) break;
        b += cp[0] < 0x80 ? 1 : cp[0] < 0x800 ? 2 : cp[0] < 0x10000 ? 3 : 4;
    }
    while (e > b) {
        size_t k = e - 1;
        while (k > b && (static_cast<unsigned char>(s[k]) & 0xC0) == 0x80) --k;
        const auto cp = code_points(s.substr(k, e - k));
        if (cp.empty() || !uspace(cp[0])) break;
        e = k;
    }
    return s.substr(b, e - b);
}

// parse_text (src/grid.rs:362-369): the first direct text child, trimmed, non-empty
bool first_text(const Tree &t, uint32_t el, std::string_view &out) {
    for (uint32_t k : t.nodes[el].kids) {
        const Node &c = t.nodes[k];
        if (c.tag) continue;
        const std::string_view x = trim(c.text);
        if (!x.empty()) {
            out = x;
            return true;
        }
    }
    return false;
}
// parse_cell_element (src/grid.rs:337-342)
bool corner_text(const Tree &t, uint32_t cell, std::string_view cls, std::string_view &out) {
    for (uint32_t k : t.nodes[cell].kids) {
        const Node &c = t.nodes[k];
        if (c.tag && c.has_cls && c.cls == cls && first_text(t, k, out)) return true;
    }
    return false;
}
bool has_class_token(const Node &n, std::string_view name) {
    if (!n.has_cls) return false;
    std::string_view c = n.cls;
    size_t i = 0;
    while (i < c.size()) {
        while (i < c.size() && is_space(c[i])) ++i;
        size_t j = i;
        while (j < c.size() && !is_space(c[j])) ++j;
        if (j > i && c.substr(i, j - i) == name) return true;
        i = j;
    }
    return false;
}
// Color32::from_hex: #rgb, #rgba, #rrggbb or #rrggbbaa
bool hex_colour(std::string_view v) {
    if (v.empty() || v[0] != '#') return false;
    const size_t n = v.size() - 1;
    if (n != 3 && n != 4 && n != 6 && n != 8) return false;
    for (size_t i = 1; i < v.size(); ++i) {
        const char c = v[i];
        if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
    }
    return true;
}
// parse_bg_color_from_style (src/grid.rs:371-385): the first background-color
// declaration of the inline style must be a hex colour
bool style_ok(const Node &n) {
    if (!n.has_style) return true;
    std::string_view s = n.style;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(';', i);
        if (j == std::string_view::npos) j = s.size();
        const std::string_view decl = s.substr(i, j - i);
        const size_t c = decl.find(':');
        if (c != std::string_view::npos && trim(decl.substr(0, c)) == "background-color")
            return hex_colour(trim(decl.substr(c + 1)));
        i = j + 1;
    }
    return true;
}
// Rust's u8::from_str syntax (optional '+', decimal digits), widened to u16
bool parse_u16(std::string_view s, uint32_t &v) {
    if (!s.empty() && s[0] == '+') s.remove_prefix(1);
    if (s.empty()) return false;
    v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return false;
        v = v * 10 + uint32_t(c - '0');
        if (v > 65535) return false;
    }
    return true;
}
bool parse_pos(std::string_view s, uint32_t &x, uint32_t &y) {
    const size_t h = s.find('#');
    return h != std::string_view::npos && parse_u16(s.substr(0, h), x) && parse_u16(s.substr(h + 1), y);
}
int homeland_of(std::string_view s) {
    if (s == "B") return MR_HOMELAND_BLUE;
    if (s == "R") return MR_HOMELAND_RED;
    if (s == "G") return MR_HOMELAND_GREEN;
    if (s == "Y") return MR_HOMELAND_YELLOW;
    return -1;
}
int border_of(std::string_view s) {
    if (s == "BR") return MR_BORDER_BR;
    if (s == "RG") return MR_BORDER_RG;
    if (s == "GY") return MR_BORDER_GY;
    if (s == "YB") return MR_BORDER_YB;
    return -1;
}
// CellIndex::try_from((bottom-right, top-right)) (src/index.rs:431-443), before build()
bool cell_index(bool has_a, std::string_view a, bool has_b, std::string_view b, mr_cell_index &c) {
    std::memset(&c, 0, sizeof(c));
    if (has_a && has_b) {
        uint32_t x, y, s;
        const int h = homeland_of(a);
        if (h >= 0 && parse_pos(b, x, y)) {
            c.kind = MR_CELL_HOMELAND;
            c.sub = uint8_t(h);
            c.x = uint16_t(x);
            c.y = uint16_t(y);
            return true;
        }
        const int bd = border_of(a);
        if (bd >= 0 && parse_u16(b, s)) {
            c.kind = MR_CELL_BORDER;
            c.sub = uint8_t(bd);
            c.x = uint16_t(s);
            return true;
        }
        return false;
    }
    if (!has_a && has_b && b == "0#0") {
        c.kind = MR_CELL_CENTER;
        return true;
    }
    return false;
}
// cell_parts (src/cell.rs:192-201) on CellElement::try_from (src/cell.rs:45-57)
uint8_t poi_of(bool has, std::string_view centre) {
    if (!has) return MR_POI_NONE;
    const auto cp = code_points(centre);
    if (cp.size() == 1 && cp[0] == 0x1F525) return MR_POI_CAMPFIRE;
    if ((cp.size() == 1 || (cp.size() == 2 && cp[1] == 0xFE0F)) && cp[0] == 0x26F2) return MR_POI_FOUNTAIN;
    if ((cp.size() == 1 || (cp.size() == 2 && cp[1] == 0xFE0F)) && cp[0] == 0x1F3DB) return MR_POI_FORUM;
    return MR_POI_NONE;
}

thread_local std::string g_parse_error;

int parse(std::string_view html, std::vector<mr_cell> &cells) {
    Tree t(html);
    uint32_t grid = 0;
    for (uint32_t i = 1; i < t.nodes.size() && !grid; ++i)
        if (t.nodes[i].tag && has_class_token(t.nodes[i], "map-grid")) grid = i;
    if (!grid) {
        g_parse_error = "No map-grid elements found";
        return MR_ERR_INVALID_GRID;
    }
    std::vector<uint32_t> mc;
    for (uint32_t k : t.nodes[grid].kids)
        if (t.nodes[k].tag && t.nodes[k].has_cls && t.nodes[k].cls == "map-cell") mc.push_back(k);
    uint32_t side = 0;
    while (uint64_t(side + 1) * (side + 1) <= mc.size()) ++side;
    if (uint64_t(side) * side != mc.size()) {
        g_parse_error = "Map grid is not square: " + std::to_string(mc.size());
        return MR_ERR_INVALID_GRID;
    }
    const int half = int(side / 2);
    cells.assign(mc.size(), mr_cell{});
    bool centre_seen = false;
    for (size_t i = 0; i < mc.size(); ++i) {
        const uint32_t e = mc[i];
        if (!style_ok(t.nodes[e])) {
            g_parse_error = "invalid background-color in map cell " + std::to_string(i);
            return MR_ERR_INVALID_GRID;
        }
        std::string_view br, tr, centre;
        const bool has_br = corner_text(t, e, "bottom-right-text", br);
        const bool has_tr = corner_text(t, e, "top-right-text", tr);
        const bool has_c = first_text(t, e, centre);
        mr_cell &c = cells[i];
        if (!cell_index(has_br, br, has_tr, tr, c.index)) {
            g_parse_error = "Can not index cell " + std::string(br) + " " + std::string(tr);
            return MR_ERR_INVALID_GRID;
        }
        c.index = mr::build_index(c.index);
        c.poi = poi_of(has_c, centre);
        // x, y run row-major from -S/2; the Center must sit at (0, 0) (src/grid.rs:122-133).
        // (For an even count the reference's row wrap differs; mr_grid_create rejects even sides.)
        const int x = int(i % side) - half, y = int(i / side) - half;
        if (c.index.kind == MR_CELL_CENTER) {
            if (x != 0 || y != 0) {
                g_parse_error = "Unexpected center position: (" + std::to_string(x) + ", " + std::to_string(y) + ")";
                return MR_ERR_INVALID_GRID;
            }
            centre_seen = true;
        }
    }
    if (!centre_seen) {
        g_parse_error = "Center is not found";
        return MR_ERR_INVALID_GRID;
    }
    return MR_OK;
}

}  // namespace

extern "C" int mr_parse_map_html(const char *html, uint64_t len, mr_cell *cells, uint32_t cap, uint32_t *n_cells) {
    if (!html || !n_cells) return MR_ERR_INVALID_ARG;
    std::vector<mr_cell> v;
    const int st = parse(std::string_view(html, size_t(len)), v);
    if (st != MR_OK) return st;
    *n_cells = uint32_t(v.size());
    if (cap < v.size() || (!cells && !v.empty())) return MR_ERR_CAPACITY;
    if (!v.empty()) std::memcpy(cells, v.data(), v.size() * sizeof(mr_cell));
    return MR_OK;
}

extern "C" const char *mr_parse_error(void) { return g_parse_error.c_str(); }

extern "C" int mr_grid_from_html(const char *html, uint64_t len, mr_grid **out) {
    if (!html || !out) return MR_ERR_INVALID_ARG;
    std::vector<mr_cell> v;
    const int st = parse(std::string_view(html, size_t(len)), v);
    if (st != MR_OK) return st;
    return mr_grid_create(v.data(), uint32_t(v.size()), out);
}
