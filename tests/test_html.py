"""MapGrid::parse (src/grid.rs:47-133, 337-389) on the host, through the C ABI
(mr_parse_map_html / mr_grid_from_html).  CPU only: parsing and grid creation
need no device.  The reference ships no HTML map fixture, so the cases below
restate its parse rules one by one; the synthetic maps' HTML (mapgen.to_html,
the same schema) must round-trip exactly."""
import pytest

from marshrutka_amd import mapgen, pathfinder as pf
from marshrutka_amd.abi import (BLUE, CELL_BORDER, CELL_CENTER, CELL_HOMELAND, MR_ERR_INVALID_GRID, POI_CAMPFIRE,
                                POI_FORUM, POI_FOUNTAIN, POI_NONE, CellIndex)

BORDER_YB = 3


def cell(br, tr, centre="", style='style="background-color:#cccccc"', extra=""):
    inner = centre + f'<div class="top-right-text">{tr}</div>'
    if br is not None:
        inner += f'<div class="bottom-right-text">{br}</div>'
    return f'<div class="map-cell" {style}>{inner}{extra}</div>'


def grid3(centre_cell=None, **kw):
    """A 3x3 map (S = 3, H = 1) in row-major order (y = -1 first)."""
    cells = [cell("B", "1#1"), cell("BR", "1"), cell("R", "1#1"),
             cell("YB", "1"), centre_cell or cell(None, "0#0"), cell("RG", "1"),
             cell("Y", "1#1"), cell("GY", "1"), cell("G", "1#1", centre="\U0001F525")]
    for i, c in kw.get("replace", {}).items():
        cells[i] = c
    return '<html><body><div class="map-grid">' + "\n".join(cells) + "</div></body></html>"


def parse(html):
    return pf.parse_map_html(html)


@pytest.mark.parametrize("size,k,clustered", [(3, 1, False), (5, 1, False), (9, 2, False), (21, 6, True),
                                              (65, 4, False)])
def test_synthetic_maps_round_trip(size, k, clustered):
    m = mapgen.SyntheticMap(size, campfires_per_homeland=k, seed=size * 7 + k, clustered=clustered)
    assert parse(mapgen.to_html(m)) == list(m.cells())
    g = pf.MapGrid.from_html(mapgen.to_html(m))
    assert g.square_size == size


def test_cell_order_identity_and_poi():
    cells = parse(grid3())
    assert len(cells) == 9
    assert cells[4] == (CellIndex(CELL_CENTER, 0, 0, 0), POI_NONE)
    assert cells[0] == (CellIndex(CELL_HOMELAND, BLUE, 1, 1), POI_NONE)
    assert cells[3] == (CellIndex(CELL_BORDER, BORDER_YB, 1, 0), POI_NONE)
    assert cells[8][1] == POI_CAMPFIRE


@pytest.mark.parametrize("centre,poi", [
    ("\U0001F525", POI_CAMPFIRE),
    ("  \U0001F525 \n", POI_CAMPFIRE),                  # str::trim
    (" \U0001F525　", POI_CAMPFIRE),          # Unicode white space
    ("⛲", POI_FOUNTAIN), ("⛲️", POI_FOUNTAIN),
    ("\U0001F3DB", POI_FORUM), ("\U0001F3DB️", POI_FORUM),
    ("\U0001F525\U0001F525", POI_NONE),                # a two-character EmojiCode, not a campfire
    ("x\U0001F525", POI_NONE), ("\U0001F525️", POI_NONE), ("camp", POI_NONE),
])
def test_centre_poi(centre, poi):
    cells = parse(grid3(replace={0: cell("B", "1#1", centre=centre)}))
    assert cells[0][1] == poi


def test_first_nonempty_text_and_corner_rules():
    # the centre is the first non-empty direct text child; nested text does not count
    c = ('<div class="map-cell"> <span>\U0001F525</span> ⛲ '
         '<div class="top-right-text"></div><div class="top-right-text"> 1#1 </div>'
         '<div class="bottom-right-text x">R</div><div class="bottom-right-text">B</div></div>')
    cells = parse(grid3(replace={0: c}))
    # corner class must match exactly ("bottom-right-text x" is skipped), empty corners are skipped
    assert cells[0] == (CellIndex(CELL_HOMELAND, BLUE, 1, 1), POI_FOUNTAIN)


def test_tolerant_markup():
    html = grid3().replace('<div class="map-grid">',
                           '<!DOCTYPE html><!-- comment <div class="map-cell"> --><br>'
                           '<DIV CLASS="other map-grid" id=x>')
    html = html.replace('class="map-cell" style="background-color:#cccccc"',
                        "class='map-cell' data-x=1 style='color: red; background-color: #ABC'", 1)
    assert len(parse(html)) == 9


def test_only_exact_map_cell_children_count():
    extra = '<div class="map-cell extra">ignored</div><p>text</p>'
    html = grid3().replace('<div class="map-grid">', '<div class="map-grid">' + extra)
    assert len(parse(html)) == 9


def test_canonicalisation_and_numbers():
    # CellIndexBuilder::build: "B 0#1" is the YB border at shift 1 (src/index.rs:257-312);
    # numbers follow Rust's u8::from_str ('+' sign and leading zeros accepted)
    cells = parse(grid3(replace={3: cell("B", "0#1"), 0: cell("B", "+01#1")}))
    assert cells[3][0] == CellIndex(CELL_BORDER, BORDER_YB, 1, 0)
    assert cells[0][0] == CellIndex(CELL_HOMELAND, BLUE, 1, 1)
    # the Center written as a homeland cell at 0#0 is still the Center
    assert parse(grid3(centre_cell=cell("B", "0#0")))[4][0] == CellIndex(CELL_CENTER, 0, 0, 0)


@pytest.mark.parametrize("html,what", [
    ('<div class="grid"></div>', "No map-grid"),
    (grid3().replace(cell("B", "1#1"), "", 1), "not square"),
    (grid3(replace={1: cell("BR", "1", style='style="background-color:red"')}), "background-color"),
    (grid3(replace={1: cell("BR", "1", style='style="background-color:#12345"')}), "background-color"),
    (grid3(replace={1: cell("XX", "1")}), "Can not index"),
    (grid3(replace={1: cell("BR", "1#1")}), "Can not index"),
    (grid3(replace={1: cell(None, "1")}), "Can not index"),
    (grid3(centre_cell=cell("B", "1#1")), "Center is not found"),
    (grid3(replace={0: cell(None, "0#0"), 4: cell("B", "1#1")}), "Unexpected center position"),
])
def test_parse_errors(html, what):
    with pytest.raises(pf.EngineError) as e:
        parse(html)
    assert e.value.status == MR_ERR_INVALID_GRID
    assert what in str(e.value)


def test_grid_from_html_rejects_campfireless_homeland():
    # the reference reaches unreachable!() (src/grid.rs:209); the engine reports it
    html = grid3().replace("\U0001F525", "")
    with pytest.raises(pf.EngineError) as e:
        pf.MapGrid.from_html(html)
    assert e.value.status == MR_ERR_INVALID_GRID
