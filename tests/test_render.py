"""The app's command table (src/app.rs:481-561) rendered by the host library
(mr_render_schedule), against hand-derived rows and against the test-side
restatement in oracle/py_ref.py over every golden label.  CPU only."""
import pytest

import py_ref
from golden_util import fixture_names, load
from marshrutka_amd import pathfinder as pf
from marshrutka_amd.abi import CellIndex, Command, TotalCost

CENTER = CellIndex.center()


def B(x, y):
    return CellIndex.parse(f"B {x}#{y}")


def label(cmds):
    return TotalCost(0, 0, 0, cmds)


def test_kat5_rows():
    # KAT5: Std{540,3} B2#2->BR1, Central{20} BR1->RG1, Std{540,3} RG1->G2#2;
    # arrive at 12:00:00, 5 s between commands
    br1, rg1, g22 = CellIndex.parse("BR 1"), CellIndex.parse("RG 1"), CellIndex.parse("G 2#2")
    cmds = [Command(2, 540, 3, 0, 0, B(2, 2), br1), Command(1, 20, 0, 0, 0, br1, rg1),
            Command(2, 540, 3, 0, 0, rg1, g22)]
    assert pf.render_schedule(label(cmds), 12 * 3600, 5) == [
        ("/go_direct_br_1", "9m", "9m5s", "11:41:25"),      # 12:00:00 - 3 x (t + 5 s), back to front
        ("/go_direct_rg_1", "20s", "9m30s", "11:50:30"),
        ("/go_direct_g_2_2", "9m", "18m35s", "11:50:55"),
    ]


def test_fleetfoot_scrolls_caravans_and_midnight_wrap():
    cf = B(3, 3)
    cmds = [Command(0, 0, 0, 0, 0, cf, cf),                      # NoMove rows are skipped
            Command(4, 0, 0, 50, 0, cf, B(1, 1)),               # SoE
            Command(2, 180 * 7, 7, 0, 1, B(1, 1), B(4, 4)),     # Fleetfoot 1: ceil(1260*50/53) = 1189
            Command(3, 1440, 0, 12, 0, B(4, 4), CENTER),        # caravan
            Command(5, 0, 0, 75, 0, CENTER, B(2, 2)),           # SHQ
            Command(6, 0, 0, 100, 0, B(2, 2), CENTER)]          # SFm
    rows = pf.render_schedule(label(cmds), 60, 0)
    assert [r[0] for r in rows] == ["/use_soe", "/go_direct_b_4_4", "/car_0_0", "/use_shq", "/use_sfm"]
    assert [r[1] for r in rows] == ["0s", "19m49s", "24m", "0s", "0s"]
    assert rows[-1][2] == "43m49s"
    assert rows[0][3] == "23:17:11"  # 00:01:00 - 43m49s wraps past midnight


def test_duration_display_pinned():
    import ctypes as C
    buf = C.create_string_buffer(32)
    for s, txt in ((63 * 60 + 10, "1h3m10s"), (0, "0s"), (86400 + 61, "1d1m1s"), (59, "59s")):
        assert pf.lib().mr_duration_display(s, buf, 32) == 0
        assert buf.value.decode() == txt == py_ref.duration_str(s)


@pytest.mark.parametrize("name", fixture_names())
def test_golden_labels_render_like_the_restatement(name):
    _, _, runs = load(name)
    n = 0
    for _, expected in runs:
        for e in expected:
            if e is None:
                continue
            legs, money, time_s, cmds = e
            lab = TotalCost(legs, money, time_s, [
                Command(k, t, lg, mn, ff, CellIndex(*fr), CellIndex(*to)) for k, t, lg, mn, ff, fr, to in cmds])
            lj = {"commands": [{"kind": k, "time_s": t, "legs": lg, "money": mn, "fleetfoot": ff, "from": fr, "to": to}
                               for k, t, lg, mn, ff, fr, to in cmds]}
            for arrive, pause in ((0, 0), (12 * 3600 + 34, 7)):
                assert pf.render_schedule(lab, arrive, pause) == py_ref.render_schedule(lj, arrive, pause)
            n += 1
    assert n > 0
