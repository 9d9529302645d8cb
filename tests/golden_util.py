"""Helpers to load tests/golden/*.json fixtures (inputs + expected outputs)."""
import glob
import json
import os

from marshrutka_amd.abi import CellIndex, Params
from marshrutka_amd.mapgen import SyntheticMap

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.json")))


def load(name):
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        d = json.load(f)
    m = SyntheticMap.from_json(d["map"])
    queries = [(CellIndex(*a), CellIndex(*b)) for a, b in d["queries"]]
    runs = [(Params.from_json(r["params"]), r["expected"]) for r in d["runs"]]
    return m, queries, runs


def as_expected(label):
    """TotalCost -> the fixture's list form."""
    if label is None:
        return None
    return [label.legs, label.money, label.time_s,
            [[c.kind, c.time_s, c.legs, c.money, c.fleetfoot,
              [c.from_.kind, c.from_.sub, c.from_.x, c.from_.y],
              [c.to.kind, c.to.sub, c.to.x, c.to.y]] for c in label.commands]]
