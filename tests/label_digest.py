"""Vectorised label digests for full-size parity checks (test infrastructure).

A label's command list is hashed exactly as the oracle's `label_digest`
(oracle/mr_oracle.cpp): each 40 B mr_command as five little-endian u64 words
(reserved bytes zero), h = Horner over the words with P, the list's digest
H = Horner over the commands' h with Q, everything mod 2^64.  Comparing
(legs, money, time, command count, digest) per label compares whole labels with
numpy instead of one Python object per label, which is what makes every-cell
checks at 1025^2 and 4097^2 affordable.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from marshrutka_amd.abi import mr_command, mr_result

P = np.uint64(0x9E3779B97F4A7C15)
Q = np.uint64(0xC2B2AE3D27D4EB4F)

RESULT_DT = np.dtype([("legs", "<u4"), ("money", "<u4"), ("time_s", "<i8"), ("n", "<u4"), ("off", "<u4"),
                      ("status", "<i4"), ("reserved", "<u4")])
assert RESULT_DT.itemsize == C.sizeof(mr_result)


def command_hashes(pool, n_cmds: int) -> np.ndarray:
    """h per command of the first n_cmds entries of an mr_command array (ctypes
    array, bytes-like or numpy view of 40 B records)."""
    w = np.frombuffer(pool, dtype="<u8", count=n_cmds * 5).reshape(n_cmds, 5)
    h = np.zeros(n_cmds, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(5):
            h = h * P + w[:, j]
    return h


def digests(results, pool, n: int, pool_len: int = 0) -> dict:
    """Per label of an mr_result array (n entries; its commands at
    pool[command_offset ...]): legs, money, time_s, n_commands, status, digest."""
    r = np.frombuffer(results, dtype=RESULT_DT, count=n)
    ncmd = r["n"].astype(np.int64)
    ok = (r["status"] == 0)
    ncmd = np.where(ok, ncmd, 0)
    total = int(ncmd.sum())
    if pool_len == 0:
        pool_len = int((r["off"].astype(np.int64) + ncmd).max()) if n else 0
    h = command_hashes(pool, pool_len) if pool_len else np.zeros(0, np.uint64)
    starts = np.repeat(r["off"].astype(np.int64), ncmd)
    within = np.arange(total, dtype=np.int64) - np.repeat(np.cumsum(ncmd) - ncmd, ncmd)
    lab = np.repeat(np.arange(n, dtype=np.int64), ncmd)
    e = np.repeat(ncmd, ncmd) - 1 - within  # Q^(len-1-j)
    maxe = int(e.max()) + 1 if total else 1
    powq = np.ones(maxe, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(1, maxe):
            powq[i] = powq[i - 1] * Q
        terms = h[starts + within] * powq[e]
        cs = np.concatenate([[np.uint64(0)], np.cumsum(terms, dtype=np.uint64)])
        ends = np.cumsum(ncmd)
        dig = cs[ends] - cs[ends - ncmd]
    del lab
    return {"legs": r["legs"].copy(), "money": r["money"].copy(), "time_s": r["time_s"].copy(),
            "n_commands": np.where(ok, r["n"], 0).astype(np.uint32), "status": r["status"].copy(),
            "digest": np.where(ok, dig, np.uint64(0))}


CMD_DT = np.dtype([("kind", "u1"), ("r0", "u1", (3,)), ("legs", "<u4"), ("money", "<u4"), ("fleetfoot", "<u4"),
                   ("time_s", "<i8"), ("from", "<u8"), ("to", "<u8")])
assert CMD_DT.itemsize == C.sizeof(mr_command)


def cell_keys(cells_array) -> np.ndarray:
    """The 8-byte mr_cell_index of every cell (mapgen cells_array) as one u64 each,
    comparable with the `from`/`to` words of CMD_DT."""
    raw = np.ascontiguousarray(cells_array).view(np.uint8).reshape(len(cells_array), -1)[:, :8]
    return np.ascontiguousarray(raw).view("<u8").ravel()


def label_properties(results, pool, n: int, src_keys, dst_keys, fleetfoot_ratio=None) -> dict:
    """Size-independent properties of n labels (mr_result array + command pool) that
    every reference label has (src/cost.rs:208-315): found; the commands form a chain
    from the query's source to its destination; no two adjacent StandardMoves or
    CentralMoves (runs merge); legs and money are the commands' sums and time is the
    sum of AggregatedCost::time (a StandardMove run's raw time through the Fleetfoot
    ceil, fleetfoot_ratio=(num, den)).  Returns counts of violations per property."""
    r = np.frombuffer(results, dtype=RESULT_DT, count=n)
    ncmd = r["n"].astype(np.int64)
    total = int(ncmd.sum())
    end = int((r["off"].astype(np.int64) + ncmd).max()) if n else 0
    cm = np.frombuffer(pool, dtype=CMD_DT, count=end)
    first = r["off"].astype(np.int64)
    last = first + ncmd - 1
    idx = np.repeat(first, ncmd) + (np.arange(total) - np.repeat(np.cumsum(ncmd) - ncmd, ncmd))
    lab = np.repeat(np.arange(n), ncmd)
    c = cm[idx]
    out = {"not_ok": int((r["status"] != 0).sum()), "empty": int((ncmd == 0).sum())}
    ok = ncmd > 0
    out["bad_from"] = int((cm["from"][first[ok]] != np.asarray(src_keys)[ok]).sum())
    out["bad_to"] = int((cm["to"][last[ok]] != np.asarray(dst_keys)[ok]).sum())
    same = lab[1:] == lab[:-1]
    out["broken_chain"] = int((same & (c["to"][:-1] != c["from"][1:])).sum())
    out["unmerged_run"] = int((same & (c["kind"][:-1] == c["kind"][1:]) & ((c["kind"][1:] == 1) |
                                                                            (c["kind"][1:] == 2))).sum())
    t = c["time_s"].astype(np.int64)
    if fleetfoot_ratio is not None:
        num, den = fleetfoot_ratio
        std = c["kind"] == 2
        t = np.where(std, (t * num + den - 1) // den, t)
    for f, vals in (("legs", c["legs"].astype(np.int64)), ("money", c["money"].astype(np.int64)), ("time_s", t)):
        s = np.zeros(n, dtype=np.int64)
        np.add.at(s, lab, vals)
        out["bad_" + f] = int((s != r[f].astype(np.int64)).sum())
    return out


FIELDS = ("status", "legs", "money", "time_s", "n_commands", "digest")
R = np.uint64(0xFF51AFD7ED558CCD)


def cell_hashes(d: dict) -> np.ndarray:
    """One u64 per label over every compared field (Horner with P, mod 2^64)."""
    h = np.zeros(np.asarray(d["digest"]).shape, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for f in FIELDS:
            h = h * P + np.asarray(d[f]).astype(np.int64).astype(np.uint64)
    return h


def row_checksums(d: dict, side: int) -> np.ndarray:
    """A checksum per grid row of one source's row-major labels (Horner with R over
    the row's cell hashes): a whole 4097^2 all-destinations answer in 32 KB, for
    golden fixtures (tests/golden/make_full_scale.py)."""
    h = cell_hashes(d).reshape(side, side)
    powr = np.ones(side, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(side - 2, -1, -1):
            powr[i] = powr[i + 1] * R
        return (h * powr[None, :]).sum(axis=1, dtype=np.uint64)


def mismatches(got: dict, exp: dict, idx_got=None, idx_exp=None) -> np.ndarray:
    """Indices (into the compared selection) where any field differs."""
    bad = None
    for f in FIELDS:
        a = got[f] if idx_got is None else got[f][idx_got]
        b = exp[f] if idx_exp is None else exp[f][idx_exp]
        d = np.asarray(a).astype(np.int64) != np.asarray(b).astype(np.int64) if f != "digest" else \
            np.asarray(a) != np.asarray(b)
        bad = d if bad is None else (bad | d)
    return np.nonzero(bad)[0]
