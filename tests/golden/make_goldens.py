#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE itself (oracle/_ref/libref.so).

libref.so is the reference's own src/query.c index.c multimap.c utils.c compiled
unchanged (oracle/Makefile). This script feeds it the SURVEY.md §8(c) synthetic
inputs through its real operator API (select_column -> fetch_column -> sum /
average / min / max, hash_join, nested_loop_join, shared_select) and records:

  goldens.json          scalar goldens: K, FNV-1a-64 of the position list, sums,
                        avg (value + IEEE bits), min/max, join pair hashes
  col_n65536_s42.bin    the 64K-row int32 input column (seed 42)
  pos_n65536_s42_sel*.bin   the reference's position lists for it

and cross-checks every value it also finds in SURVEY.md §8(c) (the survey's
numbers were produced by the same reference). Run here, where /root/reference
exists:  python tests/golden/make_goldens.py [--big]
(--big adds the N = 1e9 rows: ~8 GB RAM, a few minutes.)
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
from refapi import Api, make_column  # noqa: E402

# SURVEY.md §8(c) values (reference query.c), used to pin this run.
SURVEY = {
    (65536, 0.01): (652, 0x16960983675B5D2E, 10898381, 0x40D052D3BAE54CF5, 16385, 17038),
    (65536, 0.5): (32988, 0x7A7CC0284FEC86F3, 1080189697, 0x40DFFA3B6A612902, 16385, 49151),
    (65536, 1.0): (49351, 0xD4CD561C731E1EC5, 2018438094, 0x40E3F874744CCB13, 16385, 65535),
    (10_000_000, 0.01): (99906, 0x094395C47FF9FFC6, 254750907685, 0x41437448FE867C47, 2500000,
                         2599999),
    (10_000_000, 0.5): (5001206, 0x714AF0C30EBD65E5, 25002529069401, 0x41531220FEE4F4BE, 2500000,
                        7499995),
    (1_000_000_000, 0.01): (10001128, 0x38B1E2BAC2A24D13, 2550280400734742, 0x41AE65F5D84F6C66,
                            250000000, 259999999),
    (1_000_000_000, 0.5): (499982359, 0xF847EE6039FF377E, 249990219230110093, 0x41BDCD5D7F647815,
                           250000000, 749999999),
}
SURVEY_COLSUM = {65536: 2150627798, 10_000_000: 49997058392193,
                 1_000_000_000: 500016416298104597}
SURVEY_JOIN = {1 << 16: (32925, 0x12473D57AA0A87A5), 1 << 20: (524057, 0x14781DB9879F41D7),
               1 << 24: (8384728, 0x06459D15CFB9499A)}
SURVEY_CFG3 = {10_000_000: (99906, 499302949274, 0x41531097D6D028EB, 43, 9999799),
               1_000_000_000: (10001128, 5000678708721025, 0x41BDCD91CD940DB4, 142, 999999983)}
SURVEY_CFG4 = {42: (10001128, 2550280400734742), 43: (9998889, 2549721978156000),
               44: (10000200, 2550057357687352), 45: (9998973, 2549734091221315),
               46: (10000794, 2550193354897805), 47: (10004418, 2551125348316285),
               48: (9997914, 2549456017591494), 49: (10003437, 2550884911353056)}


def dbits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def bounds(n: int, sel: float):
    lo = int(0.25 * n)
    return lo, lo + int(sel * n)


def select_chain(api: Api, n: int, seed: int, sel: float, fetch_seed: int | None = None):
    d = refcpu.gen_uniform(n, seed)
    col = make_column(d)
    lo, hi = bounds(n, sel)
    pos = api.select_column(col, lo, hi)
    if fetch_seed is None:
        vals = api.fetch_column(col, pos)
    else:
        d2 = refcpu.gen_uniform(n, fetch_seed)
        vals = api.fetch_column(make_column(d2), pos)
        del d2
    row = {"n": n, "seed": seed, "sel": sel, "low": lo, "high": hi, "k": int(len(pos)),
           "pos_fnv1a64": f"{refcpu.fnv1a64(pos):016x}", "sum": api.sum_result(vals)}
    avg = api.average(vals)
    row.update({"avg": avg, "avg_bits": f"{dbits(avg):016x}", "min": api.min(vals),
                "max": api.max(vals)})
    if fetch_seed is not None:
        row["fetch_seed"] = fetch_seed
    return row, d, pos


def check(cond: bool, what: str) -> None:
    if not cond:
        raise SystemExit(f"golden pin FAILED: {what}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also the N = 1e9 rows")
    args = ap.parse_args()
    if not refcpu.have_reference():
        raise SystemExit("oracle/_ref/libref.so missing: run make -C oracle here first")
    api = Api(refcpu.reference())
    out = {"generator": "tests/golden/make_goldens.py via oracle/_ref/libref.so "
                        "(reference src/query.c index.c multimap.c utils.c, gcc -O2)",
           "data": "col[i] = (int32)(sm64(seed*0x100000001B3 + i) % N); "
                   "low = int(0.25 N), high = low + int(sel N)",
           "select": [], "column_sum": {}, "config3": [], "config4": [], "join": []}
    sizes = [65536, 10_000_000] + ([1_000_000_000] if args.big else [])
    for n in sizes:
        for sel in ([0.01, 0.5, 1.0] if n == 65536 else [0.01, 0.5]):
            row, d, pos = select_chain(api, n, 42, sel)
            s = SURVEY.get((n, sel))
            if s:
                check((row["k"], int(row["pos_fnv1a64"], 16), row["sum"], int(row["avg_bits"], 16),
                       row["min"], row["max"]) == s, f"select n={n} sel={sel}: {row}")
            out["select"].append(row)
            print("select", row, flush=True)
            if n == 65536:
                d.tofile(os.path.join(HERE, "col_n65536_s42.bin"))
                pos.astype(np.int32).tofile(os.path.join(HERE, f"pos_n65536_s42_sel{sel}.bin"))
            del d, pos
        d = refcpu.gen_uniform(n, 42)
        cs = api.sum_column(make_column(d))
        del d
        check(cs == SURVEY_COLSUM[n], f"column sum n={n}: {cs}")
        out["column_sum"][str(n)] = cs
        # config 3: select col0 (seed 42) at 1%, fetch col1 (seed 43), avg
        if n in SURVEY_CFG3:
            row, _, _ = select_chain(api, n, 42, 0.01, fetch_seed=43)
            s = SURVEY_CFG3[n]
            check((row["k"], row["sum"], int(row["avg_bits"], 16), row["min"], row["max"]) == s,
                  f"config3 n={n}: {row}")
            out["config3"].append(row)
            print("config3", row, flush=True)
    if args.big:
        for seed in range(42, 50):
            n = 1_000_000_000
            d = refcpu.gen_uniform(n, seed)
            lo, hi = bounds(n, 0.01)
            pos = api.select_column(make_column(d), lo, hi)
            vals = d[pos]
            row = {"n": n, "seed": seed, "sel": 0.01, "low": lo, "high": hi, "k": int(len(pos)),
                   "sum": api.sum_result(vals)}
            check((row["k"], row["sum"]) == SURVEY_CFG4[seed], f"config4 seed {seed}: {row}")
            out["config4"].append(row)
            print("config4", row, flush=True)
            del d, pos, vals
        tk = sum(r["k"] for r in out["config4"])
        ts = sum(r["sum"] for r in out["config4"])
        out["config4_combined"] = {"k": tk, "sum": ts, "avg": ts / tk}
    for logn in (16, 20):
        n = 1 << logn
        a, b = refcpu.gen_join(n, "build"), refcpu.gen_join(n, "probe")
        p = refcpu.gen_join(n, "iota")
        o1, o2 = api.join(a, p, b, p, "hash")
        row = {"n": n, "kind": "hash", "m": int(len(o1)),
               "pairs_fnv1a64": f"{refcpu.fnv1a64_pairs(o1, o2):016x}"}
        check((row["m"], int(row["pairs_fnv1a64"], 16)) == SURVEY_JOIN[n], f"join {row}")
        out["join"].append(row)
        print("join", row, flush=True)
    # small many-to-many joins (duplicate keys on both sides), hash and nested loop
    for kind in ("hash", "nested"):
        rng = np.random.default_rng(7)
        c1 = rng.integers(0, 50, 3000, dtype=np.int32)
        c2 = rng.integers(0, 60, 2000, dtype=np.int32)
        p1 = np.arange(3000, dtype=np.int32) * 3
        p2 = np.arange(2000, dtype=np.int32) * 7
        o1, o2 = api.join(c1, p1, c2, p2, kind)
        out["join"].append({"n": 3000, "kind": kind, "dup": "rng7 c1<50 c2<60",
                            "m": int(len(o1)),
                            "pairs_fnv1a64": f"{refcpu.fnv1a64_pairs(o1, o2):016x}"})
        print("join", out["join"][-1], flush=True)
    # 2^24 / 2^28 joins take the reference minutes to hours (per-slot mallocs); their
    # values come from SURVEY.md §8(c) (computed there by the reference) and are
    # re-derived by the oracle restatement in tests/test_oracle.py (2^24).
    out["join_survey"] = [{"n": n, "kind": "hash", "m": m, "pairs_fnv1a64": f"{h:016x}",
                           "source": "SURVEY.md §8(c), reference query.c"}
                          for n, (m, h) in sorted({**SURVEY_JOIN,
                                                   1 << 28: (134232477, 0x93EDF69D334A9827)}.items())
                          if n >= 1 << 24]
    path = os.path.join(HERE, "goldens.json")
    if os.path.exists(path) and not args.big:
        old = json.load(open(path))
        for key in ("config4", "config4_combined"):
            if key in old:
                out[key] = old[key]
        out["select"] += [r for r in old.get("select", []) if r["n"] == 1_000_000_000]
        out["config3"] += [r for r in old.get("config3", []) if r["n"] == 1_000_000_000]
        if "1000000000" in old.get("column_sum", {}):
            out["column_sum"]["1000000000"] = old["column_sum"]["1000000000"]
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
