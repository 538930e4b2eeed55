#!/usr/bin/env python3
"""shared_select goldens at BASELINE's full size from the REFERENCE.

oracle/_ref/libref.so is the reference's src/query.c (+ index.c, multimap.c, utils.c)
compiled unchanged (oracle/Makefile). Its own shared_select (query.c:439-583: three
threads, per-query position lists concatenated in thread order) runs here over the
SURVEY §8(c) seed-42 column of 1e9 rows, with the query sets tests/test_gpu_fullsize.py
sends to libmq:

  q16 / q150   16 / 150 ranges of 0.1 % (width N/1000), lows from default_rng(5)
  q16_dense    16 ranges of 10 % (default_rng(9)), range 3 nested inside range 2 and
               range 4 a single value: 1.6 (query, row) pairs a row

and records per query low, high, K and the FNV-1a-64 of the position list into
tests/golden/shared_goldens.json. Run here, where /root/reference exists (≈ 10 GB RAM,
a few minutes):  python tests/golden/make_shared_goldens.py
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
from refapi import Api, make_column  # noqa: E402

N = 1_000_000_000
# the 1 % select on this column (pins the column generator)
SEL1 = (250_000_000, 260_000_000, 10_001_128, 0x38B1E2BAC2A24D13)


def query_set(q, width, seed):
    """The same sets as tests/test_gpu_fullsize.py:query_set."""
    rng = np.random.default_rng(seed)
    lows = rng.integers(0, N - width, q).astype(np.int32)
    return lows, (lows + width).astype(np.int32)


def sets():
    out = {}
    out["q16"] = query_set(16, N // 1000, 5)
    out["q150"] = query_set(150, N // 1000, 5)
    lows, highs = query_set(16, N // 10, 9)
    lows[3], highs[3] = lows[2] + 1000, highs[2] - 1000
    lows[4], highs[4] = 777_777_777, 777_777_778
    out["q16_dense"] = (lows, highs)
    return out


def main() -> None:
    if not refcpu.have_reference():
        raise SystemExit("oracle/_ref/libref.so missing: run make -C oracle here first")
    api = Api(refcpu.reference())
    d = refcpu.gen_uniform(N, 42)
    col = make_column(d)
    pos = api.select_column(col, SEL1[0], SEL1[1])
    if (len(pos), refcpu.fnv1a64(pos)) != (SEL1[2], SEL1[3]):
        raise SystemExit("golden pin FAILED: the 1 % select differs from SURVEY §8(c)")
    del pos
    res = {"generator": "tests/golden/make_shared_goldens.py via oracle/_ref/libref.so "
                        "(reference src/query.c shared_select, gcc -O2)",
           "data": "col = SURVEY §8(c) seed 42, N = 1e9 (pinned by the 1 % select's K + FNV)",
           "n": N, "sets": {}}
    for name, (lows, highs) in sets().items():
        t0 = time.perf_counter()
        outs = api.shared_select(col, lows, highs)
        dt = time.perf_counter() - t0
        rows = [{"low": int(lows[j]), "high": int(highs[j]), "k": int(len(o)),
                 "pos_fnv1a64": f"{refcpu.fnv1a64(o):016x}"} for j, o in enumerate(outs)]
        del outs
        res["sets"][name] = {"q": len(rows), "reference_s": round(dt, 1), "queries": rows}
        print(name, len(rows), "queries", round(dt, 1), "s", flush=True)
    path = os.path.join(HERE, "shared_goldens.json")
    json.dump(res, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
