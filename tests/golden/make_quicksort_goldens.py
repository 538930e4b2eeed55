#!/usr/bin/env python3
"""Generate tests/golden/quicksort_goldens.json from the REFERENCE's own quicksort.

The index build's exact tie order (index.c:25-46, Lomuto, pivot = values[high]) at
the sizes build_index applies it to (up to MQ_INDEX_EXACT_MAX = 2^27 rows, DESIGN.md
§3.7). Each case is the SURVEY §8(c) uniform column (rc_gen_uniform(n, seed, modulus),
the generator mq_gen_uniform reproduces on the device) sorted by the `quicksort`
symbol of oracle/_ref/libdbm.so (the reference's index.c compiled unchanged), with
positions 0..n-1 as init_column_index prepares them (:89-100). Recorded:
  col_fnv        FNV-1a-64 of the input column (pins the generator)
  values_fnv     FNV of the sorted int32 values
  positions_fnv  FNV of the u64 positions (equal values in the quicksort's order)
  ties           number of i with values[i] == values[i+1]
Each sort runs in a child process (the recursion is the reference's; 2^27 rows take
about a minute here). Run where /root/reference exists:
  python tests/golden/make_quicksort_goldens.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
import refload  # noqa: E402

# (log2 n, seed, modulus): uniform [0, n) (about one value in three repeats), a
# narrower range (about 8 rows a value), and 4096 values of 1024 rows each (long
# equal runs: the reference's recursion on them is quadratic, still seconds here)
CASES = [(22, 42, None), (22, 43, 1 << 19), (22, 44, 4096), (24, 42, None), (27, 42, None)]


def fnv(x: np.ndarray) -> str:
    return f"{refcpu.fnv1a64(np.ascontiguousarray(x)):016x}"


def one(lg: int, seed: int, modulus) -> dict:
    n = 1 << lg
    col = refcpu.gen_uniform(n, seed, modulus or n, nthreads=8)
    v, p = refload.quicksort(col)
    return {"log2n": lg, "n": n, "seed": seed, "modulus": modulus or n, "col_fnv": fnv(col),
            "values_fnv": fnv(v), "positions_fnv": fnv(p.astype(np.uint64)),
            "ties": int(np.count_nonzero(v[1:] == v[:-1]))}


def main() -> None:
    if len(sys.argv) == 4:  # child: one case, JSON on stdout
        lg, seed, mod = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
        print(json.dumps(one(lg, seed, mod or None)))
        return
    assert refload.have(), "build oracle/_ref/libdbm.so first (make -C oracle)"
    refcpu.build()
    out = []
    for lg, seed, mod in CASES:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), str(lg), str(seed), str(mod or 0)],
                           check=True, capture_output=True, text=True)
        out.append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(out[-1], flush=True)
    with open(os.path.join(HERE, "quicksort_goldens.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
