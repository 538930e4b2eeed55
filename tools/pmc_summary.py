#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counter CSVs in a directory (not product code).
  python tools/pmc_summary.py [--parts P] DIR [kernel-substring ...]
--parts P splits each kernel's dispatches (in dispatch order) into P equal consecutive
parts, for runs that time P configurations one after another (shared_prof.py 16,150).
Prints, per kernel (name shortened), dispatches and the mean of every counter found in
DIR/*_counter_collection.csv, with FETCH_SIZE x 2 as read bytes (gfx950, MI355X_MICROARCH.md)
and WRITE_SIZE in bytes."""
import collections
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402

args = sys.argv[1:]
parts = 1
if args and args[0] == "--parts":
    parts, args = int(args[1]), args[2:]
d = args[0]
want = args[1:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "*_counter_collection.csv"))):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        k = short(r["Kernel_Name"])
        if want and not any(w in k for w in want):
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
split = {}
for k, c in vals.items():
    for p in range(parts):
        tag = k if parts == 1 else f"{k} [{p + 1}/{parts}]"
        split[tag] = {nm: v[p * len(v) // parts:(p + 1) * len(v) // parts] or v for nm, v in c.items()}
for k in sorted(split):
    c = split[k]
    n = max(len(v) for v in c.values())
    out = []
    for name in sorted(c):
        m = statistics.mean(c[name])
        if name == "FETCH_SIZE":
            out.append(f"read_GB={m * 2048 / 1e9:.3f}")
        elif name == "WRITE_SIZE":
            out.append(f"write_GB={m * 1024 / 1e9:.3f}")
        else:
            out.append(f"{name}={m:.4g}")
    print(f"{k[:60]:60s} n={n} " + " ".join(out))
