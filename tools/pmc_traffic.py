#!/usr/bin/env python3
"""HBM traffic per launch from separate rocprofv3 --pmc passes (MI355X_MICROARCH.md §HBM).

  rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D -o fetch --output-format csv -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D -o write --output-format csv -- python3 bench.py ...
  python tools/pmc_traffic.py D [--rows N] [--out profiles/pmc_traffic.json]

Per dispatch of each kernel: FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced stream,
so read bytes = FETCH_SIZE x 1024 x 2; write bytes = WRITE_SIZE x 1024 (exact for
16-B streaming stores; k_scan's only stores are its 32-B partials). The
correction is the guide's; it is applied to k_scan, whose loads are all
dwordx4 streams.
"""
import argparse
import collections
import csv
import json
import os
import statistics


def per_kernel(path, counter):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def short(name):
    """Kernel name without return type, namespaces or parameter list (template
    arguments kept; they may contain parentheses, e.g. k_scan<(Mode)0, true>)."""
    s = name.replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    depth = 0
    for i, c in enumerate(s):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0 and i > 0:
            return s[:i]
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.dir, "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.dir, "write_counter_collection.csv"), "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "bench.py --steps 3 --warmup 1 --no-cpu --no-extra",
           "correction": "read = FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count on wide streams)",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f = statistics.mean(fetch.get(name, [0.0]))
        w = statistics.mean(write.get(name, [0.0]))
        res["kernels"][short(name)] = {
            "dispatches": len(fetch.get(name, [])), "fetch_kib_raw": f, "write_kib": w,
            "read_bytes_corrected": f * 1024 * 2, "write_bytes": w * 1024}
    # the headline kernel: the k_scan instantiation bench.py launches per step
    # (with --no-extra that is the only k_scan in the run)
    scan = sorted((k for k in fetch if short(k).startswith("k_scan<")),
                  key=lambda k: -len(fetch[k]))
    if scan:
        f = statistics.mean(fetch[scan[0]])
        w = statistics.mean(write.get(scan[0], [0.0]))
        hbm = f * 1024 * 2 + w * 1024
        res["k_scan"] = {"kernel": short(scan[0]), "rows": a.rows, "hbm_bytes_per_launch": hbm,
                         "algorithmic_bytes_per_launch": 4 * a.rows,
                         "ratio_to_algorithmic": hbm / (4 * a.rows)}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res.get("k_scan"), indent=1))


if __name__ == "__main__":
    main()
