#!/usr/bin/env python3
"""Many-to-many join goldens from the REFERENCE's own hash_join.

oracle/_ref/libref.so is the reference's src/query.c + multimap.c (+ index.c, utils.c)
compiled unchanged (oracle/Makefile). Keys: the config-5 many-to-many variant of
oracle/refcpu.c (rc_gen_join_build_dup: every build key twice, rows i and i + n/2;
rc_gen_join_probe_dup: about half the probes hit, two matches each); positions are
identity (2^16 .. 2^24). Records M and the FNV-1a-64 of the interleaved (out1, out2) pairs into
tests/golden/goldens.json under "join_dup".
Run here, where /root/reference exists:  python tests/golden/make_join_dup_goldens.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
from refapi import Api  # noqa: E402


def main() -> None:
    if not refcpu.have_reference():
        raise SystemExit("oracle/_ref/libref.so missing: run make -C oracle here first")
    api = Api(refcpu.reference())
    rows = []
    for logn in (16, 20, 22, 24):
        n = 1 << logn
        a, b = refcpu.gen_join(n, "build_dup"), refcpu.gen_join(n, "probe_dup")
        p = refcpu.gen_join(n, "iota")
        t0 = time.perf_counter()
        o1, o2 = api.join(a, p, b, p, "hash")
        dt = time.perf_counter() - t0
        rows.append({"n": n, "kind": "hash", "keys": "build_dup x probe_dup", "m": int(len(o1)),
                     "pairs_fnv1a64": f"{refcpu.fnv1a64_pairs(o1, o2):016x}",
                     "reference_s": round(dt, 3)})
        print(rows[-1], flush=True)
    path = os.path.join(HERE, "goldens.json")
    g = json.load(open(path))
    g["join_dup"] = rows
    json.dump(g, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
