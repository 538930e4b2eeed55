#!/usr/bin/env python3
"""Generate tests/golden/index_goldens.json from the REFERENCE's own index build.

oracle/refload.py drives oracle/_ref/libdbm.so (src/db_manager.c + utils.c +
index.c compiled unchanged): create the table, create(idx, ...) per the case's
spec, load the case's CSV with load_db, then build_index(db) as server.c:125 does.
For every case of tests/indexcases.py this records the reference's result as it is
(equal values in its quicksort's own order):
  in_fnv                   FNV-1a-64 of the CSV text (pins the input generator)
  ix<j>_values/_positions  FNV of the index arrays (values int32, positions u64)
  hist<j>_*                bin_size, values[100], counts[100] (unclustered)
  cols                     FNV of every column after the build
Run here, where /root/reference exists:  python tests/golden/make_index_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
import refload  # noqa: E402
from indexcases import cases, csv_text  # noqa: E402


def fnv(x) -> str:
    return f"{refcpu.fnv1a64(np.ascontiguousarray(x)):016x}"


def digest(c: dict, spec) -> dict:
    d = {"cols": [fnv(col.astype(np.int32)) for col in c["cols"]]}
    for j, clustered in spec:
        d[f"ix{j}_values"] = fnv(np.asarray(c[f"ix{j}_values"], dtype=np.int32))
        d[f"ix{j}_positions"] = fnv(np.asarray(c[f"ix{j}_positions"], dtype=np.uint64))
        if not clustered:
            d[f"hist{j}_bin_size"] = int(c[f"hist{j}_bin_size"])
            d[f"hist{j}_values"] = [int(v) for v in c[f"hist{j}_values"]]
            d[f"hist{j}_counts"] = [int(v) for v in c[f"hist{j}_counts"]]
    return d


def main() -> None:
    assert refload.have(), "build oracle/_ref/libdbm.so first (make -C oracle)"
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, cols, spec in cases():
            text = csv_text(cols)
            path = os.path.join(tmp, f"{name}.csv")
            open(path, "wb").write(text)
            r = refload.load(path, len(cols), ",".join(f"{j}:{'c' if c else 'u'}" for j, c in spec))
            assert r["code"] == 0 and r["rows"] == cols.shape[1], name
            out[name] = {"in_fnv": f"{refcpu.fnv1a64_bytes(text):016x}", "spec": spec, **digest(r, spec)}
            print(name)
    with open(os.path.join(HERE, "index_goldens.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
