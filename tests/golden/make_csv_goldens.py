#!/usr/bin/env python3
"""Generate tests/golden/csv_goldens.json from the REFERENCE's own load path.

oracle/_ref/libdbm.so is the reference's src/db_manager.c + utils.c + index.c
compiled unchanged (oracle/Makefile); oracle/refload.py drives it as the server
does for create(db) / create(tbl) / create(col) x ncols / load(file). For every
input of tests/csvcases.py this script writes "<header>\\n<data>" to a scratch file,
loads it with the reference's load_db and records, per case:
  in_fnv        FNV-1a-64 of the data bytes (pins the input generator)
  rows, table_length   the table after load_db (+ insert_row's capacity doubling)
  lead[j]       rows of column j before the first row that has token j: the
                reference reads its uninitialised row[] there (stack garbage), so
                those cells are excluded from the comparison
  col_fnv[j]    FNV-1a-64 of column j's int32 rows [lead[j], rows) (little-endian)
  minmax[j]     the column's (min, max) as insert_row folded them (null when
                lead[j] > 0: it includes the garbage)
  head[j]       the first 16 values of column j (readable spot check)
Run here, where /root/reference exists:  python tests/golden/make_csv_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import refcpu  # noqa: E402
import refload  # noqa: E402
from csvcases import cases, leading_unset  # noqa: E402


def header(ncols: int) -> bytes:
    return (",".join(f"db.tbl.c{j}" for j in range(ncols)) + "\n").encode()


def main() -> None:
    assert refload.have(), "build oracle/_ref/libdbm.so first (make -C oracle)"
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, ncols, data in cases():
            path = os.path.join(tmp, f"{name}.csv")
            with open(path, "wb") as f:
                f.write(header(ncols) + data)
            r = refload.load(path, ncols)
            assert r["code"] == 0, name
            cols = r["cols"]
            lead = leading_unset(data, ncols)
            assert len(cols) == 0 or cols.shape[1] == r["rows"]
            out[name] = {
                "ncols": ncols,
                "in_fnv": f"{refcpu.fnv1a64_bytes(data):016x}",
                "rows": int(r["rows"]),
                "table_length": int(r["table_length"]),
                "lead": lead,
                "col_fnv": [f"{refcpu.fnv1a64(cols[j][lead[j]:]):016x}" for j in range(ncols)],
                "minmax": [[int(a), int(b)] if lead[j] == 0 else None
                           for j, (a, b) in enumerate(r["minmax"])],
                "head": [[int(v) for v in cols[j][lead[j]:lead[j] + 16]] for j in range(ncols)],
            }
            print(f"{name:24s} ncols={ncols:2d} bytes={len(data):7d} rows={r['rows']}")
    with open(os.path.join(HERE, "csv_goldens.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
