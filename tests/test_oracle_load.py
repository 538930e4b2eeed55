"""Pin the load-path restatement (oracle/refcpu.c rc_load_csv) before trusting it.

  1. against tests/golden/csv_goldens.json, produced by the reference's own
     load_db / insert_row (src/db_manager.c:164-199,240-322, compiled unchanged into
     oracle/_ref/libdbm.so and driven by oracle/refload.py);
  2. against that reference build directly, on fresh fuzz inputs (when present).
Cells the reference leaves uninitialised (a column before the first row that has
its token: db_manager.c:304 `int row[col_count]`) are excluded; the restatement
writes 0 there. CPU only.
"""
import json
import os
import tempfile

import numpy as np
import pytest

from csvcases import cases, leading_unset

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "csv_goldens.json")))
CASES = {name: (ncols, data) for name, ncols, data in cases()}


def check_against_golden(name, cols, minmax, rows):
    g = GOLD[name]
    import refcpu
    assert rows == g["rows"], name
    for j in range(g["ncols"]):
        lead = g["lead"][j]
        assert f"{refcpu.fnv1a64(np.ascontiguousarray(cols[j][lead:rows])):016x}" == g["col_fnv"][j], (name, j)
        assert [int(v) for v in cols[j][lead:lead + 16]] == g["head"][j], (name, j)
        assert np.all(cols[j][:lead] == 0), (name, j)  # the restatement's choice for the UB cells
        if g["minmax"][j] is not None:
            assert [int(minmax[j][0]), int(minmax[j][1])] == g["minmax"][j], (name, j)


def test_csv_inputs_match_goldens(refcpu):
    assert set(CASES) == set(GOLD)
    for name, (ncols, data) in CASES.items():
        assert f"{refcpu.fnv1a64_bytes(data):016x}" == GOLD[name]["in_fnv"], name
        assert leading_unset(data, ncols) == GOLD[name]["lead"], name


@pytest.mark.parametrize("name", sorted(CASES))
def test_load_restatement_vs_goldens(refcpu, name):
    ncols, data = CASES[name]
    cols, mm = refcpu.load_csv(data, ncols)
    check_against_golden(name, cols, mm, cols.shape[1] if ncols else 0)


def test_header_len(refcpu):
    assert refcpu.csv_header_len(b"db.t.a,db.t.b\n1,2\n") == 14
    assert refcpu.csv_header_len(b"x" * 2000) == 1023  # fgets(line, 1024)
    assert refcpu.csv_header_len(b"abc") == 3


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref",
                                                    "libdbm.so")), reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_load_restatement_vs_reference_fuzz(refcpu, seed):
    """Fresh inputs, straight through the reference's load_db."""
    import refload
    rng = np.random.default_rng(seed)
    alphabet = np.frombuffer(b"0123456789" * 8 + b",,,-+ \t\n\n\x00", dtype=np.uint8)
    parts = []
    for _ in range(200):
        k = int(rng.integers(0, 60 if rng.random() < 0.97 else 2500))
        parts.append(alphabet[rng.integers(0, len(alphabet), k)].tobytes() + b"\n")
    data = b"".join(parts)
    ncols = int(rng.integers(1, 7))
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "f.csv")
        with open(path, "wb") as f:
            f.write((",".join(f"db.tbl.c{j}" for j in range(ncols)) + "\n").encode() + data)
        r = refload.load(path, ncols)
    cols, mm = refcpu.load_csv(data, ncols)
    assert r["rows"] == cols.shape[1]
    lead = leading_unset(data, ncols)
    for j in range(ncols):
        assert np.array_equal(r["cols"][j][lead[j]:], cols[j][lead[j]:]), j
        if lead[j] == 0:
            assert list(r["minmax"][j]) == list(mm[j]), j
