"""Runs the REFERENCE's own load path — TEST INFRASTRUCTURE ONLY.

oracle/_ref/libdbm.so is src/db_manager.c + src/utils.c + src/index.c compiled
unchanged by oracle/Makefile. This script drives it exactly as the server does for
`create(db,...)`, `create(tbl,...)`, `create(col,...)` and `load(...)`
(server.c:80-127): create_db -> create_table -> create_column x ncols -> load_db.
It then reads back the table (row_count, table_length) and every column's rows and
min/max. The catalog writes files under ./database/, so it runs in a scratch
directory, in a child process (the reference keeps global state: current_db).

    python oracle/refload.py <csv> <ncols> <out.npz>
The CSV's header must name db "db" and table "tbl" (db.tbl.c0,...).
Used by tests/test_oracle.py (pins oracle/refcpu.c's rc_load_csv) and by
tests/golden/make_csv_goldens.py. Never imported by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDBM = os.path.join(HERE, "_ref", "libdbm.so")


class Status(C.Structure):
    _fields_ = [("code", C.c_int), ("error_message", C.c_char_p)]


class Column(C.Structure):  # cs165_api.h:129-144 (128 bytes)
    _fields_ = [("name", C.c_char * 64), ("data", C.POINTER(C.c_int)), ("fd", C.c_int),
                ("row_count", C.c_size_t), ("sorted", C.c_bool), ("clustered", C.c_bool),
                ("has_index", C.c_bool), ("index", C.c_void_p), ("btree_node", C.c_void_p),
                ("histogram", C.c_void_p), ("max", C.c_int), ("min", C.c_int)]


class Table(C.Structure):  # cs165_api.h:110-116
    _fields_ = [("name", C.c_char * 64), ("columns", C.POINTER(Column)), ("col_count", C.c_size_t),
                ("row_count", C.c_size_t), ("table_length", C.c_size_t)]


class Db(C.Structure):  # cs165_api.h:127-132
    _fields_ = [("name", C.c_char * 64), ("tables", C.POINTER(Table)), ("tables_size", C.c_size_t),
                ("tables_capacity", C.c_size_t)]


class ColumnIndex(C.Structure):  # cs165_api.h:117-120
    _fields_ = [("values", C.POINTER(C.c_int)), ("positions", C.POINTER(C.c_size_t))]


class Histogram(C.Structure):  # cs165_api.h:71-75
    _fields_ = [("bin_size", C.c_int), ("values", C.c_int * 100), ("counts", C.c_size_t * 100)]


def have() -> bool:
    return os.path.exists(LIBDBM)


def run(csv_path: str, ncols: int, index_spec: str = "") -> dict:
    """Child-process entry: the reference's load of csv_path into a fresh table.
    index_spec "j:c,k:u" declares create(idx, col j, sorted, clustered) / col k
    unclustered before the load; then build_index runs as server.c:125 does."""
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "database"))
        os.chdir(tmp)
        L = C.CDLL(LIBDBM)
        L.create_db.restype = Status
        L.create_db.argtypes = [C.c_char_p]
        L.create_table.argtypes = [C.POINTER(Db), C.c_char_p, C.c_size_t, C.POINTER(Status)]
        L.create_column.argtypes = [C.POINTER(Table), C.c_char_p, C.c_bool, C.POINTER(Status)]
        L.load_db.argtypes = [C.POINTER(Db), C.c_char_p, C.POINTER(Status)]
        st = L.create_db(b"db")
        assert st.code == 0
        db = C.POINTER(Db).in_dll(L, "current_db")
        s = Status()
        L.create_table(db, b"tbl", ncols, C.byref(s))
        assert s.code == 0
        tbl = C.pointer(db.contents.tables[0])
        for j in range(ncols):
            L.create_column(tbl, f"c{j}".encode(), False, C.byref(s))
            assert s.code == 0, j
        L.create_index.argtypes = [C.POINTER(Column), C.c_bool, C.c_bool, C.POINTER(Status)]
        L.build_index.argtypes = [C.POINTER(Db)]
        spec = [(int(a), b == "c") for a, b in (x.split(":") for x in index_spec.split(",") if x)]
        for j, clustered in spec:
            L.create_index(C.pointer(tbl.contents.columns[j]), clustered, True, C.byref(s))
        s = Status()
        import time
        t0 = time.perf_counter()
        L.load_db(db, csv_path.encode(), C.byref(s))
        load_s = time.perf_counter() - t0
        if spec and s.code == 0:
            L.build_index(db)
        t = tbl.contents
        rows = int(t.row_count)
        cols = np.zeros((ncols, rows), dtype=np.int32)
        mm = np.zeros((ncols, 2), dtype=np.int32)
        for j in range(ncols):
            c = t.columns[j]
            if rows:
                cols[j] = np.ctypeslib.as_array(c.data, shape=(rows,))
            mm[j] = (c.min, c.max)
        out = {"code": int(s.code), "rows": rows, "table_length": int(t.table_length),
               "cols": cols, "minmax": mm, "load_s": np.float64(load_s)}
        for j, clustered in spec:
            c = t.columns[j]
            ix = C.cast(c.index, C.POINTER(ColumnIndex)).contents
            out[f"ix{j}_values"] = np.ctypeslib.as_array(ix.values, shape=(rows,)).copy()
            out[f"ix{j}_positions"] = np.ctypeslib.as_array(ix.positions, shape=(rows,)).copy()
            if not clustered:
                h = C.cast(c.histogram, C.POINTER(Histogram)).contents
                out[f"hist{j}_bin_size"] = np.int64(h.bin_size)
                out[f"hist{j}_values"] = np.array(h.values[:], dtype=np.int64)
                out[f"hist{j}_counts"] = np.array(h.counts[:], dtype=np.uint64)
        return out


def quicksort(col: np.ndarray):
    """The reference's own quicksort (index.c:25-46, in libdbm.so) on a copy of col with
    positions 0..n-1, as init_column_index prepares them (:89-100). In-process: keep n
    small (its recursion depth reaches n on sorted or duplicate-heavy input)."""
    L = C.CDLL(LIBDBM)
    L.quicksort.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.quicksort.restype = None
    v = np.array(col, dtype=np.int32, copy=True)
    p = np.arange(len(v), dtype=np.uint64)
    if len(v):
        L.quicksort(v.ctypes.data, p.ctypes.data, 0, len(v) - 1)
    return v, p


def load(csv_path: str, ncols: int, index_spec: str = "") -> dict:
    """The reference's load (and index build) of csv_path, run in a child process."""
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "out.npz")
        subprocess.run([sys.executable, os.path.abspath(__file__), os.path.abspath(csv_path),
                        str(ncols), out, index_spec], check=True, stdout=subprocess.DEVNULL)
        z = np.load(out)
        return {k: (z[k] if z[k].ndim else z[k].item()) for k in z.files}


if __name__ == "__main__":
    r = run(sys.argv[1], int(sys.argv[2]), sys.argv[4] if len(sys.argv) > 4 else "")
    np.savez(sys.argv[3], **r)
