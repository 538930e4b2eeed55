"""Drive the reference operator API (query.h:20-50) of ANY library that exports it.

The same helpers run the reference's own compiled query.c (oracle/_ref/libref.so)
and libmq.so, so a parity test reads like the reference's call sequence in
server.c:137-434: build a Column, call select_column, fetch_column, sum, ...
Results are copied into numpy arrays and the callee's malloc'd memory is freed
with libc free(), as client_context.c:31-90 does.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "mq_binding" not in sys.modules:
    _spec = importlib.util.spec_from_file_location(
        "mq_binding", os.path.join(ROOT, "analytical-database_amd", "mq.py"))
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules["mq_binding"] = _mod
    _spec.loader.exec_module(_mod)
mq = sys.modules["mq_binding"]

_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]
_libc.free.restype = None


def make_column(data: np.ndarray, name: bytes = b"col") -> "mq.Column":
    """A Column over a numpy int32 array (kept alive by the caller)."""
    col = mq.Column()
    col.name = name
    col.data = data.ctypes.data_as(C.POINTER(C.c_int))
    col.fd = -1
    col.row_count = len(data)
    col.sorted = col.clustered = col.has_index = False
    if len(data):
        col.min = int(data.min())
        col.max = int(data.max())
    return col


def make_result(values: np.ndarray, data_type: int = mq.INT):
    """A Result whose payload is a malloc'd copy (the callee may free()/alias it)."""
    values = np.ascontiguousarray(values)
    r = mq.Result()
    r.num_tuples = len(values)
    r.data_type = data_type
    buf = _libc.malloc
    buf.restype = C.c_void_p
    buf.argtypes = [C.c_size_t]
    p = buf(max(values.nbytes, 1))
    C.memmove(p, values.ctypes.data, values.nbytes)
    r.payload = p
    return r


def free_result_struct(r) -> None:
    if r.payload:
        _libc.free(r.payload)
        r.payload = None


def take(rp, free: bool = True) -> np.ndarray:
    """Copy a returned Result* into numpy (by its data_type) and free it."""
    if not rp:
        raise RuntimeError("operator returned NULL")
    r = rp.contents
    n = int(r.num_tuples)
    dt = {mq.INT: np.int32, mq.LONG: np.int64, mq.FLOAT: np.float32, mq.DOUBLE: np.float64}[
        r.data_type]
    out = np.empty(n, dtype=dt)
    if n:
        C.memmove(out.ctypes.data, r.payload, out.nbytes)
    if free:
        _libc.free(r.payload)
        _libc.free(C.cast(rp, C.c_void_p))
    return out


def _b(v):
    return None if v is None else C.pointer(C.c_int(int(v)))


class Api:
    """Reference-API calls against one library (libref.so or libmq.so)."""

    def __init__(self, lib: C.CDLL):
        self.lib = lib

    def _st(self):
        return mq.Status(0, None)

    def select_column(self, col, low=None, high=None):
        st = self._st()
        rp = self.lib.select_column(C.byref(col), _b(low), _b(high), C.byref(st))
        assert st.code == mq.OK, "select_column failed"
        return take(rp)

    def select_result(self, vals: np.ndarray, pos: np.ndarray, low=None, high=None):
        rv, rpos = make_result(vals), make_result(pos)
        st = self._st()
        rp = self.lib.select_result(C.byref(rv), C.byref(rpos), _b(low), _b(high), C.byref(st))
        assert st.code == mq.OK
        out = take(rp)
        free_result_struct(rv)
        free_result_struct(rpos)
        return out

    def fetch_column(self, col, pos: np.ndarray):
        rpos = make_result(pos)
        st = self._st()
        rp = self.lib.fetch_column(C.byref(col), C.byref(rpos), C.byref(st))
        assert st.code == mq.OK
        out = take(rp)
        free_result_struct(rpos)
        return out

    def _unary(self, fn, vals: np.ndarray, dtype=mq.INT):
        r = make_result(vals, dtype)
        st = self._st()
        rp = fn(C.byref(r), C.byref(st))
        assert st.code == mq.OK
        out = take(rp)
        free_result_struct(r)
        return out[0]

    def average(self, vals):
        return float(self._unary(self.lib.average, vals))

    def min(self, vals):
        return int(self._unary(self.lib.min, vals))

    def max(self, vals):
        return int(self._unary(self.lib.max, vals))

    def sum_result(self, vals):
        r = make_result(vals)
        g = mq.GeneralizedColumn()
        g.column_type = mq.RESULT
        g.column_pointer.result = C.pointer(r)
        st = self._st()
        rp = self.lib.sum(C.byref(g), C.byref(st))
        assert st.code == mq.OK
        out = take(rp)
        free_result_struct(r)
        return int(out[0])

    def sum_column(self, col):
        g = mq.GeneralizedColumn()
        g.column_type = mq.COLUMN
        g.column_pointer.column = C.pointer(col)
        st = self._st()
        rp = self.lib.sum(C.byref(g), C.byref(st))
        assert st.code == mq.OK
        return int(take(rp)[0])

    def _binary(self, fn, a, b):
        ra, rb = make_result(a), make_result(b)
        st = self._st()
        rp = fn(C.byref(ra), C.byref(rb), C.byref(st))
        assert st.code == mq.OK
        out = take(rp)
        free_result_struct(ra)
        free_result_struct(rb)
        return out

    def add(self, a, b):
        return self._binary(self.lib.add, a, b)

    def sub(self, a, b):
        return self._binary(self.lib.sub, a, b)

    def shared_select(self, col, lows, highs):
        q = len(lows)
        ops = (mq.SelectOperator * q)()
        for i in range(q):
            ops[i].low = int(lows[i])
            ops[i].high = int(highs[i])
            ops[i].has_low = ops[i].has_high = 1
            ops[i].column = C.pointer(col)
        st = self._st()
        rpp = self.lib.shared_select(ops, q, C.byref(col), C.byref(st))
        assert st.code == mq.OK and rpp
        outs = [take(rpp[i]) for i in range(q)]
        _libc.free(C.cast(rpp, C.c_void_p))
        return outs

    def join(self, c1, p1, c2, p2, kind: str = "hash"):
        rs = [make_result(x) for x in (c1, p1, c2, p2)]
        st = self._st()
        fn = self.lib.hash_join if kind == "hash" else self.lib.nested_loop_join
        rpp = fn(*[C.byref(r) for r in rs], C.byref(st))
        assert st.code == mq.OK and rpp
        o1, o2 = take(rpp[0]), take(rpp[1])
        _libc.free(C.cast(rpp, C.c_void_p))
        for r in rs:
            free_result_struct(r)
        return o1, o2

    def print(self, arrays_and_types):
        rs = [make_result(a, t) for a, t in arrays_and_types]
        arr = (C.POINTER(mq.Result) * len(rs))(*[C.pointer(r) for r in rs])
        st = self._st()
        p = self.lib.print(arr, len(rs), C.byref(st))
        s = C.string_at(p).decode()
        _libc.free(p)
        for r in rs:
            free_result_struct(r)
        return s
