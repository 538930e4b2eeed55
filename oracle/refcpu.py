"""ctypes harness over the ORACLE libraries — TEST INFRASTRUCTURE ONLY.

  * librefcpu.so      — our C restatement of the reference hot path (refcpu.c)
  * _ref/libref.so    — the reference's own src/query.c index.c multimap.c utils.c,
                        compiled unchanged by oracle/Makefile (present when built
                        in the container that has /root/reference; the prebuilt .so
                        travels to the GPU box with the snapshot)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline: the product (libmq.so)
never loads it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REFCPU = os.path.join(HERE, "librefcpu.so")
REFCPU_O0 = os.path.join(HERE, "librefcpu_O0.so")
REFLIB = os.path.join(HERE, "_ref", "libref.so")
REFLIB_O0 = os.path.join(HERE, "_ref", "libref_O0.so")

_p32 = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_vp, _sz, _u64, _i32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int32
_PI32 = C.POINTER(C.c_int32)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _bind(lib: C.CDLL) -> C.CDLL:
    sigs = {
        "rc_sm64": (_u64, [_u64]),
        "rc_mix31": (C.c_uint32, [C.c_uint32]),
        "rc_gen_uniform": (None, [_vp, _sz, _u64, _u64, C.c_int]),
        "rc_gen_join_build": (None, [_vp, _sz]),
        "rc_gen_join_probe": (None, [_vp, _sz]),
        "rc_gen_join_build_dup": (None, [_vp, _sz]),
        "rc_gen_join_probe_dup": (None, [_vp, _sz]),
        "rc_iota": (None, [_vp, _sz]),
        "rc_fnv1a64": (_u64, [_vp, _sz]),
        "rc_fnv1a64_pairs": (_u64, [_vp, _vp, _sz]),
        "rc_select_scan": (_sz, [_vp, _sz, _PI32, _PI32, _vp]),
        "rc_select_scan_mt": (_sz, [_vp, _sz, _PI32, _PI32, _vp, C.c_int]),
        "rc_select_result": (_sz, [_vp, _vp, _sz, _PI32, _PI32, _vp]),
        "rc_fetch": (None, [_vp, _vp, _sz, _vp]),
        "rc_sum": (C.c_int64, [_vp, _sz]),
        "rc_avg": (C.c_double, [_vp, _sz]),
        "rc_min": (_i32, [_vp, _sz]),
        "rc_max": (_i32, [_vp, _sz]),
        "rc_add": (None, [_vp, _vp, _sz, _vp]),
        "rc_sub": (None, [_vp, _vp, _sz, _vp]),
        "rc_select_count_sum": (None, [_vp, _sz, _PI32, _PI32, C.POINTER(_u64),
                                       C.POINTER(C.c_int64), C.c_int]),
        "rc_shared_select": (C.c_int, [_vp, _sz, _vp, _vp, C.c_int, C.POINTER(_vp), _vp, C.c_int,
                                       C.c_int, _i32, _i32]),
        "rc_hash_join": (_sz, [_vp, _vp, _sz, _vp, _vp, _sz, _vp, _vp, _sz]),
        "rc_nested_loop_join": (_sz, [_vp, _vp, _sz, _vp, _vp, _sz, _vp, _vp, _sz]),
        "rc_hash_join_mt": (_sz, [_vp, _vp, _sz, _vp, _vp, _sz, _vp, _vp, _sz, C.c_int]),
        "rc_multimap_size": (_i32, [_i32]),
        "rc_csv_header_len": (_sz, [_vp, _sz]),
        "rc_load_csv": (_sz, [_vp, _sz, C.c_int, _vp, _sz, _vp]),
        "rc_index_build": (None, [_vp, _sz, _vp, _vp]),
        "rc_index_build_lomuto": (None, [_vp, _sz, _vp, _vp]),
        "rc_histogram": (None, [_vp, _sz, _i32, _i32, _vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_cache: dict[str, C.CDLL] = {}


def lib(path: str = REFCPU) -> C.CDLL:
    if path not in _cache:
        if not os.path.exists(path):
            build()
        _cache[path] = _bind(C.CDLL(path))
    return _cache[path]


def have_reference() -> bool:
    return os.path.exists(REFLIB)


def mq_binding():
    """libmq's ctypes declarations (one shared module instance, so the struct
    classes are the same objects for both libraries)."""
    import importlib.util
    import sys
    if "mq_binding" not in sys.modules:
        spec = importlib.util.spec_from_file_location(
            "mq_binding", os.path.join(os.path.dirname(HERE), "analytical-database_amd", "mq.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules["mq_binding"] = mod
        spec.loader.exec_module(mod)
    return sys.modules["mq_binding"]


def reference(path: str = REFLIB) -> C.CDLL:
    """The reference's own compiled hot path, with libmq's struct declarations."""
    if path not in _cache:
        mq = mq_binding()
        _cache[path] = mq.bind(C.CDLL(path), names=set(mq.REFERENCE_API))
    return _cache[path]


# ---------------------------------------------------------------------------
# numpy conveniences
# ---------------------------------------------------------------------------
def _a(x: np.ndarray) -> int:
    return x.ctypes.data


def _bound(v):
    return None if v is None else C.pointer(C.c_int32(int(v)))


def gen_uniform(n: int, seed: int, modulus: int | None = None, nthreads: int = 8) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    lib().rc_gen_uniform(_a(out), n, seed, n if modulus is None else modulus, nthreads)
    return out


def gen_join(n: int, kind: str) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    {"build": lib().rc_gen_join_build, "probe": lib().rc_gen_join_probe,
     "build_dup": lib().rc_gen_join_build_dup, "probe_dup": lib().rc_gen_join_probe_dup,
     "iota": lib().rc_iota}[kind](_a(out), n)
    return out


def fnv1a64(x: np.ndarray) -> int:
    x = np.ascontiguousarray(x)
    return int(lib().rc_fnv1a64(_a(x), x.nbytes))


def fnv1a64_pairs(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, dtype=np.int32)
    b = np.ascontiguousarray(b, dtype=np.int32)
    return int(lib().rc_fnv1a64_pairs(_a(a), _a(b), len(a)))


def select_scan(d: np.ndarray, low=None, high=None, nthreads: int = 1, path: str = REFCPU):
    pos = np.empty(max(len(d), 1), dtype=np.int32)
    if nthreads > 1:
        k = lib(path).rc_select_scan_mt(_a(d), len(d), _bound(low), _bound(high), _a(pos), nthreads)
    else:
        k = lib(path).rc_select_scan(_a(d), len(d), _bound(low), _bound(high), _a(pos))
    return pos[:k].copy()


def select_result(vals: np.ndarray, prev: np.ndarray, low=None, high=None):
    out = np.empty(max(len(vals), 1), dtype=np.int32)
    k = lib().rc_select_result(_a(vals), _a(prev), len(vals), _bound(low), _bound(high), _a(out))
    return out[:k].copy()


def fetch(col: np.ndarray, pos: np.ndarray) -> np.ndarray:
    out = np.empty(len(pos), dtype=np.int32)
    lib().rc_fetch(_a(col), _a(pos), len(pos), _a(out))
    return out


def agg(v: np.ndarray) -> dict:
    L = lib()
    n = len(v)
    return {"count": n, "sum": int(L.rc_sum(_a(v), n)), "avg": float(L.rc_avg(_a(v), n)),
            "min": int(L.rc_min(_a(v), n)), "max": int(L.rc_max(_a(v), n))}


def count_sum(d: np.ndarray, low=None, high=None, nthreads: int = 8, path: str = REFCPU):
    c, s = C.c_uint64(0), C.c_int64(0)
    lib(path).rc_select_count_sum(_a(d), len(d), _bound(low), _bound(high), C.byref(c),
                                  C.byref(s), nthreads)
    return int(c.value), int(s.value)


def add(a, b):
    out = np.empty(len(a), dtype=np.int32)
    lib().rc_add(_a(a), _a(b), len(a), _a(out))
    return out


def sub(a, b):
    out = np.empty(len(a), dtype=np.int32)
    lib().rc_sub(_a(a), _a(b), len(a), _a(out))
    return out


def shared_select(d: np.ndarray, lows, highs, nthreads: int = 3, split: int = 0):
    q = len(lows)
    lo = np.ascontiguousarray(lows, dtype=np.int32)
    hi = np.ascontiguousarray(highs, dtype=np.int32)
    bufs = [np.empty(max(len(d), 1), dtype=np.int32) for _ in range(q)]
    ptrs = (C.c_void_p * max(q, 1))(*[_a(b) for b in bufs])
    counts = np.zeros(max(q, 1), dtype=np.uint64)
    mn = int(d.min()) if len(d) else 0
    mx = int(d.max()) if len(d) else 0
    rc = lib().rc_shared_select(_a(d), len(d), _a(lo), _a(hi), q, ptrs, _a(counts), nthreads,
                                split, mn, mx)
    if rc != 0:
        raise ValueError("invalid value-range split (the reference reads past the column here)")
    return [bufs[i][: int(counts[i])].copy() for i in range(q)]


def hash_join(c1, p1, c2, p2, nested: bool = False):
    L = lib()
    fn = L.rc_nested_loop_join if nested else L.rc_hash_join
    m = fn(_a(c1), _a(p1), len(c1), _a(c2), _a(p2), len(c2), None, None, 0)
    o1 = np.empty(max(m, 1), dtype=np.int32)
    o2 = np.empty(max(m, 1), dtype=np.int32)
    m2 = fn(_a(c1), _a(p1), len(c1), _a(c2), _a(p2), len(c2), _a(o1), _a(o2), m)
    assert m2 == m
    return o1[:m].copy(), o2[:m].copy()


def hash_join_mt(c1, p1, c2, p2, nthreads: int):
    """rc_hash_join_mt: the join over nthreads host threads (same output as hash_join)."""
    L = lib()
    m = L.rc_hash_join_mt(_a(c1), _a(p1), len(c1), _a(c2), _a(p2), len(c2), None, None, 0, nthreads)
    o1 = np.empty(max(m, 1), dtype=np.int32)
    o2 = np.empty(max(m, 1), dtype=np.int32)
    m2 = L.rc_hash_join_mt(_a(c1), _a(p1), len(c1), _a(c2), _a(p2), len(c2), _a(o1), _a(o2), m, nthreads)
    assert m2 == m
    return o1[:m].copy(), o2[:m].copy()


def csv_header_len(text: bytes) -> int:
    buf = C.create_string_buffer(text, len(text))
    return int(lib().rc_csv_header_len(buf, len(text)))


def load_csv(text: bytes, ncols: int):
    """load_db's data-line loop (db_manager.c:304-318) over `text` (header already
    removed): returns (columns int32[ncols][rows], minmax int32[ncols][2])."""
    buf = C.create_string_buffer(text, len(text))
    L = lib()
    rows = int(L.rc_load_csv(buf, len(text), ncols, None, 0, None))
    cols = np.empty((ncols, max(rows, 1)), dtype=np.int32)
    ptrs = (C.c_void_p * max(ncols, 1))(*[cols[j].ctypes.data for j in range(ncols)])
    mm = np.empty((max(ncols, 1), 2), dtype=np.int32)
    got = int(L.rc_load_csv(buf, len(text), ncols, ptrs, rows, _a(mm)))
    assert got == rows
    return cols[:, :rows].copy(), mm[:ncols].copy()


def fnv1a64_bytes(b: bytes) -> int:
    buf = C.create_string_buffer(b, len(b))
    return int(lib().rc_fnv1a64(buf, len(b)))


def index_build(col: np.ndarray):
    """(sorted values int32, positions uint64), equal values in ascending row order."""
    col = np.ascontiguousarray(col, dtype=np.int32)
    v = np.empty(max(len(col), 1), dtype=np.int32)
    p = np.empty(max(len(col), 1), dtype=np.uint64)
    lib().rc_index_build(_a(col), len(col), _a(v), _a(p))
    return v[:len(col)].copy(), p[:len(col)].copy()


def index_build_lomuto(col: np.ndarray):
    """(sorted values int32, positions uint64) in the reference quicksort's own order
    (index.c:25-46), equal values included."""
    col = np.ascontiguousarray(col, dtype=np.int32)
    v = np.empty(max(len(col), 1), dtype=np.int32)
    p = np.empty(max(len(col), 1), dtype=np.uint64)
    lib().rc_index_build_lomuto(_a(col), len(col), _a(v), _a(p))
    return v[:len(col)].copy(), p[:len(col)].copy()


def histogram(col: np.ndarray, mn: int, bin_size: int) -> np.ndarray:
    col = np.ascontiguousarray(col, dtype=np.int32)
    out = np.zeros(101, dtype=np.uint64)
    lib().rc_histogram(_a(col), len(col), mn, bin_size, _a(out))
    return out


# ---------------------------------------------------------------------------
# J4 hashset.c restatement (pure Python: small sets only)
# ---------------------------------------------------------------------------
def _hs_home(key: int, size: int) -> int:
    """hash(key, size) = key % size (multimap.c:60-63, C remainder: truncates toward
    zero). The reference indexes keys[negative] for a negative key; the restatement
    (like libmq) starts such a probe at the wrapped remainder."""
    r = abs(key) % size
    r = -r if key < 0 else r
    return r + size if r < 0 else r


def hashset_table(keys, size: int) -> np.ndarray:
    """The slots after insert_hashset of keys in order (hashset.c:25-32): linear
    probing from the home slot while the slot is nonzero and not the key; 0 marks
    an empty slot, so inserting 0 changes nothing. A full table without the key
    stops after one lap (the reference loops forever)."""
    t = [0] * size
    for k in (int(x) for x in keys):
        i = _hs_home(k, size)
        for step in range(size):
            if t[i] == 0 or t[i] == k:
                t[i] = k
                break
            i = i + 1 if i + 1 < size else 0
    return np.array(t, dtype=np.int32)


def hashset_lookup(table: np.ndarray, key: int) -> bool:
    """lookup_hashset (hashset.c:35-45): probe as insert does; found iff the slot it
    stops at is nonzero (so 0 is never a member)."""
    size = len(table)
    i = _hs_home(int(key), size)
    for _ in range(size):
        v = int(table[i])
        if v == 0 or v == key:
            return v != 0
        i = i + 1 if i + 1 < size else 0
    return False


def hashset_elements(table: np.ndarray) -> np.ndarray:
    """get_hashset_elements (hashset.c:48-65): the nonzero slots in slot order."""
    return table[table != 0]
