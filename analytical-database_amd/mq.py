"""ctypes binding for libmq.so (include/mq_device.h, include/mq_query.h).

Host-side mirror of the reference operator interface for Python callers
(tests, bench). The product is the C-ABI library; this module only declares
its signatures and the reference struct layouts
(src/include/cs165_api.h:58-206, src/include/db_manager.h:95-108).

No fallback: `load()` raises if libmq.so is missing, and every device entry
point returns MQ_ENODEV when there is no gfx950 device.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libmq.so")
INCLUDE_DIR = os.path.join(ROOT, "include")

MQ_OK, MQ_ENODEV, MQ_EINVAL, MQ_EHIP, MQ_ENOMEM, MQ_ECAP = 0, -1, -2, -3, -4, -5
INT, LONG, FLOAT, DOUBLE = 0, 1, 2, 3
OK, ERROR = 0, 1
RESULT, COLUMN = 0, 1


class MqAgg(C.Structure):
    _fields_ = [("count", C.c_uint64), ("sum", C.c_int64), ("min", C.c_int32),
                ("max", C.c_int32), ("_pad", C.c_uint64)]


class ColumnIndex(C.Structure):
    _fields_ = [("values", C.POINTER(C.c_int)), ("positions", C.POINTER(C.c_size_t))]


class Column(C.Structure):  # cs165_api.h:77-92
    _fields_ = [("name", C.c_char * 64), ("data", C.POINTER(C.c_int)), ("fd", C.c_int),
                ("row_count", C.c_size_t), ("sorted", C.c_bool), ("clustered", C.c_bool),
                ("has_index", C.c_bool), ("index", C.POINTER(ColumnIndex)),
                ("btree_node", C.c_void_p), ("histogram", C.c_void_p), ("max", C.c_int),
                ("min", C.c_int)]


class Status(C.Structure):  # cs165_api.h:160-163
    _fields_ = [("code", C.c_int), ("error_message", C.c_char_p)]


class Result(C.Structure):  # cs165_api.h:179-183
    _fields_ = [("num_tuples", C.c_size_t), ("data_type", C.c_int), ("payload", C.c_void_p)]


class GeneralizedColumnPointer(C.Union):
    _fields_ = [("result", C.POINTER(Result)), ("column", C.POINTER(Column))]


class GeneralizedColumn(C.Structure):  # cs165_api.h:203-206
    _fields_ = [("column_type", C.c_int), ("column_pointer", GeneralizedColumnPointer)]


class SelectOperator(C.Structure):  # db_manager.h:95-108
    _fields_ = [("select_type", C.c_int), ("handle", C.c_char * 64), ("low", C.c_int),
                ("high", C.c_int), ("has_low", C.c_int), ("has_high", C.c_int),
                ("db", C.c_void_p), ("table", C.c_void_p), ("column", C.POINTER(Column)),
                ("col_result", C.POINTER(Result)), ("pos_result", C.POINTER(Result)),
                ("comparator", C.c_void_p)]


class Table(C.Structure):  # cs165_api.h:110-116
    _fields_ = [("name", C.c_char * 64), ("columns", C.POINTER(Column)), ("col_count", C.c_size_t),
                ("row_count", C.c_size_t), ("table_length", C.c_size_t)]


class Db(C.Structure):  # cs165_api.h:127-132
    _fields_ = [("name", C.c_char * 64), ("tables", C.POINTER(Table)), ("tables_size", C.c_size_t),
                ("tables_capacity", C.c_size_t)]


ABI_LAYOUT = {  # SURVEY.md §8(b), measured on the reference with gcc 11 / x86-64
    "Result": (Result, 24, {"num_tuples": 0, "data_type": 8, "payload": 16}),
    "Column": (Column, 128, {"data": 64, "fd": 72, "row_count": 80, "sorted": 88,
                             "clustered": 89, "has_index": 90, "index": 96,
                             "btree_node": 104, "histogram": 112, "max": 120, "min": 124}),
    "Status": (Status, 16, {"code": 0, "error_message": 8}),
    "GeneralizedColumn": (GeneralizedColumn, 16, {"column_type": 0, "column_pointer": 8}),
    "SelectOperator": (SelectOperator, 136, {"handle": 4, "low": 68, "high": 72,
                                             "has_low": 76, "has_high": 80, "db": 88,
                                             "table": 96, "column": 104, "col_result": 112,
                                             "pos_result": 120, "comparator": 128}),
    "Table": (Table, 96, {"columns": 64, "col_count": 72, "row_count": 80, "table_length": 88}),
    "Db": (Db, 88, {"tables": 64, "tables_size": 72, "tables_capacity": 80}),
}

_vp, _u64, _i32, _sz, _int = C.c_void_p, C.c_uint64, C.c_int32, C.c_size_t, C.c_int
_PR = C.POINTER(Result)
_PS = C.POINTER(Status)

_SIGS = {
    # runtime
    "mq_init": (_int, [_int]),
    "mq_device_count": (_int, []),
    "mq_last_error": (C.c_char_p, []),
    "mq_version": (C.c_char_p, []),
    "mq_malloc": (_int, [C.POINTER(_vp), _sz]),
    "mq_free": (_int, [_vp]),
    "mq_pool_malloc": (_int, [C.POINTER(_vp), _sz]),
    "mq_pool_free": (_int, [_vp]),
    "mq_pool_free_on": (_int, [_vp, _vp]),
    "mq_device_sync": (_int, []),
    "mq_memcpy_h2d": (_int, [_vp, _vp, _sz, _vp]),
    "mq_memcpy_d2h": (_int, [_vp, _vp, _sz, _vp]),
    "mq_memcpy_d2d": (_int, [_vp, _vp, _sz, _vp]),
    "mq_memcpy_d2h_staged": (_int, [_vp, _vp, _sz, _vp]),
    "mq_host_prefault": (None, [_vp, _sz]),
    "mq_host_prefault_wait": (None, []),
    "mq_stream_create": (_int, [C.POINTER(_vp)]),
    "mq_stream_destroy": (_int, [_vp]),
    "mq_thread_release": (None, []),
    "mq_fetch_at": (_int, [_vp, _i32, _vp, _u64, _vp, _vp]),
    "mq_memset": (_int, [_vp, _int, _sz, _vp]),
    "mq_stream_sync": (_int, [_vp]),
    "mq_default_stream": (_vp, []),
    "mq_scan_workspace_bytes": (_sz, [_u64]),
    "mq_scan_geometry": (None, [_u64, C.POINTER(C.c_uint32), C.POINTER(_u64)]),
    # data
    "mq_gen_uniform": (_int, [_vp, _u64, _u64, _u64, _vp]),
    "mq_gen_join_keys": (_int, [_vp, _u64, _int, _vp]),
    "mq_gen_iota": (_int, [_vp, _u64, _vp]),
    # operators
    "mq_select_agg": (_int, [_vp, _u64, _int, _i32, _int, _i32, _vp, _vp, _sz, _vp]),
    "mq_select_partials": (_int, [_vp, _u64, _int, _i32, _int, _i32, _int, _vp, _sz,
                                  C.POINTER(C.c_uint32), _vp]),
    "mq_combine_partials": (_int, [_vp, C.c_uint32, _vp, _vp]),
    "mq_select_sum": (_int, [_vp, _u64, _int, _i32, _int, _i32, _vp, _vp, _sz, _vp]),
    "mq_format_workspace_bytes": (_sz, [_u64]),
    "mq_format_int32": (_int, [_vp, _u64, _vp, C.POINTER(C.c_uint64), _vp, _sz, _vp]),
    "mq_trim": (None, []),
    "mq_format_csv_workspace_bytes": (_sz, [_u64, _int]),
    "mq_format_csv_int32": (_int, [_vp, _int, _u64, _vp, C.POINTER(C.c_uint64), _vp, _sz, _vp]),
    "mq_csv_workspace_bytes": (_sz, [_u64, _int]),
    "mq_csv_count_rows": (_int, [_vp, _u64, _int, C.POINTER(_u64), _vp, _sz, _vp]),
    "mq_csv_parse_int32": (_int, [_vp, _u64, _int, _vp, _u64, _vp, _vp, _sz, _vp]),
    "mq_stream_read": (_int, [_vp, _u64, _vp, _sz, C.POINTER(C.c_uint64), _vp]),
    "mq_hashset_lookup": (_int, [_vp, _i32, _vp, _u64, _vp, _vp]),
    "mq_hashset_elements": (_int, [_vp, _u64, _vp, _vp, _vp, _sz, _vp]),
    "mq_random_read": (_int, [_vp, _int, _u64, _vp, _vp]),
    "mq_select_fetch_agg": (_int, [_vp, _vp, _u64, _int, _i32, _int, _i32, _vp, _vp, _sz, _vp]),
    "mq_select_positions_at": (_int, [_vp, _vp, _u64, _i32, _int, _i32, _int, _i32, _vp, _vp, _vp, _sz,
                                      _vp]),
    "mq_select_positions": (_int, [_vp, _vp, _u64, _int, _i32, _int, _i32, _vp, _vp, _vp, _sz,
                                   _vp]),
    "mq_select_positions_download": (_int, [_vp, _u64, _int, _i32, _int, _i32, _int, _vp, _vp,
                                            C.POINTER(_u64), C.POINTER(_u64), _vp, _sz, _vp]),
    "mq_index_select": (_int, [_vp, _vp, _u64, _i32, _i32, _vp, _vp, _vp]),
    "mq_fetch": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "mq_index_build": (_int, [_vp, _u64, _vp, _vp, _vp]),
    "mq_index_build_lomuto": (_int, [_vp, _u64, _vp, _vp, _vp]),
    "mq_index_build_ref": (_int, [_vp, _u64, _vp, _vp, _u64, C.POINTER(_int), _vp]),
    "mq_gather_u64": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "mq_histogram": (_int, [_vp, _u64, _i32, _i32, _vp, _vp]),
    "mq_reduce": (_int, [_vp, _u64, _vp, _vp, _sz, _vp]),
    "mq_add": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "mq_sub": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "mq_shared_select_workspace_bytes": (_sz, [_u64, _int]),
    "mq_shared_select": (_int, [_vp, _u64, _vp, _vp, _int, _vp, _vp, _vp, _sz, _vp]),
    "mq_shared_select_count": (_int, [_vp, _u64, _vp, _vp, _int, _vp, _vp, _sz, _vp]),
    "mq_shared_select_write": (_int, [_vp, _vp, _vp]),
    "mq_shared_select_count_at": (_int, [_vp, _u64, _i32, _vp, _vp, _int, _vp, _vp, _sz, _vp]),
    "mq_hash_join": (_int, [_vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _u64, C.POINTER(_u64),
                            _vp]),
    "mq_join_build": (_int, [_vp, _vp, _u64, C.POINTER(_vp), _vp]),
    "mq_join_probe": (_int, [_vp, _vp, _u64, C.POINTER(_u64), _vp]),
    "mq_join_write": (_int, [_vp, _vp, _vp, _vp, _vp]),
    "mq_join_free": (_int, [_vp]),
    "mq_join_counts": (_int, [_vp, _vp, _vp]),
    # key-partitioned join (mq_pjoin.hip, mq_shard.c)
    "mq_pjoin_bucket": (C.c_uint32, [_i32, _int]),
    "mq_pjoin_partition": (_int, [_vp, _vp, _u64, _int, _vp, _vp, _vp, C.POINTER(_u64), _vp]),
    "mq_pjoin_place": (_int, [_vp, _vp, _vp, _vp, _u64, _u64, _vp, _vp, _vp]),
    "mq_memcpy_peer": (_int, [_vp, _int, _vp, _int, _sz, _vp]),
    "mq_enable_peer": (_int, [_int]),
    "mq_shard_join": (_int, [C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_u64), C.POINTER(_vp), C.POINTER(_vp),
                             C.POINTER(_u64), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_u64)]),
    "mq_shard_devices": (_int, [C.POINTER(_int), _int]),
    "mq_shard_join_times": (None, [C.POINTER(C.c_double)]),
    "mq_shard_join_inject_failure": (None, [C.c_int]),
    # reference API (query.h:20-50)
    "select_result": (_PR, [_PR, _PR, C.POINTER(_int), C.POINTER(_int), _PS]),
    "select_column": (_PR, [C.POINTER(Column), C.POINTER(_int), C.POINTER(_int), _PS]),
    "select_column_scan": (_PR, [C.POINTER(Column), C.POINTER(_int), C.POINTER(_int), _PS]),
    "select_column_sorted_index": (_PR, [C.POINTER(Column), _int, _int, _PS]),
    "fetch_column": (_PR, [C.POINTER(Column), _PR, _PS]),
    "print": (C.c_void_p, [C.POINTER(_PR), _int, _PS]),
    "average": (_PR, [_PR, _PS]),
    "sum": (_PR, [C.POINTER(GeneralizedColumn), _PS]),
    "add": (_PR, [_PR, _PR, _PS]),
    "sub": (_PR, [_PR, _PR, _PS]),
    "min": (_PR, [_PR, _PS]),
    "max": (_PR, [_PR, _PS]),
    "shared_select": (C.POINTER(_PR), [C.POINTER(SelectOperator), _int, C.POINTER(Column), _PS]),
    "nested_loop_join": (C.POINTER(_PR), [_PR, _PR, _PR, _PR, _PS]),
    "hash_join": (C.POINTER(_PR), [_PR, _PR, _PR, _PR, _PS]),
    "log_result": (None, [_PR]),
    "should_use_index": (C.c_bool, [C.POINTER(Column), _int, _int]),
    # load path (db_manager.h:254)
    "load_db": (None, [C.POINTER(Db), C.c_char_p, _PS]),
    "build_index": (None, [C.POINTER(Db)]),
    # residency
    "mq_column_attach": (_int, [C.POINTER(Column), _vp]),
    "mq_column_upload": (_int, [C.POINTER(Column)]),
    "mq_column_invalidate": (None, [C.POINTER(Column)]),
    "mq_result_device_ptr": (_vp, [_PR]),
    "mq_release_all": (None, []),
    "mq_shard_config": (_int, [_int, C.POINTER(_int), _int, _u64]),
    "mq_transfer_seconds": (C.c_double, [_int]),
    "mq_residency_stats": (None, [C.c_void_p]),
    # write guards (csrc/mq_guard.h; internal, bound for the guard tests)
    "mq_guard_arm": (C.c_uint64, [_vp, _sz, _int]),
    "mq_guard_clean": (_int, [C.c_uint64, _vp, _sz]),
    "mq_guard_release": (None, [C.c_uint64]),
    "mq_guard_forget_range": (None, [C.c_size_t, _sz]),
    "mq_guard_retry_test": (_int, [C.c_uint32, C.c_uint32, _int]),
}

MQ_GUARD_FILE, MQ_GUARD_CHUNK = 0, 1


class Residency(C.Structure):  # include/mq_query.h mq_residency
    _fields_ = [(n, C.c_uint64) for n in (
        "column_uploads", "column_bytes", "result_uploads", "result_bytes", "guards_armed",
        "guard_clean", "guard_stale", "guards_live", "remap_probe", "columns_resident",
        "shadows_resident", "shadow_bytes", "shards", "shard_columns", "shard_shadows", "shard_ops",
        "shard_uploads")]


def residency(lib=None) -> dict:
    r = Residency()
    (lib or load()).mq_residency_stats(C.byref(r))
    return {n: int(getattr(r, n)) for n, _ in Residency._fields_}

# The reference-API signatures shared with the reference's own library (oracle/_ref).
REFERENCE_API = ["select_result", "select_column", "select_column_scan",
                 "select_column_sorted_index", "fetch_column", "print", "average", "sum", "add",
                 "sub", "min", "max", "shared_select", "nested_loop_join", "hash_join",
                 "log_result", "should_use_index"]


class MqError(RuntimeError):
    pass


def bind(lib: C.CDLL, names=None, strict: bool = True) -> C.CDLL:
    for name, (res, args) in _SIGS.items():
        if names is not None and name not in names:
            continue
        if not strict and not hasattr(lib, name):  # an older build loaded for an A/B
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libmq.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None or path != LIB_PATH:
        if not os.path.exists(path):
            raise MqError(f"libmq.so not built at {path}; run __graft_entry__.build()")
        lib = bind(C.CDLL(path), strict=path == LIB_PATH)
        if path != LIB_PATH:
            return lib
        _LIB = lib
    return _LIB


def check(rc: int, what: str = "libmq") -> None:
    if rc != MQ_OK:
        msg = load().mq_last_error().decode(errors="replace")
        raise MqError(f"{what} failed ({rc}): {msg}")


def header_functions() -> list[str]:
    """Every function declared in include/*.h (for the export test)."""
    names = []
    for fn in sorted(os.listdir(INCLUDE_DIR)):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE_DIR, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in ("if", "while", "return", "sizeof"):
                names.append(name)
    return sorted(set(names))


# ---------------------------------------------------------------------------
# small conveniences for torch-owned device buffers (plumbing only)
# ---------------------------------------------------------------------------
def ptr(t) -> int:
    """Device pointer of a torch tensor (or an int)."""
    return t if isinstance(t, int) else t.data_ptr()


def stream_of(torch_stream) -> int:
    return int(torch_stream.cuda_stream) if torch_stream is not None else 0


def bounds(low, high):
    """(has_low, low, has_high, high) from Python values; None = unbounded."""
    return (0 if low is None else 1, 0 if low is None else int(low),
            0 if high is None else 1, 0 if high is None else int(high))
