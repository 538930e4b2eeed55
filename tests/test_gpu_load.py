"""The load path on gfx950 (mq_csv_count_rows / mq_csv_parse_int32, csrc/mq_csv.hip)
against the oracle and the reference's goldens — bit-exact.

  * every tests/csvcases.py input: all cells and min/max equal the restatement
    (oracle/refcpu.c rc_load_csv), and the reference's own load_db goldens
    (tests/golden/csv_goldens.json) outside the cells it leaves uninitialised;
  * unaligned text pointers (the byte-load staging path);
  * multi-chunk inputs with long lines, missing and extra tokens vs the oracle;
  * mq_format_csv_int32 vs Python's "%d" formatting;
  * full size (config 3's 1e9-row 4-column table as CSV text, ~40 GB in HBM):
    format -> parse round trip returns the columns exactly.
"""
import ctypes as C

import numpy as np
import pytest

from csvcases import cases
from devbuf import Dev
from refapi import mq
from test_oracle_load import GOLD, check_against_golden

pytestmark = pytest.mark.gpu
CASES = {name: (ncols, data) for name, ncols, data in cases()}


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    return L


def gpu_load(L, dtext_ptr, n, ncols):
    """count -> allocate -> parse; returns (cols [ncols, rows], minmax [ncols, 2])."""
    ws = Dev(L.mq_csv_workspace_bytes(n, ncols))
    rows = C.c_uint64()
    mq.check(L.mq_csv_count_rows(dtext_ptr, n, ncols, C.byref(rows), ws.ptr, ws.nbytes, None),
             "mq_csv_count_rows")
    rows = rows.value
    dcols = [Dev(max(rows, 1) * 4) for _ in range(ncols)]
    ptrs = (C.c_void_p * max(ncols, 1))(*[d.ptr for d in dcols])
    mm = Dev(max(ncols, 1) * 8)
    mq.check(L.mq_csv_parse_int32(dtext_ptr, n, ncols, ptrs, rows, mm.ptr, ws.ptr, ws.nbytes, None),
             "mq_csv_parse_int32")
    cols = np.stack([d.get(np.int32, rows) for d in dcols]) if ncols else np.zeros((0, rows), np.int32)
    return cols, mm.get(np.int32, 2 * ncols).reshape(ncols, 2)


def text_dev(data: bytes, offset: int = 0) -> Dev:
    return Dev.of(np.frombuffer(data, dtype=np.uint8) if data else np.zeros(0, np.uint8),
                  offset_elems=offset)


@pytest.mark.parametrize("name", sorted(CASES))
def test_load_cases_vs_oracle_and_goldens(lib, refcpu, name):
    ncols, data = CASES[name]
    d = text_dev(data)
    cols, mm = gpu_load(lib, d.ptr, len(data), ncols)
    want, want_mm = refcpu.load_csv(data, ncols)
    assert cols.shape == want.shape, name
    assert np.array_equal(cols, want), name
    if want.shape[1]:
        assert np.array_equal(mm, want_mm), name
    else:
        assert all(tuple(m) == (2 ** 31 - 1, -(2 ** 31)) for m in mm)
    check_against_golden(name, cols, mm, cols.shape[1])


@pytest.mark.parametrize("offset", [1, 3, 7, 13])
def test_load_unaligned_text(lib, refcpu, offset):
    for name in ("long_lines", "fuzz_small", "random_4col", "missing_extra"):
        ncols, data = CASES[name]
        d = text_dev(data, offset)
        cols, mm = gpu_load(lib, d.ptr, len(data), ncols)
        want, want_mm = refcpu.load_csv(data, ncols)
        assert np.array_equal(cols, want) and np.array_equal(mm, want_mm), (name, offset)


def _multichunk_text(seed: int, lines: int, long_every: int, ragged: bool) -> tuple[bytes, int]:
    rng = np.random.default_rng(seed)
    ncols = 4
    vals = rng.integers(-2 ** 31, 2 ** 31, size=(lines, ncols + 2), dtype=np.int64)
    k = rng.integers(1, ncols + 3, lines) if ragged else np.full(lines, ncols)
    out = []
    for i in range(lines):
        row = ",".join(str(int(v)) for v in vals[i, :k[i]])
        if long_every and i % long_every == long_every - 1:
            row = row + "," + " " * int(rng.integers(900, 4000)) + str(int(vals[i, 0]))
        out.append(row + "\n")
    return "".join(out).encode(), ncols


@pytest.mark.parametrize("long_every,ragged", [(0, False), (0, True), (97, False), (13, True)])
def test_load_multichunk_vs_oracle(lib, refcpu, long_every, ragged):
    data, ncols = _multichunk_text(11 + long_every, 60_000, long_every, ragged)
    assert len(data) > 40 * 16384
    d = text_dev(data)
    cols, mm = gpu_load(lib, d.ptr, len(data), ncols)
    want, want_mm = refcpu.load_csv(data, ncols)
    assert np.array_equal(cols, want) and np.array_equal(mm, want_mm)


_TOKENS = ["0", "-0", "", "-", "7", "-7", "0000000000", "4294967295", "9999999999", "-9999999999",
           "2147483647", "-2147483648", "123456789", "-12345", "00042"]
_IRREGULAR = [" 5", "+5", "5 ", "12345678901", "1-2", "5\r", "\t9"]


def _token_text(seed: int, lines: int, ncols: int, irregular_every: int) -> bytes:
    """Rows of ncols tokens of 0-10 digits (k_csv_parse's token-parallel form), with
    every irregular_every-th row made irregular (isspace, '+', junk, 11 digits,
    a missing or an extra token) so that its chunk takes the row-wise parse."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(lines):
        k = ncols
        toks = []
        for _ in range(k):
            r = rng.random()
            if r < 0.15:
                toks.append(_TOKENS[int(rng.integers(len(_TOKENS)))])
            else:
                toks.append(str(int(rng.integers(-10 ** int(rng.integers(1, 10)), 10 ** int(rng.integers(1, 11))))))
        if irregular_every and i % irregular_every == irregular_every - 1:
            kind = int(rng.integers(3))
            if kind == 0:
                toks[int(rng.integers(ncols))] = _IRREGULAR[int(rng.integers(len(_IRREGULAR)))]
            elif kind == 1 and ncols > 1:
                toks = toks[:-1]
            else:
                toks.append("31")
        out.append(",".join(toks) + "\n")
    return "".join(out).encode()


@pytest.mark.parametrize("ncols", [1, 2, 3, 4, 5, 7, 8, 16, 17])
@pytest.mark.parametrize("irregular_every", [0, 701])
def test_load_token_parallel_vs_oracle(lib, refcpu, ncols, irregular_every):
    """The token-parallel parse (every row ncols tokens of [-]digits{0..10}) and its
    per-chunk fall-back to the row-wise parse, against the oracle."""
    data = _token_text(100 + ncols, max(4000, 600_000 // (ncols * 7)), ncols, irregular_every)
    assert len(data) > 16 * 16384
    for offset in (0, 5):
        d = text_dev(data, offset)
        cols, mm = gpu_load(lib, d.ptr, len(data), ncols)
        want, want_mm = refcpu.load_csv(data, ncols)
        assert np.array_equal(cols, want), (ncols, irregular_every, offset)
        assert np.array_equal(mm, want_mm), (ncols, irregular_every, offset)


def test_load_token_parallel_short_tokens(lib, refcpu):
    """One-digit tokens: more separators per chunk than the token list holds (the
    row-wise parse), and the text's end without a final '\n'."""
    rng = np.random.default_rng(9)
    rows = ["%d,%d,%d" % tuple(rng.integers(0, 10, 3)) for _ in range(50_000)]
    data = ("\n".join(rows)).encode()
    d = text_dev(data)
    cols, mm = gpu_load(lib, d.ptr, len(data), 3)
    want, want_mm = refcpu.load_csv(data, 3)
    assert np.array_equal(cols, want) and np.array_equal(mm, want_mm)


def _format(L, dcols, rows):
    ncols = len(dcols)
    ws = Dev(L.mq_format_csv_workspace_bytes(rows, ncols))
    out = Dev(max(rows * ncols * 12, 16))
    ptrs = (C.c_void_p * ncols)(*[d.ptr for d in dcols])
    n = C.c_uint64()
    mq.check(L.mq_format_csv_int32(ptrs, ncols, rows, out.ptr, C.byref(n), ws.ptr, ws.nbytes, None),
             "mq_format_csv_int32")
    return out, n.value


def test_format_csv_vs_python(lib):
    rng = np.random.default_rng(5)
    rows = 5000
    host = [rng.integers(-2 ** 31, 2 ** 31, rows, dtype=np.int64).astype(np.int32) for _ in range(3)]
    host[0][:4] = [0, -1, 2 ** 31 - 1, -(2 ** 31)]
    out, n = _format(lib, [Dev.of(h) for h in host], rows)
    want = "".join(f"{a},{b},{c}\n" for a, b, c in zip(*host)).encode()
    assert out.get(np.uint8, n).tobytes() == want


@pytest.mark.big
def test_load_roundtrip_config3_table_1e9(lib):
    """Config 3's table (4 x 1e9 int32, seeds 42-45) as CSV text in HBM, parsed back:
    every cell equal (FNV of each column), min/max equal to the columns' own."""
    n = 1_000_000_000
    L = lib
    cols = []
    for s in range(4):
        c = Dev(n * 4)
        mq.check(L.mq_gen_uniform(c.ptr, n, 42 + s, n, None))
        cols.append(c)
    text, nbytes = _format(L, cols, n)
    got_cols, mm = gpu_load_dev(L, text.ptr, nbytes, 4, n)
    for j in range(4):
        mq.check(L.mq_sub(cols[j].ptr, got_cols[j].ptr, n, got_cols[j].ptr, None))
        a = Dev(32)
        ws = Dev(L.mq_scan_workspace_bytes(n))
        mq.check(L.mq_reduce(got_cols[j].ptr, n, a.ptr, ws.ptr, ws.nbytes, None))
        agg = mq.MqAgg.from_buffer_copy(a.get(np.uint8, 32).tobytes())
        assert (agg.min, agg.max) == (0, 0), j  # original - parsed == 0 everywhere
        b = Dev(32)
        mq.check(L.mq_reduce(cols[j].ptr, n, b.ptr, ws.ptr, ws.nbytes, None))
        orig = mq.MqAgg.from_buffer_copy(b.get(np.uint8, 32).tobytes())
        assert tuple(mm[j]) == (orig.min, orig.max), j


def gpu_load_dev(L, dtext_ptr, n, ncols, rows_expected):
    ws = Dev(L.mq_csv_workspace_bytes(n, ncols))
    rows = C.c_uint64()
    mq.check(L.mq_csv_count_rows(dtext_ptr, n, ncols, C.byref(rows), ws.ptr, ws.nbytes, None))
    assert rows.value == rows_expected
    dcols = [Dev(rows.value * 4) for _ in range(ncols)]
    ptrs = (C.c_void_p * ncols)(*[d.ptr for d in dcols])
    mm = Dev(ncols * 8)
    mq.check(L.mq_csv_parse_int32(dtext_ptr, n, ncols, ptrs, rows.value, mm.ptr, ws.ptr, ws.nbytes,
                                  None))
    return dcols, mm.get(np.int32, 2 * ncols).reshape(ncols, 2)


# ---------------------------------------------------------------------------
# the drop-in load_db (mq_query.c) through the reference's own types
# ---------------------------------------------------------------------------
def _table(ncols, capacity, rows_before=0, seed=0):
    """A Db with one table 'tbl' of ncols columns (host buffers of `capacity` rows),
    as create_db / create_table / create_column leave it (db_manager.c:34-148),
    optionally holding rows_before rows already."""
    rng = np.random.default_rng(seed)
    bufs = [np.zeros(capacity, dtype=np.int32) for _ in range(ncols)]
    cols = (mq.Column * ncols)()
    for j in range(ncols):
        c = cols[j]
        c.name = f"c{j}".encode()
        c.data = bufs[j].ctypes.data_as(C.POINTER(C.c_int))
        c.fd = -1
        c.max, c.min = -(2 ** 31), 2 ** 31 - 1
        if rows_before:
            bufs[j][:rows_before] = rng.integers(-1000, 1000, rows_before)
            c.row_count = rows_before
            c.max, c.min = int(bufs[j][:rows_before].max()), int(bufs[j][:rows_before].min())
    t = mq.Table()
    t.name = b"tbl"
    t.columns = cols
    t.col_count, t.row_count, t.table_length = ncols, rows_before, capacity
    db = mq.Db()
    db.name = b"db"
    db.tables = C.pointer(t)
    db.tables_size, db.tables_capacity = 1, 1
    return db, t, cols, bufs


def _write_csv(tmp_path, name, ncols, data, header=None):
    path = tmp_path / f"{name}.csv"
    hdr = header if header is not None else (",".join(f"db.tbl.c{j}" for j in range(ncols)) + "\n").encode()
    path.write_bytes(hdr + data)
    return str(path)


@pytest.mark.parametrize("name", ["basic", "long_lines", "missing_extra", "random_4col", "fuzz_small"])
def test_load_db_dropin_vs_reference(lib, refcpu, tmp_path, name):
    """load_db into a table with room for every row (the server's save_data /
    start_data are not linked into this process): rows, values, min/max as the
    reference's load_db + insert_row leave them, and the columns stay resident."""
    ncols, data = CASES[name]
    path = _write_csv(tmp_path, name, ncols, data)
    want, want_mm = refcpu.load_csv(data, ncols)
    rows = want.shape[1]
    db, t, cols, bufs = _table(ncols, max(rows, 1))
    st = mq.Status(0, None)
    lib.load_db(C.byref(db), path.encode(), C.byref(st))
    assert st.code == mq.OK
    assert t.row_count == rows and all(cols[j].row_count == rows for j in range(ncols))
    g = GOLD[name]
    for j in range(ncols):
        assert np.array_equal(bufs[j][:rows], want[j]), j
        if g["minmax"][j] is not None:
            assert [cols[j].min, cols[j].max] == g["minmax"][j], j
    check_against_golden(name, np.stack([b[:rows] for b in bufs]), [(c.min, c.max) for c in cols], rows)
    # resident: a select on column 0 needs no upload
    lib.mq_transfer_seconds(1)
    lo, hi = C.c_int(-10 ** 6), C.c_int(10 ** 6)
    r = lib.select_column(C.byref(cols[0]), C.byref(lo), C.byref(hi), C.byref(st))
    assert st.code == mq.OK and r
    k = r.contents.num_tuples
    assert k == int(((want[0] >= -10 ** 6) & (want[0] < 10 ** 6)).sum())


def test_load_db_appends_and_reports_errors(lib, refcpu, tmp_path):
    ncols, data = CASES["random_4col"]
    want, _ = refcpu.load_csv(data, ncols)
    rows = want.shape[1]
    db, t, cols, bufs = _table(ncols, rows + 100, rows_before=100, seed=3)
    before = [b[:100].copy() for b in bufs]
    mm_before = [(c.min, c.max) for c in cols]
    path = _write_csv(tmp_path, "app", ncols, data)
    st = mq.Status(0, None)
    lib.load_db(C.byref(db), path.encode(), C.byref(st))
    assert st.code == mq.OK and t.row_count == rows + 100
    for j in range(ncols):
        assert np.array_equal(bufs[j][:100], before[j]) and np.array_equal(bufs[j][100:], want[j])
        assert cols[j].min == min(mm_before[j][0], int(want[j].min()))
        assert cols[j].max == max(mm_before[j][1], int(want[j].max()))
    # wrong db / table name in the header, missing file: ERROR, table untouched (:253-295)
    for hdr in (b"other.tbl.c0\n", b"db.nope.c0\n", b"dbtbl\n"):
        p = _write_csv(tmp_path, "bad", ncols, b"1,2,3,4\n", header=hdr)
        st = mq.Status(0, None)
        lib.load_db(C.byref(db), p.encode(), C.byref(st))
        assert st.code == mq.ERROR and t.row_count == rows + 100
    st = mq.Status(0, None)
    lib.load_db(C.byref(db), str(tmp_path / "missing.csv").encode(), C.byref(st))
    assert st.code == mq.ERROR
    # growth needs the server's save_data/start_data: without them, ERROR
    db2, t2, _, _ = _table(ncols, 16)
    st = mq.Status(0, None)
    lib.load_db(C.byref(db2), path.encode(), C.byref(st))
    assert st.code == mq.ERROR and t2.row_count == 0
