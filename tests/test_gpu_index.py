"""The index build on gfx950 (mq_index_build / mq_index_build_lomuto /
mq_index_build_ref / mq_gather_u64 / mq_histogram, csrc/mq_index.hip, and the
build_index drop-in in mq_query.c) — bit-exact against the oracle: the stable radix
sort against the stable restatement, the Lomuto order against the restatement of
the reference quicksort (pinned to the reference's own quicksort symbol), and the
drop-in against the reference's own build_index goldens, equal values included.
"""
import ctypes as C

import numpy as np
import pytest

from devbuf import Dev
from indexcases import cases, model
from refapi import mq
from test_oracle_index import _lomuto_inputs, check_index_result

pytestmark = pytest.mark.gpu
CASES = {name: (cols, spec) for name, cols, spec in cases()}


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    return L


def gpu_index(L, col: np.ndarray):
    n = len(col)
    d = Dev.of(col.astype(np.int32))
    v, p = Dev(max(n, 1) * 4), Dev(max(n, 1) * 8)
    mq.check(L.mq_index_build(d.ptr, n, v.ptr, p.ptr, None), "mq_index_build")
    return v.get(np.int32, n), p.get(np.uint64, n)


@pytest.mark.parametrize("n,lo,hi", [(0, 0, 1), (1, 0, 1), (1000, -5, 5), (4097, -2**31, 2**31 - 1),
                                     (100_003, 0, 1000), (1_000_000, -2**31, 2**31 - 1)])
def test_index_build_vs_oracle(lib, refcpu, n, lo, hi):
    rng = np.random.default_rng(n)
    col = rng.integers(lo, hi, n, dtype=np.int64).astype(np.int32) if n else np.zeros(0, np.int32)
    if n > 4:
        col[:3] = [-2**31, 2**31 - 1, 0]
    v, p = gpu_index(lib, col)
    wv, wp = refcpu.index_build(col)
    assert np.array_equal(v, wv) and np.array_equal(p, wp)


def _wide_range_inputs():
    """Columns that take radix_sort_index's MSD form (n >= 2^22 rows, key range over
    24 bits, csrc/mq_isort.hip) or its shortened LSD form, with the shapes that steer
    the MSD levels: ranges split twice or three times, finisher ranges of one key
    (copied out in row order), ranges above the LDS capacity with no key bits left,
    one or two LDS passes, a nonzero range minimum."""
    rng = np.random.default_rng(77)
    n = (1 << 22) + 17
    yield "full_int32_4M", rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32)
    yield "b25_5M", rng.integers(0, 1 << 25, 5_000_000).astype(np.int32)
    yield "b30_offset_6M", (rng.integers(0, 1 << 30, 6_000_000) - 123_456_789).astype(np.int32)
    c = rng.integers(0, 1 << 30, n).astype(np.int32)
    c[rng.random(n) < 0.5] = 7  # one key holds half the rows: a finisher range far above kCap
    yield "half_one_value_4M", c
    c = (rng.integers(0, 1 << 22, n) << 8).astype(np.int32)  # low 8 bits zero: ties everywhere
    yield "low_bits_zero_4M", c
    c = rng.integers(0, 1 << 30, n).astype(np.int32)
    c[: n // 4] = rng.integers(0, 1 << 12, n // 4)  # a dense corner: ranges split three levels
    yield "skewed_corner_4M", c
    yield "b23_lsd3_4M", (rng.integers(0, 1 << 23, n) + 10**9).astype(np.int32)
    yield "b8_lsd1_4M", (rng.integers(0, 200, n) - 100).astype(np.int32)
    yield "sorted_desc_4M", np.arange(n, 0, -1, dtype=np.int64).astype(np.int32) * 64
    c = rng.integers(0, 1 << 30, n).astype(np.int32)
    hot = rng.choice(n, 3000, replace=False)
    c[hot[:1000]] = 123_456_789  # keys on more than kTieMax rows inside ranges of many
    c[hot[1000:2000]] = 987_654_321  # keys: the counting finisher hands them to the ranked one
    c[hot[2000:]] = c[hot[2000:]] | 1
    yield "hot_keys_4M", c


@pytest.mark.parametrize("form", ["default", "msd"])
@pytest.mark.parametrize("name,col", list(_wide_range_inputs()), ids=lambda x: x if isinstance(x, str) else "")
def test_index_build_wide_range_vs_oracle(lib, refcpu, name, col, form, monkeypatch):
    """form "msd": MQ_INDEX_MSD_MIN=0 takes the MSD form at these sizes too (by default
    it starts at 2^24 rows)."""
    if form == "msd":
        monkeypatch.setenv("MQ_INDEX_MSD_MIN", "0")
    v, p = gpu_index(lib, col)
    wv, wp = refcpu.index_build(col)
    assert np.array_equal(v, wv), name
    assert np.array_equal(p, wp), name


@pytest.mark.parametrize("which", ["values_only", "positions_only"])
def test_index_build_msd_one_output(lib, refcpu, which, monkeypatch):
    """mq_index_build takes NULL for either output (mq_device.h); the MSD form's
    finishers and the copied one-key ranges honour it too."""
    monkeypatch.setenv("MQ_INDEX_MSD_MIN", "0")
    rng = np.random.default_rng(91)
    n = (1 << 22) + 3
    col = rng.integers(0, 1 << 30, n).astype(np.int32)
    col[rng.random(n) < 0.2] = 5  # a one-key range far above the LDS capacity
    d = Dev.of(col)
    v, p = Dev(n * 4), Dev(n * 8)
    wv, wp = refcpu.index_build(col)
    if which == "values_only":
        mq.check(lib.mq_index_build(d.ptr, n, v.ptr, None, None))
        assert np.array_equal(v.get(np.int32, n), wv)
    else:
        mq.check(lib.mq_index_build(d.ptr, n, None, p.ptr, None))
        assert np.array_equal(p.get(np.uint64, n), wp)


@pytest.mark.parametrize("n", [(1 << 24) - 1, 1 << 24])
def test_index_build_form_boundary(lib, refcpu, n):
    """Either side of the default MSD threshold (2^24 rows), a 31-bit key range."""
    rng = np.random.default_rng(n)
    col = rng.integers(-2**30, 2**30, n).astype(np.int32)
    v, p = gpu_index(lib, col)
    wv, wp = refcpu.index_build(col)
    assert np.array_equal(v, wv) and np.array_equal(p, wp)


def gpu_lomuto(L, col: np.ndarray):
    n = len(col)
    d = Dev.of(col.astype(np.int32)) if n else Dev(4)
    v, p = Dev(max(n, 1) * 4), Dev(max(n, 1) * 8)
    mq.check(L.mq_index_build_lomuto(d.ptr, n, v.ptr, p.ptr, None), "mq_index_build_lomuto")
    return v.get(np.int32, n), p.get(np.uint64, n)


def _more_lomuto_inputs():
    rng = np.random.default_rng(5)
    # one value >= the pivot followed by a long run below it: a 4999-step swap chain
    # (pointer doubling past kChainCap)
    yield "long_chain", np.concatenate([[10**6], np.arange(1, 5000), [10**6 - 1]]).astype(np.int32)
    yield "chains_mixed", np.concatenate([rng.integers(900, 1000, 40), rng.integers(0, 100, 3000),
                                          [500]]).astype(np.int32)
    yield "dups_200k", rng.integers(0, 1000, 200_000).astype(np.int32)
    yield "distinctish_300k", rng.integers(-2**31, 2**31 - 1, 300_000, dtype=np.int64).astype(np.int32)
    yield "few_values_100k", rng.integers(0, 3, 100_000).astype(np.int32)
    yield "runs_sorted_blocks", np.repeat(rng.permutation(2000), 20).astype(np.int32)


@pytest.mark.parametrize("name,col", list(_lomuto_inputs()) + list(_more_lomuto_inputs()))
def test_index_build_lomuto_vs_oracle(lib, refcpu, name, col):
    """The reference quicksort's order (index.c:25-46), equal values included."""
    v, p = gpu_lomuto(lib, col)
    wv, wp = refcpu.index_build_lomuto(col)
    assert np.array_equal(v, wv), name
    assert np.array_equal(p, wp), name


def test_index_build_ref_policy(lib, refcpu):
    """distinct values -> the radix result (one order exists); ties -> the Lomuto order
    up to exact_max rows, ascending row order beyond it."""
    rng = np.random.default_rng(8)
    for col, ties in ((rng.permutation(50_000).astype(np.int32), False),
                      (rng.integers(0, 500, 50_000).astype(np.int32), True)):
        n = len(col)
        d, v, p = Dev.of(col), Dev(n * 4), Dev(n * 8)
        for exact_max, want_exact in ((1 << 40, 1), (1000, 0 if ties else 1)):
            ex = C.c_int(-1)
            mq.check(lib.mq_index_build_ref(d.ptr, n, v.ptr, p.ptr, exact_max, C.byref(ex), None))
            assert ex.value == want_exact
            wv, wp = (refcpu.index_build_lomuto(col) if want_exact else refcpu.index_build(col))
            assert np.array_equal(v.get(np.int32, n), wv) and np.array_equal(p.get(np.uint64, n), wp)


def test_gather_and_histogram_vs_oracle(lib, refcpu):
    rng = np.random.default_rng(9)
    col = rng.integers(-10**6, 10**6, 300_000).astype(np.int32)
    dc = Dev.of(col)
    for m in (1, 7, 2047, 2049, 200_013):  # full steps of 8 x 256 rows and the ragged last one
        pos = rng.integers(0, len(col), m).astype(np.uint64)
        dp, out = Dev.of(pos), Dev(len(pos) * 4)
        mq.check(lib.mq_gather_u64(dc.ptr, dp.ptr, len(pos), out.ptr, None))
        assert np.array_equal(out.get(np.int32, len(pos)), col[pos.astype(np.int64)]), m
    for mn, bs in ((int(col.min()), (int(col.max()) - int(col.min())) // 99), (0, 7), (-10, -3)):
        h = Dev(101 * 8)
        mq.check(lib.mq_histogram(dc.ptr, len(col), mn, bs, h.ptr, None))
        assert np.array_equal(h.get(np.uint64, 101), refcpu.histogram(col, mn, bs)), (mn, bs)
    h = Dev(101 * 8)
    assert lib.mq_histogram(dc.ptr, len(col), 0, 0, h.ptr, None) == mq.MQ_EINVAL


def _db(cols: np.ndarray, spec):
    """A table as the server holds it after load_db, with create(idx,...) applied."""
    ncols, n = cols.shape
    bufs = [np.ascontiguousarray(cols[j].astype(np.int32)) for j in range(ncols)]
    cs = (mq.Column * ncols)()
    for j in range(ncols):
        c = cs[j]
        c.name = f"c{j}".encode()
        c.data = bufs[j].ctypes.data_as(C.POINTER(C.c_int))
        c.row_count = n
        c.max, c.min = int(bufs[j].max()), int(bufs[j].min())
    for j, clustered in spec:
        cs[j].has_index, cs[j].clustered, cs[j].sorted = True, clustered, True
    t = mq.Table()
    t.name = b"tbl"
    t.columns = cs
    t.col_count, t.row_count, t.table_length = ncols, n, n
    db = mq.Db()
    db.name = b"db"
    db.tables = C.pointer(t)
    db.tables_size = db.tables_capacity = 1
    return db, t, cs, bufs


class Histogram(C.Structure):  # cs165_api.h:71-75
    _fields_ = [("bin_size", C.c_int), ("values", C.c_int * 100), ("counts", C.c_size_t * 100)]


@pytest.mark.parametrize("name", sorted(CASES))
def test_build_index_dropin(lib, refcpu, name):
    cols, spec = CASES[name]
    db, t, cs, bufs = _db(cols, spec)
    lib.build_index(C.byref(db))
    n = cols.shape[1]
    got = {"cols": np.stack(bufs)}
    for j, clustered in spec:
        ix = cs[j].index.contents
        got[f"ix{j}_values"] = np.ctypeslib.as_array(ix.values, shape=(n,)).copy()
        got[f"ix{j}_positions"] = np.ctypeslib.as_array(ix.positions, shape=(n,)).copy()
        if not clustered:
            h = C.cast(cs[j].histogram, C.POINTER(Histogram)).contents
            got[f"hist{j}_bin_size"] = h.bin_size
            got[f"hist{j}_values"] = np.array(h.values[:], dtype=np.int64)
            got[f"hist{j}_counts"] = np.array(h.counts[:], dtype=np.uint64)
    want = model(refcpu, cols, spec)
    for k, v in want.items():  # bit-exact vs the quicksort restatement
        assert np.array_equal(np.asarray(got[k]), np.asarray(v)), (name, k)
    check_index_result(refcpu, name, got)  # and vs the reference's own build, exactly
    # the index and the reordered columns are resident: a sorted-index select and a
    # select on a reordered column agree with the host arrays
    st = mq.Status(0, None)
    j0 = spec[0][0]
    lo, hi = int(want[f"ix{j0}_values"][n // 4]), int(want[f"ix{j0}_values"][n // 2])
    r = lib.select_column_sorted_index(C.byref(cs[j0]), lo, hi, C.byref(st))
    assert st.code == mq.OK and r
    k = r.contents.num_tuples
    pos = np.ctypeslib.as_array(C.cast(r.contents.payload, C.POINTER(C.c_int32)), shape=(k,))
    v = want[f"ix{j0}_values"]
    a, b = np.searchsorted(v, lo), np.searchsorted(v, hi)
    assert k == b - a
    assert np.array_equal(pos, want[f"ix{j0}_positions"][a:b].astype(np.int32))
    other = (j0 + 1) % cols.shape[0]
    lo2, hi2 = C.c_int(int(np.median(bufs[other]))), C.c_int(2**31 - 1)
    r2 = lib.select_column_scan(C.byref(cs[other]), C.byref(lo2), C.byref(hi2), C.byref(st))
    k2 = r2.contents.num_tuples
    p2 = np.ctypeslib.as_array(C.cast(r2.contents.payload, C.POINTER(C.c_int32)), shape=(k2,))
    assert np.array_equal(p2, np.flatnonzero(bufs[other] >= lo2.value).astype(np.int32))


@pytest.mark.big
def test_index_build_1e9_properties(lib):
    """Full size: the 1e9-row uniform column (seed 42). Sorted values ascending, the
    positions a permutation that maps to them, ties in ascending row order."""
    n = 1_000_000_000
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, 42, n, None))
    v, p = Dev(n * 4), Dev(n * 8)
    mq.check(lib.mq_index_build(col.ptr, n, v.ptr, p.ptr, None))
    g = Dev(n * 4)
    mq.check(lib.mq_gather_u64(col.ptr, p.ptr, n, g.ptr, None))
    # gathered == sorted values (difference all zero), values ascending
    d = Dev(n * 4)
    mq.check(lib.mq_sub(g.ptr, v.ptr, n, d.ptr, None))
    ws = Dev(lib.mq_scan_workspace_bytes(n))
    a = Dev(32)
    mq.check(lib.mq_reduce(d.ptr, n, a.ptr, ws.ptr, ws.nbytes, None))
    agg = mq.MqAgg.from_buffer_copy(a.get(np.uint8, 32).tobytes())
    assert (agg.min, agg.max) == (0, 0)
    vs = v.get(np.int32, n)
    assert np.all(vs[1:] >= vs[:-1])
    ps = p.get(np.uint64, n)
    tie = vs[1:] == vs[:-1]
    assert np.all(ps[1:][tie] > ps[:-1][tie])
    seen = np.zeros(n, dtype=np.bool_)
    seen[ps.astype(np.int64)] = True
    assert seen.all()


def _qs_cases():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "quicksort_goldens.json")
    for c in json.load(open(path)):
        marks = [pytest.mark.big] if c["n"] > (1 << 24) else []
        yield pytest.param(c, marks=marks, id=f"2^{c['log2n']}_s{c['seed']}_m{c['modulus']}")


@pytest.mark.parametrize("case", list(_qs_cases()))
def test_index_build_lomuto_full_size(lib, refcpu, case):
    """the exact tie order at the sizes build_index applies it to
    (up to MQ_INDEX_EXACT_MAX = 2^27 rows), against the reference's own quicksort
    (tests/golden/quicksort_goldens.json, made by the `quicksort` symbol of the
    reference's index.c, make_quicksort_goldens.py). Both entry points:
    mq_index_build_lomuto, and mq_index_build_ref (the build_index policy: radix sort,
    tie check, then the Lomuto restatement) with exact_max = 2^27. Up to 2^24 rows the
    arrays are also compared element by element with the restatement
    rc_index_build_lomuto (refcpu.c, itself pinned to the same symbol)."""
    n = case["n"]
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, case["seed"], case["modulus"], None))
    h = col.get(np.int32, n)
    assert f"{refcpu.fnv1a64(h):016x}" == case["col_fnv"]
    v, p = Dev(n * 4), Dev(n * 8)
    mq.check(lib.mq_index_build_lomuto(col.ptr, n, v.ptr, p.ptr, None), "mq_index_build_lomuto")
    hv, hp = v.get(np.int32, n), p.get(np.uint64, n)
    assert f"{refcpu.fnv1a64(hv):016x}" == case["values_fnv"]
    assert f"{refcpu.fnv1a64(hp):016x}" == case["positions_fnv"]
    if n <= (1 << 24):
        wv, wp = refcpu.index_build_lomuto(h)
        assert np.array_equal(hv, wv) and np.array_equal(hp, wp)
    del hv, hp
    ex = C.c_int(-1)
    mq.check(lib.mq_memset(v.ptr, 0, n * 4, None))
    mq.check(lib.mq_memset(p.ptr, 0, n * 8, None))
    mq.check(lib.mq_index_build_ref(col.ptr, n, v.ptr, p.ptr, 1 << 27, C.byref(ex), None))
    assert ex.value == 1
    assert f"{refcpu.fnv1a64(v.get(np.int32, n)):016x}" == case["values_fnv"]
    assert f"{refcpu.fnv1a64(p.get(np.uint64, n)):016x}" == case["positions_fnv"]


_VARIANT_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1]]
from devbuf import Dev
from refapi import mq
L = mq.load()
mq.check(L.mq_init(0))
d = np.load(sys.argv[2])
out = {}
for name in d.files:
    col = d[name]
    n = len(col)
    c, v, p = Dev.of(col), Dev(n * 4), Dev(n * 8)
    mq.check(L.mq_index_build_lomuto(c.ptr, n, v.ptr, p.ptr, None))
    out[name + "_v"], out[name + "_p"] = v.get(np.int32, n), p.get(np.uint64, n)
np.savez(sys.argv[3], **out)
"""


@pytest.mark.parametrize("small,cap", [("512", "1"), ("2048", "3"), ("1024", "100000")])
def test_index_build_lomuto_variants(refcpu, tmp_path, small, cap):
    """The same order with the other small-range finishers (MQ_LQ_SMALL) and chain
    caps (MQ_LQ_CAP=1: pointer doubling in every range of every level; 100000: none),
    in a child process (both are read once per process)."""
    import os
    import subprocess
    import sys
    rng = np.random.default_rng(11)
    cols = {"long_chain": np.concatenate([[10**6], np.arange(1, 20000), [10**6 - 1]]).astype(np.int32),
            "dups": rng.integers(0, 500, 150_000).astype(np.int32),
            "distinct": rng.integers(-2**31, 2**31 - 1, 250_000, dtype=np.int64).astype(np.int32),
            "sorted_desc": np.arange(5000, 0, -1).astype(np.int32),
            "two_values": rng.integers(0, 2, 70_000).astype(np.int32)}
    np.savez(tmp_path / "in.npz", **cols)
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MQ_LQ_SMALL=small, MQ_LQ_CAP=cap)
    subprocess.run([sys.executable, "-c", _VARIANT_CHILD, here, str(tmp_path / "in.npz"), str(tmp_path / "out.npz")],
                   env=env, check=True, timeout=240)
    got = np.load(tmp_path / "out.npz")
    for name, col in cols.items():
        wv, wp = refcpu.index_build_lomuto(col)
        assert np.array_equal(got[name + "_v"], wv), name
        assert np.array_equal(got[name + "_p"], wp), name
