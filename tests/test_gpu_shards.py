"""Row shards inside libmq (-m gpu): a column split into G row ranges, each on its own
device thread and stream (csrc/mq_shard.c), behind the unchanged reference API.

SURVEY.md §8(e): per-shard positions are local rows plus the shard base, concatenated
in shard order; {count, sum, min, max} fold across shards. VERDICT r01 next-3: a
2-way row split forced on device 0 must be bit-exact to the oracle (refcpu, pinned to
the reference's own query.c). On a one-GPU box every shard sits on device 0 with its
own stream; on a multi-GPU node the same code spreads them (MQ_DEVICES). The layout is
set with mq_shard_config, so this runs in the one pytest process.
"""
import ctypes as C
import mmap
import os

import numpy as np
import pytest

from refapi import _libc, make_column, make_result, mq, take

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    yield L
    L.mq_release_all()
    assert L.mq_shard_config(0, None, 0, 0) == 0  # back to the environment's layout


def config(lib, g, min_rows=0, devices=None):
    devs = devices or [0] * g  # every shard on device 0: the split itself is under test
    arr = (C.c_int * len(devs))(*devs)
    assert lib.mq_shard_config(g, arr, len(devs), min_rows) == 0


def st():
    return mq.Status(0, None)


def _b(v):
    return None if v is None else C.pointer(C.c_int(int(v)))


def select(lib, col, lo, hi):
    s = st()
    rp = lib.select_column(C.byref(col), _b(lo), _b(hi), C.byref(s))
    assert s.code == mq.OK and rp
    return rp


def fetch(lib, col, rp):
    s = st()
    out = lib.fetch_column(C.byref(col), rp, C.byref(s))
    assert s.code == mq.OK and out
    return out


def agg(lib, rp):
    """sum / avg / min / max of a Result through the API"""
    g = mq.GeneralizedColumn()
    g.column_type = mq.RESULT
    g.column_pointer.result = rp
    s = st()
    out = {"sum": int(take(lib.sum(C.byref(g), C.byref(s)))[0])}
    out["avg"] = float(take(lib.average(rp, C.byref(s)))[0])
    out["min"] = int(take(lib.min(rp, C.byref(s)))[0])
    out["max"] = int(take(lib.max(rp, C.byref(s)))[0])
    assert s.code == mq.OK
    return out


def sum_column(lib, col):
    g = mq.GeneralizedColumn()
    g.column_type = mq.COLUMN
    g.column_pointer.column = C.pointer(col)
    s = st()
    out = lib.sum(C.byref(g), C.byref(s))
    assert s.code == mq.OK
    return int(take(out)[0])


def memfd_column(values):
    """A column in a MAP_SHARED file mapping, as the reference's start_data maps them
    (db_manager.c:736-790), so the shards keep it resident between operators."""
    fd = os.memfd_create("shardcol")
    os.ftruncate(fd, max(values.nbytes, 4))
    m = mmap.mmap(fd, max(values.nbytes, 4), mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    a = np.frombuffer(m, dtype=np.int32)[:len(values)]
    a[:] = values
    return a, m, make_column(a)


BOUNDS = [(None, None), (None, 1000), (250_000, None), (250_000, 310_000), (0, 1), (500, 500),
          (-(2 ** 31), 2 ** 31 - 1), (900_000, 10 ** 9)]


@pytest.mark.parametrize("g", [2, 3])
def test_select_fetch_agg_on_shards(lib, refcpu, g):
    config(lib, g)
    n = 3_000_001  # ragged: not a multiple of the 1024-row split unit
    v0 = refcpu.gen_uniform(n, 42, 1_000_000)
    v1 = refcpu.gen_uniform(n, 43)
    c0, c1 = make_column(v0, b"c0"), make_column(v1, b"c1")
    ops0 = mq.residency(lib)["shard_ops"]
    for lo, hi in BOUNDS:
        want = refcpu.select_scan(v0, lo, hi)
        rp = select(lib, c0, lo, hi)
        assert np.array_equal(take(rp, free=False), want), (g, lo, hi)
        rf = fetch(lib, c1, rp)
        vals = v1[want]
        assert np.array_equal(take(rf, free=False), vals)
        if len(vals):
            w = refcpu.agg(vals)
            got = agg(lib, rf)
            assert (got["sum"], got["min"], got["max"]) == (w["sum"], w["min"], w["max"])
            assert got["avg"] == w["avg"]
        take(rp)
        take(rf)
    assert sum_column(lib, c0) == int(v0.astype(np.int64).sum())
    r = mq.residency(lib)
    assert r["shards"] == g and r["shard_ops"] > ops0


def test_shard_residency_and_rewrite(lib, refcpu):
    """File-backed columns stay resident on the shards across operators; an in-place
    rewrite (the reference's clustered reorder, index.c:105-114) is seen."""
    config(lib, 2)
    n = 2_000_000
    a, m, col = memfd_column(refcpu.gen_uniform(n, 44))
    lo, hi = n // 4, n // 4 + n // 50
    assert np.array_equal(take(select(lib, col, lo, hi)), refcpu.select_scan(a, lo, hi))
    up = mq.residency(lib)["shard_uploads"]
    assert np.array_equal(take(select(lib, col, lo, hi)), refcpu.select_scan(a, lo, hi))
    assert mq.residency(lib)["shard_uploads"] == up, "resident shards uploaded again"
    a[:] = a[::-1].copy()
    assert np.array_equal(take(select(lib, col, lo, hi)), refcpu.select_scan(a, lo, hi))
    assert mq.residency(lib)["shard_uploads"] == up + 1
    assert sum_column(lib, col) == int(a.astype(np.int64).sum())
    col.data = None
    del a
    lib.mq_release_all()


def test_sharded_column_stays_resident_after_upload(lib, refcpu):
    """mq_column_upload of a column the shards serve, then select -> fetch -> sum three
    times (the chain of bench.py --inproc): one shard upload, no re-upload per operator.
    (Found by --inproc: the one-device copy's write guard made the shard copy's guard
    fail to arm, so every operator uploaded the shards again.)"""
    config(lib, 2)
    n = 2_000_000
    a, m, col = memfd_column(refcpu.gen_uniform(n, 46))
    lo, hi = n // 4, n // 4 + n // 50
    up0 = mq.residency(lib)["shard_uploads"]
    assert lib.mq_column_upload(C.byref(col)) == 0
    assert mq.residency(lib)["shard_uploads"] == up0 + 1
    want = refcpu.select_scan(a, lo, hi)
    for _ in range(3):
        rp = select(lib, col, lo, hi)
        assert np.array_equal(take(rp, free=False), want)
        rf = fetch(lib, col, rp)
        assert agg(lib, rf)["sum"] == int(a[want].astype(np.int64).sum())
        take(rp)
        take(rf)
    assert mq.residency(lib)["shard_uploads"] == up0 + 1, "shards uploaded again"
    # the one-device path (a column below the shard threshold is not this one) takes the
    # column back whole after the shards drop it
    config(lib, 1)
    assert np.array_equal(take(select(lib, col, lo, hi)), want)
    col.data = None
    del a
    lib.mq_release_all()


def test_fetch_with_foreign_positions(lib, refcpu):
    """Positions that did not come from the shards (value order, duplicates, the
    caller's own payload) take the one-device path."""
    config(lib, 2)
    n = 1_500_000
    v = refcpu.gen_uniform(n, 45)
    col = make_column(v)
    pos = refcpu.gen_uniform(200_000, 46, n)
    r = make_result(pos)
    assert np.array_equal(take(fetch(lib, col, C.pointer(r))), v[pos])


@pytest.mark.parametrize("q", [2, 5, 20, 300])
def test_shared_select_on_shards(lib, refcpu, q):
    """shared_select (query.c:439-583) over a 2-way split: one query as an ordered
    select, more as count + write per shard (elementary intervals), Q > 256 in chunks."""
    config(lib, 2)
    n = 2_500_003
    v = refcpu.gen_uniform(n, 47, 100_000)
    rng = np.random.default_rng(q)
    lows = rng.integers(-10, 100_000, q).astype(np.int32)
    highs = (lows + rng.integers(-5, 3_000, q)).astype(np.int32)
    col = make_column(v)
    ops = (mq.SelectOperator * q)()
    for j in range(q):
        ops[j].low, ops[j].high = int(lows[j]), int(highs[j])
    s = st()
    out = lib.shared_select(ops, q, C.byref(col), C.byref(s))
    assert s.code == mq.OK and out
    want = refcpu.shared_select(v, lows, highs, split=0)
    for j in range(q):
        assert np.array_equal(take(out[j]), want[j]), j
    _libc.free(C.cast(out, C.c_void_p))


def test_config3_on_shards(lib, refcpu):
    """SURVEY §8(c) config 3 at 1e8 rows on a 2-way split: select col0 1 %, fetch col1,
    avg, against the oracle; the K and sum equal a one-device run."""
    config(lib, 2)
    n = 100_000_000
    c0 = refcpu.gen_uniform(n, 42, nthreads=16)
    c1 = refcpu.gen_uniform(n, 43, nthreads=16)
    col0, col1 = make_column(c0, b"c0"), make_column(c1, b"c1")
    lo, hi = n // 4, n // 4 + n // 100
    rp = select(lib, col0, lo, hi)
    pos = take(rp, free=False)
    assert np.array_equal(pos, refcpu.select_scan(c0, lo, hi, nthreads=16))
    rf = fetch(lib, col1, rp)
    w = refcpu.agg(c1[pos])
    got = agg(lib, rf)
    assert (got["sum"], got["min"], got["max"], got["avg"]) == (w["sum"], w["min"], w["max"], w["avg"])
    take(rp)
    take(rf)
    config(lib, 1)
    rp1 = select(lib, col0, lo, hi)
    assert np.array_equal(take(rp1), pos)


@pytest.mark.parametrize("g", [20, 40])
def test_many_shards_on_one_device(lib, refcpu, g):
    """VERDICT r02 weak-4 / ADVICE r02: more row shards on one device than the old 16
    arrival-counter slots. Every shard's worker runs mq_reduce / mq_select_positions on
    its own stream at the same time, so the in-kernel combines of up to g launches are
    in flight together; sum / avg / min / max of the column and of a select -> fetch
    chain must be bit-exact against the oracle. A second layout change stops and
    restarts all workers (their pinned staging is released, mq_thread_release)."""
    config(lib, g)
    n = 4_000_037
    v0 = refcpu.gen_uniform(n, 48, 1_000_000)
    v1 = refcpu.gen_uniform(n, 49)
    c0, c1 = make_column(v0, b"c0"), make_column(v1, b"c1")
    for rep in range(3):
        assert sum_column(lib, c0) == int(v0.astype(np.int64).sum()), rep
        assert sum_column(lib, c1) == int(v1.astype(np.int64).sum()), rep
        lo, hi = 100_000 * rep, 100_000 * rep + 40_000
        want = refcpu.select_scan(v0, lo, hi)
        rp = select(lib, c0, lo, hi)
        assert np.array_equal(take(rp, free=False), want), rep
        rf = fetch(lib, c1, rp)
        w = refcpu.agg(v1[want])
        got = agg(lib, rf)
        assert (got["sum"], got["min"], got["max"], got["avg"]) == (w["sum"], w["min"], w["max"], w["avg"]), rep
        take(rp)
        take(rf)
    assert mq.residency(lib)["shards"] == g
    lib.mq_release_all()


def test_bad_shard_device_falls_back(lib, refcpu):
    """a layout naming a device that does not exist is refused by
    mq_shard_config; the operators keep running on one device."""
    arr = (C.c_int * 2)(0, 10_000)
    assert lib.mq_shard_config(2, arr, 2, 0) != 0
    n = 2_000_003
    v = refcpu.gen_uniform(n, 50, 1_000_000)
    col = make_column(v)
    assert np.array_equal(take(select(lib, col, 1000, 90_000)), refcpu.select_scan(v, 1000, 90_000))
    assert sum_column(lib, col) == int(v.astype(np.int64).sum())
