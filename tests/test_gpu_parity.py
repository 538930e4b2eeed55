"""libmq's HIP path vs the oracle — bit-exact (integer/index work) — on gfx950.

Every test calls through the C-ABI (include/mq_device.h, include/mq_query.h):
  * device API on seeded inputs at oracle-sized N, edge cases (empty, ragged,
    unaligned, NULL bounds, inverted/empty/full ranges, INT32 extremes);
  * the committed golden fixtures (tests/golden/, produced by the reference);
  * the drop-in query API side by side with the reference's own compiled
    query.c (oracle/_ref/libref.so) where that library is present;
  * at BASELINE's full size (1e9 rows): goldens plus size-independent
    properties (range additivity, sortedness, fetch-in-range).
"""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from devbuf import Dev
from refapi import Api, make_column, mq, take

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
I32MIN, I32MAX = -(2 ** 31), 2 ** 31 - 1
BOUNDS = [(None, None), (10, None), (None, 10), (-5, 5), (5, 5), (7, 3), (I32MIN, I32MAX),
          (I32MIN, None), (None, I32MAX), (I32MAX, None), (None, I32MIN), (0, 1), (-20, 20)]
SIZES = [0, 1, 3, 5, 1023, 1024, 1025, 4096 * 4 + 3, 65536 + 7, 1 << 20, 3_000_001]


def dbits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    return L


def _agg(L, dcol_ptr, n, lo, hi, fused_val_ptr=None):
    ws = Dev(L.mq_scan_workspace_bytes(n))
    out = Dev(32)
    hl, l, hh, h = mq.bounds(lo, hi)
    if fused_val_ptr is None:
        mq.check(L.mq_select_agg(dcol_ptr, n, hl, l, hh, h, out.ptr, ws.ptr, ws.nbytes, None))
    else:
        mq.check(L.mq_select_fetch_agg(dcol_ptr, fused_val_ptr, n, hl, l, hh, h, out.ptr, ws.ptr,
                                       ws.nbytes, None))
    return mq.MqAgg.from_buffer_copy(out.get(np.uint8, 32).tobytes())


def _positions(L, dcol_ptr, n, lo, hi, payload_ptr=None):
    ws = Dev(L.mq_scan_workspace_bytes(n))
    pos = Dev(max(n, 1) * 4)
    cnt = Dev(8)
    hl, l, hh, h = mq.bounds(lo, hi)
    mq.check(L.mq_select_positions(dcol_ptr, payload_ptr, n, hl, l, hh, h, pos.ptr, cnt.ptr, ws.ptr,
                                   ws.nbytes, None))
    k = int(cnt.get(np.uint64, 1)[0])
    return pos.get(np.int32, k)


def _data(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.integers(-25, 25, n, dtype=np.int32)
    if n > 8:
        d[1], d[2], d[n - 1] = I32MIN, I32MAX, I32MAX - 1
    return d


@pytest.mark.parametrize("n", SIZES)
def test_select_agg_and_positions_vs_oracle(lib, refcpu, n):
    d = _data(n, n)
    for off in (0, 1):  # 16-B aligned column and an unaligned (+4 B) one
        dd = Dev.of(d, offset_elems=off)
        for lo, hi in BOUNDS:
            want = refcpu.select_scan(d, lo, hi)
            got = _positions(lib, dd.ptr, n, lo, hi)
            assert np.array_equal(got, want), (n, off, lo, hi)
            a = _agg(lib, dd.ptr, n, lo, hi)
            vals = d[want]
            assert a.count == len(want), (n, off, lo, hi)
            assert a.sum == int(vals.astype(np.int64).sum()), (n, off, lo, hi)
            if len(vals):
                assert (a.min, a.max) == (int(vals.min()), int(vals.max()))
            else:
                assert (a.min, a.max) == (I32MAX, I32MIN)
            c, sm = _select_sum(lib, dd.ptr, n, lo, hi)
            assert (c, sm) == (a.count, a.sum), (n, off, lo, hi)


@pytest.mark.parametrize("out_off", [1, 2, 3])
def test_positions_into_unaligned_output(lib, refcpu, out_off):
    """The output pointer 4 / 8 / 12 B past a 16-byte boundary: the batched bitmap
    expansion (round 4) flushes its LDS ring as 16-byte stores placed by the output
    address, so a base that is not 16-byte aligned shifts every flush. Dense ranges
    (bitmap mode) and a sparse one, positions and the payload form."""
    n = 3_000_017
    d = _data(n, 77)
    pay = (np.arange(n, dtype=np.int64) * 7 - 5).astype(np.int32)
    dd, dp = Dev.of(d), Dev.of(pay)
    ws = Dev(lib.mq_scan_workspace_bytes(n))
    out = Dev((n + 8) * 4)
    cnt = Dev(8)
    for lo, hi in ((-25, 25), (-10, 10), (0, 0), (24, 24)):
        want = refcpu.select_scan(d, lo, hi)
        for payload in (None, dp.ptr):
            hl, l, hh, h = mq.bounds(lo, hi)
            mq.check(lib.mq_select_positions(dd.ptr, payload, n, hl, l, hh, h, out.ptr + 4 * out_off, cnt.ptr,
                                             ws.ptr, ws.nbytes, None))
            k = int(cnt.get(np.uint64, 1)[0])
            got = out.get(np.int32, k + out_off)[out_off:]
            assert k == len(want), (out_off, lo, hi, payload is not None)
            assert np.array_equal(got, pay[want] if payload else want), (out_off, lo, hi, payload is not None)


def _select_sum(L, dcol_ptr, n, lo, hi, ws=None, out=None):
    """mq_select_sum: one launch, partials folded by the last block to arrive."""
    ws = ws or Dev(L.mq_scan_workspace_bytes(n))
    out = out or Dev(32)
    hl, l, hh, h = mq.bounds(lo, hi)
    mq.check(L.mq_select_sum(dcol_ptr, n, hl, l, hh, h, out.ptr, ws.ptr, ws.nbytes, None))
    a = mq.MqAgg.from_buffer_copy(out.get(np.uint8, 32).tobytes())
    return a.count, a.sum


def test_select_sum_in_kernel_combine_repeated(lib, refcpu):
    """The arrival counters reset themselves: many back-to-back launches (every
    slot is reused several times), grids from 1 block to a full wave, and
    launches queued without a host sync in between, each matching the oracle."""
    sizes = [1, 1024 * 3, 1024 * 7 + 5, 1024 * 9, 1 << 16, 1 << 20, 3_000_001, 12_345_678]
    data = {n: _data(n, 1000 + n) for n in sizes}
    devs = {n: Dev.of(d) for n, d in data.items()}
    want = {}
    for n, d in data.items():
        v = d[refcpu.select_scan(d, -5, 5)]
        want[n] = (len(v), int(v.astype(np.int64).sum()))
    for rep in range(20):
        for n in sizes:
            assert _select_sum(lib, devs[n].ptr, n, -5, 5) == want[n], (rep, n)
    # queued: 80 launches into separate outputs, one sync at the end
    ws = [Dev(lib.mq_scan_workspace_bytes(n)) for n in sizes]
    outs = [[Dev(32) for _ in sizes] for _ in range(10)]
    hl, l, hh, h = mq.bounds(-5, 5)
    for r in range(10):
        for i, n in enumerate(sizes):
            mq.check(lib.mq_select_sum(devs[n].ptr, n, hl, l, hh, h, outs[r][i].ptr, ws[i].ptr,
                                       ws[i].nbytes, None))
    for r in range(10):
        for i, n in enumerate(sizes):
            a = mq.MqAgg.from_buffer_copy(outs[r][i].get(np.uint8, 32).tobytes())
            assert (a.count, a.sum) == want[n], (r, n)


def test_select_sum_in_kernel_combine_32_streams(lib, refcpu):
    """the in-kernel combine's arrival counters belong to the
    launch's stream, so launches in flight on many streams at once never share them
    (a pool of 16 slots handed out in rotation did). 32 streams, each with its own
    workspace, queue 6 mq_select_sum launches back to back and alternate with the
    fused fetch + aggregate (mq_select_fetch_agg, the other in-kernel combine); no
    host sync until every launch is queued; every result equals the oracle."""
    nstreams, reps = 32, 6
    sizes = [1024 * 5 + 3, 1 << 18, 1_000_003, 4_000_037]
    data = {n: _data(n, 2000 + n) for n in sizes}
    aux = {n: _data(n, 3000 + n) for n in sizes}
    devs = {n: Dev.of(d) for n, d in data.items()}
    dauxs = {n: Dev.of(a) for n, a in aux.items()}
    want, want_aux = {}, {}
    for n, d in data.items():
        p = refcpu.select_scan(d, -5, 5)
        want[n] = (len(p), int(d[p].astype(np.int64).sum()))
        a = aux[n][p]
        want_aux[n] = (len(a), int(a.astype(np.int64).sum()), int(a.min()), int(a.max()))
    streams = []
    for _ in range(nstreams):
        sp = C.c_void_p()
        mq.check(lib.mq_stream_create(C.byref(sp)))
        streams.append(sp.value)
    big = max(sizes)
    ws = [Dev(lib.mq_scan_workspace_bytes(big)) for _ in range(nstreams)]
    outs = [[Dev(32) for _ in range(reps)] for _ in range(nstreams)]
    hl, l, hh, h = mq.bounds(-5, 5)
    plan = []
    for r in range(reps):
        for s in range(nstreams):
            n = sizes[(s + r) % len(sizes)]
            fused = (s + r) % 3 == 0
            if fused:
                mq.check(lib.mq_select_fetch_agg(devs[n].ptr, dauxs[n].ptr, n, hl, l, hh, h,
                                                 outs[s][r].ptr, ws[s].ptr, ws[s].nbytes, streams[s]))
            else:
                mq.check(lib.mq_select_sum(devs[n].ptr, n, hl, l, hh, h, outs[s][r].ptr,
                                           ws[s].ptr, ws[s].nbytes, streams[s]))
            plan.append((s, r, n, fused))
    for sp in streams:
        mq.check(lib.mq_stream_sync(sp))
    for s, r, n, fused in plan:
        a = mq.MqAgg.from_buffer_copy(outs[s][r].get(np.uint8, 32).tobytes())
        if fused:
            assert (a.count, a.sum, a.min, a.max) == want_aux[n], (s, r, n)
        else:
            assert (a.count, a.sum) == want[n], (s, r, n)
    for sp in streams:
        mq.check(lib.mq_stream_destroy(sp))


@pytest.mark.parametrize("n", [0, 7, 4097, 200_003, 3_000_017])
def test_select_result_payload_vs_oracle(lib, refcpu, n):
    rng = np.random.default_rng(n + 1)
    vals = rng.integers(-100, 100, n, dtype=np.int32)
    prev = np.sort(rng.choice(10 ** 7, n, replace=False)).astype(np.int32)
    dv, dp = Dev.of(vals), Dev.of(prev)
    for lo, hi in BOUNDS:
        assert np.array_equal(_positions(lib, dv.ptr, n, lo, hi, dp.ptr),
                              refcpu.select_result(vals, prev, lo, hi)), (n, lo, hi)


def test_positions_stage_repeated_queued(lib, refcpu):
    """k_select_stage: waves switch from the LDS buffer to bitmap mode at different
    points (selectivities from 0.1 % to 100 %); blocks combine counts across the
    grid at the end. Every launch (three queued back to back, one sync) must
    equal the oracle's list word for word."""
    n = 20_000_003
    rng = np.random.default_rng(77)
    d = rng.integers(0, 1000, n, dtype=np.int32)
    dd = Dev.of(d)
    cases = [(0, 1), (0, 10), (0, 250), (100, 600), (0, 999), (0, 1000), (500, 501)]
    want = {c: refcpu.select_scan(d, *c) for c in cases}
    ws = Dev(lib.mq_scan_workspace_bytes(n))
    outs = [Dev(n * 4) for _ in range(3)]
    cnts = [Dev(8) for _ in range(3)]
    for rep in range(3):
        for lo, hi in cases:
            hl, l, hh, h = mq.bounds(lo, hi)
            for i in range(3):  # three launches queued, one sync
                mq.check(lib.mq_select_positions(dd.ptr, None, n, hl, l, hh, h, outs[i].ptr,
                                                 cnts[i].ptr, ws.ptr, ws.nbytes, None))
            for i in range(3):
                k = int(cnts[i].get(np.uint64, 1)[0])
                assert k == len(want[(lo, hi)]), (rep, lo, hi, i)
                assert np.array_equal(outs[i].get(np.int32, k), want[(lo, hi)]), (rep, lo, hi, i)


@pytest.mark.parametrize("k", [0, 1, 5, 4096, 100_003])
def test_fetch_vs_oracle(lib, refcpu, k):
    rng = np.random.default_rng(k)
    col = rng.integers(I32MIN, I32MAX, 500_000, dtype=np.int32)
    pos = np.sort(rng.integers(0, len(col), k)).astype(np.int32)
    dc, dpos, out = Dev.of(col), Dev.of(pos), Dev(max(k, 1) * 4)
    mq.check(lib.mq_fetch(dc.ptr, dpos.ptr, k, out.ptr, None))
    assert np.array_equal(out.get(np.int32, k), refcpu.fetch(col, pos))
    # unaligned positions / output pointers take the scalar path
    if k > 1:
        dpos2 = Dev.of(pos, offset_elems=1)
        out2 = Dev(k * 4 + 8)
        mq.check(lib.mq_fetch(dc.ptr, dpos2.ptr, k, out2.ptr + 4, None))
        assert np.array_equal(out2.get(np.int32, k, byte_offset=4), refcpu.fetch(col, pos))


@pytest.mark.parametrize("n", [0, 1, 3, 4, 1001, 1 << 18])
def test_add_sub_vs_oracle(lib, refcpu, n):
    rng = np.random.default_rng(n)
    a = rng.integers(I32MIN, I32MAX, n, dtype=np.int32)
    b = rng.integers(I32MIN, I32MAX, n, dtype=np.int32)
    da, db, out = Dev.of(a), Dev.of(b), Dev(max(n, 1) * 4)
    mq.check(lib.mq_add(da.ptr, db.ptr, n, out.ptr, None))
    assert np.array_equal(out.get(np.int32, n), refcpu.add(a, b))
    mq.check(lib.mq_sub(da.ptr, db.ptr, n, out.ptr, None))
    assert np.array_equal(out.get(np.int32, n), refcpu.sub(a, b))


def test_fused_select_fetch_agg_vs_oracle(lib, refcpu):
    """config 3 fused (k_scan_gather); dense selections overflow the per-wave LDS buffer
    many times."""
    for n in (1, 1023, 4099, 2_000_003):
        d0, d1 = refcpu.gen_uniform(n, 42), refcpu.gen_uniform(n, 43)
        d1[: min(n, 3)] = [I32MIN, I32MAX, -1][: min(n, 3)]
        for off in (0, 1):
            D0, D1 = Dev.of(d0, offset_elems=off), Dev.of(d1, offset_elems=off)
            for lo, hi in ((n // 4, n // 4 + n // 100 + 1), (None, n // 2), (0, None), (5, 5),
                           (None, None)):
                pos = refcpu.select_scan(d0, lo, hi)
                vals = d1[pos]
                a = _agg(lib, D0.ptr, n, lo, hi, fused_val_ptr=D1.ptr)
                assert a.count == len(pos) and a.sum == int(vals.astype(np.int64).sum()), (n, lo, hi)
                if len(vals):
                    assert (a.min, a.max) == (int(vals.min()), int(vals.max())), (n, lo, hi)
                else:
                    assert (a.min, a.max) == (I32MAX, I32MIN)


def test_generators_match_oracle(lib, refcpu):
    n = 1 << 20
    out = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(out.ptr, n, 42, n, None))
    assert np.array_equal(out.get(np.int32, n), refcpu.gen_uniform(n, 42))
    for kind, name in ((0, "build"), (1, "probe")):
        mq.check(lib.mq_gen_join_keys(out.ptr, n, kind, None))
        assert np.array_equal(out.get(np.int32, n), refcpu.gen_join(n, name))
    mq.check(lib.mq_gen_iota(out.ptr, n, None))
    assert np.array_equal(out.get(np.int32, n), np.arange(n, dtype=np.int32))


def test_golden_fixture_64k(lib):
    d = np.fromfile(os.path.join(GOLD, "col_n65536_s42.bin"), dtype=np.int32)
    dd = Dev.of(d)
    for sel in (0.01, 0.5, 1.0):
        want = np.fromfile(os.path.join(GOLD, f"pos_n65536_s42_sel{sel}.bin"), dtype=np.int32)
        lo = int(0.25 * 65536)
        assert np.array_equal(_positions(lib, dd.ptr, 65536, lo, lo + int(sel * 65536)), want)


def _device_chain(lib, refcpu, n, seed, lo, hi, fetch_seed=None):
    """select_column_scan -> fetch_column -> reduce, all on the device."""
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, seed, n, None))
    ws = Dev(lib.mq_scan_workspace_bytes(n))
    pos, cnt = Dev(n * 4), Dev(8)
    mq.check(lib.mq_select_positions(col.ptr, None, n, 1, lo, 1, hi, pos.ptr, cnt.ptr, ws.ptr,
                                     ws.nbytes, None))
    k = int(cnt.get(np.uint64, 1)[0])
    src = col
    if fetch_seed is not None:
        src = Dev(n * 4)
        mq.check(lib.mq_gen_uniform(src.ptr, n, fetch_seed, n, None))
    vals = Dev(max(k, 1) * 4)
    mq.check(lib.mq_fetch(src.ptr, pos.ptr, k, vals.ptr, None))
    out = Dev(32)
    mq.check(lib.mq_reduce(vals.ptr, k, out.ptr, ws.ptr, ws.nbytes, None))
    a = mq.MqAgg.from_buffer_copy(out.get(np.uint8, 32).tobytes())
    fnv = refcpu.fnv1a64(pos.get(np.int32, k))
    # fused paths must agree with the chain
    fa = _agg(lib, col.ptr, n, lo, hi, None if fetch_seed is None else src.ptr)
    assert (fa.count, fa.sum, fa.min, fa.max) == (k, a.sum, a.min, a.max)
    return k, fnv, a


def _check_row(r, k, fnv, a):
    assert k == r["k"]
    if "pos_fnv1a64" in r:
        assert f"{fnv:016x}" == r["pos_fnv1a64"]
    assert a.sum == r["sum"] and a.min == r["min"] and a.max == r["max"]
    assert f"{dbits(a.sum / k):016x}" == r["avg_bits"]  # query.c:314, one double division


def test_goldens_10m(lib, refcpu, goldens):
    for r in goldens["select"]:
        if r["n"] == 10_000_000:
            _check_row(r, *_device_chain(lib, refcpu, r["n"], r["seed"], r["low"], r["high"]))
    for r in goldens["config3"]:
        if r["n"] == 10_000_000:
            _check_row(r, *_device_chain(lib, refcpu, r["n"], r["seed"], r["low"], r["high"],
                                         fetch_seed=r["fetch_seed"]))
    n = 10_000_000
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, 42, n, None))
    a = _agg(lib, col.ptr, n, None, None)
    assert a.sum == goldens["column_sum"][str(n)]


@pytest.mark.big
def test_goldens_1e9(lib, refcpu, goldens):
    for r in goldens["select"]:
        if r["n"] == 1_000_000_000:
            _check_row(r, *_device_chain(lib, refcpu, r["n"], r["seed"], r["low"], r["high"]))
    for r in goldens["config3"]:
        if r["n"] == 1_000_000_000:
            _check_row(r, *_device_chain(lib, refcpu, r["n"], r["seed"], r["low"], r["high"],
                                         fetch_seed=r["fetch_seed"]))


@pytest.mark.big
def test_config4_per_seed_and_combined_1e9(lib, goldens):
    n = 1_000_000_000
    col = Dev(n * 4)
    tk = ts = 0
    for r in goldens["config4"]:
        mq.check(lib.mq_gen_uniform(col.ptr, n, r["seed"], n, None))
        a = _agg(lib, col.ptr, n, r["low"], r["high"])
        assert (a.count, a.sum) == (r["k"], r["sum"]), r["seed"]
        tk += a.count
        ts += a.sum
    c = goldens["config4_combined"]
    assert (tk, ts) == (c["k"], c["sum"])


@pytest.mark.big
def test_full_size_properties_1e9(lib):
    """Size-independent checks at BASELINE's N: range additivity of count and sum,
    strictly ascending positions, every fetched value inside the range."""
    n = 1_000_000_000
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, 42, n, None))
    whole = _agg(lib, col.ptr, n, 100_000_000, 900_000_000)
    left = _agg(lib, col.ptr, n, 100_000_000, 400_000_000)
    right = _agg(lib, col.ptr, n, 400_000_000, 900_000_000)
    assert whole.count == left.count + right.count and whole.sum == left.sum + right.sum
    everything = _agg(lib, col.ptr, n, None, None)
    assert everything.count == n and everything.min >= 0 and everything.max < n
    lo, hi = 123_456_789, 133_456_789
    pos = _positions(lib, col.ptr, n, lo, hi)
    assert len(pos) == _agg(lib, col.ptr, n, lo, hi).count
    assert np.all(np.diff(pos.astype(np.int64)) > 0)
    dp, vals = Dev.of(pos), Dev(len(pos) * 4)
    mq.check(lib.mq_fetch(col.ptr, dp.ptr, len(pos), vals.ptr, None))
    v = vals.get(np.int32, len(pos))
    assert v.min() >= lo and v.max() < hi


def _check_positions_exact(lib, col, n, lo, hi, pos):
    """count == the fused count, strictly ascending, every row's value in range:
    together these say pos is exactly the reference's list (query.c:100-104)."""
    assert len(pos) == _agg(lib, col.ptr, n, lo, hi).count, (lo, hi)
    if len(pos) == 0:
        return
    assert np.all(np.diff(pos.astype(np.int64)) > 0), (lo, hi)
    assert pos[0] >= 0 and pos[-1] < n
    dp, vals = Dev.of(pos), Dev(len(pos) * 4)
    mq.check(lib.mq_fetch(col.ptr, dp.ptr, len(pos), vals.ptr, None))
    v = vals.get(np.int32, len(pos))
    assert v.min() >= lo and v.max() < hi, (lo, hi)


@pytest.mark.big
def test_positions_spill_boundary_1e9(lib):
    """k_select_stage's three regimes at full size: LDS ring only, ring + spill to
    the workspace (density below 1/32 with more than 1024 matches per wave), and
    the switch to bitmap mode (past 1/32), on a uniform column and on a bursty one
    (4096 equal rows per value, so a wave's matches arrive in dense runs)."""
    n = 1_000_000_000
    col = Dev(n * 4)
    mq.check(lib.mq_gen_uniform(col.ptr, n, 42, n, None))
    for sel in (0.005, 0.02, 0.03, 0.0325, 0.04):
        lo = n // 3
        hi = lo + int(sel * n)
        _check_positions_exact(lib, col, n, lo, hi, _positions(lib, col.ptr, n, lo, hi))
    bursty = (np.arange(n, dtype=np.int32) // 4096) % 1000
    col = Dev.of(bursty)
    del bursty
    for lo, hi in ((0, 3), (0, 30), (500, 532), (0, 40)):
        _check_positions_exact(lib, col, n, lo, hi, _positions(lib, col.ptr, n, lo, hi))


# ---------------------------------------------------------------------------
# the drop-in query API (mq_query.c) against the reference's own query.c
# ---------------------------------------------------------------------------
needs_ref = pytest.mark.skipif(not os.path.exists(os.path.join(
    os.path.dirname(HERE), "oracle", "_ref", "libref.so")), reason="oracle/_ref not built")


@needs_ref
@pytest.mark.parametrize("n", [5, 1025, 100_000])
def test_query_api_vs_reference(lib, refcpu, n):
    ref, mine = Api(refcpu.reference()), Api(lib)
    d = _data(n, 7 * n)
    col = make_column(d)
    for lo, hi in BOUNDS:
        p_ref, p_mine = ref.select_column(col, lo, hi), mine.select_column(col, lo, hi)
        assert np.array_equal(p_ref, p_mine), (n, lo, hi)
        if not len(p_ref):
            continue
        v_ref, v_mine = ref.fetch_column(col, p_ref), mine.fetch_column(col, p_mine)
        assert np.array_equal(v_ref, v_mine)
        assert ref.sum_result(v_ref) == mine.sum_result(v_mine)
        assert dbits(ref.average(v_ref)) == dbits(mine.average(v_mine))
        assert ref.min(v_ref) == mine.min(v_mine) and ref.max(v_ref) == mine.max(v_mine)
        assert np.array_equal(ref.select_result(v_ref, p_ref, -3, 3),
                              mine.select_result(v_mine, p_mine, -3, 3))
        assert np.array_equal(ref.add(v_ref, v_ref), mine.add(v_mine, v_mine))
        assert np.array_equal(ref.sub(v_ref, p_ref), mine.sub(v_mine, p_mine))
    assert ref.sum_column(col) == mine.sum_column(col)


@needs_ref
@pytest.mark.parametrize("segs", [2, 3, 7, 64])
@pytest.mark.parametrize("n", [5, 1025, 100_000, 3_000_017])
def test_query_api_select_pipelined_vs_reference(lib, refcpu, monkeypatch, n, segs):
    """select_column's pipelined path (mq_select_positions_download: row segments, each
    downloaded while the next ones scan, into a payload over-allocated for n rows and
    shrunk to K) forced on small columns (MQ_SELECT_PIPE_MIN), including segments with
    no rows (n < 1024 * segs) and the bound matrix; then fetch / sum / select_result on
    its shadow, all equal to the reference build."""
    monkeypatch.setenv("MQ_SELECT_PIPE_MIN", "1")
    monkeypatch.setenv("MQ_SELECT_SEGS", str(segs))
    ref, mine = Api(refcpu.reference()), Api(lib)
    d = _data(n, 11 * n + segs)
    col = make_column(d)
    for lo, hi in BOUNDS:
        p_ref, p_mine = ref.select_column(col, lo, hi), mine.select_column(col, lo, hi)
        assert np.array_equal(p_ref, p_mine), (n, segs, lo, hi)
        if not len(p_ref):
            continue
        v_ref, v_mine = ref.fetch_column(col, p_ref), mine.fetch_column(col, p_mine)
        assert np.array_equal(v_ref, v_mine)
        assert ref.sum_result(v_ref) == mine.sum_result(v_mine)
        assert np.array_equal(ref.select_result(v_ref, p_ref, -3, 3),
                              mine.select_result(v_mine, p_mine, -3, 3))


def test_query_api_select_pipelined_large(lib, refcpu):
    """The default pipelined select (4 segments from 2^26 rows) on 2^26 + 4097 rows at
    0.1 %, 1 %, 30 % and 100 %: positions equal the oracle's; the fetch that follows
    reads the shadow (no result upload)."""
    n = (1 << 26) + 4097
    d = refcpu.gen_uniform(n, 42, n)
    col = make_column(d)
    api = Api(lib)
    for sel in (0.001, 0.01, 0.3, 1.0):
        lo = n // 5
        hi = lo + int(sel * n) if sel < 1 else n
        if sel == 1.0:
            lo = 0
        p = api.select_column(col, lo, hi)
        want = refcpu.select_scan(d, lo, hi)
        assert np.array_equal(p, want), sel
    up0 = mq.residency(lib)["result_uploads"]
    s = mq.Status(0, None)
    lo_c, hi_c = C.pointer(C.c_int(n // 5)), C.pointer(C.c_int(n // 5 + n // 100))
    r = lib.select_column(C.byref(col), lo_c, hi_c, C.byref(s))
    f = lib.fetch_column(C.byref(col), r, C.byref(s))
    assert s.code == mq.OK
    assert mq.residency(lib)["result_uploads"] == up0
    pos = take(r)
    assert np.array_equal(take(f), d[pos])


@needs_ref
def test_query_api_shared_select_vs_reference(lib, refcpu):
    ref, mine = Api(refcpu.reference()), Api(lib)
    n = 50_000
    d = refcpu.gen_uniform(n, 5, modulus=n)
    col = make_column(d)
    rng = np.random.default_rng(2)
    lows = rng.integers(0, n, 25).astype(np.int32)
    highs = (lows + rng.integers(0, n // 4, 25)).astype(np.int32)
    for a, b in zip(ref.shared_select(col, lows, highs), mine.shared_select(col, lows, highs)):
        assert np.array_equal(a, b)


@needs_ref
def test_query_api_sorted_index_vs_reference(lib, refcpu):
    """select_column on an indexed column takes the sorted-index path (query.c:165-220)."""
    ref, mine = Api(refcpu.reference()), Api(lib)
    rng = np.random.default_rng(4)
    d = rng.integers(0, 500, 20_000, dtype=np.int32)
    order = np.argsort(d, kind="stable")
    values = np.ascontiguousarray(d[order])
    positions = np.ascontiguousarray(order.astype(np.uint64))
    ix = mq.ColumnIndex()
    ix.values = values.ctypes.data_as(C.POINTER(C.c_int))
    ix.positions = positions.ctypes.data_as(C.POINTER(C.c_size_t))
    col = make_column(d)
    col.has_index = True
    col.index = C.pointer(ix)
    # low >= values[0] (the reference reads out of bounds below that)
    for lo, hi in ((0, 10), (3, 3), (7, 2), (100, 499), (250, 251), (0, 1000), (499, 600)):
        assert np.array_equal(ref.select_column(col, lo, hi), mine.select_column(col, lo, hi)), \
            (lo, hi)


@needs_ref
@pytest.mark.parametrize("kind", ["hash", "nested"])
def test_query_api_join_vs_reference(lib, refcpu, kind):
    ref, mine = Api(refcpu.reference()), Api(lib)
    rng = np.random.default_rng(11)
    for n1, n2, kr in ((4, 9, 3), (100, 257, 10), (3000, 2000, 50), (513, 4000, 5)):
        c1 = rng.integers(0, kr, n1, dtype=np.int32)
        c2 = rng.integers(0, kr, n2, dtype=np.int32)
        p1 = rng.integers(0, 10 ** 6, n1, dtype=np.int32)
        p2 = rng.integers(0, 10 ** 6, n2, dtype=np.int32)
        w1, w2 = ref.join(c1, p1, c2, p2, kind)
        g1, g2 = mine.join(c1, p1, c2, p2, kind)
        assert np.array_equal(g1, w1) and np.array_equal(g2, w2), (kind, n1, n2, kr)


def test_query_api_print_and_empty(lib):
    mine = Api(lib)
    assert mine.print([(np.array([3, -7, 12], np.int32), mq.INT),
                       (np.array([1234567890123], np.int64), mq.LONG),
                       (np.array([2.0 / 3.0], np.float64), mq.DOUBLE)]) == "3\n-7\n12,1234567890123,0.67"
    assert mine.print([(np.array([], np.int32), mq.INT)]) == ""
    col = make_column(np.arange(100, dtype=np.int32))
    assert len(mine.select_column(col, 500, 600)) == 0


def _int_edge_values(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.integers(I32MIN, I32MAX, n, dtype=np.int64, endpoint=True).astype(np.int32)
    edge = [I32MIN, I32MAX, 0, -1, 1, 9, 10, -9, -10, 99, 100, 999999999, 1000000000, -1000000000]
    v[:min(n, len(edge))] = edge[:min(n, len(edge))]
    v[len(edge):len(edge) + n // 4] = rng.integers(-1000, 1000, max(0, min(n // 4, n - len(edge))))
    return v


@pytest.mark.parametrize("n", [0, 1, 2, 15, 100_003, 1 << 20])
def test_format_int32_vs_printf(lib, n):
    v = _int_edge_values(n, n)
    d = Dev.of(v)
    out = Dev(max(12 * n, 1))
    ws = Dev(max(lib.mq_format_workspace_bytes(n), 1))
    ln = C.c_uint64()
    mq.check(lib.mq_format_int32(d.ptr, n, out.ptr, C.byref(ln), ws.ptr, ws.nbytes, None))
    want = "\n".join("%d" % x for x in v.tolist()).encode()
    assert ln.value == len(want)
    assert out.get(np.uint8, ln.value).tobytes() == want if n else ln.value == 0


@needs_ref
def test_query_api_print_large_vs_reference(lib, refcpu):
    """GPU formatting of big INT results (>= 32768 tuples) next to host-formatted
    LONG / DOUBLE / small INT results: the same bytes as the reference's print."""
    ref, mine = Api(refcpu.reference()), Api(lib)
    parts = [(_int_edge_values(100_003, 1), mq.INT),
             (np.array([1234567890123, -5], np.int64), mq.LONG),
             (np.array([2.0 / 3.0, -1.005], np.float64), mq.DOUBLE),
             (np.array([7, -8], np.int32), mq.INT),
             (_int_edge_values(40_000, 2), mq.INT)]
    assert mine.print(parts) == ref.print(parts)


# ---------------------------------------------------------------------------
# J1 hash join (device API) vs the oracle and the reference goldens
# ---------------------------------------------------------------------------
def _dev_join(lib, c1, p1, c2, p2):
    n1, n2 = len(c1), len(c2)
    D = [Dev.of(x) for x in (c1, p1, c2, p2)]
    h = C.c_void_p()
    mq.check(lib.mq_join_build(D[0].ptr, D[1].ptr, n1, C.byref(h), None), "join_build")
    m = C.c_uint64()
    mq.check(lib.mq_join_probe(h, D[2].ptr, n2, C.byref(m), None), "join_probe")
    m = m.value
    o1, o2 = Dev(max(m, 1) * 4), Dev(max(m, 1) * 4)
    mq.check(lib.mq_join_write(h, D[3].ptr, o1.ptr, o2.ptr, None), "join_write")
    mq.check(lib.mq_join_free(h), "join_free")
    return o1.get(np.int32, m), o2.get(np.int32, m)


JOIN_PATHS = {"winruns": {}, "sorted": {"MQ_JOIN_WINRUNS": "0"},
              "cas": {"MQ_JOIN_RUNS": "0"},
              # the windowed runs table probed by random bucket reads / window by window in LDS
              # (round 5: the default from 2^20 build rows, forced here from 2^16)
              "winruns_table": {"MQ_JOIN_PART": "0"},
              "winruns_part": {"MQ_JOIN_PART_MIN": "65536", "MQ_JOIN_PART_DIV": "1000000"},
              # ... with the short runs' build positions carried to the write (run2, the
              # default) or only the packed runs (MQ_JOIN_RUN2=0: the write reads the runs)
              "winruns_part_packed": {"MQ_JOIN_PART_MIN": "65536", "MQ_JOIN_PART_DIV": "1000000",
                                      "MQ_JOIN_RUN2": "0"}}


@pytest.mark.parametrize("path", list(JOIN_PATHS))
@pytest.mark.parametrize("case", ["unique", "dups", "skew", "neg", "tiny", "empty", "marker",
                                  "unique_partitioned", "dups_partitioned",
                                  "ragged_hits", "dups_short_runs", "dups_run_of_15"])
def test_hash_join_vs_oracle(lib, refcpu, monkeypatch, case, path):
    """Duplicate keys: winruns (default) partitions the build rows by window and finds
    each window's runs in LDS (k_win_build_runs); a window over 6144 rows or 3072 keys,
    or a key on 15+ rows, falls back to: sorted,
    the sorted runs behind the windowed table of distinct keys (MQ_JOIN_WINRUNS=0);
    cas: the global-CAS table of run heads (MQ_JOIN_RUNS=0, the last fallback)."""
    for k, v in JOIN_PATHS[path].items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(hash(case) % 1000)
    if case == "unique":
        c1 = rng.permutation(200_000).astype(np.int32)
        c2 = rng.integers(0, 400_000, 150_000, dtype=np.int32)
    elif case == "dups":
        c1 = rng.integers(0, 5000, 100_000, dtype=np.int32)
        c2 = rng.integers(0, 6000, 30_000, dtype=np.int32)
    elif case == "skew":  # one huge group plus a long tail
        c1 = np.where(rng.random(50_000) < 0.5, 7, rng.integers(0, 10 ** 6, 50_000)).astype(np.int32)
        c2 = np.concatenate([[7, 7, 3], rng.integers(0, 10 ** 6, 2000)]).astype(np.int32)
    elif case == "neg":
        c1 = rng.integers(-(2 ** 31), 2 ** 31 - 1, 20_000, dtype=np.int64).astype(np.int32)
        c1[:4] = [-(2 ** 31), 2 ** 31 - 1, 0, -1]
        c2 = np.concatenate([c1[::3], rng.integers(-100, 100, 500)]).astype(np.int32)
    elif case == "tiny":  # the reference's full-table hang shapes (multimap.c:65-71)
        c1 = np.array([5, 9], dtype=np.int32)
        c2 = np.array([1, 9, 5, 5, 2], dtype=np.int32)
    elif case == "marker":  # unique keys, one build row {key -1, position -1} = the
        c1 = (rng.permutation(3000) - 1500).astype(np.int32)  # packed table's empty word
        c2 = rng.integers(-1600, 1600, 5000, dtype=np.int32)
    elif case == "ragged_hits":  # unique keys, probe rows 64k+1 with hits at the word edges
        c1 = rng.permutation(1000).astype(np.int32)
        c2 = np.concatenate([np.arange(129), rng.integers(500, 2000, 64 * 7 + 1), [999]]).astype(np.int32)
    elif case == "dups_short_runs":  # > 2^16 rows, runs of 1..14 rows in input order
        # (spread keys: the oracle's `key % size` multimap goes quadratic on dense ones)
        keys = rng.choice(1 << 30, 90_000, replace=False).astype(np.int32)
        c1 = np.repeat(keys[:60_000], rng.integers(1, 15, 60_000))[:300_000]
        c1 = c1[rng.permutation(len(c1))]
        c2 = np.concatenate([rng.choice(keys[:60_000], 100_000), keys[60_000:80_000]]).astype(np.int32)
    elif case == "dups_run_of_15":  # one key on 15 rows: not packable, the window flags
        keys = rng.choice(1 << 30, 250_000, replace=False).astype(np.int32)
        c1 = keys[:200_000].copy()
        c1[1 + rng.choice(len(c1) - 1, 14, replace=False)] = c1[0]
        c2 = rng.choice(keys, 100_000)
        c2[:5] = c1[0]
    elif case in ("unique_partitioned", "dups_partitioned"):
        # > 2^22 build rows: the window-partitioned insert. Keys from the spread
        # config-5 generator: the oracle restates the reference's `key % size`
        # multimap, which goes quadratic on dense or arithmetic key runs.
        c1 = rng.permutation(refcpu.gen_join(5_000_000, "build"))
        c2 = refcpu.gen_join(3_000_000, "probe")
        if case == "dups_partitioned":  # one duplicate, seen only after partitioning
            c1[4_999_999] = c1[17]
    else:
        c1 = np.array([], dtype=np.int32)
        c2 = np.array([1, 2], dtype=np.int32)
    p1 = rng.integers(0, 10 ** 7, len(c1), dtype=np.int32)
    p2 = rng.integers(0, 10 ** 7, len(c2), dtype=np.int32)
    if case == "marker":
        p1[np.nonzero(c1 == -1)[0][0]] = -1
    g1, g2 = _dev_join(lib, c1, p1, c2, p2)
    w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2), case
    if len(c2) and len(c1):  # swapped roles (nested_loop_join's build side)
        h1, h2 = _dev_join(lib, c2, p2, c1, p1)
        if len(c1) * len(c2) <= 10 ** 10:  # the oracle's nested loop is O(n1 * n2)
            v1, v2 = refcpu.hash_join(c1, p1, c2, p2, nested=True)
            assert np.array_equal(h2, v1) and np.array_equal(h1, v2), case
        else:  # nested == swapped hash join, pinned by the smaller cases above
            v2, v1 = refcpu.hash_join(c2, p2, c1, p1)
            assert np.array_equal(h2, v1) and np.array_equal(h1, v2), case


JOIN_PROBE_MODES = {"table": {"MQ_JOIN_PART": "0"},  # the global table + random bucket reads
                    "part": {"MQ_JOIN_PART_MIN": "65536", "MQ_JOIN_PART_DIV": "1000000"},
                    "part_wide": {"MQ_JOIN_PART_MIN": "65536", "MQ_JOIN_PART_DIV": "1000000", "MQ_JOIN_NARROW": "0"},
                    "part_materialized": {"MQ_JOIN_PART_MIN": "65536", "MQ_JOIN_PART_DIV": "1"}}


@pytest.mark.parametrize("mode", list(JOIN_PROBE_MODES))
@pytest.mark.parametrize("case", ["n2_1", "n2_63", "n2_65", "n2_4097", "all_miss", "all_hit_dup_probe",
                                  "negative_extremes", "one_pass", "two_passes", "marker", "dup_probed",
                                  "dup_unprobed", "overfull_window", "payload_extremes"])
def test_hash_join_partitioned_probe(lib, refcpu, monkeypatch, mode, case):
    """Unique builds (round 5): the probe keys partitioned by table window like the build
    rows, each window joined in LDS (k_win_join), the results taken back to probe order
    by the inverted passes (k_pwin_gather), as u32 payloads with a miss marker outside the
    payloads' range ("part_wide": MQ_JOIN_NARROW=0, u64 {payload, hit}, also what a build
    whose payloads hold both INT32 extremes takes); "part_materialized" makes the probe side too
    small for that (MQ_JOIN_PART_DIV), so the checked windows are stored as the global
    table first; "table" is the random-read probe. One LSD pass (build < 2^20 rows: at
    most 256 windows) and two (2^21 build rows: 512 windows, a second digit); a build row
    equal to the table's empty word sends the build to the duplicate paths. The build is
    not checked up front: a probe key that meets a duplicate build key, or a window of
    more than 6144 build rows, flags, and the join is built again without the partition
    (dup_probed, overfull_window); a duplicate no probe row meets leaves the output
    unchanged (dup_unprobed)."""
    monkeypatch.setenv("MQ_JOIN_SAMPLE", "0")  # (the sampled duplicate check would catch none here)
    for k, v in JOIN_PROBE_MODES[mode].items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(abs(hash((case, mode))) % 2 ** 32)
    n1 = (1 << 21) + 333 if case == "two_passes" else 200_003
    c1 = rng.permutation(refcpu.gen_join(n1, "build"))
    if case.startswith("n2_"):
        n2 = int(case[3:])
        c2 = np.concatenate([rng.choice(c1, n2 // 2), rng.integers(-2 ** 31, 2 ** 31 - 1, n2 - n2 // 2)])
        c2 = c2.astype(np.int64).astype(np.int32)[rng.permutation(n2)]
    elif case == "all_miss":
        c2 = refcpu.gen_join(n1 * 4, "build")[n1:n1 + 300_000]  # mix31 is a bijection: never built
        c1 = rng.permutation(refcpu.gen_join(n1 * 4, "build")[:n1])
    elif case == "all_hit_dup_probe":
        c2 = rng.choice(c1, 500_000)  # every probe row hits, keys repeat on the probe side
    elif case == "negative_extremes":
        c1 = (rng.choice(1 << 32, n1, replace=False).astype(np.int64) - 2 ** 31).astype(np.int32)
        c1[:2] = [-2 ** 31, 2 ** 31 - 1]
        c2 = np.concatenate([c1[::5], [-2 ** 31, 2 ** 31 - 1, 0, -1], rng.integers(-100, 100, 1000)]).astype(np.int32)
    elif case == "marker":  # {key -1, position -1} is the table's empty word
        c1 = (rng.permutation(n1) - n1 // 2).astype(np.int32)
        c2 = rng.integers(-n1, n1, 150_000).astype(np.int32)
    elif case in ("dup_probed", "dup_unprobed"):
        c1[n1 - 5] = c1[100]  # one key on two build rows
        c2 = rng.choice(c1, 300_000)
        c2 = np.where(c2 == c1[100], c1[7], c2) if case == "dup_unprobed" else c2
        c2 = np.concatenate([c2, [c1[100]]] if case == "dup_probed" else [c2]).astype(np.int32)
    elif case == "overfull_window":  # 7000 build keys homed in one 8192-slot window
        slots = 1 << 19  # 200_003 rows: 2^19 slots, 64 windows
        i = np.arange(7000, dtype=np.uint64)
        hw = (np.uint64(5) << np.uint64(13)) | (i & np.uint64(8191)) | ((i + np.uint64(1)) << np.uint64(19))
        crafted = _inv_fmix32(hw & np.uint64(0xFFFFFFFF))
        c1 = np.unique(np.concatenate([crafted, c1[:n1 - 7000]]))
        c1 = c1[rng.permutation(len(c1))]
        c2 = np.concatenate([rng.choice(c1, 100_000), crafted[:500]]).astype(np.int32)
    else:
        c2 = np.concatenate([rng.choice(c1, 700_000), refcpu.gen_join(1 << 20, "probe")]).astype(np.int32)
        c2 = c2[rng.permutation(len(c2))]
    p1 = rng.integers(-10 ** 7, 10 ** 7, len(c1), dtype=np.int32)
    p2 = rng.integers(0, 10 ** 7, len(c2), dtype=np.int32)
    if case == "marker":
        p1[np.nonzero(c1 == -1)[0][0]] = -1
    if case == "payload_extremes":  # no int32 is free to mark a miss: the u64 results
        p1[:2] = [-2 ** 31, 2 ** 31 - 1]
    if case == "two_passes":  # a payload of INT32_MAX: the miss marker becomes INT32_MIN
        p1[3] = 2 ** 31 - 1
    g1, g2 = _dev_join(lib, c1, p1, c2, p2)
    w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2), (case, mode)


def _inv_fmix32(h):
    """Inverse of libmq's table hash (the murmur3 finaliser, mq_join.hip hash32), so a
    test can pick the home slot of every key."""
    M = np.uint64(0xFFFFFFFF)
    x = h.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(pow(0xC2B2AE35, -1, 1 << 32))) & M
    x ^= (x >> np.uint64(13)) ^ (x >> np.uint64(26))
    x = (x * np.uint64(pow(0x85EBCA6B, -1, 1 << 32))) & M
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32).view(np.int32)


@pytest.mark.parametrize("probe", ["table", "part"])
@pytest.mark.parametrize("dup", [False, True])
def test_hash_join_clustered_window(lib, refcpu, monkeypatch, dup, probe):
    """One 8192-slot window of the unique table holds a 5000-slot cluster: 5000 keys
    homed in 16 buckets at its start, so probes of those keys (hits) and of other keys
    homed there (misses) follow chains of up to ~5000 slots through the per-wave
    continuation queue (requeued every step, then drained at the end; the in-step
    drain runs when more than 128 rows wait), past the full buckets' overflow marks.
    dup: every cluster key twice (the runs table behind the same windowed build).
    probe "part": the partitioned probe (unique builds), whose LDS lookups follow the
    same chains inside the window."""
    for k, v in JOIN_PROBE_MODES["part" if probe == "part" else "table"].items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(4242)
    n_rand, n_cl = 295_000, 5000
    slots = 1 << 20  # the table of ~300K build rows: 2^20 slots, 128 windows of 8192
    w0 = 7
    i = np.arange(n_cl, dtype=np.uint64)
    home = np.uint64(w0 * 8192) + np.uint64(4) * (i % np.uint64(16))
    h_cl = home | ((i // np.uint64(16)) << np.uint64(20))  # distinct, all homed in 16 buckets
    h_rand = rng.choice(1 << 32, size=3 * n_rand, replace=False).astype(np.uint64)
    h_rand = h_rand[((h_rand & np.uint64(slots - 1)) >> np.uint64(13)) != np.uint64(w0)][:n_rand]
    k_cl, k_rand = _inv_fmix32(h_cl), _inv_fmix32(h_rand)
    c1 = np.concatenate([k_rand, k_cl, k_cl if dup else k_cl[:0]])
    c1 = c1[rng.permutation(len(c1))]
    # probes: cluster hits, misses homed in the cluster's buckets, random hits and misses
    j = np.arange(3000, dtype=np.uint64)
    h_miss = (np.uint64(w0 * 8192) + np.uint64(4) * (j % np.uint64(16))) | ((np.uint64(400) + j) << np.uint64(20))
    c2 = np.concatenate([rng.choice(k_cl, 3000), _inv_fmix32(h_miss), rng.choice(k_rand, 100_000),
                         rng.integers(-2 ** 31, 2 ** 31 - 1, 50_000, dtype=np.int64).astype(np.int32)])
    c2 = c2[rng.permutation(len(c2))]
    p1 = rng.integers(0, 10 ** 7, len(c1), dtype=np.int32)
    p2 = rng.integers(0, 10 ** 7, len(c2), dtype=np.int32)
    g1, g2 = _dev_join(lib, c1, p1, c2, p2)
    w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
    assert len(w1) >= 3000 * (2 if dup else 1)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2)


def test_hash_join_scratch_reuse_and_trim(lib, refcpu):
    """Join scratch comes from libmq's caching pool: back-to-back joins of
    different sizes reuse (and outgrow) blocks, mq_trim() releases them, and every
    result still matches the oracle."""
    rng = np.random.default_rng(77)
    for rep, (n1, n2) in enumerate([(300_000, 200_000), (100_000, 400_000), (300_000, 200_000),
                                    (70_000, 5_000), (500_000, 100_000)]):
        c1 = rng.permutation(refcpu.gen_join(n1, "build"))
        c2 = refcpu.gen_join(n2, "probe")
        p1 = rng.integers(0, 10 ** 7, n1, dtype=np.int32)
        p2 = rng.integers(0, 10 ** 7, n2, dtype=np.int32)
        g1, g2 = _dev_join(lib, c1, p1, c2, p2)
        w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
        assert np.array_equal(g1, w1) and np.array_equal(g2, w2), rep
        if rep == 2:
            lib.mq_trim()


def _join_golden(lib, refcpu, n, dup=False, keep=False):
    D = {k: Dev(n * 4) for k in ("a", "b", "p")}
    mq.check(lib.mq_gen_join_keys(D["a"].ptr, n, 2 if dup else 0, None))
    mq.check(lib.mq_gen_join_keys(D["b"].ptr, n, 3 if dup else 1, None))
    mq.check(lib.mq_gen_iota(D["p"].ptr, n, None))
    h = C.c_void_p()
    mq.check(lib.mq_join_build(D["a"].ptr, D["p"].ptr, n, C.byref(h), None))
    m = C.c_uint64()
    mq.check(lib.mq_join_probe(h, D["b"].ptr, n, C.byref(m), None))
    m = m.value
    o1, o2 = Dev(m * 4), Dev(m * 4)
    mq.check(lib.mq_join_write(h, D["p"].ptr, o1.ptr, o2.ptr, None))
    mq.check(lib.mq_join_free(h))
    g1, g2 = o1.get(np.int32, m), o2.get(np.int32, m)
    if keep:
        return m, refcpu.fnv1a64_pairs(g1, g2), g1, g2
    return m, refcpu.fnv1a64_pairs(g1, g2)


def test_hash_join_goldens(lib, refcpu, goldens):
    rows = [r for r in goldens["join"] if "dup" not in r] + \
           [r for r in goldens["join_survey"] if r["n"] <= 1 << 24]
    for r in rows:
        m, h = _join_golden(lib, refcpu, r["n"])
        assert (m, f"{h:016x}") == (r["m"], r["pairs_fnv1a64"]), r["n"]


@pytest.mark.parametrize("path", list(JOIN_PATHS))
@pytest.mark.parametrize("sample", [True, False])
def test_hash_join_dup_goldens(lib, refcpu, goldens, monkeypatch, path, sample):
    """Many-to-many config 5 (every build key twice, tests/golden/make_join_dup_goldens.py):
    the duplicate-key build paths (JOIN_PATHS) against the reference's own hash_join.
    sample: builds of 2^20 rows and up go straight to the runs build when a sample of
    the keys has a duplicate; MQ_JOIN_SAMPLE=0: the unique attempt first, abandoned on
    the duplicate."""
    for k, v in JOIN_PATHS[path].items():
        monkeypatch.setenv(k, v)
    if not sample:
        monkeypatch.setenv("MQ_JOIN_SAMPLE", "0")
    for r in goldens["join_dup"]:
        m, h = _join_golden(lib, refcpu, r["n"], dup=True)
        assert (m, f"{h:016x}") == (r["m"], r["pairs_fnv1a64"]), r["n"]


@pytest.mark.big
def test_hash_join_dup_2e28_properties(lib, refcpu):
    """2^28 x 2^28 many-to-many (beyond the reference's reach): every pair joins equal
    keys, pairs are probe-major with build positions ascending inside a probe row (the
    multimap's insertion order, query.c:669-681), and M equals the number of
    (probe, build) key matches counted on the host."""
    n = 1 << 28
    m, _, o1, o2 = _join_golden(lib, refcpu, n, dup=True, keep=True)
    a, b = refcpu.gen_join(n, "build_dup"), refcpu.gen_join(n, "probe_dup")
    # the n/2 distinct build keys (mix31 is a bijection) each occur twice
    assert m == 2 * int(np.isin(b, a[: n // 2]).sum())
    assert np.array_equal(a[o1], b[o2])
    assert np.all(o2[1:] >= o2[:-1])
    same = o2[1:] == o2[:-1]
    assert np.all(o1[1:][same] > o1[:-1][same])


@pytest.mark.big
def test_hash_join_golden_2e28(lib, refcpu, goldens):
    r = [x for x in goldens["join_survey"] if x["n"] == 1 << 28][0]
    m, h = _join_golden(lib, refcpu, r["n"])
    assert (m, f"{h:016x}") == (r["m"], r["pairs_fnv1a64"])


# ---------------------------------------------------------------------------
# S11 shared_select (device API): Q predicates, two passes, exact-size outputs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("twopass", [False, True])
@pytest.mark.parametrize("n,q", [(0, 3), (1, 2), (5, 1), (4099, 7), (100_003, 150), (1 << 20, 256),
                                 (3_000_017, 20), (2_000_003, 2), (2_000_003, 5),
                                 # round-5 boundaries: 3 -> 4 count blocks a CU (Q 8 / 9),
                                 # output pointers as scatter arguments (Q 32 / 33)
                                 (1_000_003, 8), (1_000_003, 9), (1_000_003, 32), (1_000_003, 33)])
def test_shared_select_vs_oracle(lib, refcpu, monkeypatch, n, q, twopass):
    """Every Q takes the elementary-interval kernels: the single pass (pairs listed by the
    count pass, k_ssp_scatter), or the column pass (MQ_SS_TWOPASS=1 forces it; a pair-slice
    overflow takes it)."""
    if twopass:
        monkeypatch.setenv("MQ_SS_TWOPASS", "1")
    rng = np.random.default_rng(n + q)
    d = rng.integers(-1000, 1000, n, dtype=np.int32)
    if n > 8:
        d[:3] = [I32MIN, I32MAX, 0]
    lows = rng.integers(-1100, 1000, q).astype(np.int32)
    highs = (lows + rng.integers(-50, 400, q)).astype(np.int32)  # some empty / inverted
    if q > 3:
        lows[0], highs[0] = I32MIN, I32MAX   # everything but INT_MAX
        lows[1], highs[1] = 5, 5             # empty
        lows[2], highs[2] = -3, 900          # wide, overlapping
    want = [refcpu.select_scan(d, int(lows[j]), int(highs[j])) for j in range(q)]
    dd = Dev.of(d)
    ws = Dev(lib.mq_shared_select_workspace_bytes(n, q))
    k = (C.c_uint64 * q)()
    lo_c = (C.c_int32 * q)(*lows.tolist())
    hi_c = (C.c_int32 * q)(*highs.tolist())
    mq.check(lib.mq_shared_select_count(dd.ptr, n, lo_c, hi_c, q, k, ws.ptr, ws.nbytes, None))
    assert [int(x) for x in k] == [len(w) for w in want]
    outs = [Dev(max(int(x), 1) * 4) for x in k]
    ptrs = (C.c_void_p * q)(*[o.ptr for o in outs])
    mq.check(lib.mq_shared_select_write(ws.ptr, ptrs, None))
    for j in range(q):
        assert np.array_equal(outs[j].get(np.int32, int(k[j])), want[j]), (n, q, j)
    # the one-call form (capacity-n outputs, device counts)
    if n and q <= 20:
        full = [Dev(n * 4) for _ in range(q)]
        dk = Dev(8 * q)
        fptrs = (C.c_void_p * q)(*[o.ptr for o in full])
        mq.check(lib.mq_shared_select(dd.ptr, n, lo_c, hi_c, q, fptrs, dk.ptr, ws.ptr, ws.nbytes, None))
        kk = dk.get(np.uint64, q)
        for j in range(q):
            assert np.array_equal(full[j].get(np.int32, int(kk[j])), want[j]), (n, q, j)


def _shared_run(lib, d, lows, highs):
    n, q = len(d), len(lows)
    dd = Dev.of(d)
    ws = Dev(lib.mq_shared_select_workspace_bytes(n, q))
    k = (C.c_uint64 * q)()
    lo_c = (C.c_int32 * q)(*[int(x) for x in lows])
    hi_c = (C.c_int32 * q)(*[int(x) for x in highs])
    mq.check(lib.mq_shared_select_count(dd.ptr, n, lo_c, hi_c, q, k, ws.ptr, ws.nbytes, None))
    outs = [Dev(max(int(x), 1) * 4) for x in k]
    ptrs = (C.c_void_p * q)(*[o.ptr for o in outs])
    mq.check(lib.mq_shared_select_write(ws.ptr, ptrs, None))
    return [outs[j].get(np.int32, int(k[j])) for j in range(q)]


@pytest.mark.parametrize("impl", ["ei", "ei_twopass", "ei_sw8"])
@pytest.mark.parametrize("case", ["sparse150", "nested", "identical", "dense", "extremes",
                                  "mixed256", "narrow_domain"])
def test_shared_select_many_queries(lib, refcpu, monkeypatch, impl, case):
    """The elementary-interval kernels: by default the count pass lists (query, row) pairs
    and k_ssp_scatter writes them (one column read), MQ_SS_TWOPASS=1 forces the column
    pass (k_ssi_write), which is also what a pair-slice overflow (the dense case) falls
    back to. Sparse and dense queries (dense tiles fall back to
    ballots inside k_ssi_write), nested and identical ranges, INT32 extremes, all 256
    queries, a 7-value domain."""
    if impl.endswith("twopass"):
        monkeypatch.setenv("MQ_SS_TWOPASS", "1")
    if impl == "ei_sw8":  # the scatter's 8-wave blocks, which the default takes for long slices only
        monkeypatch.setenv("MQ_SS_SCATTER_WAVES", "8")
    rng = np.random.default_rng(hash(case) % 2 ** 32)
    n = 1_000_003
    d = rng.integers(0, 10 ** 6, n).astype(np.int32)
    if case == "sparse150":
        lows = rng.integers(0, 10 ** 6 - 1000, 150)
        highs = lows + 1000
    elif case == "nested":
        c = rng.integers(300_000, 700_000, 40)
        w = rng.integers(1, 300_000, 40)
        lows, highs = c - w, c + w
    elif case == "identical":
        lows, highs = np.full(30, 123_456), np.full(30, 654_321)
    elif case == "dense":
        lows = rng.integers(0, 500_000, 48)
        highs = lows + rng.integers(100_000, 500_000, 48)
    elif case == "extremes":
        d[:6] = [I32MIN, I32MAX, I32MIN + 1, I32MAX - 1, 0, -1]
        lows = np.array([I32MIN, I32MIN, 0, -5, I32MAX - 1, I32MIN + 1] + list(rng.integers(0, 10 ** 6, 30)))
        highs = np.array([I32MAX, I32MIN + 2, I32MAX, 5, I32MAX, 0] + list(rng.integers(0, 10 ** 6, 30)))
    elif case == "mixed256":
        lows = rng.integers(-10, 10 ** 6, 256)
        highs = lows + rng.integers(-100, 20_000, 256)  # some empty/inverted
    else:  # narrow_domain: 7 distinct values, many queries share bounds
        d = rng.integers(0, 7, n).astype(np.int32)
        lows = rng.integers(-1, 7, 64)
        highs = lows + rng.integers(0, 4, 64)
    lows = np.asarray(lows, dtype=np.int64).astype(np.int32)
    highs = np.asarray(highs, dtype=np.int64).astype(np.int32)
    got = _shared_run(lib, d, lows, highs)
    for j in range(len(lows)):
        want = refcpu.select_scan(d, int(lows[j]), int(highs[j]))
        assert np.array_equal(got[j], want), (case, impl, j, int(lows[j]), int(highs[j]))
