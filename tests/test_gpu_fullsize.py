"""shared_select at BASELINE's full size (-m gpu, big): VERDICT r02 next-1.

S11 shared_select (src/query.c:439-583) changes behaviour with size: the count pass
lists (query, row) pairs with 24-bit row offsets into per-wave slices of one pair per
row, a slice that overflows sends the write to the column pass, and the coverage
filter's 16384-cell bitmap spans [bmin, bmax] of the queries. On
the seed-42 1e9-row column (generated on the device) every query's
output must equal mq_select_positions on the same range, which the 1e9 goldens pin
(test_gpu_parity.py): K equal, and the two position lists equal element by element
(their difference, mq_sub, reduces to min = max = 0 on the device).

Cases: Q = 16 and Q = 150 ranges of 0.1 % (the bench's sets), through the pair path,
the forced column pass (MQ_SS_TWOPASS=1), and the drop-in API with two row shards on
device 0 (host Column, host Result payloads); plus a dense Q = 16 set of 10 % ranges,
1.6 pairs per row, which overflows every pair slice.
"""
import ctypes as C

import numpy as np
import pytest

from devbuf import Dev
from refapi import _libc, make_column, mq, take

pytestmark = [pytest.mark.gpu, pytest.mark.big]

N = 1_000_000_000


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    yield L
    L.mq_release_all()
    assert L.mq_shard_config(0, None, 0, 0) == 0


@pytest.fixture(scope="module")
def col(lib):
    d = Dev(N * 4)
    mq.check(lib.mq_gen_uniform(d.ptr, N, 42, N, None))
    mq.check(lib.mq_stream_sync(None))
    yield d
    d.free()


def query_set(q, width, seed=5):
    rng = np.random.default_rng(seed)
    lows = rng.integers(0, N - width, q).astype(np.int32)
    return lows, (lows + width).astype(np.int32)


class Checker:
    """mq_select_positions of each range (the pinned single-query path) and an exact
    device comparison of another position list against it."""

    def __init__(self, lib, col):
        self.lib, self.col = lib, col
        self.ws = Dev(lib.mq_scan_workspace_bytes(N))
        self.cnt = Dev(8)
        self.ref = Dev(N // 5 * 4)  # room for a 20 % range
        self.diff = Dev(N // 5 * 4)
        self.agg = Dev(32)

    def positions(self, lo, hi):
        L = self.lib
        mq.check(L.mq_select_positions(self.col.ptr, None, N, 1, int(lo), 1, int(hi), self.ref.ptr,
                                       self.cnt.ptr, self.ws.ptr, self.ws.nbytes, None))
        return int(self.cnt.get(np.uint64, 1)[0])

    def equal_on_device(self, other_ptr, k):
        L = self.lib
        if k == 0:
            return True
        mq.check(L.mq_sub(other_ptr, self.ref.ptr, k, self.diff.ptr, None))
        mq.check(L.mq_reduce(self.diff.ptr, k, self.agg.ptr, self.ws.ptr, self.ws.nbytes, None))
        a = mq.MqAgg.from_buffer_copy(self.agg.get(np.uint8, 32).tobytes())
        return (a.count, a.min, a.max) == (k, 0, 0)


def run_device(lib, col, lows, highs):
    q = len(lows)
    ws = Dev(lib.mq_shared_select_workspace_bytes(N, q))
    k = (C.c_uint64 * q)()
    lo_c = (C.c_int32 * q)(*lows.tolist())
    hi_c = (C.c_int32 * q)(*highs.tolist())
    mq.check(lib.mq_shared_select_count(col.ptr, N, lo_c, hi_c, q, k, ws.ptr, ws.nbytes, None))
    outs = [Dev(max(int(x), 1) * 4) for x in k]
    ptrs = (C.c_void_p * q)(*[o.ptr for o in outs])
    mq.check(lib.mq_shared_select_write(ws.ptr, ptrs, None))
    mq.check(lib.mq_stream_sync(None))
    ws.free()
    return [int(x) for x in k], outs


@pytest.mark.parametrize("twopass", [False, True], ids=["pairs", "twopass"])
@pytest.mark.parametrize("q", [16, 150])
def test_shared_select_1e9_vs_select_positions(lib, col, monkeypatch, q, twopass):
    if twopass:
        monkeypatch.setenv("MQ_SS_TWOPASS", "1")
    lows, highs = query_set(q, N // 1000)
    ks, outs = run_device(lib, col, lows, highs)
    chk = Checker(lib, col)
    for j in range(q):
        kw = chk.positions(lows[j], highs[j])
        assert ks[j] == kw, (q, j)
        assert chk.equal_on_device(outs[j].ptr, kw), (q, j)
        outs[j].free()


def test_shared_select_1e9_pair_slice_overflow(lib, col):
    """16 ranges of 10 % each: 1.6 (query, row) pairs per row, more than a wave's
    slice holds (one pair per row), so the write runs the column pass on the count
    pass's offsets. Two of the ranges are nested and one is a single value."""
    lows, highs = query_set(16, N // 10, seed=9)
    lows[3], highs[3] = lows[2] + 1000, highs[2] - 1000
    lows[4], highs[4] = 777_777_777, 777_777_778
    ks, outs = run_device(lib, col, lows, highs)
    assert sum(ks) > 1.5 * N
    chk = Checker(lib, col)
    for j in range(16):
        kw = chk.positions(lows[j], highs[j])
        assert ks[j] == kw, j
        assert chk.equal_on_device(outs[j].ptr, kw), j
        outs[j].free()


def test_shared_select_1e9_api_two_shards(lib, col):
    """The drop-in shared_select (query.h) over a host Column, split into two row
    shards on device 0 (mq_shard_config): Q = 150 host payloads, each equal to the
    single-query device path's positions."""
    host = col.get(np.int32, N)
    c = make_column(host)
    arr = (C.c_int * 2)(0, 0)
    assert lib.mq_shard_config(2, arr, 2, 0) == 0
    try:
        q = 150
        lows, highs = query_set(q, N // 1000)
        ops = (mq.SelectOperator * q)()
        for j in range(q):
            ops[j].low, ops[j].high = int(lows[j]), int(highs[j])
        s = mq.Status(0, None)
        out = lib.shared_select(ops, q, C.byref(c), C.byref(s))
        assert s.code == mq.OK and out
        assert mq.residency(lib)["shards"] == 2
        chk = Checker(lib, col)
        for j in range(q):
            kw = chk.positions(lows[j], highs[j])
            got = take(out[j])
            assert len(got) == kw, j
            assert np.array_equal(got, chk.ref.get(np.int32, kw)), j
        _libc.free(C.cast(out, C.c_void_p))
    finally:
        lib.mq_release_all()
        assert lib.mq_shard_config(0, None, 0, 0) == 0
        c.data = None
        del host
