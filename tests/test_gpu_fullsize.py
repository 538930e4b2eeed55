"""shared_select at BASELINE's full size (-m gpu, big): VERDICT r02 next-1, r05 next-6.

S11 shared_select (src/query.c:439-583) changes behaviour with size: the count pass
lists (query, row) pairs with 24-bit row offsets into per-wave slices of one pair per
row, a slice that overflows sends the write to the column pass, and the coverage
filter's cell table spans [bmin, bmax] of the queries. On the seed-42
1e9-row column (generated on the device) every query's K and the FNV-1a-64
of its position list must equal the REFERENCE's own shared_select on the same column
and queries (tests/golden/shared_goldens.json, made by tests/golden/make_shared_goldens.py
through oracle/_ref/libref.so, the reference's query.c compiled unchanged).

Cases: Q = 16 and Q = 150 ranges of 0.1 % (the bench's sets), through the pair path,
the forced column pass (MQ_SS_TWOPASS=1), and the drop-in API with two row shards on
device 0 (host Column, host Result payloads); plus a dense Q = 16 set of 10 % ranges,
1.6 pairs per row, which overflows every pair slice.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from devbuf import Dev
from refapi import _libc, make_column, mq, take

pytestmark = [pytest.mark.gpu, pytest.mark.big]

N = 1_000_000_000
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "shared_goldens.json")


@pytest.fixture(scope="module")
def sgold():
    g = json.load(open(GOLDEN))
    assert g["n"] == N
    return g["sets"]


def check_set(refcpu, sgold, name, lows, highs, ks, get):
    """K and the position list's FNV-1a-64 of every query equal the reference's; get(j)
    returns query j's positions as a host int32 array."""
    gs = sgold[name]["queries"]
    assert len(gs) == len(lows)
    for j, g in enumerate(gs):
        assert (g["low"], g["high"]) == (int(lows[j]), int(highs[j])), (name, j)
        assert ks[j] == g["k"], (name, j)
        assert f"{refcpu.fnv1a64(get(j)):016x}" == g["pos_fnv1a64"], (name, j)


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
def test_shared_select_1e9_vs_reference(lib, col, refcpu, sgold, monkeypatch, q, twopass):
    if twopass:
        monkeypatch.setenv("MQ_SS_TWOPASS", "1")
    lows, highs = query_set(q, N // 1000)
    ks, outs = run_device(lib, col, lows, highs)
    check_set(refcpu, sgold, f"q{q}", lows, highs, ks, lambda j: outs[j].get(np.int32, ks[j]))
    for o in outs:
        o.free()


def test_shared_select_1e9_pair_slice_overflow(lib, col, refcpu, sgold):
    """16 ranges of 10 % each: 1.6 (query, row) pairs per row, more than a wave's
    slice holds (one pair per row), so the write runs the column pass on the count
    pass's offsets. Two of the ranges are nested and one is a single value."""
    lows, highs = query_set(16, N // 10, seed=9)
    lows[3], highs[3] = lows[2] + 1000, highs[2] - 1000
    lows[4], highs[4] = 777_777_777, 777_777_778
    ks, outs = run_device(lib, col, lows, highs)
    assert sum(ks) > 1.5 * N
    check_set(refcpu, sgold, "q16_dense", lows, highs, ks, lambda j: outs[j].get(np.int32, ks[j]))
    for o in outs:
        o.free()


def test_shared_select_1e9_api_two_shards(lib, col, refcpu, sgold):
    """The drop-in shared_select (query.h) over a host Column, split into two row
    shards on device 0 (mq_shard_config): Q = 150 host payloads, each equal to the
    reference's shared_select output (K and FNV)."""
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
        got = [take(out[j]) for j in range(q)]
        _libc.free(C.cast(out, C.c_void_p))
        check_set(refcpu, sgold, "q150", lows, highs, [len(g) for g in got], lambda j: got[j])
    finally:
        lib.mq_release_all()
        assert lib.mq_shard_config(0, None, 0, 0) == 0
        c.data = None
        del host
