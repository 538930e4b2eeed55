"""Pin the oracle (oracle/refcpu.c) before trusting it.

  1. against the golden vectors in tests/golden/ (produced by the reference's
     own query.c, cross-checked with SURVEY.md §8(c));
  2. against the reference build itself (oracle/_ref/libref.so) on edge cases:
     NULL bounds, empty / inverted / full ranges, negative values, INT32
     extremes, ragged sizes, duplicate join keys.
CPU only (no GPU marker).
"""
import os
import struct

import numpy as np
import pytest

from refapi import Api, make_column

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
I32MIN, I32MAX = -(2 ** 31), 2 ** 31 - 1


def dbits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _rows(goldens, key, big=False):
    rows = goldens[key]
    return [r for r in rows if big or r["n"] <= 10_000_000]


def test_goldens_present(goldens):
    assert any(r["n"] == 1_000_000_000 for r in goldens["select"]), "1e9 goldens missing"
    assert goldens["config4_combined"]["k"] == 80005753
    assert goldens["config4_combined"]["sum"] == 20401453459958049


def test_oracle_matches_select_goldens(refcpu, goldens):
    for r in _rows(goldens, "select"):
        d = refcpu.gen_uniform(r["n"], r["seed"])
        pos = refcpu.select_scan(d, r["low"], r["high"])
        assert len(pos) == r["k"]
        assert f"{refcpu.fnv1a64(pos):016x}" == r["pos_fnv1a64"]
        a = refcpu.agg(refcpu.fetch(d, pos))
        assert a["sum"] == r["sum"] and a["min"] == r["min"] and a["max"] == r["max"]
        assert f"{dbits(a['avg']):016x}" == r["avg_bits"]
        c, s = refcpu.count_sum(d, r["low"], r["high"])
        assert (c, s) == (r["k"], r["sum"])


def test_oracle_matches_column_sum_and_config3(refcpu, goldens):
    for n, want in goldens["column_sum"].items():
        if int(n) > 10_000_000:
            continue
        d = refcpu.gen_uniform(int(n), 42)
        assert refcpu.agg(d)["sum"] == want
    for r in _rows(goldens, "config3"):
        d0 = refcpu.gen_uniform(r["n"], 42)
        d1 = refcpu.gen_uniform(r["n"], r["fetch_seed"])
        pos = refcpu.select_scan(d0, r["low"], r["high"])
        a = refcpu.agg(refcpu.fetch(d1, pos))
        assert (len(pos), a["sum"], a["min"], a["max"]) == (r["k"], r["sum"], r["min"], r["max"])
        assert f"{dbits(a['avg']):016x}" == r["avg_bits"]


def test_fixture_files_match_generator(refcpu):
    d = np.fromfile(os.path.join(GOLD, "col_n65536_s42.bin"), dtype=np.int32)
    assert np.array_equal(d, refcpu.gen_uniform(65536, 42))
    for sel in (0.01, 0.5, 1.0):
        want = np.fromfile(os.path.join(GOLD, f"pos_n65536_s42_sel{sel}.bin"), dtype=np.int32)
        lo = int(0.25 * 65536)
        assert np.array_equal(refcpu.select_scan(d, lo, lo + int(sel * 65536)), want)


def test_oracle_matches_join_goldens(refcpu, goldens):
    for r in goldens["join"]:
        if "dup" in r:
            rng = np.random.default_rng(7)
            c1 = rng.integers(0, 50, 3000, dtype=np.int32)
            c2 = rng.integers(0, 60, 2000, dtype=np.int32)
            p1 = np.arange(3000, dtype=np.int32) * 3
            p2 = np.arange(2000, dtype=np.int32) * 7
            o1, o2 = refcpu.hash_join(c1, p1, c2, p2, nested=(r["kind"] == "nested"))
        else:
            n = r["n"]
            p = refcpu.gen_join(n, "iota")
            o1, o2 = refcpu.hash_join(refcpu.gen_join(n, "build"), p, refcpu.gen_join(n, "probe"), p)
        assert len(o1) == r["m"]
        assert f"{refcpu.fnv1a64_pairs(o1, o2):016x}" == r["pairs_fnv1a64"]


def test_oracle_matches_join_dup_goldens(refcpu, goldens):
    """The many-to-many config-5 variant (every build key twice) against the
    reference's own hash_join (tests/golden/make_join_dup_goldens.py)."""
    for r in goldens["join_dup"]:
        n = r["n"]
        p = refcpu.gen_join(n, "iota")
        o1, o2 = refcpu.hash_join(refcpu.gen_join(n, "build_dup"), p, refcpu.gen_join(n, "probe_dup"), p)
        assert (len(o1), f"{refcpu.fnv1a64_pairs(o1, o2):016x}") == (r["m"], r["pairs_fnv1a64"]), n


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_host_cores_join_equals_restatement(refcpu, goldens, threads):
    """rc_hash_join_mt (the config-5 host-cores baseline) = rc_hash_join on the unique and
    many-to-many goldens to 2^20 and on a dense small-domain case (long runs)."""
    rows = [(r, "build", "probe") for r in goldens["join"] if "dup" not in r] + \
           [(r, "build_dup", "probe_dup") for r in goldens["join_dup"] if r["n"] <= 1 << 20]
    for r, kb, kp in rows:
        n = r["n"]
        p = refcpu.gen_join(n, "iota")
        o1, o2 = refcpu.hash_join_mt(refcpu.gen_join(n, kb), p, refcpu.gen_join(n, kp), p, threads)
        assert (len(o1), f"{refcpu.fnv1a64_pairs(o1, o2):016x}") == (r["m"], r["pairs_fnv1a64"]), (n, kb)
    rng = np.random.default_rng(threads)
    c1, c2 = rng.integers(-5, 5, 5000).astype(np.int32), rng.integers(-6, 6, 3000).astype(np.int32)
    p1, p2 = np.arange(5000, dtype=np.int32), np.arange(3000, dtype=np.int32) * 3
    w, g = refcpu.hash_join(c1, p1, c2, p2), refcpu.hash_join_mt(c1, p1, c2, p2, threads)
    assert np.array_equal(w[0], g[0]) and np.array_equal(w[1], g[1])


def test_oracle_reproduces_survey_join_2e24(refcpu, goldens):
    r = [x for x in goldens["join_survey"] if x["n"] == 1 << 24][0]
    n = r["n"]
    p = refcpu.gen_join(n, "iota")
    o1, o2 = refcpu.hash_join(refcpu.gen_join(n, "build"), p, refcpu.gen_join(n, "probe"), p)
    assert len(o1) == r["m"]
    assert f"{refcpu.fnv1a64_pairs(o1, o2):016x}" == r["pairs_fnv1a64"]


# ---------------------------------------------------------------------------
# restatement vs the reference build on edge cases
# ---------------------------------------------------------------------------
needs_ref = pytest.mark.skipif(not os.path.exists(os.path.join(
    os.path.dirname(HERE), "oracle", "_ref", "libref.so")), reason="oracle/_ref not built")

BOUNDS = [(None, None), (10, None), (None, 10), (-5, 5), (5, 5), (7, 3), (I32MIN, I32MAX),
          (I32MIN, None), (None, I32MAX), (I32MAX, None), (None, I32MIN), (0, 1)]


def _edge_data(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.integers(-20, 20, n, dtype=np.int32)
    if n > 4:
        d[0], d[1], d[2] = I32MIN, I32MAX, 0
    return d


@needs_ref
@pytest.mark.parametrize("n", [0, 1, 3, 64, 1023, 1025, 4099])
def test_select_fetch_agg_vs_reference(refcpu, n):
    api = Api(refcpu.reference())
    d = _edge_data(n, n)
    col = make_column(d)
    for lo, hi in BOUNDS:
        want = api.select_column(col, lo, hi)
        got = refcpu.select_scan(d, lo, hi)
        assert np.array_equal(got, want), (n, lo, hi)
        if n == 0:
            continue
        vals = api.fetch_column(col, want)
        assert np.array_equal(refcpu.fetch(d, want), vals)
        if len(vals):
            a = refcpu.agg(vals)
            assert a["sum"] == api.sum_result(vals)
            assert a["min"] == api.min(vals) and a["max"] == api.max(vals)
            assert dbits(a["avg"]) == dbits(api.average(vals))
    if n:
        assert refcpu.agg(d)["sum"] == api.sum_column(col)


@needs_ref
def test_select_result_vs_reference(refcpu):
    api = Api(refcpu.reference())
    rng = np.random.default_rng(3)
    vals = rng.integers(-100, 100, 5000, dtype=np.int32)
    prev = np.sort(rng.choice(10 ** 6, 5000, replace=False)).astype(np.int32)
    for lo, hi in BOUNDS:
        assert np.array_equal(refcpu.select_result(vals, prev, lo, hi),
                              api.select_result(vals, prev, lo, hi)), (lo, hi)


@needs_ref
def test_add_sub_vs_reference(refcpu):
    api = Api(refcpu.reference())
    rng = np.random.default_rng(5)
    a = rng.integers(-1000, 1000, 777, dtype=np.int32)
    b = rng.integers(-1000, 1000, 777, dtype=np.int32)
    assert np.array_equal(refcpu.add(a, b), api.add(a, b))
    assert np.array_equal(refcpu.sub(a, b), api.sub(a, b))


@needs_ref
def test_shared_select_vs_reference(refcpu):
    api = Api(refcpu.reference())
    n = 30000
    d = refcpu.gen_uniform(n, 11, modulus=n)  # values in [0,n): value-range split is valid
    col = make_column(d)
    rng = np.random.default_rng(1)
    lows = rng.integers(0, n, 40).astype(np.int32)
    highs = (lows + rng.integers(0, n // 3, 40)).astype(np.int32)
    want = api.shared_select(col, lows, highs)
    for split, threads in ((1, 3), (0, 1), (0, 7)):
        got = refcpu.shared_select(d, lows, highs, nthreads=threads, split=split)
        for q in range(40):
            assert np.array_equal(got[q], want[q]), (split, threads, q)


@needs_ref
@pytest.mark.parametrize("kind", ["hash", "nested"])
def test_join_vs_reference(refcpu, kind):
    api = Api(refcpu.reference())
    rng = np.random.default_rng(9)
    # build sides of >= 4 rows: with 1-3 distinct build keys the reference's
    # multimap is full and find_index (multimap.c:65-71) spins forever on an
    # absent probe key; those shapes are covered by test_join_small_vs_python.
    for n1, n2, kr in ((4, 9, 3), (100, 257, 10), (2000, 1500, 300), (513, 4000, 5)):
        c1 = rng.integers(0, kr, n1, dtype=np.int32)
        c2 = rng.integers(0, kr, n2, dtype=np.int32)
        p1 = rng.integers(0, 10 ** 6, n1, dtype=np.int32)
        p2 = rng.integers(0, 10 ** 6, n2, dtype=np.int32)
        w1, w2 = api.join(c1, p1, c2, p2, kind)
        g1, g2 = refcpu.hash_join(c1, p1, c2, p2, nested=(kind == "nested"))
        assert np.array_equal(g1, w1) and np.array_equal(g2, w2), (n1, n2, kr)


def _py_join(c1, p1, c2, p2):
    groups = {}
    for i, k in enumerate(c1.tolist()):
        groups.setdefault(k, []).append(int(p1[i]))
    o1, o2 = [], []
    for j, k in enumerate(c2.tolist()):
        for v in groups.get(k, []):
            o1.append(v)
            o2.append(int(p2[j]))
    return np.array(o1, dtype=np.int32), np.array(o2, dtype=np.int32)


def test_join_small_vs_python(refcpu):
    rng = np.random.default_rng(21)
    for n1, n2 in ((0, 5), (5, 0), (1, 1), (1, 4), (2, 7), (3, 3), (17, 40)):
        c1 = rng.integers(-3, 3, n1, dtype=np.int32)
        c2 = rng.integers(-4, 4, n2, dtype=np.int32)
        p1 = np.arange(n1, dtype=np.int32)
        p2 = np.arange(n2, dtype=np.int32) + 100
        w1, w2 = _py_join(c1, p1, c2, p2)
        g1, g2 = refcpu.hash_join(c1, p1, c2, p2)
        assert np.array_equal(g1, w1) and np.array_equal(g2, w2), (n1, n2)
        # nested loop = outer-major over column_one
        n1_, n2_ = _py_join(c2, p2, c1, p1)
        h1, h2 = refcpu.hash_join(c1, p1, c2, p2, nested=True)
        assert np.array_equal(h1, n2_) and np.array_equal(h2, n1_), (n1, n2)


@needs_ref
def test_print_vs_reference(refcpu):
    api = Api(refcpu.reference())
    ints = np.array([3, -7, 12], dtype=np.int32)
    longs = np.array([1234567890123], dtype=np.int64)
    dbl = np.array([2.0 / 3.0], dtype=np.float64)
    from refapi import mq
    assert api.print([(ints, mq.INT), (longs, mq.LONG), (dbl, mq.DOUBLE)]) == "3\n-7\n12,1234567890123,0.67"


def test_multimap_size_matches_reference_rule(refcpu):
    L = refcpu.lib()
    # smallest prime >= (int)(1.3 n), multimap.c:30-38
    assert L.rc_multimap_size(10) == 13
    assert L.rc_multimap_size(100) == 131
    assert L.rc_multimap_size(1 << 16) == 85199
