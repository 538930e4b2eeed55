"""The key-partitioned hash join on the GPU (-m gpu).

hash_join (query.c:652-696) over G row shards: each shard partitions its build and probe
rows by key bucket (mq_pjoin_partition), device g joins bucket g of every shard
(mq_join_*), the counts and pairs go back to the probe rows' shards and are placed
(mq_pjoin_place). On this one-GPU box all shards sit on device 0 (own threads and
streams, the exchanges device-to-device copies); on a node the same code spreads them
(mq_shard_config / MQ_DEVICES). Checked bit-exact against:
  * the reference's own hash_join outputs: the config-5 goldens 2^16..2^24 (unique) and
    the many-to-many goldens 2^16..2^22 (tests/golden/, M and the pairs' FNV-1a);
  * the oracle (refcpu.hash_join, pinned to the reference's query.c) on duplicate,
    skewed, negative, tiny and empty inputs, every build path of the local join;
  * at 2^28 (beyond the reference's reach), the many-to-many properties;
  * the drop-in hash_join / nested_loop_join with shards on, and a select -> fetch ->
    join chain whose inputs are the shards' own result pieces;
  * two processes (gloo) running dist.partitioned_join over libmq's kernels.
"""
import ctypes as C
import importlib.util
import os
import socket
import sys

import numpy as np
import pytest

from devbuf import Dev
from refapi import _libc, make_column, make_result, mq, take
from test_pjoin_dist import HostPhases, bucket

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    yield L
    L.mq_release_all()
    assert L.mq_shard_config(0, None, 0, 0) == 0


def config(lib, g, min_rows=0):
    arr = (C.c_int * g)(*([0] * g))
    assert lib.mq_shard_config(g, arr, g, min_rows) == 0


def bounds_of(n, g, seed):
    """a ragged split of n rows into g contiguous ranges (one may be empty)"""
    rng = np.random.default_rng(seed)
    b = [0] + sorted(rng.integers(0, n + 1, g - 1).tolist()) + [n]
    return b


def shard_join(lib, g, bufs, n1, n2, seed=0):
    """mq_shard_join over device buffers c1, p1, c2, p2 (Dev) split raggedly into g shards;
    returns the concatenated (out1, out2)."""
    b1, b2 = bounds_of(n1, g, seed), bounds_of(n2, g, seed + 1)
    V = C.c_void_p * g
    U = C.c_uint64 * g
    c1 = V(*[bufs[0].ptr + 4 * b1[s] for s in range(g)])
    p1 = V(*[bufs[1].ptr + 4 * b1[s] for s in range(g)])
    c2 = V(*[bufs[2].ptr + 4 * b2[s] for s in range(g)])
    p2 = V(*[bufs[3].ptr + 4 * b2[s] for s in range(g)])
    n1s = U(*[b1[s + 1] - b1[s] for s in range(g)])
    n2s = U(*[b2[s + 1] - b2[s] for s in range(g)])
    o1, o2, m = V(), V(), U()
    mq.check(lib.mq_shard_join(c1, p1, n1s, c2, p2, n2s, o1, o2, m), "mq_shard_join")
    outs = [], []
    for s in range(g):
        for k, o in enumerate((o1, o2)):
            a = np.empty(m[s], dtype=np.int32)
            if m[s]:
                mq.check(lib.mq_memcpy_d2h(a.ctypes.data, o[s], a.nbytes, None), "d2h")
            outs[k].append(a)
            lib.mq_pool_free(o[s])
    return np.concatenate(outs[0]), np.concatenate(outs[1]), list(m)


@pytest.mark.parametrize("G", [1, 2, 3, 8, 64])
@pytest.mark.parametrize("n", [0, 1, 1023, 1025, 70_001, 3_000_017])
def test_partition_is_a_stable_bucket_split(lib, G, n):
    rng = np.random.default_rng(n + G)
    keys = rng.integers(-(2 ** 31), 2 ** 31 - 1, n, dtype=np.int64).astype(np.int32)
    pay = rng.integers(0, 10 ** 9, n, dtype=np.int32)
    dk, dp = Dev.of(keys), Dev.of(pay)
    ko, po, inv = Dev(4 * max(n, 1)), Dev(4 * max(n, 1)), Dev(4 * max(n, 1))
    cnt = (C.c_uint64 * G)()
    mq.check(lib.mq_pjoin_partition(dk.ptr, dp.ptr, n, G, ko.ptr, po.ptr, inv.ptr, cnt, None))
    b = bucket(keys, G)
    order = np.argsort(b, kind="stable")
    assert list(cnt) == np.bincount(b, minlength=G).tolist()
    assert np.array_equal(ko.get(np.int32, n), keys[order])
    assert np.array_equal(po.get(np.int32, n), pay[order])
    want_inv = np.empty(n, dtype=np.int32)
    want_inv[order] = np.arange(n, dtype=np.int32)
    assert np.array_equal(inv.get(np.int32, n), want_inv)


def test_place_matches_host_restatement(lib, refcpu):
    rng = np.random.default_rng(9)
    n = 300_001
    cntp = rng.integers(0, 4, n).astype(np.int32)
    cntp[7] = 9000  # a run past the per-lane limit: copied by a block
    m = int(cntp.astype(np.int64).sum())
    o1p = rng.integers(0, 10 ** 9, m, dtype=np.int32)
    perm = rng.permutation(n).astype(np.int32)  # any bijection row -> partitioned index
    p2 = rng.integers(0, 10 ** 9, n, dtype=np.int32)
    D = [Dev.of(x) for x in (cntp, o1p, perm, p2)]
    out1, out2 = Dev(4 * m), Dev(4 * m)
    mq.check(lib.mq_pjoin_place(D[0].ptr, D[1].ptr, D[2].ptr, D[3].ptr, n, m, out1.ptr, out2.ptr, None))
    import torch
    w1, w2 = HostPhases(refcpu).place(torch.from_numpy(cntp), torch.from_numpy(o1p), torch.from_numpy(perm),
                                      torch.from_numpy(p2), m)
    assert np.array_equal(out1.get(np.int32, m), w1.numpy())
    assert np.array_equal(out2.get(np.int32, m), w2.numpy())


def _golden_inputs(lib, n, dup):
    D = [Dev(n * 4) for _ in range(4)]
    mq.check(lib.mq_gen_join_keys(D[0].ptr, n, 2 if dup else 0, None))
    mq.check(lib.mq_gen_iota(D[1].ptr, n, None))
    mq.check(lib.mq_gen_join_keys(D[2].ptr, n, 3 if dup else 1, None))
    mq.check(lib.mq_gen_iota(D[3].ptr, n, None))
    return D


@pytest.mark.parametrize("g", [2, 3])
def test_shard_join_goldens(lib, refcpu, goldens, g):
    """SURVEY §8(c) config 5 and its many-to-many variant, split into g ragged row
    ranges per side: M and the pairs' FNV equal the reference's own hash_join."""
    config(lib, g)
    rows = [(r, False) for r in goldens["join"] if "dup" not in r] + \
           [(r, False) for r in goldens["join_survey"] if r["n"] <= 1 << 24] + \
           [(r, True) for r in goldens["join_dup"]]
    for i, (r, dup) in enumerate(rows):
        n = r["n"]
        D = _golden_inputs(lib, n, dup)
        o1, o2, parts = shard_join(lib, g, D, n, n, seed=i)
        assert (len(o1), f"{refcpu.fnv1a64_pairs(o1, o2):016x}") == (r["m"], r["pairs_fnv1a64"]), (n, dup)


def test_shard_join_waits_for_null_stream_writers(lib, refcpu, goldens):
    """Regression (GPUTEST_r04: M = 54 instead of 32,925): the inputs are written on the
    null stream and mq_shard_join is called at once, with no sync. The shard workers run
    on non-blocking streams, so without the entry fence (include/mq_query.h, the
    mq_shard_join stream contract) they would partition the keys before the writers
    finish. Made deterministic: 2^28-row key columns are first filled 200 times with the
    WRONG keys (the other side's), then once with the right ones, all queued on the null
    stream behind each other (~60 ms of queued writes): a worker that does not wait reads
    the wrong keys. M and the pairs' FNV must equal the reference's 2^28 golden."""
    n = 1 << 28
    r = [r for r in goldens["join_survey"] if r["n"] == n][0]
    config(lib, 2)
    D = [Dev(n * 4) for _ in range(4)]
    for _ in range(200):
        mq.check(lib.mq_gen_join_keys(D[0].ptr, n, 1, None))
        mq.check(lib.mq_gen_join_keys(D[2].ptr, n, 0, None))
    mq.check(lib.mq_gen_join_keys(D[0].ptr, n, 0, None))
    mq.check(lib.mq_gen_iota(D[1].ptr, n, None))
    mq.check(lib.mq_gen_join_keys(D[2].ptr, n, 1, None))
    mq.check(lib.mq_gen_iota(D[3].ptr, n, None))
    o1, o2, _ = shard_join(lib, 2, D, n, n, seed=11)  # no sync in between
    assert (len(o1), f"{refcpu.fnv1a64_pairs(o1, o2):016x}") == (r["m"], r["pairs_fnv1a64"])


@pytest.mark.parametrize("g,phase", [(2, 1), (2, 2), (3, 3), (1, 4)])
def test_shard_join_injected_failure_then_goldens(lib, refcpu, goldens, g, phase):
    """an allocation that fails inside a phase (mq_shard_join_inject_failure)
    must return MQ_ENOMEM with no output and only then hand the phase's buffers back to
    the pool (every worker drains its stream first, pj_end), so the next join on the
    same pool is still exact: the 2^20 golden, then the many-to-many 2^20 golden."""
    rows = [r for r in goldens["join"] if r.get("n") == 1 << 20 and "dup" not in r] + \
           [r for r in goldens["join_dup"] if r["n"] == 1 << 20]
    config(lib, g)
    n = 1 << 20
    D = _golden_inputs(lib, n, False)
    b = bounds_of(n, g, 3)
    V, U = C.c_void_p * g, C.c_uint64 * g
    ptrs = [V(*[D[k].ptr + 4 * b[s] for s in range(g)]) for k in range(4)]
    ns = U(*[b[s + 1] - b[s] for s in range(g)])
    o1, o2, m = V(), V(), U()
    lib.mq_shard_join_inject_failure(phase)
    try:
        rc = lib.mq_shard_join(ptrs[0], ptrs[1], ns, ptrs[2], ptrs[3], ns, o1, o2, m)
    finally:
        lib.mq_shard_join_inject_failure(0)
    assert rc == mq.MQ_ENOMEM
    for r, dup in ((rows[0], False), (rows[1], True)):
        D = _golden_inputs(lib, n, dup)
        a1, a2, _ = shard_join(lib, g, D, n, n, seed=5)
        assert (len(a1), f"{refcpu.fnv1a64_pairs(a1, a2):016x}") == (r["m"], r["pairs_fnv1a64"]), dup


CASES = ["unique", "dups", "skew", "neg", "tiny", "empty_build", "empty_probe", "dups_long", "unique_big"]


@pytest.mark.parametrize("g", [2, 3])
@pytest.mark.parametrize("case", CASES)
def test_shard_join_vs_oracle(lib, refcpu, monkeypatch, g, case):
    config(lib, g)
    rng = np.random.default_rng(sum(case.encode()) + g)
    if case == "unique":
        c1 = rng.permutation(200_000).astype(np.int32)
        c2 = rng.integers(0, 400_000, 150_000, dtype=np.int32)
    elif case == "dups":
        c1 = rng.integers(0, 5000, 100_000, dtype=np.int32)
        c2 = rng.integers(0, 6000, 30_000, dtype=np.int32)
    elif case == "skew":
        c1 = np.where(rng.random(50_000) < 0.5, 7, rng.integers(0, 10 ** 6, 50_000)).astype(np.int32)
        c2 = np.concatenate([[7, 7, 3], rng.integers(0, 10 ** 6, 2000)]).astype(np.int32)
    elif case == "neg":
        c1 = rng.integers(-(2 ** 31), 2 ** 31 - 1, 20_000, dtype=np.int64).astype(np.int32)
        c1[:4] = [-(2 ** 31), 2 ** 31 - 1, 0, -1]
        c2 = np.concatenate([c1[::3], rng.integers(-100, 100, 500)]).astype(np.int32)
    elif case == "tiny":
        c1 = np.array([5, 9], dtype=np.int32)
        c2 = np.array([1, 9, 5, 5, 2], dtype=np.int32)
    elif case == "empty_build":
        c1 = np.zeros(0, np.int32)
        c2 = np.array([1, 2, 3], np.int32)
    elif case == "empty_probe":
        c1 = np.array([1, 2, 3], np.int32)
        c2 = np.zeros(0, np.int32)
    elif case == "dups_long":  # a key on 6000 rows: the per-row write's long-run path
        keys = rng.choice(1 << 30, 100_000, replace=False).astype(np.int32)
        c1 = np.concatenate([keys[:80_000], np.full(6000, keys[5], np.int32)])
        c1 = c1[rng.permutation(len(c1))]
        c2 = np.concatenate([[keys[5]] * 3, rng.choice(keys, 50_000)]).astype(np.int32)
    else:  # > 2^22 build rows per side in all: the windowed builds on each device
        c1 = rng.permutation(refcpu.gen_join(5_000_000, "build"))
        c2 = refcpu.gen_join(3_000_000, "probe")
    p1 = rng.integers(0, 10 ** 7, len(c1), dtype=np.int32)
    p2 = rng.integers(0, 10 ** 7, len(c2), dtype=np.int32)
    D = [Dev.of(x) for x in (c1, p1, c2, p2)]
    g1, g2, _ = shard_join(lib, g, D, len(c1), len(c2), seed=len(c1))
    w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2), case


@pytest.mark.big
def test_shard_join_dup_2e28_properties(lib, refcpu):
    """2^28 x 2^28 many-to-many over two shards: every pair joins equal keys, pairs are
    probe-major with build positions ascending inside a probe row, and M equals the
    (probe, build) key matches counted on the host."""
    config(lib, 2)
    n = 1 << 28
    D = _golden_inputs(lib, n, True)
    o1, o2, parts = shard_join(lib, 2, D, n, n, seed=5)
    a, b = refcpu.gen_join(n, "build_dup"), refcpu.gen_join(n, "probe_dup")
    assert len(o1) == 2 * int(np.isin(b, a[: n // 2]).sum())
    assert np.array_equal(a[o1], b[o2])
    assert np.all(o2[1:] >= o2[:-1])
    same = o2[1:] == o2[:-1]
    assert np.all(o1[1:][same] > o1[:-1][same])


def _api_join(lib, c1, p1, c2, p2, fn):
    rs = [make_result(x) for x in (c1, p1, c2, p2)]
    s = mq.Status(0, None)
    out = getattr(lib, fn)(*[C.pointer(r) for r in rs], C.byref(s))
    assert s.code == mq.OK and out
    a, b = take(out[0]), take(out[1])
    _libc.free(C.cast(out, C.c_void_p))
    return a, b


@pytest.mark.parametrize("g", [2, 3])
def test_query_api_join_on_shards(lib, refcpu, g):
    """hash_join / nested_loop_join through the drop-in with shards on (probe sides of
    at least min_rows rows take the partitioned path): equal to the oracle."""
    config(lib, g, min_rows=1000)
    rng = np.random.default_rng(31 + g)
    c1 = rng.integers(0, 40_000, 120_000, dtype=np.int32)
    c2 = rng.integers(0, 50_000, 90_001, dtype=np.int32)
    p1 = rng.integers(0, 10 ** 7, len(c1), dtype=np.int32)
    p2 = rng.integers(0, 10 ** 7, len(c2), dtype=np.int32)
    ops0 = mq.residency(lib)["shard_ops"]
    g1, g2 = _api_join(lib, c1, p1, c2, p2, "hash_join")
    w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2)
    assert mq.residency(lib)["shard_ops"] >= ops0 + 2  # both outputs came from the shards
    # nested_loop_join == the hash join with roles swapped (query.c:585-650)
    h1, h2 = _api_join(lib, c2[:20_000], p2[:20_000], c1[:3000], p1[:3000], "nested_loop_join")
    v1, v2 = refcpu.hash_join(c2[:20_000], p2[:20_000], c1[:3000], p1[:3000], nested=True)
    assert np.array_equal(h1, v1) and np.array_equal(h2, v2)


def test_select_fetch_join_chain_on_shards(lib, refcpu):
    """select -> fetch on two columns of each table, then hash_join of the fetched keys
    with the selected positions: the join takes the shards' own result pieces as inputs
    (no upload), and the output equals the oracle's chain."""
    config(lib, 2, min_rows=1000)
    n = 2_000_003
    a_key = refcpu.gen_uniform(n, 61, 300_000)
    b_key = refcpu.gen_uniform(n, 62, 300_000)
    ca, cb = make_column(a_key, b"ak"), make_column(b_key, b"bk")
    s = mq.Status(0, None)
    lo, hi = C.pointer(C.c_int(0)), C.pointer(C.c_int(150_000))
    pa = lib.select_column(C.byref(ca), lo, hi, C.byref(s))
    pb = lib.select_column(C.byref(cb), lo, C.pointer(C.c_int(40_000)), C.byref(s))
    fa = lib.fetch_column(C.byref(ca), pa, C.byref(s))
    fb = lib.fetch_column(C.byref(cb), pb, C.byref(s))
    assert s.code == mq.OK
    up0 = mq.residency(lib)["result_uploads"]
    out = lib.hash_join(fa, pa, fb, pb, C.byref(s))
    assert s.code == mq.OK and out
    assert mq.residency(lib)["result_uploads"] == up0
    g1, g2 = take(out[0]), take(out[1])
    _libc.free(C.cast(out, C.c_void_p))
    wpa = refcpu.select_scan(a_key, 0, 150_000)
    wpb = refcpu.select_scan(b_key, 0, 40_000)
    w1, w2 = refcpu.hash_join(a_key[wpa], wpa, b_key[wpb], wpb)
    assert np.array_equal(g1, w1) and np.array_equal(g2, w2)
    for r in (pa, pb, fa, fb):
        take(r)


def _mp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import refcpu
    from refapi import mq as mqm
    spec = importlib.util.spec_from_file_location("mq_dist", os.path.join(ROOT, "analytical-database_amd", "dist.py"))
    mqd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mqd)
    L = mqm.load()
    mqm.check(L.mq_init(0), "mq_init")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 20
    out = {}
    for dup in (False, True):
        c1 = refcpu.gen_join(n, "build_dup" if dup else "build")
        c2 = refcpu.gen_join(n, "probe_dup" if dup else "probe")
        p = np.arange(n, dtype=np.int32)
        a, b = mqd.shard_rows(n, rank, world)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x[a:b])).to(dev)
        o1, o2 = mqd.partitioned_join(mqd.LibmqPhases(L, mqm), t(c1), t(p), t(c2), t(p))
        out[dup] = (o1.cpu().numpy(), o2.cpu().numpy())
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_processes_partitioned_join_over_libmq(refcpu, goldens):
    """dist.partitioned_join with libmq's kernels in each of two processes (both on
    device 0, exchanges over gloo): the concatenated output equals the 2^20 goldens."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 1 << 20
    for dup in (False, True):
        g1 = np.concatenate([res[r][dup][0] for r in range(2)])
        g2 = np.concatenate([res[r][dup][1] for r in range(2)])
        rows = goldens["join_dup"] if dup else [r for r in goldens["join"] if "dup" not in r]
        want = [r for r in rows if r["n"] == n]
        assert want, (n, dup)
        assert (len(g1), f"{refcpu.fnv1a64_pairs(g1, g2):016x}") == (want[0]["m"], want[0]["pairs_fnv1a64"]), dup
