"""The key-partitioned hash join's exchange and ordering logic over real process groups
(gloo, CPU; SURVEY.md §8(e) "radix-partitioning by key with an all-to-all").

analytical-database_amd/dist.py partitioned_join runs the protocol of
csrc/mq_pjoin.hip one process per rank: partition both sides by key bucket, all_to_all
bucket g to rank g, local join, all_to_all the counts and pairs back, place. Here its
device steps are host stand-ins (numpy; the local join is the oracle's hash_join, pinned
to the reference's own query.c), so what is under test is the driver itself: split
sizes, segment offsets, the two exchanges and the final placement. The concatenation of
every rank's output must equal the reference's hash_join of the whole input
(query.c:652-696: probe-major, build-insertion order) for 2 and 3 ranks, ragged and
empty row ranges, duplicate, skewed and negative keys. The same driver over libmq's
kernels runs in tests/test_gpu_pjoin.py (-m gpu).
"""
import importlib.util
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dist_mod():
    spec = importlib.util.spec_from_file_location("mq_dist", os.path.join(ROOT, "analytical-database_amd", "dist.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def bucket(keys: np.ndarray, G: int) -> np.ndarray:
    """mq_pjoin.hip pj_part restated: lowbias32 of key ^ 0x9E3779B9, then (h * G) >> 32."""
    h = keys.astype(np.int64).astype(np.uint32) ^ np.uint32(0x9E3779B9)
    h = h.astype(np.uint64)
    M = np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & M
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & M
    h ^= h >> np.uint64(16)
    return ((h * np.uint64(G)) >> np.uint64(32)).astype(np.int64)


class HostPhases:
    """The device steps of partitioned_join as numpy stand-ins (test infrastructure)."""

    def __init__(self, refcpu):
        self.refcpu = refcpu

    def partition(self, keys, pay, G, want_inv):
        k = keys.numpy()
        b = bucket(k, G)
        order = np.argsort(b, kind="stable")
        inv = np.empty(len(k), dtype=np.int32)
        inv[order] = np.arange(len(k), dtype=np.int32)
        counts = np.bincount(b, minlength=G).astype(np.int64)
        return (torch.from_numpy(k[order].copy()), None if pay is None else torch.from_numpy(pay.numpy()[order].copy()),
                torch.from_numpy(inv) if want_inv else None, torch.from_numpy(counts))

    def local_join(self, bk, bp, pk):
        n2 = pk.numel()
        o1, rows = self.refcpu.hash_join(bk.numpy(), bp.numpy(), pk.numpy(), np.arange(n2, dtype=np.int32))
        cnt = np.bincount(rows, minlength=n2).astype(np.int32) if n2 else np.zeros(0, np.int32)
        return torch.from_numpy(cnt), torch.from_numpy(np.ascontiguousarray(o1, dtype=np.int32))

    def place(self, cntp, o1p, inv, p2, m):
        cntp, o1p, inv, p2 = cntp.numpy().astype(np.int64), o1p.numpy(), inv.numpy(), p2.numpy()
        poff = np.concatenate([[0], np.cumsum(cntp)[:-1]]) if len(cntp) else cntp
        cnt_row = cntp[inv]
        start = poff[inv]  # row r's pairs in the partitioned stream
        src = np.repeat(start, cnt_row) + (np.arange(m) - np.repeat(np.cumsum(cnt_row) - cnt_row, cnt_row))
        return torch.from_numpy(o1p[src].astype(np.int32)), torch.from_numpy(np.repeat(p2, cnt_row).astype(np.int32))


def cases():
    rng = np.random.default_rng(2024)
    out = {}
    c1 = rng.integers(0, 3000, 40_000, dtype=np.int32)  # duplicates: runs in insertion order
    c2 = rng.integers(0, 3500, 25_000, dtype=np.int32)
    out["dups"] = (c1, c2)
    c1 = rng.permutation(60_000).astype(np.int32)  # unique build keys, about half the probes hit
    c2 = rng.integers(0, 120_000, 50_000, dtype=np.int32)
    out["unique"] = (c1, c2)
    c1 = np.where(rng.random(20_000) < 0.3, 7, rng.integers(-(2 ** 31), 2 ** 31 - 1, 20_000)).astype(np.int32)
    c2 = np.concatenate([[7, 7, -1], rng.choice(c1, 3000)]).astype(np.int32)  # a hot key, negatives
    out["skew"] = (c1, c2)
    out["tiny"] = (np.array([5, 9, 5], np.int32), np.array([1, 9, 5, 5, 2], np.int32))
    out["empty_build"] = (np.zeros(0, np.int32), np.array([1, 2, 3], np.int32))
    return out


def splits(n, world, kind):
    """contiguous row ranges in rank order: even, or ragged with an empty range"""
    if kind == "even":
        b = [n * r // world for r in range(world + 1)]
    else:
        b = [0] + sorted(np.random.default_rng(n + world).integers(0, n + 1, world - 1).tolist()) + [n]
        if world > 2:
            b[1] = b[0]  # rank 0 holds no rows
    return b


def _worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu
    refcpu.build()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mqd = _dist_mod()
    ph = HostPhases(refcpu)
    res = {}
    for name, (c1, c2) in cases().items():
        p1 = (np.arange(len(c1)) * 3 + 11).astype(np.int32)
        p2 = (np.arange(len(c2)) * 5 + 7).astype(np.int32)
        b1, b2 = splits(len(c1), world, kind), splits(len(c2), world, kind)
        t = lambda a, b, r: torch.from_numpy(np.ascontiguousarray(a[b[r]:b[r + 1]]))
        o1, o2 = mqd.partitioned_join(ph, t(c1, b1, rank), t(p1, b1, rank), t(c2, b2, rank), t(p2, b2, rank))
        res[name] = (o1.numpy().copy(), o2.numpy().copy())
    q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,kind", [(2, "even"), (2, "ragged"), (3, "ragged")])
def test_partitioned_join_exchange_matches_reference(refcpu, world, kind):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for name, (c1, c2) in cases().items():
        p1 = (np.arange(len(c1)) * 3 + 11).astype(np.int32)
        p2 = (np.arange(len(c2)) * 5 + 7).astype(np.int32)
        w1, w2 = refcpu.hash_join(c1, p1, c2, p2)
        g1 = np.concatenate([res[r][name][0] for r in range(world)])
        g2 = np.concatenate([res[r][name][1] for r in range(world)])
        assert np.array_equal(g1, w1) and np.array_equal(g2, w2), (name, world, kind)
        # each rank's part is the pairs of its own probe rows
        b2 = splits(len(c2), world, kind)
        for r in range(world):
            own = set(p2[b2[r]:b2[r + 1]].tolist())
            assert set(res[r][name][1].tolist()) <= own, (name, r)


def test_bucket_restatement_matches_libmq():
    """The numpy bucket function above is libmq's own (mq_pjoin_bucket, a host symbol:
    no device needed), for G = 1..8 and 64 on keys including the int32 extremes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from refapi import mq
    lib = mq.load()
    keys = np.concatenate([np.array([0, -1, 1, 2 ** 31 - 1, -(2 ** 31)], np.int32),
                           np.random.default_rng(5).integers(-(2 ** 31), 2 ** 31 - 1, 3000, dtype=np.int64).astype(np.int32)])
    for G in (1, 2, 3, 5, 8, 64):
        want = bucket(keys, G)
        got = np.array([lib.mq_pjoin_bucket(int(k), G) for k in keys])
        assert np.array_equal(got, want), G
        if G > 1:  # and it spreads
            assert np.bincount(want, minlength=G).min() > len(keys) / G / 2
