"""Multi-GPU combine for sharded scans.

One process per GPU. Each rank scans its own shard — a row range of one column,
or (config 4) its own column of a batched query — with libmq, producing an
mq_agg {count, sum, min, max} in HBM. The only exchange is the final aggregate
combine: one all-reduce of 16 bytes ({count, sum}, int64 SUM) and, when min/max
are wanted, one more of 16 bytes (MAX over {-min, max}). With backend "nccl"
this is RCCL over xGMI; the same code runs on "gloo" for CPU tests.

avg is computed after the combine as one double division of the combined int64
sum by the combined count, exactly as query.c:314 does on one node, so the
multi-GPU avg is bit-identical to the single-GPU one.

Position lists never move: a row-sharded select's global list is the
concatenation of the per-rank lists (local row + shard base) in rank order,
which is the order shared_select's thread concatenation produces
(query.c:563-574).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

I32MAX, I32MIN = 2 ** 31 - 1, -(2 ** 31)


def agg_tensor(device) -> torch.Tensor:
    """A 32-byte buffer laid out as mq_agg: [count u64, sum i64, (min i32|max i32), pad]."""
    return torch.zeros(4, dtype=torch.int64, device=device)


def unpack(agg: torch.Tensor) -> dict:
    a = agg.cpu()
    mm = a[2:3].view(torch.int32)
    return {"count": int(a[0]), "sum": int(a[1]), "min": int(mm[0]), "max": int(mm[1])}


def combine_count_sum(agg: torch.Tensor, group=None) -> None:
    """In place: agg[0:2] <- SUM over ranks (the one collective on the scan path)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(agg[0:2], op=dist.ReduceOp.SUM, group=group)


def combine_full(agg: torch.Tensor, group=None) -> dict:
    """count/sum/min/max over all ranks; returns host values plus avg."""
    combine_count_sum(agg, group)
    mm = agg[2:3].view(torch.int32).to(torch.int64)
    ext = torch.stack([-mm[0], mm[1]])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(ext, op=dist.ReduceOp.MAX, group=group)
    c, s = int(agg[0]), int(agg[1])
    return {"count": c, "sum": s, "min": int(-ext[0]), "max": int(ext[1]),
            "avg": (float(s) / float(c)) if c else float("nan")}


def shard_rows(n: int, rank: int, world: int, align: int = 1024) -> tuple[int, int]:
    """Contiguous row range [lo, hi) of rank's shard, boundaries on `align` rows."""
    per = -(-n // world)
    per = -(-per // align) * align
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


# ---------------------------------------------------------------------------
# Key-partitioned hash join, one process per GPU (SURVEY.md §8(e) "next"; the
# protocol of csrc/mq_pjoin.hip). The in-process form over libmq's
# row-shard workers is mq_shard_join (peer copies); this is the same steps with
# all_to_all exchanges: RCCL over xGMI with backend "nccl", gloo (through host
# memory) otherwise.
# ---------------------------------------------------------------------------
def _a2a(t: torch.Tensor, in_splits, out_splits, group=None) -> torch.Tensor:
    """all_to_all_single of a 1-D tensor; device tensors go through host memory when
    the backend cannot move them (gloo)."""
    out_n = int(sum(out_splits))
    if dist.get_world_size(group) == 1:
        return t[:out_n].clone()
    stage = t.is_cuda and dist.get_backend(group) != "nccl"
    src = t.cpu() if stage else t
    out = torch.empty(out_n, dtype=t.dtype, device=src.device)
    dist.all_to_all_single(out, src.contiguous(), output_split_sizes=[int(x) for x in out_splits],
                           input_split_sizes=[int(x) for x in in_splits], group=group)
    return out.to(t.device) if stage else out


def _a2a_counts(counts: torch.Tensor, group=None) -> torch.Tensor:
    """counts[b] (rows this rank sends to rank b) -> the rows each rank sends here."""
    G = dist.get_world_size(group)
    if G == 1:
        return counts.clone()
    stage = counts.is_cuda and dist.get_backend(group) != "nccl"
    src = counts.cpu() if stage else counts
    out = torch.empty_like(src)
    dist.all_to_all_single(out, src.contiguous(), group=group)
    return out


def partitioned_join(phases, c1, p1, c2, p2, group=None):
    """hash_join (query.c:652-696) over the ranks of `group`, keys partitioned.

    c1 / p1: this rank's build rows (keys, build positions), c2 / p2 its probe rows;
    each side split into contiguous row ranges in rank order (any sizes). Returns this
    rank's (out1, out2): the reference's pairs of its probe rows, in the reference's
    order, so the concatenation over ranks is hash_join's whole output.

    phases: the device steps (LibmqPhases on the GPU; the tests pass host stand-ins):
      partition(keys, pay, G, want_inv) -> (keys_out, pay_out, inv, counts int64[G])
      local_join(bk, bp, pk) -> (cnt u32-as-int32 per probe row, out1 build positions)
      place(cntp, out1p, inv, p2, m) -> (out1, out2)
    """
    G = dist.get_world_size(group) if dist.is_initialized() else 1
    # 1. partition both sides by key bucket (stable)
    bk, bp, _, cb = phases.partition(c1, p1, G, False)
    pk, _, inv, cp = phases.partition(c2, None, G, True)
    # 2. bucket g of every rank to rank g, in rank order
    rb = _a2a_counts(cb, group).tolist()
    rp = _a2a_counts(cp, group).tolist()
    cb, cp = cb.tolist(), cp.tolist()
    jk, jp = _a2a(bk, cb, rb, group), _a2a(bp, cb, rb, group)
    jq = _a2a(pk, cp, rp, group)
    # 3. local join of this rank's bucket
    cnt, o1 = phases.local_join(jk, jp, jq)
    # pairs of each source rank's rows: the sums of its segment of the counts
    seg = torch.tensor([0] + rp, dtype=torch.int64).cumsum(0).tolist()
    c64 = cnt.to(torch.int64)
    mg = torch.stack([c64[seg[s]:seg[s + 1]].sum() for s in range(G)]).to(torch.int64)
    # 4. counts and pairs back to the probe rows' home ranks
    mr = _a2a_counts(mg.to(cnt.device), group).tolist()
    mg = mg.tolist()
    cntp = _a2a(cnt, rp, cp, group)
    o1p = _a2a(o1, mg, mr, group)
    # 5. every probe row's pairs at its offset
    return phases.place(cntp, o1p, inv, p2, int(sum(mr)))


class LibmqPhases:
    """partitioned_join's steps on libmq's kernels (mq_pjoin_partition, mq_join_*,
    mq_pjoin_place), on torch-owned device buffers and torch's current stream."""

    def __init__(self, lib, mq):
        self.lib, self.mq = lib, mq

    def _st(self):
        return torch.cuda.current_stream().cuda_stream

    def partition(self, keys, pay, G, want_inv):
        import ctypes as C
        n = keys.numel()
        ko = torch.empty(max(n, 1), dtype=torch.int32, device=keys.device)
        po = torch.empty(max(n, 1), dtype=torch.int32, device=keys.device) if pay is not None else None
        inv = torch.empty(max(n, 1), dtype=torch.int32, device=keys.device) if want_inv else None
        counts = (C.c_uint64 * G)()
        self.mq.check(self.lib.mq_pjoin_partition(
            keys.data_ptr(), pay.data_ptr() if pay is not None else None, n, G, ko.data_ptr(),
            po.data_ptr() if po is not None else None, inv.data_ptr() if inv is not None else None, counts,
            self._st()), "mq_pjoin_partition")
        c = torch.tensor(list(counts), dtype=torch.int64, device=keys.device)
        return ko[:n], (po[:n] if po is not None else None), (inv[:n] if inv is not None else None), c

    def local_join(self, bk, bp, pk):
        import ctypes as C
        h = C.c_void_p()
        st = self._st()
        self.mq.check(self.lib.mq_join_build(bk.data_ptr(), bp.data_ptr(), bk.numel(), C.byref(h), st),
                      "mq_join_build")
        try:
            m = C.c_uint64()
            self.mq.check(self.lib.mq_join_probe(h, pk.data_ptr(), pk.numel(), C.byref(m), st), "mq_join_probe")
            cnt = torch.empty(max(pk.numel(), 1), dtype=torch.int32, device=pk.device)
            self.mq.check(self.lib.mq_join_counts(h, cnt.data_ptr(), st), "mq_join_counts")
            o1 = torch.empty(max(m.value, 1), dtype=torch.int32, device=pk.device)
            if m.value:
                self.mq.check(self.lib.mq_join_write(h, None, o1.data_ptr(), None, st), "mq_join_write")
            torch.cuda.current_stream().synchronize()
        finally:
            self.lib.mq_join_free(h)
        return cnt[:pk.numel()], o1[:m.value]

    def place(self, cntp, o1p, inv, p2, m):
        n = p2.numel()
        out1 = torch.empty(max(m, 1), dtype=torch.int32, device=p2.device)
        out2 = torch.empty(max(m, 1), dtype=torch.int32, device=p2.device)
        if m:
            self.mq.check(self.lib.mq_pjoin_place(cntp.data_ptr(), o1p.data_ptr(), inv.data_ptr(), p2.data_ptr(), n,
                                                  m, out1.data_ptr(), out2.data_ptr(), self._st()),
                          "mq_pjoin_place")
        return out1[:m], out2[:m]
