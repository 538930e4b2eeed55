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
