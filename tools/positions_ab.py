"""A/B of the ordered-compaction paths (MQ_POSITIONS_IMPL = stage | mask | lookback, and
stage_lanes: stage with MQ_STAGE_EXPAND=0, the lane-scattered bitmap expansion) on
1e9 rows at several selectivities, each output fully checked: K equals the fused
count, positions strictly ascending, every position's value in range (together:
exactly the reference's list)."""
import json
import os
import sys

sys.path[:0] = ['tests', 'oracle']
import torch
from refapi import mq

lib = mq.load(os.environ["MQ_LIB"]) if os.environ.get("MQ_LIB") else mq.load()
mq.check(lib.mq_init(0))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
impls = sys.argv[2].split(',') if len(sys.argv) > 2 else ['stage', 'mask', 'lookback']
col = torch.empty(n, dtype=torch.int32, device='cuda')
mq.check(lib.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
ws_b = lib.mq_scan_workspace_bytes(n)
ws = torch.empty(ws_b, dtype=torch.uint8, device='cuda')
pos = torch.empty(n, dtype=torch.int32, device='cuda')
cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
agg = torch.zeros(4, dtype=torch.int64, device='cuda')
res = {}
for sel in (0.001, 0.01, 0.1, 0.5, 1.0):
    lo = n // 4
    hi = lo + int(sel * n)
    mq.check(lib.mq_select_agg(col.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(), ws.data_ptr(), ws_b, 0))
    want = int(agg[0].item())
    for impl in impls:
        # stage_lanes: k_select_stage with the lane-scattered bitmap expansion (MQ_STAGE_EXPAND=0)
        os.environ['MQ_POSITIONS_IMPL'] = 'stage' if impl.startswith('stage') else impl
        os.environ['MQ_STAGE_EXPAND'] = '0' if impl == 'stage_lanes' else '1'

        def run():
            mq.check(lib.mq_select_positions(col.data_ptr(), None, n, 1, lo, 1, hi, pos.data_ptr(),
                                             cnt.data_ptr(), ws.data_ptr(), ws_b, 0))
        pos.fill_(-7)
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        k = int(cnt.item())
        p = pos[:k]
        ok = k == want
        if k > 1:
            ok = ok and bool((p[1:] > p[:-1]).all().item())
        if k:
            ok = ok and int(p[0]) >= 0 and int(p[-1]) < n
            v = col[p.long()]
            ok = ok and bool(((v >= lo) & (v < hi)).all().item())
        res.setdefault(impl, {})[sel] = {"ms": round(ms, 4), "k": k, "ok": ok,
                                         "gbs_alg": round((4 * n + 4 * k) / ms / 1e6, 1)}
        del p
for impl, r in res.items():
    print(impl, json.dumps(r), flush=True)
