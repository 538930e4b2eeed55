"""A/B of the ordered-compaction paths on 1e9 rows (look-back vs mask+compact), several selectivities."""
import ctypes as C, os, subprocess, sys, json
sys.path[:0] = ['tests', 'oracle']
import numpy as np
import torch
from refapi import mq
lib = mq.load(); mq.check(lib.mq_init(0))
n = 1_000_000_000
col = torch.empty(n, dtype=torch.int32, device='cuda')
mq.check(lib.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
ws_b = lib.mq_scan_workspace_bytes(n)
ws = torch.empty(ws_b, dtype=torch.uint8, device='cuda')
pos = torch.empty(n, dtype=torch.int32, device='cuda')
cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
res = {}
for sel in (0.001, 0.01, 0.1, 0.5, 1.0):
    lo = n // 4; hi = lo + int(sel * n)
    def run():
        mq.check(lib.mq_select_positions(col.data_ptr(), None, n, 1, lo, 1, hi, pos.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws_b, 0))
    for _ in range(2): run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(10): run()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    k = int(cnt.item())
    p = pos[:k]
    ok = bool((p[1:] > p[:-1]).all().item()) if k > 1 else True
    if k:
        ok = ok and int(p[0]) >= 0 and int(p[-1]) < n
    res[sel] = {"ms": round(ms, 4), "k": k, "gbs_alg": round((4 * n + 4 * k) / ms / 1e6, 1), "sorted": ok}
print(os.environ.get("MQ_POSITIONS_IMPL", "lookback"), json.dumps(res))
