"""Diagnostic (not product code): k_select_stage's phases at 10 / 50 % on 1e9 rows, positions
and select_result, with MQ_STAGE_EXPAND = 1 (default), 2 (no bitmap expansion: the scan
and prefix alone), 3 (bitmap words read and counted, nothing placed) and 4 (+ the payload
rows of every tile with a match loaded, nothing placed). HIP events, median of 5. Outputs
of modes 2-4 are incomplete by design. (Round 5 also ran a mode 5, the payload loads of
the next two tiles issued before the current two were placed: same output, no faster,
removed; profiles/r05_stage_diag5.log.)"""
import json
import os
import sys
sys.path[:0] = ['tests', 'oracle']
import torch
from refapi import mq
lib = mq.load()
mq.check(lib.mq_init(0))
n = 1_000_000_000
col = torch.empty(n, dtype=torch.int32, device='cuda'); pay = torch.empty(n, dtype=torch.int32, device='cuda')
mq.check(lib.mq_gen_uniform(col.data_ptr(), n, 42, n, 0)); mq.check(lib.mq_gen_uniform(pay.data_ptr(), n, 43, n, 0))
ws_b = lib.mq_scan_workspace_bytes(n); ws = torch.empty(ws_b, dtype=torch.uint8, device='cuda')
pos = torch.empty(n, dtype=torch.int32, device='cuda'); cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
res = {}
for mode in ("1", "2", "3", "4"):
    os.environ["MQ_STAGE_EXPAND"] = mode
    for sel in (0.1, 0.5):
        lo = n // 4; hi = lo + int(sel * n)
        for name, p in (("positions", None), ("select_result", pay.data_ptr())):
            ms = []
            for r in range(6):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(); mq.check(lib.mq_select_positions(col.data_ptr(), p, n, 1, lo, 1, hi, pos.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws_b, 0)); b.record(); b.synchronize()
                if r: ms.append(a.elapsed_time(b))
            ms.sort(); res[f"x{mode}_{sel}_{name}"] = round(ms[len(ms)//2], 3)
print(json.dumps(res))
