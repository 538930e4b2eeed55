"""Fused-scan variants on the 1e9-row column (not product code): select + count + sum
(mq_select_sum, the headline) against select + count + sum + min + max
(mq_select_agg, the API's sum/min/max of a column), HIP events, median of 10."""
import json
import sys

sys.path[:0] = ["tests", "oracle"]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load()
mq.check(L.mq_init(0))
n = 1_000_000_000
col = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
wsb = L.mq_scan_workspace_bytes(n)
ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
agg = torch.zeros(4, dtype=torch.int64, device="cuda")
lo, hi = n // 4, n // 4 + n // 100
res = {}
for name, fn in (("select_sum", L.mq_select_sum), ("select_agg", L.mq_select_agg)):
    ms = []
    for r in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mq.check(fn(col.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(), ws.data_ptr(), wsb, 0))
        b.record()
        b.synchronize()
        if r >= 2:
            ms.append(a.elapsed_time(b))
    ms.sort()
    res[name] = {"ms": ms[len(ms) // 2], "gbs": 4 * n / ms[len(ms) // 2] / 1e6}
print(json.dumps(res))
