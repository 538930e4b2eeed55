"""A/B of the config-3 fused path (not product code): mq_select_fetch_agg on the
1e9-row columns seeds 42 (select) / 43 (fetch) at 1 %, with the deferred-gather
kernel (default) and k_scan<kAux> (MQ_AUX_IMPL=inline); checks the SURVEY §8(c)
config-3 golden (K, sum, min, max) each time."""
import json
import os
import sys

sys.path[:0] = ["tests", "oracle"]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load()
mq.check(L.mq_init(0))
n = 1_000_000_000
c0 = torch.empty(n, dtype=torch.int32, device="cuda")
c1 = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(c0.data_ptr(), n, 42, n, 0))
mq.check(L.mq_gen_uniform(c1.data_ptr(), n, 43, n, 0))
wsb = L.mq_scan_workspace_bytes(n)
ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
agg = torch.zeros(4, dtype=torch.int64, device="cuda")
lo, hi = 250_000_000, 260_000_000
want = (10001128, 5000678708721025, 142, 999999983)
res = {}
for impl in ("gather", "inline", "gather"):
    if impl == "inline":
        os.environ["MQ_AUX_IMPL"] = "inline"
    else:
        os.environ.pop("MQ_AUX_IMPL", None)
    ms = []
    for r in range(11):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mq.check(L.mq_select_fetch_agg(c0.data_ptr(), c1.data_ptr(), n, 1, lo, 1, hi, agg.data_ptr(),
                                       ws.data_ptr(), wsb, 0))
        b.record()
        b.synchronize()
        if r:
            ms.append(a.elapsed_time(b))
    raw = agg.cpu()
    got = (int(raw[0]), int(raw[1]), int(raw[2].view(torch.int32)[0]) if False else None, None)
    a32 = agg.view(torch.int32).cpu()
    got = (int(raw[0]), int(raw[1]), int(a32[4]), int(a32[5]))
    ms.sort()
    res[impl] = {"ms_median": ms[len(ms) // 2], "ms_best": ms[0], "ok": got == want, "got": got}
print(json.dumps(res))
