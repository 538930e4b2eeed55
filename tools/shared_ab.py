"""A/B of shared_select on the 1e9-row column (not product code): Q range queries of
0.1 % each, count + write, elementary-interval kernels (default for Q >= 24) vs the
per-query ballot kernels (MQ_SS_IMPL=ballot); outputs compared between the two."""
import ctypes as C
import json
import os
import sys
import time

sys.path[:0] = ["tests", "oracle"]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ['MQ_LIB']) if os.environ.get('MQ_LIB') else mq.load()
mq.check(L.mq_init(0))
n = 1_000_000_000
col = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
res = {}
for q in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "24,64,150,256").split(",")]:
    rng = np.random.default_rng(5)
    lows = rng.integers(0, n - n // 1000, q).astype(np.int32)
    highs = (lows + n // 1000).astype(np.int32)
    lo_c = (C.c_int32 * q)(*lows.tolist())
    hi_c = (C.c_int32 * q)(*highs.tolist())
    wsb = L.mq_shared_select_workspace_bytes(n, q)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    row = {}
    prev = None
    for impl in ("ei", "ballot"):
        if impl == "ballot":
            os.environ["MQ_SS_IMPL"] = "ballot"
        else:
            os.environ.pop("MQ_SS_IMPL", None)
        k = (C.c_uint64 * q)()
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mq.check(L.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, 0))
            t1 = time.perf_counter()
            outs = [torch.empty(max(int(x), 1), dtype=torch.int32, device="cuda") for x in k]
            ptrs = (C.c_void_p * q)(*[o.data_ptr() for o in outs])
            mq.check(L.mq_shared_select_write(ws.data_ptr(), ptrs, 0))
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ts.append((t1 - t0, t2 - t1))
        ts.sort()
        row[impl] = {"ms_count": 1e3 * ts[1][0], "ms_write": 1e3 * ts[1][1], "k_total": int(sum(k))}
        if prev is not None:
            row["same_output"] = all(torch.equal(a, b) for a, b in zip(prev, outs))
        prev = outs
    res[f"q{q}"] = row
os.environ.pop("MQ_SS_IMPL", None)
print(json.dumps(res))
