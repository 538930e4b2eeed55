"""shared_select kernels on the 1e9-row column for rocprofv3 --kernel-trace --stats
(not product code): Q range queries of 0.1 % each, count + write, REPS times each.
  python tools/shared_prof.py [Q,Q,...] [reps]"""
import ctypes as C
import os
import sys
import time

sys.path[:0] = ["tests", "oracle"]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ["MQ_LIB"]) if os.environ.get("MQ_LIB") else mq.load()
mq.check(L.mq_init(0))
n = 1_000_000_000
col = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
qs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,16,150").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for q in qs:
    rng = np.random.default_rng(5)
    lows = rng.integers(0, n - n // 1000, q).astype(np.int32)
    highs = (lows + n // 1000).astype(np.int32)
    lo_c = (C.c_int32 * q)(*lows.tolist())
    hi_c = (C.c_int32 * q)(*highs.tolist())
    wsb = L.mq_shared_select_workspace_bytes(n, q)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    k = (C.c_uint64 * q)()
    mq.check(L.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, 0))
    outs = [torch.empty(max(int(x), 1), dtype=torch.int32, device="cuda") for x in k]
    ptrs = (C.c_void_p * q)(*[o.data_ptr() for o in outs])
    ts = []
    for rep in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mq.check(L.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, 0))
        mq.check(L.mq_shared_select_write(ws.data_ptr(), ptrs, 0))
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"q={q} ms={1e3 * ts[0]:.3f} median={1e3 * ts[len(ts) // 2]:.3f} k={sum(k)}", flush=True)
