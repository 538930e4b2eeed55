"""A/B (not product code): shared_select on the 1e9-row column for small Q, the
per-query ballot pass (default below kEiMinQ) against the k-major elementary-interval
pass forced by MQ_SS_EI_MIN=1; count + write wall time, outputs compared.
usage: python tools/ss_qsmall_ab.py 2,4,8,16 [selectivity per query, default 0.001]
(MQ_SS_EI_MIN=1000 forces the ballot pass as the A side when the default is k-major)"""
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
variants = {"ballot": {"MQ_SS_EI_MIN": "1000"}, "ei_min1": {"MQ_SS_EI_MIN": "1"}}
sel = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001
w = int(sel * n)
for q in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,16").split(",")]:
    rng = np.random.default_rng(5)
    lows = rng.integers(0, n - w, q).astype(np.int32)
    highs = (lows + w).astype(np.int32)
    lo_c = (C.c_int32 * q)(*lows.tolist())
    hi_c = (C.c_int32 * q)(*highs.tolist())
    wsb = L.mq_shared_select_workspace_bytes(n, q)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    row, prev = {}, None
    for rnd in range(2):
        for name, env in variants.items():
            for k_ in ("MQ_SS_EI_MIN",):
                os.environ.pop(k_, None)
            os.environ.update(env)
            k = (C.c_uint64 * q)()
            ts = []
            for rep in range(7):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                mq.check(L.mq_shared_select_count(col.data_ptr(), n, lo_c, hi_c, q, k, ws.data_ptr(), wsb, 0))
                outs = [torch.empty(max(int(x), 1), dtype=torch.int32, device="cuda") for x in k]
                ptrs = (C.c_void_p * q)(*[o.data_ptr() for o in outs])
                mq.check(L.mq_shared_select_write(ws.data_ptr(), ptrs, 0))
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            row[f"{name}_{rnd}"] = 1e3 * sorted(ts)[3]
            if prev is not None:
                row.setdefault("same_output", True)
                row["same_output"] &= all(torch.equal(a, b) for a, b in zip(prev, outs))
            prev = outs
    res[f"q{q}_sel{sel}"] = row
    print(json.dumps({f"q{q}_sel{sel}": row}), flush=True)
os.environ.pop("MQ_SS_EI_MIN", None)
print(json.dumps(res))
