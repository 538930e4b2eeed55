"""Load-path timing (not product code): a rows x ncols int32 table (SURVEY §8(c)
generator, seeds 42..) formatted as CSV text in HBM, then mq_csv_count_rows +
mq_csv_parse_int32 timed with HIP events on the library stream; checks the parsed
columns against the originals.
    python tools/load_bench.py [rows] [ncols] [reps]
MQ_LIB=<path to another libmq.so build> times that build instead (A/B of kernel variants).
"""
import ctypes as C
import json
import sys
import time

sys.path[:0] = ["tests", "oracle"]
import os  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ['MQ_LIB']) if os.environ.get('MQ_LIB') else mq.load()
mq.check(L.mq_init(0))
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
ncols = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda")
cols = [torch.empty(rows, dtype=torch.int32, device=dev) for _ in range(ncols)]
for j, c in enumerate(cols):
    mq.check(L.mq_gen_uniform(c.data_ptr(), rows, 42 + j, rows, 0))
fws = torch.empty(L.mq_format_csv_workspace_bytes(rows, ncols), dtype=torch.uint8, device=dev)
text = torch.empty(rows * ncols * 11 + 16, dtype=torch.uint8, device=dev)
ptrs = (C.c_void_p * ncols)(*[c.data_ptr() for c in cols])
nbytes = C.c_uint64()
mq.check(L.mq_format_csv_int32(ptrs, ncols, rows, text.data_ptr(), C.byref(nbytes), fws.data_ptr(),
                               fws.numel(), 0))
del fws
n = nbytes.value
ws = torch.empty(L.mq_csv_workspace_bytes(n, ncols), dtype=torch.uint8, device=dev)
outs = [torch.empty(rows, dtype=torch.int32, device=dev) for _ in range(ncols)]
optrs = (C.c_void_p * ncols)(*[o.data_ptr() for o in outs])
mm = torch.empty(2 * ncols, dtype=torch.int32, device=dev)
st = L.mq_default_stream()
ts = torch.cuda.ExternalStream(st)
got = C.c_uint64()
res = []
for r in range(reps + 1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a, b, c2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    a.record(ts)
    mq.check(L.mq_csv_count_rows(text.data_ptr(), n, ncols, C.byref(got), ws.data_ptr(), ws.numel(), st))
    b.record(ts)
    mq.check(L.mq_csv_parse_int32(text.data_ptr(), n, ncols, optrs, got.value, mm.data_ptr(),
                                  ws.data_ptr(), ws.numel(), st))
    c2.record(ts)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if r:
        res.append((a.elapsed_time(b), b.elapsed_time(c2), wall * 1e3))
ok = got.value == rows and all(torch.equal(o, c) for o, c in zip(outs, cols))
ok = ok and all(int(mm[2 * j]) == int(c.min()) and int(mm[2 * j + 1]) == int(c.max())
                for j, c in enumerate(cols))
med = np.median(np.array(res), axis=0)
print(json.dumps({"rows": rows, "ncols": ncols, "text_bytes": n, "ok": bool(ok),
                  "ms_count": round(float(med[0]), 3), "ms_parse": round(float(med[1]), 3),
                  "ms_wall": round(float(med[2]), 3),
                  "text_gbs": round(n / (med[0] + med[1]) / 1e6, 1),
                  "rows_per_s": rows / ((med[0] + med[1]) * 1e-3)}))
