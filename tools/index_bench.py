"""Index-build timing (not product code): mq_index_build on an n-row uniform column
(seed 42), HIP events on the library stream, median of reps after one warm-up."""
import os
import sys
import time

sys.path[:0] = ["tests", "oracle"]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ['MQ_LIB']) if os.environ.get('MQ_LIB') else mq.load()
mq.check(L.mq_init(0))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
col = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(col.data_ptr(), n, 42, n, 0))
v = torch.empty(n, dtype=torch.int32, device="cuda")
p = torch.empty(n, dtype=torch.int64, device="cuda")
st = L.mq_default_stream()
ts = torch.cuda.ExternalStream(st)
ms = []
for r in range(reps + 1):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(ts)
    mq.check(L.mq_index_build(col.data_ptr(), n, v.data_ptr(), p.data_ptr(), st))
    b.record(ts)
    torch.cuda.synchronize()
    if r:
        ms.append(a.elapsed_time(b))
ok = bool((v[1:] >= v[:-1]).all()) and bool(torch.equal(col[p], v))
ms.sort()
print({"n": n, "ms_median": ms[len(ms) // 2], "ok": ok, "rows_per_s": n / (ms[len(ms) // 2] * 1e-3)})
