"""Config-5 join timing (not product code): 2^logn x 2^logn keys of SURVEY §8(c),
build / probe / write timed separately (wall clock around each step, which ends in
a host sync), median of reps; M checked against the golden."""
import ctypes as C
import json
import statistics
import os
import sys
import time

sys.path[:0] = ["tests", "oracle"]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ['MQ_LIB']) if os.environ.get('MQ_LIB') else mq.load()
mq.check(L.mq_init(0))
logn = int(sys.argv[1]) if len(sys.argv) > 1 else 28
dup = len(sys.argv) > 2 and sys.argv[2] == "dup"  # the many-to-many variant (kinds 2 / 3)
n = 1 << logn
a = torch.empty(n, dtype=torch.int32, device="cuda")
b = torch.empty(n, dtype=torch.int32, device="cuda")
p = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_join_keys(a.data_ptr(), n, 2 if dup else 0, 0))
mq.check(L.mq_gen_join_keys(b.data_ptr(), n, 3 if dup else 1, 0))
mq.check(L.mq_gen_iota(p.data_ptr(), n, 0))
rows = []
o1 = o2 = None
for rep in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = C.c_void_p()
    mq.check(L.mq_join_build(a.data_ptr(), p.data_ptr(), n, C.byref(h), 0))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    mm = C.c_uint64()
    mq.check(L.mq_join_probe(h, b.data_ptr(), n, C.byref(mm), 0))
    t2 = time.perf_counter()
    if o1 is None:
        o1 = torch.empty(mm.value, dtype=torch.int32, device="cuda")
        o2 = torch.empty(mm.value, dtype=torch.int32, device="cuda")
    mq.check(L.mq_join_write(h, p.data_ptr(), o1.data_ptr(), o2.data_ptr(), 0))
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    mq.check(L.mq_join_free(h))
    if rep:
        rows.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
med = [1e3 * statistics.median(r[i] for r in rows) for i in range(4)]
print(json.dumps({"n": n, "m": mm.value, "ms_build": med[0], "ms_probe": med[1], "ms_write": med[2],
                  "ms_total": med[3], "dup": dup,
                  "m_ok": (mm.value == 134232477) if logn == 28 and not dup else None}))
