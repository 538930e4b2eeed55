"""Exact (Lomuto-order) index build at 2^27 rows: wall time per call and, under
rocprofv3 --kernel-trace --stats, the per-kernel split (not product code).
  python tools/lomuto_prof.py [logn] [reps]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load(os.environ["MQ_LIB"]) if os.environ.get("MQ_LIB") else mq.load()
mq.check(L.mq_init(0))
logn = int(sys.argv[1]) if len(sys.argv) > 1 else 27
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = 1 << logn
c = torch.empty(n, dtype=torch.int32, device="cuda")
mq.check(L.mq_gen_uniform(c.data_ptr(), n, 42, n, None))
v = torch.empty(n, dtype=torch.int32, device="cuda")
p = torch.empty(n, dtype=torch.int64, device="cuda")
for r in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mq.check(L.mq_index_build_lomuto(c.data_ptr(), n, v.data_ptr(), p.data_ptr(), None))
    torch.cuda.synchronize()
    print(f"rep {r}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
