"""Random-read rate against table size (not product code).

k_random_read (mq_random_read: 2^28 reads of 8 bytes at hashed slots, 8 in flight per
lane, the join probe's pattern without compares) over tables of 2^k u64 slots, from
64 MB (inside the 256 MB Infinity Cache) to 4 GB (the 2^28 join's table). If a table
that fits the Infinity Cache reads >= 2x faster than the 4 GB one, a probe partitioned
into cache-sized slices of the table could pay; otherwise it cannot.
  python tools/random_read_ic.py
"""
import json
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import torch  # noqa: E402
from refapi import mq  # noqa: E402

L = mq.load()
mq.check(L.mq_init(0))
n_reads = 1 << 28
ws = torch.empty(1, dtype=torch.int64, device="cuda")
out = []
for lg in (20, 22, 23, 24, 25, 26, 27, 29):
    t = torch.zeros(1 << lg, dtype=torch.int64, device="cuda")
    ms = []
    for i in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mq.check(L.mq_random_read(t.data_ptr(), lg, n_reads, ws.data_ptr(), None))
        b.record()
        b.synchronize()
        if i:
            ms.append(a.elapsed_time(b))
    m = statistics.median(ms)
    r = {"table_mb": (8 << lg) >> 20, "slots_log2": lg, "reads": n_reads, "ms": m, "g_reads_per_s": n_reads / m / 1e6}
    out.append(r)
    print(json.dumps(r), flush=True)
    del t
base = out[-1]["ms"]
print(json.dumps({"speedup_vs_4gb": {r["table_mb"]: base / r["ms"] for r in out}}))
