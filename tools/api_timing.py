"""Host-side timing of the drop-in API chain (config 3: select_column -> fetch_column
-> average) on resident columns, with MQ_TRACE=1 phase times on stderr.

  python tools/api_timing.py [--rows N] [--backing anon|memfd] [--reps R]
  (MQ_GUARD=0 disables the write guards; run each variant in its own process)
"""
import argparse
import ctypes as C
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import refcpu  # noqa: E402  (input generator)
from refapi import make_column, mq, _libc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--backing", default="memfd")
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    n = a.rows
    keep = []

    def column(seed):
        if a.backing == "memfd":
            fd = os.memfd_create(f"c{seed}")
            os.ftruncate(fd, 4 * n)
            m = mmap.mmap(fd, 4 * n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            os.close(fd)
            keep.append(m)
            v = np.frombuffer(m, dtype=np.int32)
        else:
            v = np.empty(n, dtype=np.int32)
        refcpu.lib().rc_gen_uniform(v.ctypes.data, n, seed, n, 16)
        return v

    c0, c1 = column(42), column(43)
    lib = mq.load(os.environ["MQ_LIB"]) if os.environ.get("MQ_LIB") else mq.load()
    mq.check(lib.mq_init(0), "init")
    col0, col1 = make_column(c0, b"c0"), make_column(c1, b"c1")
    t0 = time.perf_counter()
    mq.check(lib.mq_column_upload(C.byref(col0)), "up0")
    mq.check(lib.mq_column_upload(C.byref(col1)), "up1")
    print(f"upload {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    lo, hi = C.c_int(n // 4), C.c_int(n // 4 + n // 100)
    for rep in range(a.reps):
        st = mq.Status(0, None)
        print(f"--- rep {rep}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        rp = lib.select_column(C.byref(col0), C.byref(lo), C.byref(hi), C.byref(st))
        t1 = time.perf_counter()
        rf = lib.fetch_column(C.byref(col1), rp, C.byref(st))
        t2 = time.perf_counter()
        ra = lib.average(rf, C.byref(st))
        t3 = time.perf_counter()
        for r in (rp, rf, ra):
            _libc.free(r.contents.payload)
            _libc.free(r)
        t4 = time.perf_counter()
        print(f"rep {rep}: select {1e3*(t1-t0):.2f} fetch {1e3*(t2-t1):.2f} avg {1e3*(t3-t2):.2f} "
              f"free {1e3*(t4-t3):.2f} ms", flush=True)
    print(mq.residency(lib))


if __name__ == "__main__":
    main()
