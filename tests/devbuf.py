"""Device buffers through libmq's own allocator (GPU tests need no torch)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from refapi import mq


class Dev:
    def __init__(self, nbytes: int):
        self.lib = mq.load()
        p = C.c_void_p()
        mq.check(self.lib.mq_malloc(C.byref(p), max(int(nbytes), 16)), "mq_malloc")
        self.p = p.value
        self.nbytes = int(nbytes)

    @classmethod
    def of(cls, arr: np.ndarray, offset_elems: int = 0) -> "Dev":
        """Copy arr to the device, optionally starting offset_elems into the buffer
        (to exercise unaligned column pointers)."""
        arr = np.ascontiguousarray(arr)
        d = cls(arr.nbytes + offset_elems * arr.itemsize + 16)
        d.off = offset_elems * arr.itemsize
        if arr.nbytes:
            mq.check(d.lib.mq_memcpy_h2d(d.p + d.off, arr.ctypes.data, arr.nbytes, None), "h2d")
        return d

    off = 0

    @property
    def ptr(self) -> int:
        return self.p + self.off

    def get(self, dtype, count: int, byte_offset: int = 0) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            mq.check(self.lib.mq_stream_sync(None), "sync")
            mq.check(self.lib.mq_memcpy_d2h(out.ctypes.data, self.ptr + byte_offset, out.nbytes,
                                            None), "d2h")
        return out

    def free(self) -> None:
        if self.p:
            self.lib.mq_free(self.p)
            self.p = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
