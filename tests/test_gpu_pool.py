"""The caching device allocator's stream-ordered free (-m gpu).

mq_pool_free_on(p, stream) returns a block while work queued on `stream` may still
write it; the block must not be handed out again before that work has finished. The
join handle (mq_join_probe / mq_join_free) and the shard workers now free this way
instead of synchronising the whole device.
"""
import ctypes as C

import numpy as np
import pytest

from refapi import mq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    L = mq.load()
    mq.check(L.mq_init(0), "mq_init")
    return L


def test_ordered_free_is_not_reused_while_queued_writers_run(lib):
    """200 writes of 2^26 rows (~30 ms) queued on stream A into block X, X freed on A at
    once, then the same size allocated: while A's writes are queued X is not handed out
    (round 6, ADVICE r05: a fresh block instead of a wait, so callers on other streams
    never wait for each other; the wait is left for when no fresh block fits). A write of
    iota into the new block is its final content, and once A has finished X is reused."""
    n = 1 << 26
    lib.mq_trim()  # no other idle block of this size to pick instead
    a = C.c_void_p()
    mq.check(lib.mq_stream_create(C.byref(a)), "stream")
    x = C.c_void_p()
    mq.check(lib.mq_pool_malloc(C.byref(x), n * 4), "pool_malloc")
    for _ in range(200):
        mq.check(lib.mq_gen_join_keys(x, n, 1, a), "gen")
    mq.check(lib.mq_pool_free_on(x, a), "pool_free_on")
    y = C.c_void_p()
    mq.check(lib.mq_pool_malloc(C.byref(y), n * 4), "pool_malloc")
    assert y.value != x.value  # X's free is still in flight
    mq.check(lib.mq_gen_iota(y, n, None), "iota")
    mq.check(lib.mq_stream_sync(None), "sync")
    mq.check(lib.mq_stream_sync(a), "sync")
    out = np.empty(n, dtype=np.int32)
    mq.check(lib.mq_memcpy_d2h(out.ctypes.data, y, out.nbytes, None), "d2h")
    assert np.array_equal(out, np.arange(n, dtype=np.int32))
    z = C.c_void_p()
    mq.check(lib.mq_pool_malloc(C.byref(z), n * 4), "pool_malloc")
    assert z.value == x.value  # A has finished: X is idle again, the best fit
    lib.mq_pool_free(z)
    lib.mq_pool_free(y)
    mq.check(lib.mq_stream_destroy(a), "stream destroy")


def test_ordered_free_of_idle_block_is_reused_at_once(lib):
    """A block freed on an idle stream is reusable straight away (no new allocation)."""
    lib.mq_trim()
    a = C.c_void_p()
    mq.check(lib.mq_stream_create(C.byref(a)), "stream")
    x = C.c_void_p()
    mq.check(lib.mq_pool_malloc(C.byref(x), 1 << 20), "pool_malloc")
    mq.check(lib.mq_pool_free_on(x, a), "pool_free_on")
    mq.check(lib.mq_stream_sync(a), "sync")
    y = C.c_void_p()
    mq.check(lib.mq_pool_malloc(C.byref(y), 1 << 20), "pool_malloc")
    assert y.value == x.value
    lib.mq_pool_free(y)
    mq.check(lib.mq_stream_destroy(a), "stream destroy")


def test_mq_malloc_pointer_through_ordered_free(lib):
    """A pointer that is not the pool's (mq_malloc) is freed after its stream drains."""
    a = C.c_void_p()
    mq.check(lib.mq_stream_create(C.byref(a)), "stream")
    p = C.c_void_p()
    mq.check(lib.mq_malloc(C.byref(p), 1 << 24), "malloc")
    mq.check(lib.mq_gen_iota(p, 1 << 22, a), "iota")
    mq.check(lib.mq_pool_free_on(p, a), "pool_free_on")
    mq.check(lib.mq_device_sync(), "device sync")
    mq.check(lib.mq_stream_destroy(a), "stream destroy")
