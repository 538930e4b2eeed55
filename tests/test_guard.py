"""Write guards on host memory mirrored in HBM (csrc/mq_guard.c), checked on the CPU.

The guard is how libmq knows that a Column's rows (or a Result payload) are still
what it uploaded: the reference rewrites column data in place through the same
mmap'd pointer (src/index.c:105-114 reorder_column) and appends through it
(src/db_manager.c:190-197 insert_row). No GPU is involved here: these are host
page-protection mechanics, exercised through libmq.so's own entry points.
"""
import ctypes as C
import mmap
import os
import subprocess
import sys

import numpy as np
import pytest

from refapi import mq

PAGE = mmap.PAGESIZE
libc = C.CDLL(None, use_errno=True)
libc.malloc.restype = C.c_void_p
libc.malloc.argtypes = [C.c_size_t]
libc.free.argtypes = [C.c_void_p]
libc.mmap.restype = C.c_void_p
libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
libc.memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
libc.memset.restype = C.c_void_p


@pytest.fixture(scope="module")
def lib():
    return mq.load()


def memfd_array(n, fill=None):
    """n int32 in a MAP_SHARED memfd mapping (a file-backed column, as start_data makes)."""
    fd = os.memfd_create("mqcol")
    os.ftruncate(fd, n * 4)
    m = mmap.mmap(fd, n * 4, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    a = np.frombuffer(m, dtype=np.int32)
    a[:] = np.arange(n, dtype=np.int32) if fill is None else fill
    return a, m


def test_file_mapping_clean_until_written(lib):
    a, m = memfd_array(1 << 16)
    h = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    assert h
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 1
    assert int(a[12345]) == 12345  # reads do not disturb it
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 1
    a[40000] = -7  # an in-place store: faults once, the handler lets it through
    assert int(a[40000]) == -7
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 0
    a[40001] = -8  # the pages are writable again: no second fault needed
    lib.mq_guard_release(h)
    del a
    m.close()


def test_same_range_armed_twice_shares_one_guard(lib):
    """A column resident both whole on one device and split over row shards arms the
    same range twice: the second arm joins the first guard (a second mprotect guard
    could not arm over read-only pages); one release leaves it armed for the other
    owner, a write is seen by both, the last release lifts it."""
    a, m = memfd_array(1 << 16)
    h1 = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    h2 = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    assert h1 and h2 == h1
    lib.mq_guard_release(h1)
    assert lib.mq_guard_clean(h2, a.ctypes.data, a.nbytes) == 1  # still armed for owner 2
    h3 = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    assert h3 == h2
    a[7] = -1
    assert lib.mq_guard_clean(h2, a.ctypes.data, a.nbytes) == 0
    assert lib.mq_guard_clean(h3, a.ctypes.data, a.nbytes) == 0
    lib.mq_guard_release(h2)
    lib.mq_guard_release(h3)
    h4 = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)  # a fresh guard now
    assert h4 and lib.mq_guard_clean(h4, a.ctypes.data, a.nbytes) == 1
    lib.mq_guard_release(h4)
    a[8] = -2  # writable after the last release
    del a
    m.close()


def test_reorder_like_writes_from_c(lib):
    """A write from C code (memset, like reorder_column's memcpy) is seen too."""
    a, m = memfd_array(1 << 15)
    h = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    libc.memset(a.ctypes.data + 8 * PAGE, 0, 4 * PAGE)
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 0
    assert not a[2 * PAGE:3 * PAGE].any()
    lib.mq_guard_release(h)
    del a
    m.close()


def test_partial_edge_pages_are_compared(lib):
    """Bytes outside the whole pages (not protected) are compared with their copy."""
    a, m = memfd_array(PAGE)  # 4 pages
    sub = a[5:PAGE - 3]  # starts and ends inside a page
    h = lib.mq_guard_arm(sub.ctypes.data, sub.nbytes, mq.MQ_GUARD_FILE)
    assert h and lib.mq_guard_clean(h, sub.ctypes.data, sub.nbytes)
    a[3] = 99  # outside the range: no effect
    assert lib.mq_guard_clean(h, sub.ctypes.data, sub.nbytes) == 1
    sub[-1] = 12  # inside the range, on the unprotected tail page
    assert lib.mq_guard_clean(h, sub.ctypes.data, sub.nbytes) == 0
    lib.mq_guard_release(h)
    del a, sub
    m.close()


def test_anonymous_heap_memory_is_not_guarded(lib):
    a = np.arange(1 << 16, dtype=np.int32)
    assert lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE) == 0
    p = libc.malloc(256)  # a heap chunk (not mmapped): freeing it would leave pages behind
    assert lib.mq_guard_arm(p, 256, mq.MQ_GUARD_CHUNK) == 0
    libc.free(p)


def test_mmapped_malloc_chunk(lib):
    n = 64 << 20  # above glibc's largest mmap threshold: served by mmap, freed by munmap
    p = libc.malloc(n)
    libc.memset(p, 1, n)
    h = lib.mq_guard_arm(p, n, mq.MQ_GUARD_CHUNK)
    assert h
    assert lib.mq_guard_clean(h, p, n) == 1
    C.c_char.from_address(p + n // 2).value = b"\x07"
    assert lib.mq_guard_clean(h, p, n) == 0
    lib.mq_guard_release(h)
    libc.free(p)


def test_remapped_range_is_stale(lib):
    """munmap + a fresh mapping at the same address (same length) is not the memory
    that was guarded, even with identical bytes."""
    r = mq.residency(lib)
    if not r["remap_probe"]:
        pytest.skip("kernel without MADV_POPULATE_WRITE: remaps are not told apart")
    n = 16 * PAGE
    PROT_RW, MAP_SHARED_ANON, MAP_FIXED = 3, 0x01 | 0x20, 0x10
    p = libc.mmap(None, n, PROT_RW, MAP_SHARED_ANON, -1, 0)
    fd = os.memfd_create("mqremap")
    os.ftruncate(fd, n)
    libc.munmap(p, n)
    q = libc.mmap(p, n, PROT_RW, 0x01 | MAP_FIXED, fd, 0)
    assert q == p
    h = lib.mq_guard_arm(q, n, mq.MQ_GUARD_FILE)
    assert h and lib.mq_guard_clean(h, q, n)
    libc.munmap(q, n)
    q2 = libc.mmap(p, n, PROT_RW, 0x01 | MAP_FIXED, fd, 0)  # same file, same bytes
    assert q2 == p
    assert lib.mq_guard_clean(h, q2, n) == 0
    lib.mq_guard_release(h)
    libc.munmap(q2, n)
    os.close(fd)


def test_forget_range_lifts_guard(lib):
    a, m = memfd_array(1 << 14)
    h = lib.mq_guard_arm(a.ctypes.data, a.nbytes, mq.MQ_GUARD_FILE)
    lib.mq_guard_forget_range(a.ctypes.data + 100, 8)
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 0
    fd = os.open("/dev/zero", os.O_RDONLY)
    assert os.readv(fd, [memoryview(m)[:PAGE * 2]]) == PAGE * 2
    os.close(fd)
    lib.mq_guard_release(h)
    del a
    m.close()


def test_foreign_segfault_still_terminates(tmp_path):
    """A fault that is not a guard's goes on to the previous handler (here: the
    default action), so real crashes are not swallowed."""
    code = f"""
import ctypes as C, mmap, os, sys
sys.path.insert(0, {os.path.join(os.path.dirname(__file__))!r})
from refapi import mq
import numpy as np
lib = mq.load()
fd = os.memfd_create("x"); os.ftruncate(fd, 1 << 16)
m = mmap.mmap(fd, 1 << 16)
a = np.frombuffer(m, dtype=np.int32)
assert lib.mq_guard_arm(a.ctypes.data, a.nbytes, 0)
a[5] = 1
print("guard-write-ok", flush=True)
C.string_at(8, 8)
print("not reached", flush=True)
"""
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "guard-write-ok" in cp.stdout
    assert "not reached" not in cp.stdout
    assert cp.returncode == -11, (cp.returncode, cp.stderr[-2000:])


def test_guard_disabled_by_env(tmp_path):
    code = """
import sys; sys.path.insert(0, %r)
from refapi import mq
import mmap, os, numpy as np
lib = mq.load()
fd = os.memfd_create("x"); os.ftruncate(fd, 1 << 16)
m = mmap.mmap(fd, 1 << 16); a = np.frombuffer(m, dtype=np.int32)
print(lib.mq_guard_arm(a.ctypes.data, a.nbytes, 0))
""" % os.path.dirname(__file__)
    env = dict(os.environ, MQ_GUARD="0")
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                        env=env)
    assert cp.stdout.strip() == "0", cp.stderr[-2000:]


def test_chunk_check_needs_glibc_mmapped_header(lib):
    """a CHUNK guard is armed only on what looks exactly like glibc's
    mmapped chunk (header at a page start, IS_MMAPPED set, whole pages), so a block
    from another allocator whose size word merely has bit 1 set is refused."""
    base = libc.mmap(None, 4 * PAGE, mmap.PROT_READ | mmap.PROT_WRITE,
                     mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS, -1, 0)
    try:
        words = (C.c_size_t * (PAGE // 8)).from_address(base)
        words[7] = (3 * PAGE) | 2   # size word of a fake chunk at base + 48: not page-aligned
        assert lib.mq_guard_arm(base + 64, 2 * PAGE, mq.MQ_GUARD_CHUNK) == 0
        words[1] = 1000 | 2         # at the page start, but not a whole number of pages
        assert lib.mq_guard_arm(base + 16, 2 * PAGE, mq.MQ_GUARD_CHUNK) == 0
    finally:
        libc.munmap(base, 4 * PAGE)


def test_concurrent_first_writes_into_one_guard():
    """several threads store into the same guarded pages at once; every
    fault after the first finds the guard no longer armed and must re-execute its
    store instead of handing the signal on (which would kill the process)."""
    code = f"""
import ctypes as C, mmap, os, sys, threading
sys.path.insert(0, {os.path.join(os.path.dirname(__file__))!r})
from refapi import mq
import numpy as np
lib = mq.load()
libc = C.CDLL(None)
libc.memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
for rep in range(200):
    fd = os.memfd_create("x"); os.ftruncate(fd, 1 << 20)
    m = mmap.mmap(fd, 1 << 20); os.close(fd)
    a = np.frombuffer(m, dtype=np.uint8)
    h = lib.mq_guard_arm(a.ctypes.data, a.nbytes, 0)
    assert h
    go = threading.Barrier(8)
    def w(i):
        go.wait()
        libc.memset(a.ctypes.data + i * 4096, i + 1, 64)
    ts = [threading.Thread(target=w, args=(i,)) for i in range(8)]
    [t.start() for t in ts]; [t.join() for t in ts]
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 0
    assert all(a[i * 4096] == i + 1 for i in range(8))
    lib.mq_guard_release(h)
    del a; m.close()
print("ok", flush=True)
"""
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert cp.returncode == 0 and "ok" in cp.stdout, (cp.returncode, cp.stderr[-2000:])


def test_retry_table_slots_are_reclaimed():
    """a retried store that succeeds never clears its thread's
    entry in the fault handler's retry table. Entries are dead after RETRY_TTL_NS
    (250 ms): a full table of stale entries takes new threads again, and a thread that
    reuses an old tid does not inherit its tag. Run in a child process (fresh table)."""
    code = f"""
import sys, time
sys.path.insert(0, {os.path.join(os.path.dirname(__file__))!r})
from refapi import mq
lib = mq.load()
for t in range(1, 1025):          # 1024 threads that retried once and never came back
    assert lib.mq_guard_retry_test(t, 0x1001, 0) == 1
assert lib.mq_guard_retry_test(5000, 0x2001, 0) == 0   # full of live entries
assert lib.mq_guard_retry_test(7, 0, 1) == 0x1001
time.sleep(0.4)
assert lib.mq_guard_retry_test(7, 0, 1) == 0           # dead: a reused tid starts clean
for t in range(5000, 6024):        # every dead slot is taken over
    assert lib.mq_guard_retry_test(t, 0x3001, 0) == 1, t
assert lib.mq_guard_retry_test(9000, 0x2001, 0) == 0   # full again, of live entries
assert lib.mq_guard_retry_test(5500, 0, 1) == 0x3001
assert lib.mq_guard_retry_test(5500, 0x5001, 0) == 1   # own entry updated in place
assert lib.mq_guard_retry_test(5500, 0, 1) == 0x5001
assert lib.mq_guard_retry_test(5500, 0, 0) == 1        # cleared
assert lib.mq_guard_retry_test(5500, 0, 1) == 0
print("ok", flush=True)
"""
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert cp.returncode == 0 and "ok" in cp.stdout, (cp.returncode, cp.stdout, cp.stderr[-2000:])


def test_many_short_lived_threads_race_on_guards():
    """More than 1024 short-lived threads, in racing groups of 16 on one guarded page:
    every losing fault is retried (never handed on, which would kill the process)."""
    code = f"""
import ctypes as C, mmap, os, sys, threading
sys.path.insert(0, {os.path.join(os.path.dirname(__file__))!r})
from refapi import mq
import numpy as np
lib = mq.load()
libc = C.CDLL(None)
libc.memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
for rep in range(100):
    fd = os.memfd_create("x"); os.ftruncate(fd, 1 << 16)
    m = mmap.mmap(fd, 1 << 16); os.close(fd)
    a = np.frombuffer(m, dtype=np.uint8)
    h = lib.mq_guard_arm(a.ctypes.data, a.nbytes, 0)
    assert h
    go = threading.Barrier(16)
    def w(i):
        go.wait()
        libc.memset(a.ctypes.data + 4096 + i * 64, i + 1, 64)
    ts = [threading.Thread(target=w, args=(i,)) for i in range(16)]
    [t.start() for t in ts]; [t.join() for t in ts]
    assert lib.mq_guard_clean(h, a.ctypes.data, a.nbytes) == 0
    assert all(a[4096 + i * 64] == i + 1 for i in range(16))
    lib.mq_guard_release(h)
    del a; m.close()
print("ok", flush=True)
"""
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert cp.returncode == 0 and "ok" in cp.stdout, (cp.returncode, cp.stderr[-2000:])
