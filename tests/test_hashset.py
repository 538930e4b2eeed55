"""J4: hashset.c (src/hashset.c:11-65) — libmq's drop-in of hashset.h and its device
side (mq_hashset_lookup / mq_hashset_elements), against the reference's own
hashset.c compiled unchanged into oracle/_ref/libref.so and the restatement in
oracle/refcpu.py.

The reference mallocs the slots uninitialised (hashset.c:13); the tests zero them
after create_hashset so its 0-means-empty rule holds. Its get_hashset_elements
writes past a 16-byte buffer beyond 4 elements (hashset.c:49), so it is called only
on sets of at most 4; larger listings are checked against the table itself. A
negative key makes it index keys[negative]: negative keys are compared against the
restatement only.
"""
import ctypes as C

import numpy as np
import pytest

from refapi import mq, _libc

class _Hashset(C.Structure):
    _fields_ = [("keys", C.POINTER(C.c_int32)), ("size", C.c_int)]


def _bind(lib):
    lib.create_hashset.restype = C.POINTER(_Hashset)
    lib.create_hashset.argtypes = [C.c_int]
    lib.insert_hashset.argtypes = [C.POINTER(_Hashset), C.c_int]
    lib.insert_hashset.restype = None
    lib.lookup_hashset.argtypes = [C.POINTER(_Hashset), C.c_int]
    lib.lookup_hashset.restype = C.c_bool
    lib.get_hashset_elements.argtypes = [C.POINTER(_Hashset)]
    lib.get_hashset_elements.restype = C.POINTER(mq.Result)
    lib.free_hashset.argtypes = [C.POINTER(_Hashset)]
    lib.free_hashset.restype = None
    return lib


def _table(hs) -> np.ndarray:
    s = hs.contents
    return np.ctypeslib.as_array(s.keys, shape=(s.size,)).copy()


def _elements(lib, hs) -> np.ndarray:
    r = lib.get_hashset_elements(hs)
    assert r, "get_hashset_elements returned NULL"
    n = r.contents.num_tuples
    out = np.ctypeslib.as_array(C.cast(r.contents.payload, C.POINTER(C.c_int32)), shape=(n,)).copy() if n else \
        np.empty(0, np.int32)
    _libc.free(r.contents.payload)
    _libc.free(r)
    return out


@pytest.fixture(scope="module")
def ref(refcpu):
    if not refcpu.have_reference():
        pytest.skip("reference library not built")
    return _bind(refcpu.reference())


@pytest.fixture(scope="module")
def lib():
    return _bind(mq.load())


def _ref_create(ref, size):
    hs = ref.create_hashset(size)
    C.memset(hs.contents.keys, 0, size * 4)  # the reference leaves them uninitialised
    return hs


CASES = {
    "distinct": (101, [5, 17, 3, 99, 42, 7]),
    "collide": (10, [3, 13, 23, 33, 3, 43, 4]),        # one cluster, a duplicate, a neighbour
    "wrap": (8, [7, 15, 23, 6, 14]),                   # probes wrap past the last slot
    "zero": (16, [0, 16, 32, 0, 1]),                   # 0 is the empty marker: never stored
    "dense": (64, list(range(1, 60))),
    "big_keys": (97, [2**31 - 1, 2**31 - 98, 12345678, 97 * 1000]),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_restatement_vs_reference(ref, refcpu, name):
    size, keys = CASES[name]
    hs = _ref_create(ref, size)
    for k in keys:
        ref.insert_hashset(hs, k)
    t = _table(hs)
    assert np.array_equal(t, refcpu.hashset_table(keys, size)), name
    for k in set(keys) | {0, 1, size, 2 * size + 1, 123456}:
        assert bool(ref.lookup_hashset(hs, k)) == refcpu.hashset_lookup(t, k), (name, k)
    if np.count_nonzero(t) <= 4:  # the reference's listing buffer holds 4
        assert np.array_equal(_elements(ref, hs), refcpu.hashset_elements(t)), name
    ref.free_hashset(hs)


@pytest.mark.parametrize("name", sorted(CASES))
def test_libmq_host_api_vs_reference(ref, lib, refcpu, name):
    size, keys = CASES[name]
    a, b = _ref_create(ref, size), lib.create_hashset(size)
    for k in keys:
        ref.insert_hashset(a, k)
        lib.insert_hashset(b, k)
    ta, tb = _table(a), _table(b)
    assert np.array_equal(ta, tb), name
    for k in set(keys) | {0, 1, size, 2 * size + 1, 123456}:
        assert bool(lib.lookup_hashset(b, k)) == bool(ref.lookup_hashset(a, k)), (name, k)
    assert np.array_equal(_elements(lib, b), refcpu.hashset_elements(ta)), name  # host listing
    ref.free_hashset(a)
    lib.free_hashset(b)


def test_libmq_negative_and_full(lib, refcpu):
    """Where the reference has no defined behaviour: negative keys (keys[negative])
    and a full table (endless probe); libmq follows the restatement."""
    keys = [-1, -11, -21, 9, -5, 0, -2**31]
    b = lib.create_hashset(10)
    for k in keys:
        lib.insert_hashset(b, k)
    t = _table(b)
    assert np.array_equal(t, refcpu.hashset_table(keys, 10))
    for k in keys + [-31, 19, 1]:
        assert bool(lib.lookup_hashset(b, k)) == refcpu.hashset_lookup(t, k), k
    lib.free_hashset(b)
    full = lib.create_hashset(4)
    for k in [1, 2, 3, 4, 5]:  # the fifth finds no slot: dropped, no hang
        lib.insert_hashset(full, k)
    assert np.array_equal(_table(full), refcpu.hashset_table([1, 2, 3, 4, 5], 4))
    assert not lib.lookup_hashset(full, 5) and lib.lookup_hashset(full, 4)
    lib.free_hashset(full)


@pytest.mark.gpu
def test_gpu_elements_and_lookup(lib, refcpu):
    """A 2^20 + 7-slot set filled to ~2/3 through libmq's insert_hashset: the listing
    takes the GPU path (>= 32768 slots) and must equal the nonzero slots in order;
    mq_hashset_lookup on 3e5 probes (members, non-members, 0, negatives) must equal
    lookup_hashset's answers."""
    from devbuf import Dev
    size = (1 << 20) + 7
    rng = np.random.default_rng(11)
    keys = rng.integers(-2**31, 2**31 - 1, 700_000, dtype=np.int64).astype(np.int32)
    keys[::97] = 0
    keys[1::89] = keys[::89][: len(keys[1::89])]  # duplicates
    b = lib.create_hashset(size)
    for k in keys.tolist():
        lib.insert_hashset(b, k)
    t = _table(b)
    got = _elements(lib, b)
    assert np.array_equal(got, t[t != 0])
    probes = np.concatenate([keys[:150_000], rng.integers(-2**31, 2**31 - 1, 150_000).astype(np.int32),
                             np.array([0, -1, 1, 2**31 - 1, -2**31], np.int32)])
    dt, dp = Dev.of(t), Dev.of(probes)
    df = Dev(len(probes))
    mq.check(lib.mq_hashset_lookup(dt.ptr, size, dp.ptr, len(probes), df.ptr, None))
    found = df.get(np.uint8, len(probes)).astype(bool)
    want = np.array([lib.lookup_hashset(b, int(k)) for k in probes.tolist()], dtype=bool)
    assert np.array_equal(found, want)
    assert np.array_equal(found[:150_000], keys[:150_000] != 0)  # every inserted nonzero key is a member
    lib.free_hashset(b)
